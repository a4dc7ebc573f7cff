#!/usr/bin/env python3
"""Name the per-sample decisions a minibatch's gradient hangs on (test infrastructure, CPU, this
container only: the REFERENCE rsl_rl through tools/gen_learner_golden.py).

At the reference's own parameters at the start of minibatch i (a tools/ref_update_probe.py
output), this re-forms that minibatch (rollout_storage.py:134-182 with the injected permutation)
and lists the samples whose surrogate decision (ppo.py:250-254: max(-A r, -A clip(r, 1-e, 1+e)))
sits within `tol` (relative) of a tie, i.e. whose clip-boundary side any fp32 rounding of the
log-prob can flip. For each such sample it prints the ratio, the margin, and the change a flip
makes in every actor gradient (the sample's -A grad(r) / mb), relative to max|g| of that tensor —
to be compared with a GPU path's teacher-forced gradient error at that minibatch.

  python tools/ref_minibatch_ties.py <probe.npz> <case> <i> [<i> ...]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen_learner_golden as G  # noqa: E402
import learner_case as LC  # noqa: E402

TOL = float(os.environ.get("TOL", "3e-5"))


def main():
    probe = np.load(sys.argv[1])
    case = sys.argv[2]
    which = [int(x) for x in sys.argv[3:]]
    torch.set_num_threads(8)
    alg = G.build(case)
    scratch = {}
    G.rollout(alg, case, 0, scratch, adaptation_mode=True)
    G._Inject.perm = torch.from_numpy(LC.permutation(case, 0))
    alg.update_dagger()
    G._Inject.perm = None
    G.rollout(alg, case, 1, scratch, adaptation_mode=False)
    G._Inject.perm = torch.from_numpy(LC.permutation(case, 1))
    batches = list(alg.storage.mini_batch_generator(alg.num_mini_batches, 1))
    G._Inject.perm = None
    ac = alg.actor_critic
    named = dict(G.named_params(alg))
    clip = alg.clip_param
    for i in which:
        with torch.no_grad():
            for n, p in named.items():
                p.copy_(torch.from_numpy(probe[f"p{i}.{n}"]))
        (obs_b, priv_b, _critic_b, est_b, scan_b, actions_b, _tv, adv_b, _ret, old_logp_b, _om, _os, _h,
         _m) = batches[i % alg.num_mini_batches]
        mb = obs_b.shape[0]
        ac.update_distribution(obs_b, priv_b, est_b, scan_b, adaptation_mode=False)
        logp = ac.get_actions_log_prob(actions_b)
        ratio = torch.exp(logp - torch.squeeze(old_logp_b))
        adv = torch.squeeze(adv_b)
        s1 = -adv * ratio
        s2 = -adv * torch.clamp(ratio, 1.0 - clip, 1.0 + clip)
        gap = (s1 - s2).abs() / torch.maximum(s1.abs(), s2.abs()).clamp_min(1e-30)
        j = 2 * i  # the probe's surrogate torch.max arguments of this minibatch
        dev_a = float(np.abs(s1.detach().numpy() - probe[f"maxa{j}"]).max()) if f"maxa{j}" in probe.files else -1.0
        print(f"minibatch {i}: recomputed surrogate vs the probe's: max |diff| {dev_a:.3e}; smallest relative "
              f"margin {float(gap[s1 != s2].min()):.3e}; clipped-branch samples {int((s2 > s1).sum())}")
        near = torch.nonzero((gap <= TOL) & (s1 != s2)).flatten().tolist()
        ties = int(((s1 == s2) & ((ratio <= 1 - clip) | (ratio >= 1 + clip))).sum())
        print(f"minibatch {i}: {mb} samples, {len(near)} within {TOL:g} of a clip tie (plus {ties} exact ties at "
              f"the bounds)")
        actor = {n: p for n, p in named.items() if n.startswith("actor.")}
        for s in near:
            ac.zero_grad(set_to_none=True)
            r = ratio[s]
            (-adv[s] * r / mb).backward(retain_graph=True)
            side = "unclipped" if float(s1[s]) > float(s2[s]) else "clipped"
            print(f"  sample {s}: ratio {float(ratio[s]):.9f} adv {float(adv[s]):+.4f}, reference takes the {side} "
                  f"branch by {float(gap[s]):.2e} (relative)")
            for n, p in actor.items():
                if p.grad is None:
                    continue
                ref = probe[f"g{i}.{n}"]
                rel = float(p.grad.abs().max()) / (float(np.abs(ref).max()) + 1e-30)
                print(f"    a flip changes {n:18s} by {rel:.3e} of max|g|")


if __name__ == "__main__":
    main()
