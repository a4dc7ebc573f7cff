#!/usr/bin/env python3
"""Probe of the REFERENCE rsl_rl update's rounding sensitivity (test infrastructure, CPU, this
container only: imports /root/reference/rsl_rl through tools/gen_learner_golden.py).

Runs one learner case (tests/learner_case.py: rollout A, DAgger, rollout B, then PPO.update)
and records, per minibatch of the update:
  * the pre-clip gradients of every parameter (hooked at clip_grad_norm_) and both norms;
  * the parameters at the minibatch's start;
  * the per-sample decisions of the two torch.max calls of ppo.py:254 (surrogate vs clipped
    surrogate) and ppo.py:261 (value loss vs clipped value loss), as bit masks, plus the
    per-sample ratio, advantage and value terms they compare.

  python tools/ref_update_probe.py <case> <threads> <out.npz> [perturb] [noise]

`perturb` > 0 multiplies the initial weights of actor.0 by (1 + perturb * 2^-23), a one-ulp-scale
change, so that two runs differ only by rounding. `noise` > 0 multiplies every pre-clip gradient
of every minibatch by (1 + noise * N(0, 1)) per entry (a stand-in for a GPU path's per-entry
rounding, ~1e-5 relative), seeded. tools/ref_update_compare.py diffs two outputs.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import gen_learner_golden as G  # noqa: E402  (patches Normal.sample / randperm for injection)
import learner_case as LC  # noqa: E402


def main():
    case, threads, out_path = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    perturb = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
    noise = float(sys.argv[5]) if len(sys.argv) > 5 else 0.0
    gen = torch.Generator().manual_seed(99)
    torch.set_num_threads(threads)
    alg = G.build(case)
    if perturb:
        with torch.no_grad():
            alg.actor_critic.actor[0].weight.mul_(1.0 + perturb * 2.0 ** -23)
    names_of = {id(p): n for n, p in G.named_params(alg)}
    scratch = {}
    G.rollout(alg, case, 0, scratch, adaptation_mode=True)
    G._Inject.perm = torch.from_numpy(LC.permutation(case, 0))
    alg.update_dagger()
    G._Inject.perm = None
    G.rollout(alg, case, 1, scratch, adaptation_mode=False)
    alg.total_updates = LC.TOTAL_UPDATES

    rec = {"grads": [], "params": [], "norm_est": [], "norm_main": [], "max_masks": [], "max_args": []}
    orig_clip = nn.utils.clip_grad_norm_
    orig_max = torch.max
    cur = {}

    def clip_hook(params, max_norm, *a, **k):
        params = list(params)
        est = all(names_of[id(p)].startswith("estimator.") for p in params)
        if est:  # first call of a minibatch: the main parameters are still at the minibatch's start
            cur.clear()
            cur["params"] = {n: p.detach().numpy().copy() for n, p in G.named_params(alg)}
            cur["grads"] = {}
        for p in params:
            if p.grad is not None:
                cur["grads"][names_of[id(p)]] = p.grad.detach().numpy().copy()
                if noise:
                    with torch.no_grad():
                        p.grad.mul_(1.0 + noise * torch.randn(p.grad.shape, generator=gen))
        total = orig_clip(params, max_norm, *a, **k)
        rec["norm_est" if est else "norm_main"].append(float(total))
        if not est:
            rec["grads"].append(cur["grads"])
            rec["params"].append(cur["params"])
        return total

    def max_hook(*a, **k):
        if len(a) == 2 and isinstance(a[1], torch.Tensor) and a[0].dim() >= 1:
            x, y = a[0].detach(), a[1].detach()
            rec["max_masks"].append(np.packbits((x >= y).reshape(-1).numpy()))
            rec["max_args"].append((x.reshape(-1).numpy().copy(), y.reshape(-1).numpy().copy()))
        return orig_max(*a, **k)

    nn.utils.clip_grad_norm_ = clip_hook
    torch.max = max_hook
    G._Inject.perm = torch.from_numpy(LC.permutation(case, 1))
    losses = alg.update()
    G._Inject.perm = None
    torch.max = orig_max
    nn.utils.clip_grad_norm_ = orig_clip
    out = {"losses": np.array(losses, dtype=np.float64), "norm_est": np.array(rec["norm_est"]),
           "norm_main": np.array(rec["norm_main"])}
    for i, (g, p) in enumerate(zip(rec["grads"], rec["params"])):
        for n, v in g.items():
            out[f"g{i}.{n}"] = v
        for n, v in p.items():
            out[f"p{i}.{n}"] = v
    for j, (m, (x, y)) in enumerate(zip(rec["max_masks"], rec["max_args"])):
        out[f"mask{j}"] = m
        out[f"maxa{j}"] = x
        out[f"maxb{j}"] = y
    np.savez(out_path, **out)
    print(f"{case} threads={threads} perturb={perturb}: losses {losses}, {len(rec['grads'])} minibatches -> {out_path}")


if __name__ == "__main__":
    main()
