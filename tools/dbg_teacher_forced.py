"""Teacher-forced and free-running comparison of the GPU update with the REFERENCE's own
per-minibatch state (dev tool, GPU box).

Input: a tools/ref_update_probe.py output (the reference rsl_rl's parameters at the start of
every minibatch and its pre-clip gradients), copied to the path given. The learner case's
sequence (tests/learner_replay.py: rollout A, DAgger, rollout B) runs on this build, then:
  teacher-forced  for every minibatch i: ALL parameters := the reference's at minibatch i's
                  start, one phase A (forward, loss heads, backward), gradients vs the
                  reference's (worst per-tensor max|dg| / max|g|)
  free-running    the update's eager loop from the reference's initial state; after every
                  optimizer step the parameters vs the reference's at the next minibatch's start
for the S8 path and the autograd path.

  python tools/dbg_teacher_forced.py <probe.npz> [case]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import learner_case as LC  # noqa: E402
import learner_replay as R  # noqa: E402

probe = np.load(sys.argv[1])
case = sys.argv[2] if len(sys.argv) > 2 else "go2_c2"
dev = "cuda:0"
nmb = len(probe["norm_main"])


def prepared(use_s8):
    alg = R.build(case, dev, use_graphs=False)
    alg.use_s8 = use_s8
    R.rollout(alg, case, 0, {}, True, dev)
    perm0 = torch.from_numpy(LC.permutation(case, 0)).to(dev)
    alg._next_perm = lambda n: perm0
    alg.update_dagger()
    R.rollout(alg, case, 1, {}, False, dev)
    alg.total_updates = LC.TOTAL_UPDATES
    alg._reg_coef.fill_(alg.reg_coef())
    alg._perm.copy_(torch.from_numpy(LC.permutation(case, 1)).to(dev))
    return alg


def load_params(alg, i):
    with torch.no_grad():
        for n, p in R.named_params(alg):
            p.copy_(torch.from_numpy(probe[f"p{i}.{n}"]).to(dev))


def grad_err(alg, i):
    worst, wn = 0.0, ""
    for n, p in R.named_params(alg):
        if n.startswith("adaptation"):
            continue
        ref = torch.from_numpy(probe[f"g{i}.{n}"]).to(dev)
        e = float((p.grad - ref).abs().max() / (ref.abs().max() + 1e-30))
        if e > worst:
            worst, wn = e, n
    return worst, wn


def param_err(alg, i):
    worst, wn = 0.0, ""
    for n, p in R.named_params(alg):
        ref = torch.from_numpy(probe[f"p{i}.{n}"]).to(dev)
        e = float((p - ref).abs().max())
        if e > worst:
            worst, wn = e, n
    return worst, wn


for use_s8 in (True, False):
    label = "S8" if use_s8 else "autograd"
    alg = prepared(use_s8)
    load_params(alg, 0)
    alg._precompute()
    slices = alg._minibatches()
    print(f"== {label}: teacher-forced (reference parameters at every minibatch's start)")
    for i in range(nmb):
        load_params(alg, i)
        alg._minibatch_grads(slices[i % len(slices)])
        e, n = grad_err(alg, i)
        print(f"  minibatch {i:2d}: worst grad err {e:.3e} ({n})")
    print(f"== {label}: free-running from the reference's initial state (eager update loop)")
    alg = prepared(use_s8)
    load_params(alg, 0)
    alg._precompute()
    slices = alg._minibatches()
    for i in range(nmb):
        alg._minibatch_grads(slices[i % len(slices)])
        e, n = grad_err(alg, i)
        alg._minibatch_step()
        pe, pn = param_err(alg, i + 1) if i + 1 < nmb else (0.0, "")
        print(f"  minibatch {i:2d}: grad err {e:.3e} ({n}); params after its step vs reference "
              f"{pe:.3e} ({pn})")
    sys.stdout.flush()
