"""S8 vs autograd minibatch path WITH the optimizer steps in between (the update's real
sequence): per-minibatch gradient agreement — where does the divergence start (dev tool)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

import learner_case as LC  # noqa: E402
import learner_replay as R  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "go2_c2"
dev = "cuda:0"
runs = {}
# (path, legacy dW block budget): the third run is the autograd path with a different split-K
# (LGX_DW_SLOTS: a different fp32 summation order only) — the update's own sensitivity
for key in (False, "legacy_again", True):
    s8 = key is True
    alg = R.build(case, dev, use_graphs=False)
    alg.use_s8 = s8
    R.rollout(alg, case, 1, {}, False, dev)
    alg.total_updates = LC.TOTAL_UPDATES
    alg._reg_coef.fill_(alg.reg_coef())
    alg._perm.copy_(torch.from_numpy(LC.permutation(case, 1)).to(dev))
    alg._precompute()
    seq = []
    for ep in range(alg.num_learning_epochs):
        for idx in alg._minibatches():
            alg._minibatch_grads(idx)
            g = {n: p.grad.detach().clone() for n, p in R.named_params(alg) if not n.startswith("adaptation")}
            alg._minibatch_step()
            pr = {n: p.detach().clone() for n, p in R.named_params(alg) if not n.startswith("adaptation")}
            m = alg.exp_avg.clone()
            seq.append((g, pr, m))
    runs[key] = seq


def report(a, b, label):
    print(f"== {label}")
    for k, ((g0, p0, m0), (g1, p1, m1)) in enumerate(zip(runs[a], runs[b])):
        ge = sorted(((n, float((g1[n] - g).abs().max() / (g.abs().max() + 1e-30))) for n, g in g0.items()),
                    key=lambda x: -x[1])[:2]
        pe = max(float((p1[n] - p).abs().max()) for n, p in p0.items())
        me = float((m1 - m0).abs().max() / (m0.abs().max() + 1e-30))
        print(f"minibatch {k}: worst grad rel err {[(n, f'{e:.2e}') for n, e in ge]}  max |dparam| {pe:.2e}  "
              f"exp_avg rel {me:.2e}")


report(False, "legacy_again", "autograd path, run 1 vs the same configuration again (run 2)")
report("legacy_again", True, "run 2 (autograd) vs S8 (run 3)")
