"""One minibatch's gradients: GPU (HIP GEMMs) vs CPU torch, per segment (dev tool)."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from test_ppo_update import _fill, _make  # noqa: E402
from test_gpu_learner import _to_gpu  # noqa: E402

base = _make("adaptive")
cpu = _to_gpu(base, use_graphs=False, device="cpu")
gpu = _to_gpu(base, use_graphs=False)
for alg in (cpu, gpu):
    _fill(alg, 40)
idx_c = torch.arange(32)
cpu._minibatch_grads(idx_c)
gpu._minibatch_grads(idx_c.cuda())
gc, gg = cpu.grads, gpu.grads
for name in ("main", "estimator", "adaptation"):
    a = gc.segment(name).double()
    b = gg.segment(name).double().cpu()
    d = (a - b).abs()
    rel = d / (a.abs() + 1e-12)
    sign = ((a > 0) != (b > 0)) & (a.abs() > 0)
    print(name, "n", a.numel(), "max|a|", float(a.abs().max()), "max abs diff", float(d.max()),
          "median rel", float(rel.median()), "p99 rel", float(torch.quantile(rel, 0.99)), "sign flips", int(sign.sum()),
          "norm rel", float((a - b).norm() / a.norm()))
print("losses", cpu._losses.tolist(), gpu._losses.tolist())
# per-parameter
for (n, p), (_, q) in zip(list(cpu.actor_critic.named_parameters()) + list(cpu.estimator.named_parameters()),
                          list(gpu.actor_critic.named_parameters()) + list(gpu.estimator.named_parameters())):
    if p.grad is None:
        continue
    a, b = p.grad.double(), q.grad.double().cpu()
    print(f"{n:45s} rel {float((a - b).norm() / (a.norm() + 1e-30)):.2e}")
