"""Per-layer timing: liblgx_mlp GEMMs vs torch/hipBLASLt for the learner's shapes (dev tool)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

B = 24576
layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (572, 128), (128, 64), (132, 128), (29, 64)]


def t(fn, it=20):
    """GPU time per call: `it` calls captured in one hipGraph, replayed (no host overhead)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * it) * 1e3


torch.set_float32_matmul_precision("high")
tot_h = tot_t = 0.0
for (i, o) in layers:
    X = torch.randn(B, i, device="cuda")
    W = torch.randn(o, i, device="cuda") * 0.05
    b = torch.randn(o, device="cuda")
    dY = torch.randn(B, o, device="cuda")
    Y = torch.nn.functional.elu(torch.randn(B, i, device="cuda"))
    fl = 2 * B * i * o
    h = {"fwd": t(lambda: H.linear_forward(X, W, b, True)), "dX": t(lambda: H.linear_input_grad(dY, W, Y)),
         "dW": t(lambda: H.linear_weight_grad(dY, X))}
    r = {"fwd": t(lambda: torch.nn.functional.elu(torch.addmm(b, X, W.t()))),
         "dX": t(lambda: (dY @ W) * torch.where(Y > 0, 1.0, Y + 1)),
         "dW": t(lambda: (dY.t() @ X, dY.sum(0)))}
    tot_h += sum(h.values())
    tot_t += sum(r.values())
    print((i, o), " ".join(f"{k}: hip {h[k]:.0f}us ({fl / h[k] / 1e6:.0f}TF) torch {r[k]:.0f}us" for k in h))
print(f"sum hip {tot_h:.0f}us torch {tot_t:.0f}us")
