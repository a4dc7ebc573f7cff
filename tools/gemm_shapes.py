"""Per-layer learner GEMM timings (B = 24576 minibatch rows) — dev tool."""
import time
import torch

B = 24576
layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (572, 128), (128, 64), (132, 128)]


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = time.time()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.time() - s) / it * 1e6


tot = {}
for prec in ("highest", "high"):
    torch.set_float32_matmul_precision(prec)
    for (i, o) in layers:
        X = torch.randn(B, i, device="cuda")
        W = torch.randn(o, i, device="cuda") * 0.05
        b = torch.randn(o, device="cuda")
        dY = torch.randn(B, o, device="cuda")
        fl = 2 * B * i * o
        r = {"fwd": t(lambda: torch.addmm(b, X, W.t())), "dX": t(lambda: dY @ W), "dW": t(lambda: dY.t() @ X)}
        for S in (4, 8, 16, 32):
            r[f"dW_s{S}"] = t(lambda: torch.bmm(dY.view(S, B // S, o).transpose(1, 2), X.view(S, B // S, i)).sum(0))
        r["db"] = t(lambda: dY.sum(0))
        print(prec, (i, o), " ".join(f"{k}={v:.0f}us/{fl / v / 1e6:.0f}TF" if k != "db" else f"db={v:.0f}us" for k, v in r.items()))
