"""Time the learner's GEMM shapes under fp32 precision modes (dev tool)."""
import torch
import time

torch.manual_seed(0)
M = 24576
shapes = [(M, 627, 512), (M, 736, 512), (M, 512, 256), (M, 572, 256)]


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = time.time()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.time() - s) / it * 1e3


def split(x):
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return hi, lo


for (m, k, n) in shapes:
    a = torch.randn(m, k, device="cuda")
    b = torch.randn(k, n, device="cuda") * 0.05
    ref = (a.double() @ b.double())
    out = {}
    for mode in ("highest", "high", "medium"):
        torch.set_float32_matmul_precision(mode)
        ms = t(lambda: a @ b)
        err = ((a @ b).double() - ref).abs().max().item()
        out[mode] = (ms, err)
    torch.set_float32_matmul_precision("highest")
    ah, al = split(a)
    bh, bl = split(b)

    def x3():
        return (ah @ bh).float() + (ah @ bl).float() + (al @ bh).float()
    ms3 = t(x3)
    err3 = (x3().double() - ref).abs().max().item()
    bfms = t(lambda: ah @ bh)
    flops = 2 * m * k * n
    print(f"{m}x{k}x{n}: " + " ".join(f"{k_}={v[0]:.3f}ms({flops / v[0] / 1e9:.0f}TF,err{v[1]:.1e})" for k_, v in out.items())
          + f" bf16x3(bf16-out)={ms3:.3f}ms err{err3:.1e} bf16={bfms:.3f}ms")
print(torch.__version__, torch.version.hip)
try:
    a = torch.randn(64, 64, device="cuda", dtype=torch.bfloat16)
    r = torch.mm(a, a, out_dtype=torch.float32)
    print("mm out_dtype ok", r.dtype)
except Exception as e:
    print("mm out_dtype unsupported:", type(e).__name__, str(e)[:100])
