"""EXPERIMENT: tools/exp/gemm_ring.hip (fp32 LDS-DMA ring, split at fragment read) vs the
product forward GEMM on the update's forward shapes; error vs fp64 (|C - C64| / sum|a b|).
Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/exp/gemm_ring.hip -o tools/exp/libgr.so"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402
from bench_mlp_t import t  # noqa: E402

L = C.CDLL(os.path.join(ROOT, "tools", "exp", "libgr.so"))
L.gr_ring_fwd.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                          C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
B = 24576
torch.manual_seed(0)
for (i, o) in [(736, 512), (627, 512), (512, 256), (256, 128), (128, 64)]:
    X = torch.randn(B, i, device="cuda")
    W = torch.randn(o, i, device="cuda") * 0.05
    b = torch.randn(o, device="cuda")
    Y = torch.empty(B, o, device="cuda")
    ref = torch.nn.functional.elu(X.double() @ W.double().t() + b.double())
    den = X.double().abs() @ W.double().abs().t() + 1e-6
    res = []
    for ns in (0, 1, 2):
        def run(ns=ns):
            rc = L.gr_ring_fwd(X.data_ptr(), i, W.data_ptr(), i, b.data_ptr(), Y.data_ptr(), o, B, o, i, ns,
                               C.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
        Y.zero_()
        run()
        torch.cuda.synchronize()
        err = ((Y.double() - ref).abs() / den).max().item()
        res.append((ns, t(run), err))
    t_old = t(lambda: H.linear_forward(X, W, b, True))
    yo = H.linear_forward(X, W, b, True)
    err_old = ((yo.double() - ref).abs() / den).max().item()
    fl = 2 * B * i * o
    print(f"{i}x{o}: product {t_old:.1f} us ({fl / t_old / 1e6:.0f} TF, err {err_old:.1e}); " + "; ".join(
        f"ring v{ns} {tt:.1f} us ({fl / tt / 1e6:.0f} TF, err {e:.1e})" for ns, tt, e in res), flush=True)
