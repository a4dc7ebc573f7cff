"""EXPERIMENT: time tools/exp/gemm_glds.hip (pre-split bf16 planes + global_load_lds) against
the product forward GEMM (lgx_mlp.hip) on the update's largest forward shapes, and check it
against fp64. Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/exp/gemm_glds.hip
-o tools/exp/libgx.so"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402
from bench_mlp_t import t  # noqa: E402

L = C.CDLL(os.path.join(ROOT, "tools", "exp", "libgx.so"))
L.gx_fwd_planes.argtypes = [C.c_void_p] * 2 + [C.c_int64] + [C.c_void_p] * 2 + [C.c_int64] + [C.c_void_p] * 2 + \
    [C.c_int64, C.c_int, C.c_int, C.c_int, C.c_void_p]
L.gx_fwd_planes1.argtypes = L.gx_fwd_planes.argtypes
L.gx_fwd_f32.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                         C.c_int, C.c_int, C.c_int, C.c_void_p]


def planes(x, kpad):
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    out = []
    for p in (hi, lo):
        q = torch.zeros(x.shape[0], kpad, dtype=torch.bfloat16, device=x.device)
        q[:, :x.shape[1]] = p
        out.append(q)
    return out


B = 24576
torch.manual_seed(0)
for (i, o) in [(736, 512), (640, 512), (512, 256), (256, 128)]:
    X = torch.randn(B, i, device="cuda")
    W = torch.randn(o, i, device="cuda") * 0.05
    b = torch.randn(o, device="cuda")
    kp = (i + 31) // 32 * 32
    Xh, Xl = planes(X, kp)
    Wh, Wl = planes(W, kp)
    Y = torch.empty(B, o, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run():
        rc = L.gx_fwd_planes(Xh.data_ptr(), Xl.data_ptr(), kp, Wh.data_ptr(), Wl.data_ptr(), kp, b.data_ptr(),
                             Y.data_ptr(), o, B, o, kp, C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
    def run1():
        rc = L.gx_fwd_planes1(Xh.data_ptr(), Xl.data_ptr(), kp, Wh.data_ptr(), Wl.data_ptr(), kp, b.data_ptr(),
                              Y.data_ptr(), o, B, o, kp, C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
    run1()
    torch.cuda.synchronize()
    ref0 = torch.nn.functional.elu(X.double() @ W.double().t() + b.double())
    err1 = ((Y.double() - ref0).abs() / (X.double().abs() @ W.double().abs().t() + 1e-6)).max().item()
    t_1 = t(run1)
    run()
    torch.cuda.synchronize()
    ref = torch.nn.functional.elu(X.double() @ W.double().t() + b.double())
    err = ((Y.double() - ref).abs() / (X.double().abs() @ W.double().abs().t() + 1e-6)).max().item()
    t_new = t(run)
    t_old = t(lambda: H.linear_forward(X, W, b, True))
    Xp = torch.zeros(B, kp, device="cuda")
    Xp[:, :i] = X
    Wp = torch.zeros(o, kp, device="cuda")
    Wp[:, :i] = W
    Y32 = torch.empty(B, o, device="cuda")

    def run32():
        rc = L.gx_fwd_f32(Xp.data_ptr(), kp, Wp.data_ptr(), kp, b.data_ptr(), Y32.data_ptr(), o, B, o, kp,
                          C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
    run32()
    torch.cuda.synchronize()
    err32 = ((Y32.double() - ref).abs() / (X.double().abs() @ W.double().abs().t() + 1e-6)).max().item()
    t_32 = t(run32)
    fl = 2 * B * i * o
    print(f"{i}x{o}: planes+glds {t_new:.1f} us ({fl / t_new / 1e6:.0f} TF fp32-eq), product {t_old:.1f} us "
          f"({fl / t_old / 1e6:.0f} TF); exact f32 mfma {t_32:.1f} us ({fl / t_32 / 1e6:.0f} TF); "
          f"single-buffer planes {t_1:.1f} us ({fl / t_1 / 1e6:.0f} TF, err {err1:.1e}); "
          f"max err / sum|a b| planes {err:.2e} f32 {err32:.2e}", flush=True)
