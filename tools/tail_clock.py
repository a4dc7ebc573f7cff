"""Phase clocks of lgx_loss_heads_tail (dev tool, GPU): LGX_MLP_LIB=legged_gym_custom_amd/lib/dev/liblgx_mlp_clock.so (lgx_mlp.hip
built with -DLGX_TAIL_CLOCK) runs the launch at the go2 minibatch size (24,576 rows, A 12, H 128)
and prints per-block cycles of: input loads | last layers' forward | PPO head rows | input
gradients | column sums | block sum | total, plus the launch time (HIP events).
Usage: LGX_MLP_LIB=legged_gym_custom_amd/lib/dev/liblgx_mlp_clock.so PYTHONPATH=. python tools/tail_clock.py"""
import ctypes as C

import numpy as np
import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S

dev = "cuda:0"
B, A, Hd, L, E = 24576, 12, 128, 20, 3
g = torch.Generator(device=dev).manual_seed(1)
r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
y8, yc8 = S.to_s8_torch(torch.nn.functional.elu(r(B, Hd))), S.to_s8_torch(torch.nn.functional.elu(r(B, Hd)))
W, b, Wc, bc = 0.1 * r(A, Hd), r(A), 0.1 * r(1, Hd), r(1)
std = r(A).abs() + 0.5
actions, old_logp, adv, tv, ret = r(B, A), r(B, 1), r(B, 1), r(B, 1), r(B, 1)
old_mu, old_sigma = r(B, A), r(B, A).abs() + 0.5
p_lat, a_lat, pred, t_est = r(B, L), r(B, L), r(B, E), r(B, E)
seeds = torch.tensor([1.0, 1.3, -0.01, 0.05, 1.0], device=dev)
nt, nblk = (B + 31) // 32, (B + 255) // 256
z = lambda *s: torch.zeros(*s, device=dev)  # noqa: E731
ws, wsa, out, out_aux, dstd, dp = z(19 * nt), z(2 * nblk), z(8), z(2), z(A), z(B, L)
cnt, cnta = torch.zeros(1, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int32, device=dev)
dmu8, dv8, de8 = S.empty(B, A, dev), S.empty(B, 1, dev), S.empty(B, E, dev)
cs_mu, cs_v, cs_e = z(nt, A), z(nt, 1), z(nblk, E)
dy8, dyc8, cs_y, cs_yc, mu, val = S.empty(B, Hd, dev), S.empty(B, Hd, dev), z(nt, Hd), z(nt, Hd), z(B, A), z(B, 1)
h = H.HeadArgs(mu=mu.data_ptr(), value=val.data_ptr(), std=std.data_ptr(), actions=actions.data_ptr(),
               old_logp=old_logp.data_ptr(), adv=adv.data_ptr(), target_values=tv.data_ptr(), returns=ret.data_ptr(),
               old_mu=old_mu.data_ptr(), old_sigma=old_sigma.data_ptr(), B=B, A=A, clip=0.2, clipped_value=1,
               out=out.data_ptr(), g=seeds.data_ptr(), dstd=dstd.data_ptr(), ws=ws.data_ptr(), counter=cnt.data_ptr())
x = H.AuxArgs(p=p_lat.data_ptr(), a=a_lat.data_ptr(), L=L, e=pred.data_ptr(), t=t_est.data_ptr(), E=E, B=B,
              out=out_aux.data_ptr(), g=seeds.data_ptr() + 12, dp=dp.data_ptr(), ws=wsa.data_ptr(),
              counter=cnta.data_ptr(), ld_p=L)
s8 = H.HeadsS8Args(dmu_s8=dmu8.data_ptr(), ld_dmu=dmu8.shape[1], dmu_cs=cs_mu.data_ptr(), dvalue_s8=dv8.data_ptr(),
                   ld_dvalue=dv8.shape[1], dvalue_cs=cs_v.data_ptr(), de_s8=de8.data_ptr(), ld_de=de8.shape[1],
                   de_cs=cs_e.data_ptr())
t = H.HeadsTailArgs(y=y8.data_ptr(), ld_y=y8.shape[1], W=W.data_ptr(), b=b.data_ptr(), dy=dy8.data_ptr(),
                    ld_dy=dy8.shape[1], dy_cs=cs_y.data_ptr(), yc=yc8.data_ptr(), ld_yc=yc8.shape[1], Wc=Wc.data_ptr(),
                    bc=bc.data_ptr(), dyc=dyc8.data_ptr(), ld_dyc=dyc8.shape[1], dyc_cs=cs_yc.data_ptr(),
                    mu_out=mu.data_ptr(), value_out=val.data_ptr(), H=Hd, Hc=Hd)
Lb = H.lib()


def run():
    H._check(Lb.lgx_loss_heads_tail(C.byref(h), C.byref(x), C.byref(s8), C.byref(t), H._stream()), "tail")


for _ in range(5):
    run()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(20):
    run()
ev[1].record()
torch.cuda.synchronize()
print(f"lgx_loss_heads_tail: {ev[0].elapsed_time(ev[1]) * 1000 / 20:.1f} us per launch ({nt} PPO blocks + {nblk} aux)")
if hasattr(Lb, "lgx_tail_set_clock"):
    Lb.lgx_tail_set_clock.argtypes = [C.c_void_p]
    buf = torch.zeros(nt * 8, dtype=torch.int32, device=dev)
    Lb.lgx_tail_set_clock(buf.data_ptr())
    run()
    torch.cuda.synchronize()
    Lb.lgx_tail_set_clock(None)
    d = buf.view(nt, 8).cpu().numpy().astype(np.int64)
    names = ["loads", "forward", "head rows", "input grads", "col sums", "block sum", "total"]
    print("  per block (cycles, mean / max): " + "  ".join(f"{n} {d[:, q].mean():.0f}/{d[:, q].max()}"
                                                             for q, n in enumerate(names)))
