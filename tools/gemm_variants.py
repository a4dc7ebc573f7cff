"""Time the learner's dominant GEMM launches for the liblgx_mlp.so named by LGX_MLP_LIB
(dev tool for comparing kernel variants): critic layer-0 forward, an input-gradient
launch, and the whole-backward weight-gradient group (the go2 update's 17 dW GEMMs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402
from bench_mlp_t import t  # noqa: E402

B = 24576
torch.manual_seed(0)
X = torch.randn(B, 736, device="cuda")
W = torch.randn(512, 736, device="cuda") * 0.05
b = torch.randn(512, device="cuda")
g1 = torch.randn(B, 256, device="cuda")
W1 = torch.randn(256, 512, device="cuda") * 0.05
Y0 = torch.nn.functional.elu(torch.randn(B, 512, device="cuda"))
# (in, out) of every layer of the go2 update: actor, critic, privileged/scan encoders, estimator
layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (512, 256), (256, 128), (128, 1),
          (29, 64), (64, 20), (20, 20), (132, 128), (128, 64), (64, 32), (572, 128), (128, 64), (64, 3)]
data = [(torch.randn(B, o, device="cuda"), torch.randn(B, i, device="cuda"), torch.zeros(o, i, device="cuda"),
         torch.zeros(o, device="cuda")) for i, o in layers]


Xa = torch.randn(B, 627, device="cuda")
Wa = torch.randn(512, 627, device="cuda") * 0.05
ya, yc = torch.empty(B, 512, device="cuda"), torch.empty(B, 512, device="cuda")
fwd_args = [H._fwd_args(Xa, Wa, b, True, ya), H._fwd_args(X, W, b, True, yc)]
g2 = torch.randn(B, 256, device="cuda")
W2 = torch.randn(256, 512, device="cuda") * 0.05
dxa, dxc = torch.empty(B, 512, device="cuda"), torch.empty(B, 512, device="cuda")
dx_args = [H._dx_args(g1, W1, Y0, dxa), H._dx_args(g2, W2, Y0, dxc)]
W1t, W2t = W1.t().contiguous(), W2.t().contiguous()


def _dxt(g, Wt, y, dx):  # the same input gradient with W transposed (k-contiguous B)
    M, N = g.shape
    return H.GemmArgs(A=g.data_ptr(), lda=g.stride(0), a_kcontig=1, B=Wt.data_ptr(), ldb=Wt.stride(0), b_kcontig=1,
                      C=dx.data_ptr(), ldc=dx.stride(0), M=M, N=Wt.shape[0], K=N, epilogue=H.EPI_DELU,
                      act=y.data_ptr(), ld_act=y.stride(0), split_k=1)


dxt_args = [_dxt(g1, W1t, Y0, dxa), _dxt(g2, W2t, Y0, dxc)]


def dw_group():
    with H.deferred_weight_grads():
        for dy, x, dW, db in data:
            H.linear_weight_grad(dy, x, dW, db, accumulate=True)


Xs = torch.randn(B, 128, device="cuda")
Ws = torch.randn(64, 128, device="cuda") * 0.3
bs = torch.randn(64, device="cuda")
Xr = X[:4096].contiguous()
# ELU epilogue accuracy: x @ I + b over a sweep of pre-activations in [-20, 5]
z = torch.linspace(-20, 5, 4096 * 64, device="cuda").view(4096, 64)
eye = torch.eye(64, device="cuda")
yz = H.linear_forward(z, eye, torch.zeros(64, device="cuda"), True)
ref = torch.nn.functional.elu(z.double())
ulp = ((yz.double() - ref).abs() / (ref.abs() * 2.0 ** -23 + 1e-30)).max().item()
r = {"fwd736x512": t(lambda: H.linear_forward(X, W, b, True)),
     "fwd128x64": t(lambda: H.linear_forward(Xs, Ws, bs, True)),
     "fwd4096r": t(lambda: H.linear_forward(Xr, W, b, True)),
     "dx256to512": t(lambda: H.linear_input_grad(g1, W1, Y0)),
     "fwdgroup": t(lambda: H.run_group(fwd_args)),
     "dxgroup": t(lambda: H.run_group(dx_args)),
     "dxgroupT": t(lambda: H.run_group(dxt_args)),
     "dWgroup": t(dw_group, it=5)}
fl = {"fwd736x512": 2 * B * 736 * 512, "fwd128x64": 2 * B * 128 * 64, "fwd4096r": 2 * 4096 * 736 * 512, "dx256to512": 2 * B * 256 * 512,
      "fwdgroup": 2 * B * 512 * (627 + 736), "dxgroup": 2 * 2 * B * 256 * 512, "dxgroupT": 2 * 2 * B * 256 * 512,
      "dWgroup": sum(2 * B * i * o for i, o in layers)}
print(os.path.basename(os.environ.get("LGX_MLP_LIB", "default")), "BN", os.environ.get("LGX_GROUP_BN", "auto"), f"elu max {ulp:.1f} ulp", " ".join(
    f"{k} {v:.1f}us ({fl[k] / v / 1e6:.0f}TF)" for k, v in r.items()), flush=True)
