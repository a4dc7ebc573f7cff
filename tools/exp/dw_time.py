"""Weight-gradient group (go2 update, 17 layers, 24576 rows) and the L1 forward: us per launch
with the library named by LGX_MLP_LIB (dev tool for build-flag variants)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

B = 24576
layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (512, 256), (256, 128), (128, 1),
          (29, 64), (64, 20), (20, 20), (132, 128), (128, 64), (64, 32), (572, 128), (128, 64), (64, 3)]
data = [(torch.randn(B, o, device="cuda"), torch.randn(B, i, device="cuda"), torch.zeros(o, i, device="cuda"),
         torch.zeros(o, device="cuda")) for i, o in layers]


def dw():
    with H.deferred_weight_grads():
        for dy, x, dW, db in data:
            H.linear_weight_grad(dy, x, dW, db, accumulate=True)


X = torch.randn(B, 736, device="cuda")
W = torch.randn(512, 736, device="cuda") * 0.05
b = torch.zeros(512, device="cuda")
Y = torch.empty(B, 512, device="cuda")


def fwd():
    H.linear_forward(X, W, b, True, out=Y)


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


print(f"{os.environ.get('LGX_MLP_LIB', 'product')}: dW group {t(dw):.1f} us (incl. split-K reduce), "
      f"fwd 736x512 {t(fwd):.1f} us", flush=True)
