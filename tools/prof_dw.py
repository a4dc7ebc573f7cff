"""The go2 update's weight-gradient group launch x 20 (for rocprofv3 --pmc; dev tool)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

B = 24576
layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (512, 256), (256, 128), (128, 1),
          (29, 64), (64, 20), (20, 20), (132, 128), (128, 64), (64, 32), (572, 128), (128, 64), (64, 3)]
data = [(torch.randn(B, o, device="cuda"), torch.randn(B, i, device="cuda"), torch.zeros(o, i, device="cuda"),
         torch.zeros(o, device="cuda")) for i, o in layers]
for _ in range(int(os.environ.get("ITERS", "20"))):
    with H.deferred_weight_grads():
        for dy, x, dW, db in data:
            H.linear_weight_grad(dy, x, dW, db, accumulate=True)
torch.cuda.synchronize()
print("done")
