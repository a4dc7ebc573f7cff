"""The three big learner GEMMs (critic layer 0 shapes, B = 24576) x 20 each, for rocprofv3."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

B, i, o = 24576, 736, 512
X = torch.randn(B, i, device="cuda")
W = torch.randn(o, i, device="cuda") * 0.05
b = torch.randn(o, device="cuda")
dY = torch.randn(B, o, device="cuda")
Y = torch.nn.functional.elu(torch.randn(B, i, device="cuda"))
for _ in range(20):
    H.linear_forward(X, W, b, True)
torch.cuda.synchronize()
for _ in range(20):
    H.linear_input_grad(dY, W, Y)
torch.cuda.synchronize()
for _ in range(20):
    H.linear_weight_grad(dY, X)
torch.cuda.synchronize()
print("done")
