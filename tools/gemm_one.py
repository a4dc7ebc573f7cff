"""Run one learner GEMM shape repeatedly (dev tool for rocprofv3 --pmc passes).
SHAPE=in,out MODE=fwd|dx|dw IT=50"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

B = int(os.environ.get("ROWS", "24576"))
i, o = (int(x) for x in os.environ.get("SHAPE", "736,512").split(","))
mode = os.environ.get("MODE", "fwd")
X = torch.randn(B, i, device="cuda")
W = torch.randn(o, i, device="cuda") * 0.05
b = torch.randn(o, device="cuda")
dY = torch.randn(B, o, device="cuda")
Y = torch.nn.functional.elu(torch.randn(B, i, device="cuda"))
fn = {"fwd": lambda: H.linear_forward(X, W, b, True), "dx": lambda: H.linear_input_grad(dY, W, Y),
      "dw": lambda: H.linear_weight_grad(dY, X)}[mode]
for _ in range(int(os.environ.get("IT", "50"))):
    fn()
torch.cuda.synchronize()
print("done")
