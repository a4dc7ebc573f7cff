"""lgx_gather_rows at the update's shape (dev tool; run under rocprofv3 --kernel-trace --stats):
98304 rows of the storage's 12 buffers packed (a), with obs into a 628-float-pitch actor-input
buffer (b), and with est also into it (c); 10 launches each, in that order."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

R = 98304
widths = [572, 29, 736, 3, 132, 12, 1, 1, 1, 1, 12, 12]
srcs = [torch.randn(R, w, device="cuda") for w in widths]
perm = torch.randperm(R, device="cuda")
buf = torch.empty(R, int(os.environ.get("PITCH", "628")), device="cuda")
variant = os.environ.get("V", "abc")
for v in variant:
    for _ in range(10):
        if v == "a":
            H.gather_rows(srcs, perm)
        elif v == "b":
            H.gather_rows(srcs, perm, [buf[:, :572]] + [None] * 11)
        else:
            H.gather_rows(srcs + [srcs[3]], perm, [buf[:, :572]] + [None] * 11 + [buf[:, 624:627]])
    torch.cuda.synchronize()
print("done")
