"""lgx_adaptation_forward at the update's 98,304 rows and the rollout's 4,096 (dev tool): us per
launch, HIP events over 50 launches, median of 5 rounds, on the history read in place from
go2's obs rows. Library: the product one or LGX_MLP_LIB (a build variant; round 6 timed an LDS-staged
form against the product kernel with it, profiles/r06_adapt_fwd_lds_experiment.txt).
Usage: python tools/adapt_fwd_timing.py"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoder  # noqa: E402

dev = "cuda:0"
torch.manual_seed(0)
enc = AdaptationEncoder(num_proprio=52, history_buffer_length=10, output_dim=20).to(dev)
res = {}
for B in (98304, 4096):
    obs = torch.randn(B, 572, device=dev)
    hist = obs[:, 52:].reshape(-1, 10, 52)
    ts = []
    with torch.no_grad():
        for rnd in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(50):
                enc(hist)
            b.record()
            b.synchronize()
            if rnd:
                ts.append(a.elapsed_time(b) * 1000 / 50)
    res[B] = round(statistics.median(ts), 1)
print(json.dumps({"lib": os.environ.get("LGX_MLP_LIB", "product"), "fwd2": os.environ.get("LGX_ADAPT_FWD2", "1"),
                  "us_per_launch": res}))
