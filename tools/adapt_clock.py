"""Phase clocks of lgx_adaptation_train (dev tool, GPU): LGX_MLP_LIB=exp/mlp_adclk.so (lgx_mlp.hip
-DLGX_ADAPT_CLOCK) at the go2 DAgger minibatch (24,576 rows). Phases per block (summed over its
chunks): stage-in, 4 forward stages, loss, fc_final dW, dpre2, conv2 dW, dpre1, conv1 dW, dpre0,
fc_encoder dW. Usage: LGX_MLP_LIB=exp/mlp_adclk.so PYTHONPATH=. python tools/adapt_clock.py"""
import ctypes as C

import numpy as np
import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoder

B, P, Hh = 24576, 52, 10
mod = AdaptationEncoder(num_proprio=P, history_buffer_length=Hh).to("cuda:0")
obs = torch.randn(B, P * (Hh + 1), device="cuda:0")
target = torch.randn(B, 20, device="cuda:0")
NP = sum(p.numel() for p in H.adaptation_param_order(mod))
BLK = 512  # ppo.DAGGER_BLOCKS
grid = H.adapt_train_grid(B, BLK)
gws, lws = torch.empty(grid * NP, device="cuda:0"), torch.empty(grid, device="cuda:0")
for _ in range(3):
    H.adaptation_train(mod, obs, P * Hh, target, gws, lws, BLK)
e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
e[0].record()
for _ in range(5):
    H.adaptation_train(mod, obs, P * Hh, target, gws, lws, BLK)
e[1].record()
torch.cuda.synchronize()
print(f"lgx_adaptation_train: {e[0].elapsed_time(e[1]) * 200:.1f} us per launch, grid {grid}")
L = H.lib()
if hasattr(L, "lgx_adapt_set_clock"):
    L.lgx_adapt_set_clock.argtypes = [C.c_void_p]
    buf = torch.zeros(grid * 16, dtype=torch.int32, device="cuda:0")
    L.lgx_adapt_set_clock(buf.data_ptr())
    H.adaptation_train(mod, obs, P * Hh, target, gws, lws, BLK)
    torch.cuda.synchronize()
    L.lgx_adapt_set_clock(None)
    d = buf.view(grid, 16).cpu().numpy().astype(np.int64)
    names = ["stage-in", "fwd0", "fwd1", "fwd2", "fwd3", "loss", "dWf", "dpre2", "dW2", "dpre1", "dW1", "dpre0", "dW0"]
    tot = d[:, :13].sum(1)
    print("  per block (ticks, mean): " + "  ".join(f"{n} {d[:, q].mean():.0f}" for q, n in enumerate(names)) +
          f"  | total {tot.mean():.0f}")
