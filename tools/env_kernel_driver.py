"""Launch the env-step kernel K times on the bench workload (Go2 flat, 4096 envs, actions
~N(0,1) clipped, Philox seed 1234) — the command profiled for PMC HBM traffic."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

N = int(os.environ.get("N", "4096"))
K = int(os.environ.get("K", "20"))
a = get_args(["--task=go2", "--headless", f"--num_envs={N}", "--sim_device=cuda:0", "--rl_device=cuda:0", "--seed=1"])
env, _ = task_registry.make_env("go2", a)
g = torch.Generator(device="cuda:0").manual_seed(1234)
acts = torch.clamp(torch.randn(K, env.num_envs, env.num_actions, device="cuda:0", generator=g), -3.14, 3.14)
stream = torch.cuda.current_stream()
torch.cuda.synchronize()
for i in range(K):
    env.actions_in.copy_(acts[i])
    env.common_step_counter += 1
    env._native.step(env.seed, env.common_step_counter, stream.cuda_stream)
torch.cuda.synchronize()
print("env kernel launches:", K, "envs:", N)
