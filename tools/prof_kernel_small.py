"""Run a handful of env-step launches (for rocprofv3 counter collection)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

N = int(os.environ.get("N", "4096"))
args = get_args(["--task=go2", "--headless", f"--num_envs={N}", "--sim_device=cuda:0", "--rl_device=cuda:0"])
env, _ = task_registry.make_env("go2", args)
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
for _ in range(int(os.environ.get("STEPS", "10"))):
    env.step(torch.randn(N, 12, device="cuda", generator=g).clamp(-3, 3))
torch.cuda.synchronize()
print("done")
