"""Profile one rollout + one PPO update of the drop-in runner (torch.profiler)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
torch.set_float32_matmul_precision(os.environ.get("PREC", "high"))
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

N = int(os.environ.get("N", "4096"))
args = get_args(["--task=go2", "--headless", f"--num_envs={N}", "--sim_device=cuda:0", "--rl_device=cuda:0"])
env, _ = task_registry.make_env("go2", args)
_, tcfg = task_registry.get_cfgs("go2")
runner, _ = task_registry.make_alg_runner(env, args=args, train_cfg=tcfg, log_root=None)
runner.learn(2, init_at_random_ep_len=True)
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    t = time.time()
    runner.learn(1)
    torch.cuda.synchronize()
    print("iteration wall", time.time() - t, runner.last_perf)
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=35, max_name_column_width=70))
print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=15, max_name_column_width=70))
