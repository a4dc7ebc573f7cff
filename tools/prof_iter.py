"""Run K full learning iterations of the drop-in runner after warm-up (dev tool: profile
it with rocprofv3 --kernel-trace and read the trace with tools/trace_gaps.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

torch.set_float32_matmul_precision("high")
task = os.environ.get("TASK", "go2")
n = int(os.environ.get("N", "4096"))
a = get_args([f"--task={task}", "--headless", f"--num_envs={n}", "--sim_device=cuda:0", "--rl_device=cuda:0"])
env, _ = task_registry.make_env(task, a)
_, tcfg = task_registry.get_cfgs(task)
runner, _ = task_registry.make_alg_runner(env, args=a, train_cfg=tcfg, log_root=None)
runner.learn(3, init_at_random_ep_len=True)  # dagger, eager + captures, replay
torch.cuda.synchronize()
runner.learn(int(os.environ.get("K", "3")))
torch.cuda.synchronize()
print("done", runner.last_perf)
