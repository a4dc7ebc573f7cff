"""Replay the captured rollout graph (24 steps) K times — profiled with rocprofv3 (dev tool)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

torch.set_float32_matmul_precision("high")
a = get_args(["--task=go2", "--headless", "--num_envs=4096", "--sim_device=cuda:0", "--rl_device=cuda:0"])
env, _ = task_registry.make_env("go2", a)
_, tcfg = task_registry.get_cfgs("go2")
runner, _ = task_registry.make_alg_runner(env, args=a, train_cfg=tcfg, log_root=None)
runner.learn(3, init_at_random_ep_len=True)  # dagger, eager + captures, replay
torch.cuda.synchronize()
print("graphs:", list(runner._graphs))
for _ in range(int(os.environ.get("K", "10"))):
    with torch.inference_mode():
        runner._rollout(False, False)
    runner.alg.storage.clear()
torch.cuda.synchronize()
print("done")
