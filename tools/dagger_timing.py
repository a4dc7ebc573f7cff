"""Per-iteration wall times of the go2 runner over 22 iterations, marking the DAgger ones
(it % dagger_update_freq == 0) — dev tool for the bench window's representativeness."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

torch.set_float32_matmul_precision("high")
a = get_args(["--task=go2", "--headless", "--num_envs=4096", "--sim_device=cuda:0", "--rl_device=cuda:0", "--seed=1"])
env, _ = task_registry.make_env("go2", a)
_, tcfg = task_registry.get_cfgs("go2")
runner, _ = task_registry.make_alg_runner(env, args=a, train_cfg=tcfg, log_root=None)
runner.learn(2, init_at_random_ep_len=True)
dag = []
_upd = runner.alg.update_dagger


def timed_update_dagger(*a, **k):  # the DAgger update's own cost, synchronised around it
    torch.cuda.synchronize()
    t = time.time()
    r = _upd(*a, **k)
    torch.cuda.synchronize()
    dag.append(time.time() - t)
    return r


runner.alg.update_dagger = timed_update_dagger
times = []
for i in range(22):
    it = runner.current_learning_iteration
    torch.cuda.synchronize()
    t0 = time.time()
    runner.learn(1)
    torch.cuda.synchronize()
    times.append((it, time.time() - t0))
freq = runner.dagger_update_freq
d = [t for it, t in times if it % freq == 0]
n = [t for it, t in times if it % freq != 0]
ppo = sum(n) / len(n)
print("dagger every", freq, "| dagger iters ms:", [round(x * 1e3, 1) for x in d],
      "| ppo iters mean ms: %.1f" % (1e3 * ppo), "| update_dagger ms:", [round(x * 1e3, 2) for x in dag])
if d and dag:
    print("dagger iteration / (ppo iteration + update_dagger) = %.3f" % (d[-1] / (ppo + dag[-1])))
