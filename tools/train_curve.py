"""Learning-curve sanity run (dev tool): the go2 runner for ITERS iterations with episode
tracking on; prints the mean episode reward / length of the last <=100 episodes and the
tracking reward every 25 iterations. A working learner shows the reward rising."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

torch.set_float32_matmul_precision("high")
task = os.environ.get("TASK", "go2")
iters = int(os.environ.get("ITERS", "300"))
a = get_args([f"--task={task}", "--headless", "--num_envs=4096", "--sim_device=cuda:0", "--rl_device=cuda:0",
              "--seed=1"])
env, _ = task_registry.make_env(task, a)
_, tcfg = task_registry.get_cfgs(task)
runner, _ = task_registry.make_alg_runner(env, args=a, train_cfg=tcfg, log_root=None)
runner.log_dir = tempfile.mkdtemp()  # device-side episode tracking on
runner.log = lambda locs, width=80, pad=35: None  # no tensorboard writer needed
runner.save = lambda path, infos=None: None
runner.learn(1, init_at_random_ep_len=True)
for k in range(iters // 25):
    runner.learn(25)
    rew, ln, ep = runner._host_stats()
    mr = sum(rew) / max(1, len(rew))
    ml = sum(ln) / max(1, len(ln))
    print(f"it {runner.current_learning_iteration:4d}  mean reward {mr:8.3f}  mean length {ml:7.1f}  "
          f"fps {runner.last_perf['fps']:.0f}", flush=True)
