"""train.py — same flow as the reference's legged_gym/scripts/train.py:39-49:
make_env -> make_alg_runner -> learn(max_iterations, init_at_random_ep_len=True), at the
reference's matmul precision ('high', train.py:37). Multi-GPU: launch one process per GPU
with torch.distributed.run; envs shard over ranks, rank 0 logs and saves."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import isaacgym  # noqa: E402,F401  (placeholder, kept for line-for-line drop-in)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from legged_gym.envs import *  # noqa: E402,F401,F403
from legged_gym.utils import get_args, task_registry  # noqa: E402

torch.set_float32_matmul_precision("high")


def train(args):
    env, env_cfg = task_registry.make_env(name=args.task, args=args)
    ppo_runner, train_cfg = task_registry.make_alg_runner(env=env, name=args.task, args=args)
    ppo_runner.learn(num_learning_iterations=train_cfg.runner.max_iterations, init_at_random_ep_len=True)


def main(argv=None):
    args = get_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        args.sim_device = args.rl_device = f"cuda:{local}"
        args.sim_device_id = local
    try:
        train(args)
    finally:
        if world > 1:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
