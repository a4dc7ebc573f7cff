"""play.py — the reference's legged_gym/scripts/play.py:12-105 flow: one env on a 1x1
terrain without randomisation, the latest checkpoint of the task's experiment loaded,
the policy exported as TorchScript (policy / adaptation_module / estimator /
scan_encoder, helpers.py:180-214), then the inference policy (adaptation mode) driven
for 10 episodes' worth of steps with state and reward logging. Headless: no viewer,
camera or frame recording; the state plot is written as a PNG."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import isaacgym  # noqa: E402,F401  (placeholder, kept for line-for-line drop-in)
import torch  # noqa: E402

from legged_gym_custom_amd import LEGGED_GYM_ROOT_DIR  # noqa: E402
from legged_gym.envs import *  # noqa: E402,F401,F403
from legged_gym.utils import Logger, export_policy_as_jit, get_args, task_registry  # noqa: E402

EXPORT_POLICY = True
SHOW_PLOTS = False


def play(args, num_steps=None, root=None):
    root = root or LEGGED_GYM_ROOT_DIR
    env_cfg, train_cfg = task_registry.get_cfgs(name=args.task)
    env_cfg.env.num_envs = min(env_cfg.env.num_envs, 1)
    env_cfg.terrain.num_rows = 1
    env_cfg.terrain.num_cols = 1
    env_cfg.terrain.curriculum = False
    env_cfg.noise.add_noise = True
    env_cfg.domain_rand.randomize_friction = False
    env_cfg.domain_rand.randomize_base_mass = False
    env_cfg.domain_rand.randomize_center_of_mass = False
    env_cfg.domain_rand.randomize_motor_strength = False
    env_cfg.domain_rand.push_robots = False
    env_cfg.commands.zero_command = False
    env, _ = task_registry.make_env(name=args.task, args=args, env_cfg=env_cfg)

    train_cfg.runner.resume = True
    ppo_runner, train_cfg = task_registry.make_alg_runner(env=env, name=args.task, args=args, train_cfg=train_cfg,
                                                          log_root=os.path.join(root, "logs", train_cfg.runner.experiment_name))
    policy = ppo_runner.get_inference_policy(device=env.device)
    export_path = None
    if EXPORT_POLICY:
        export_path = os.path.join(root, "logs", train_cfg.runner.experiment_name, "exported", "policies")
        export_policy_as_jit(ppo_runner.alg.actor_critic, ppo_runner.alg.estimator, export_path)

    logger = Logger(env.dt)
    robot, joint = 0, 1
    stop_state_log = 100
    stop_rew_log = int(env.max_episode_length) + 1
    obs = env.get_observations()
    priv = env.get_privileged_observations()
    est = env.get_estimated_observations()
    scan = env.get_scan_observations()
    steps = num_steps if num_steps is not None else 10 * int(env.max_episode_length)
    with torch.inference_mode():
        for i in range(steps):
            actions = policy(obs, priv, est, scan, adaptation_mode=True)
            obs, priv, _, est, scan, _, _, infos = env.step(actions)
            if i < stop_state_log:
                logger.log_states({
                    "dof_pos_target": actions[robot, joint].item() * env.cfg.control.action_scale,
                    "dof_pos": env.dof_pos[robot, joint].item(),
                    "dof_vel": env.dof_vel[robot, joint].item(),
                    "dof_torque": env.torques[robot, joint].item(),
                    "command_x": env.commands[robot, 0].item(),
                    "command_y": env.commands[robot, 1].item(),
                    "command_yaw": env.commands[robot, 2].item(),
                    "base_vel_x": env.base_lin_vel[robot, 0].item(),
                    "base_vel_y": env.base_lin_vel[robot, 1].item(),
                    "base_vel_z": env.base_lin_vel[robot, 2].item(),
                    "base_vel_yaw": env.base_ang_vel[robot, 2].item(),
                    "contact_forces_z": env.contact_forces[robot, env.feet_indices, 2].cpu().numpy(),
                })
            elif i == stop_state_log and SHOW_PLOTS:
                logger.plot_states()
            if 0 < i < stop_rew_log:
                if infos["episode"]:
                    n = int(env.reset_buf.sum().item())
                    if n > 0:
                        logger.log_rewards(infos["episode"], n)
            elif i == stop_rew_log:
                logger.print_rewards()
    return env, ppo_runner, logger, export_path


def main(argv=None):
    torch.set_float32_matmul_precision("high")
    return play(get_args(argv))


if __name__ == "__main__":
    main()
