"""Helpers to replay tests/golden/*.npz fixtures (recorded from the reference's own
tensor code by tools/gen_golden.py) through the oracle or the HIP library."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def num_steps(d):
    t = 0
    while f"steps.{t}.csc_in" in d:
        t += 1
    return t


def step(d, t, key):
    return d[f"steps.{t}.{key}"]


def go2_setup(num_envs, task="go2"):
    from legged_gym_custom_amd.envs import task_registry_configs
    from legged_gym_custom_amd import model as mdl, params as prm
    env_cfg, _ = task_registry_configs(task)
    m = mdl.load_model(env_cfg.asset.file, env_cfg.asset.foot_name)
    P = prm.build_task_params(env_cfg, m, num_envs, go2=True)
    return env_cfg, m, P
