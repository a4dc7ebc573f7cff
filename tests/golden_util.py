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


def terrain_for(env_cfg, np_seed=1):
    """The task's Terrain (legged_gym_custom_amd.utils.terrain, pinned bit-exact to the
    reference in test_terrain.py) and its packed collision mesh, or (None, None)."""
    t = env_cfg.terrain
    if t.mesh_type not in ("heightfield", "trimesh"):
        return None, None
    from legged_gym_custom_amd.utils.terrain import Terrain
    from legged_gym_custom_amd.utils import terrain_utils
    np.random.seed(np_seed)
    ter = Terrain(t, env_cfg.env.num_envs)
    mesh = terrain_utils.pack_mesh(ter.heightsamples, t.horizontal_scale, t.vertical_scale,
                                   t.slope_treshold if t.mesh_type == "trimesh" else None)
    return ter, mesh


def go2_setup(num_envs, task="go2", terrain=None, sea_seed=None, cfg_hook=None):
    """(env_cfg, model, task params) for a task; `sea_seed` installs the synthetic SEA
    actuator net (legged_gym_custom_amd.actuator.random_sea_weights) the ANYmal fixtures
    were recorded with."""
    from legged_gym_custom_amd.envs import task_registry_configs
    from legged_gym_custom_amd import model as mdl, params as prm
    env_cfg, _ = task_registry_configs(task)
    if cfg_hook is not None:
        cfg_hook(env_cfg)
    m = mdl.load_model(env_cfg.asset.file, env_cfg.asset.foot_name)
    shape = (terrain.tot_rows, terrain.tot_cols) if terrain is not None else None
    if env_cfg.terrain.mesh_type not in ("heightfield", "trimesh"):
        env_cfg.terrain.curriculum = False  # LeggedRobot._parse_cfg (legged_robot.py:950-951)
    P = prm.build_task_params(env_cfg, m, num_envs, go2=task.startswith("go2"), terrain_shape=shape)
    if sea_seed is not None:
        from legged_gym_custom_amd import actuator as act
        act.fill_task_params(P, act.random_sea_weights(int(sea_seed)))
    return env_cfg, m, P


def fixture_setup(d, task):
    """Everything a replay needs from a fixture: (env_cfg, model, params, terrain tuple
    for OracleEnv.set_terrain / Twin, sea flag)."""
    import hashlib
    N = int(d["num_envs"])
    ter = tw = None
    if "terrain_levels" in d:
        from legged_gym_custom_amd.envs import task_registry_configs
        env_cfg = task_registry_configs(task)[0]
        env_cfg.env.num_envs = N
        ter, mesh = terrain_for(env_cfg, int(d["np_seed"]))
        assert hashlib.sha1(ter.heightsamples.tobytes()).hexdigest() == str(d["height_samples_sha1"])
        tw = (ter.heightsamples, mesh, d["terrain_levels"], d["terrain_types"], d["terrain_origins"])
    sea = int(d["sea_seed"]) if "sea_seed" in d else None
    cfg, m, P = go2_setup(N, task, terrain=ter, sea_seed=sea, cfg_hook=curriculum_hook(d))
    return cfg, m, P, tw, sea is not None


def curriculum_hook(d):
    """The command-curriculum settings a fixture was recorded with (tools/gen_golden.py), or None."""
    if "command_ranges0" not in d:
        return None
    r, c = d["command_ranges0"], d["curriculum_cfg"]

    def hook(cfg):
        cm = cfg.commands
        cm.curriculum = True
        cm.ranges.lin_vel_x, cm.ranges.lin_vel_y = [float(r[0]), float(r[1])], [float(r[2]), float(r[3])]
        cm.ranges.ang_vel_yaw, cm.ranges.heading = [float(r[4]), float(r[5])], [float(r[6]), float(r[7])]
        for k, v in zip(("vel_increment", "max_forward_vel", "max_reverse_vel", "max_curriculum"), c):
            if not np.isnan(v):
                setattr(cm, k, float(v))
    return hook


def enable_curriculum(oracle_env, d):
    """Bind the command-curriculum buffers (lgx_buffers.command_ranges, curriculum_vals,
    command_range_log) of an oracle.OracleEnv from a fixture."""
    N = oracle_env.P.num_envs
    oracle_env.a["command_ranges"] = np.array(d["command_ranges0"], dtype=np.float64)
    oracle_env.a["curriculum_vals"] = np.zeros(N, np.float32)
    r = oracle_env.a["command_ranges"]
    go2 = oracle_env.P.command_curriculum == 1  # (LeggedRobot._init_buffers' initial extras values)
    oracle_env.a["command_range_log"] = np.array([r[1], r[0], r[3], r[5]] if go2 else [r[1], r[3], r[5], 0.0],
                                                 np.float32)
    oracle_env.rebind()
