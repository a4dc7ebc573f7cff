"""Terrain on the GPU: the env kernel's trimesh contact against the C
oracle's double-precision restatement, and the whole env built on generated terrain.

* one full step (physics + post-physics) on a small rough field (slopes, rough slopes,
  stairs, obstacles; trimesh with slope-threshold walls), robots dropped onto it:
  kernel vs oracle, same tolerances as the plane case (test_gpu_parity.py);
* Go2Robot on go2_parkour's terrain and on a rough curriculum field at N=4096: finite
  state, robots supported by the mesh (contact normal force ~ weight), a parkour course
  spawn at the start platform, terrain_level extras present, bitwise determinism.
"""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu


def _rough_cfg(n, mesh="trimesh"):
    from legged_gym_custom_amd.envs import task_registry_configs
    cfg = task_registry_configs("go2")[0]
    cfg.env.num_envs = n
    t = cfg.terrain
    t.mesh_type = mesh
    t.curriculum = True
    t.num_rows, t.num_cols = 3, 4
    t.terrain_length = t.terrain_width = 8.0
    t.max_init_terrain_level = 2
    t.terrain_proportions = [0.25, 0.25, 0.15, 0.15, 0.2, 0.0, 0.0]
    return cfg


def _ground(ter, x, y):
    t = ter.cfg
    ix = np.clip(((x + t.border_size) / t.horizontal_scale).astype(int), 0, ter.tot_rows - 1)
    iy = np.clip(((y + t.border_size) / t.horizontal_scale).astype(int), 0, ter.tot_cols - 1)
    return ter.heightsamples[ix, iy] * t.vertical_scale


@pytest.mark.parametrize("mesh", ["trimesh", "heightfield"])
def test_full_step_on_terrain_matches_oracle(mesh):
    terrain_step_vs_oracle(mesh, "cuda")


def terrain_step_vs_oracle(mesh, device):
    from native_util import Twin
    from legged_gym_custom_amd import model as mdl, params as prm
    n = 64
    cfg = _rough_cfg(n, mesh)
    ter, words = G.terrain_for(cfg, np_seed=3)
    m = mdl.load_model(cfg.asset.file, cfg.asset.foot_name)
    P = prm.build_task_params(cfg, m, n, go2=True, terrain_shape=(ter.tot_rows, ter.tot_cols))
    P.push_robots = 0
    P.curriculum = 0
    tw = Twin(P, mdl.to_struct(m), P.num_reward_terms + P.has_termination_reward, terrain=(ter.heightsamples, words),
              device=device)
    rng = np.random.default_rng(11)
    a = tw.a
    a["friction"][:] = rng.uniform(0.3, 1.2, n)
    a["mass_params"][:, 0] = rng.uniform(0, 3, n)
    a["kp_kd"][:] = rng.uniform(0.8, 1.2, a["kp_kd"].shape)
    # robots over every tile, feet near the surface (stairs / slopes / obstacle edges)
    tiles = rng.integers(0, 3, n), rng.integers(0, 4, n)
    x = (tiles[0] + rng.uniform(0.1, 0.9, n)) * 8.0
    y = (tiles[1] + rng.uniform(0.1, 0.9, n)) * 8.0
    root = a["root_states"]
    root[:, 0], root[:, 1] = x, y
    root[:, 2] = _ground(ter, x, y) + rng.uniform(0.26, 0.36, n)
    ax = rng.normal(size=(n, 3))
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    ang = rng.uniform(0, 0.2, n)
    root[:, 3:6] = ax * np.sin(ang / 2)[:, None]
    root[:, 6] = np.cos(ang / 2)
    root[:, 7:13] = rng.normal(0, 0.2, (n, 6))
    q0 = np.array(P.default_dof_pos[:12], np.float32)
    a["dof_state"][:, :, 0] = q0 + rng.normal(0, 0.1, (n, 12))
    a["dof_state"][:, :, 1] = rng.normal(0, 0.5, (n, 12))
    a["actions_in"][:] = rng.normal(0, 0.5, (n, 12))
    a["episode_length"][:] = rng.integers(0, 900, n)
    a["commands"][:, :3] = rng.uniform(-1, 1, (n, 3))
    tw.push()
    tw.o.step(3, 11)
    tw.native.step(3, 11, tw.stream())
    tw.sync()
    ok = a["reset"] == 0
    assert ok.sum() > n // 2
    # the terrain actually carried load
    fz = a["contact_forces"][:, :, 2].sum(1)
    assert (fz[ok] > 1.0).mean() > 0.5
    assert np.array_equal(tw.gpu("reset"), a["reset"])
    np.testing.assert_allclose(tw.gpu("torques"), a["torques"], atol=2e-2, rtol=1e-3)
    np.testing.assert_allclose(tw.gpu("root_states")[ok], a["root_states"][ok], atol=2e-3, rtol=1e-3)
    np.testing.assert_allclose(tw.gpu("dof_state")[ok], a["dof_state"][ok], atol=2e-3, rtol=1e-3)
    np.testing.assert_allclose(tw.gpu("contact_forces")[ok], a["contact_forces"][ok], atol=0.5, rtol=2e-2)
    np.testing.assert_allclose(tw.gpu("measured_heights"), a["measured_heights"], atol=1e-6)
    np.testing.assert_allclose(tw.gpu("obs")[ok], a["obs"][ok], atol=2e-3, rtol=1e-3)


def _run_env(cfg, steps=100):
    import torch
    from legged_gym_custom_amd.envs.go2.go2 import Go2Robot
    from legged_gym_custom_amd.utils.helpers import SimParams, class_to_dict, set_seed
    set_seed(1)
    env = Go2Robot(cfg, SimParams(class_to_dict(cfg.sim)), 1, "cuda:0", True)
    env.reset()
    z = torch.zeros(env.num_envs, 12, device="cuda")
    for _ in range(steps):
        env.step(z)
    torch.cuda.synchronize()
    return env


def _weight_ratio(env, mask):
    fz = env.contact_forces[:, :, 2].sum(1)
    mass = 15.0 + env.privileged_mass_params[:, 0]
    return (fz / (mass * 9.81))[mask]


def test_go2_rough_curriculum_env_stands():
    import torch
    cfg = _rough_cfg(4096)
    cfg.domain_rand.push_robots = False
    cfg.noise.add_noise = False
    env = _run_env(cfg)
    assert env.height_samples.dtype == torch.int16
    assert torch.isfinite(env.root_states).all() and torch.isfinite(env.obs_buf).all()
    ground = torch.from_numpy(_ground(env.terrain, env.root_states[:, 0].cpu().numpy(),
                                      env.root_states[:, 1].cpu().numpy())).cuda()
    clearance = env.root_states[:, 2] - ground
    standing = (clearance > 0.15) & (clearance < 0.45) & (env.projected_gravity[:, 2] < -0.8)
    assert standing.float().mean() > 0.8, clearance.mean()
    assert (_weight_ratio(env, standing).median() - 1.0).abs() < 0.15
    assert "terrain_level" in env.extras["episode"]
    assert env.terrain_levels.max() <= 2
    env2 = _run_env(cfg)
    assert torch.equal(env.root_states, env2.root_states)


def test_go2_parkour_env_builds_and_stands():
    import torch
    from legged_gym_custom_amd.envs import task_registry_configs
    cfg = task_registry_configs("go2_parkour")[0]
    cfg.env.num_envs = 4096
    cfg.domain_rand.push_robots = False
    cfg.noise.add_noise = False
    env = _run_env(cfg, steps=60)
    assert tuple(env.height_samples.shape) == (3860, 2500)
    assert torch.isfinite(env.root_states).all()
    # spawn: tile start + (2, 0) +- 1 m, on the flat start platform (height 0)
    rel = env.root_states[:, :2] - env.env_origins[:, :2]
    assert (rel[:, 0] > 0.5).all() and (rel[:, 0] < 3.5).all()
    h = env.root_states[:, 2]
    standing = (h > 0.2) & (h < 0.45)
    assert standing.float().mean() > 0.9
    assert (_weight_ratio(env, standing).median() - 1.0).abs() < 0.1
    # the scan sees the first gap ahead for no-one yet (5 m away): all zero heights here
    assert env.measured_heights.abs().max() < 1e-6


def test_anymal_rough_env_with_actuator_net(tmp_path):
    """anymal_c_rough end to end on the GPU: rough curriculum trimesh, 187-point scan in
    the 235-dim proprio (history 5 -> obs 1410), SEA actuator net loaded from a
    TorchScript archive (synthetic weights, written here) and run in the kernel; reset
    envs leave the step with zero LSTM state (anymal.py:56-60)."""
    import torch
    from legged_gym_custom_amd import actuator as act
    from legged_gym_custom_amd.envs import task_registry_configs
    from legged_gym_custom_amd.envs.anymal_c.anymal import Anymal
    from legged_gym_custom_amd.utils.helpers import SimParams, class_to_dict, set_seed
    path = str(tmp_path / "sea.pt")
    act.save_sea_archive(act.random_sea_weights(1, scale=0.3), path)
    cfg = task_registry_configs("anymal_c_rough")[0]
    cfg.env.num_envs = 1024
    cfg.terrain.num_rows, cfg.terrain.num_cols = 6, 6   # max_init_terrain_level 5 < num_rows
    cfg.control.actuator_net_file = path
    set_seed(1)
    env = Anymal(cfg, SimParams(class_to_dict(cfg.sim)), 1, "cuda:0", True)
    env.reset()
    assert env.obs_buf.shape == (1024, 1410)
    z = torch.zeros(env.num_envs, 12, device="cuda")
    resets = 0
    for _ in range(30):
        env.step(z)
        resets += int(env.reset_buf.sum())
    torch.cuda.synchronize()
    assert torch.isfinite(env.obs_buf).all() and torch.isfinite(env.sea_hidden_state).all()
    assert env.sea_hidden_state.abs().sum() > 0
    r = env.reset_buf.nonzero().flatten()
    if len(r):
        assert env.sea_hidden_state_per_env[:, r].abs().max() == 0
        assert env.sea_cell_state_per_env[:, r].abs().max() == 0
    heights = env.obs_buf[:, -187:]
    assert heights.abs().max() > 0  # the scan sees the terrain


def test_anymal_missing_actuator_archive_fails_loudly(tmp_path):
    from legged_gym_custom_amd.envs import task_registry_configs
    from legged_gym_custom_amd.envs.anymal_c.anymal import Anymal
    from legged_gym_custom_amd.utils.helpers import SimParams, class_to_dict
    cfg = task_registry_configs("anymal_c_flat")[0]
    cfg.env.num_envs = 8
    cfg.control.actuator_net_file = str(tmp_path / "missing.pt")
    with pytest.raises(FileNotFoundError):
        Anymal(cfg, SimParams(class_to_dict(cfg.sim)), 1, "cuda:0", True)
