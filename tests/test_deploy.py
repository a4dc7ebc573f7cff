"""Deploy observation builder + scan replay (deploy/base/deploy_base.py,
config_parser.py): a sim-to-sim cross-check of the observation layout.

The numpy controller (wxyz quaternion, no noise) is fed the same robot state the env saw,
and its 52-dim observation must equal the env's current-observation slice (go2.py:506-
515), here computed by the C oracle that is pinned to the reference's golden vectors
(test_oracle_golden.py). CPU only."""
import numpy as np
import pytest
import torch

import golden_util as G

YAML = """
model_name: "test_model"
policy_path: "{LEGGED_GYM_ROOT_DIR}/deploy/networks/go2/*model/policy.pt"
adaptation_path: "{LEGGED_GYM_ROOT_DIR}/deploy/networks/go2/*model/adaptation_module.pt"
estimator_path: "{LEGGED_GYM_ROOT_DIR}/deploy/networks/go2/*model/estimator.pt"
scan_encoder_path: "{LEGGED_GYM_ROOT_DIR}/deploy/networks/go2/*model/scan_encoder.pt"
xml_path: "{LEGGED_GYM_ROOT_DIR}/resources/robots/go2/mujoco/scene.xml"
num_actions: 12
num_proprio: 52
buffer_length: 10
num_scan_obs: 132
period: 0.45
fr_offset: 0.0
bl_offset: 0.0
fl_offset: 0.5
br_offset: 0.5
msg_type: "go"
lowcmd_topic: "rt/lowcmd"
lowstate_topic: "rt/lowstate"
simulation_dt: 0.005
control_decimation: 4
leg_joint2motor_idx: [3, 4, 5, 0, 1, 2, 9, 10, 11, 6, 7, 8]
kps: [40.0, 40.0, 40.0, 40.0, 40.0, 40.0, 40.0, 40.0, 40.0, 40.0, 40.0, 40.0]
kds: [1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0]
default_angles: [0.1, 0.8, -1.5, -0.1, 0.8, -1.5, 0.1, 1.0, -1.5, -0.1, 1.0, -1.5]
pitch_offset: 0.0
roll_offset: 0.0
lin_vel_scale: 2.0
ang_vel_scale: 0.25
dof_pos_scale: 1.0
dof_vel_scale: 0.05
action_scale: 0.25
clip_observations: 100.0
clip_actions: 3.14
rc_scale: [1.0, 1.0, 1.0]
"""


@pytest.fixture
def cfg(tmp_path):
    from legged_gym_custom_amd.deploy.base.config_parser import ConfigParser
    p = tmp_path / "go2.yaml"
    p.write_text(YAML)
    return ConfigParser(str(p))


def test_config_parser_paths_and_derived_fields(cfg):
    from legged_gym_custom_amd import LEGGED_GYM_ROOT_DIR
    assert cfg.policy_path == f"{LEGGED_GYM_ROOT_DIR}/deploy/networks/go2/test_model/policy.pt"
    assert cfg.num_obs == 52 * 11
    assert cfg.control_dt == pytest.approx(0.02)
    np.testing.assert_array_equal(cfg.cmd_scale, np.array([2.0, 2.0, 0.25], np.float32))


def _controller(cfg):
    from legged_gym_custom_amd.deploy.base.deploy_base import BaseController
    z = lambda *a: torch.zeros(1, 1)  # noqa: E731  (networks unused by the obs builder)
    return BaseController(cfg, scan_replay_path=None, networks=(z, z, z, z))


def test_deploy_observation_equals_env_observation(cfg):
    """Same state in, same 52 numbers out: env (oracle) vs deploy builder."""
    import driver
    from legged_gym_custom_amd import model as mdl
    n = 48
    env_cfg, m, P = G.go2_setup(n, "go2")
    P.add_noise = 0
    P.push_robots = 0
    o = driver.OracleEnv(P, mdl.to_struct(m), P.num_reward_terms + P.has_termination_reward)
    a = o.a
    rng = np.random.default_rng(4)
    root = a["root_states"]
    root[:, 2] = 0.3
    ax = rng.normal(size=(n, 3))
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    ang = rng.uniform(0, 0.5, n)
    root[:, 3:6] = ax * np.sin(ang / 2)[:, None]
    root[:, 6] = np.cos(ang / 2)
    root[:, 7:13] = rng.normal(0, 0.5, (n, 6))
    q0 = np.array(P.default_dof_pos[:12], np.float32)
    a["dof_state"][:, :, 0] = q0 + rng.normal(0, 0.2, (n, 12))
    a["dof_state"][:, :, 1] = rng.normal(0, 1.5, (n, 12))
    a["commands"][:, :3] = rng.uniform(-1, 1, (n, 3))
    a["commands"][:4, :3] = 0.05  # below the 0.2 gait-phase threshold
    a["episode_length"][:] = rng.integers(2, 450, n)  # no resampling step (ep % 500)
    a["actions_in"][:] = rng.normal(0, 1.0, (n, 12))
    o.clip_actions()
    o.compute_torques()
    o.post_physics(seed=1, step=17)
    ok = a["reset"] == 0
    assert ok.sum() > n // 2
    dt = P.dt
    for e in np.nonzero(ok)[0]:
        c = _controller(cfg)
        q = a["root_states"][e, 3:7]
        c.base_quat = np.array([q[3], q[0], q[1], q[2]], np.float32)  # xyzw -> wxyz
        c.ang_vel = a["base_ang_vel"][e].copy()
        c.qj = a["dof_state"][e, :, 0].copy()
        c.dqj = a["dof_state"][e, :, 1].copy()
        c.cmd = a["commands"][e, :3].copy()
        c.actions = a["actions"][e].copy()
        obs = c.build_observation(float(a["episode_length"][e]) * dt)
        np.testing.assert_allclose(obs[0, -52:].numpy(), a["obs"][e, -52:], atol=2e-5, rtol=1e-5,
                                   err_msg=f"env {e}")
        # the reference's attributes of the same tick (deploy_base.py:184,219-220)
        np.testing.assert_allclose([c.roll, c.pitch], obs[0, -52 + 3:-52 + 5].numpy(), atol=1e-6)
        assert np.isfinite(c.yaw)


def test_history_fill_then_roll(cfg):
    c = _controller(cfg)
    c.base_quat = np.array([1, 0, 0, 0], np.float32)
    assert c.first_step_ever
    o1 = c.build_observation(0.0)
    assert not c.first_step_ever
    assert torch.all(o1[0, :52 * 10] == 0)  # network input: zero history on the first tick
    first = c.obs_history.copy()
    assert np.all(first == first[0])         # then filled with the first observation
    c.qj = c.qj + 0.1
    c.build_observation(0.02)
    np.testing.assert_array_equal(c.obs_history[:-1], first[1:])
    assert not np.array_equal(c.obs_history[-1], first[0])


def test_scan_replay_state_machine(cfg, tmp_path):
    from legged_gym_custom_amd.deploy.base.deploy_base import BaseController, parse_scan_replay
    scans = [np.full(132, 0.01 * (i + 1)) for i in range(5)]
    text = "[0.25]\n\n" + "\n\n".join("[" + " ".join(f"{v:.8f}" for v in s) + "]" for s in scans)
    p = tmp_path / "scan.txt"
    p.write_text(text)
    sync, vecs = parse_scan_replay(text)
    assert sync == 0.25 and len(vecs) == 5
    z = lambda *a: torch.zeros(1, 1)  # noqa: E731
    c = BaseController(cfg, scan_replay_path=str(p), networks=(z, z, z, z))
    c.phase = 0.5
    assert torch.all(c._get_scan_obs() == 0) and c.mode == "NORMAL"
    c.jump_button_pressed = True
    assert torch.all(c._get_scan_obs() == 0) and c.mode == "WAITING"   # phase not synced yet
    c.phase = 0.252
    fed = [c._get_scan_obs() for _ in range(4)]
    np.testing.assert_allclose(fed[0].numpy()[0], scans[0], rtol=1e-6)
    np.testing.assert_allclose(fed[3].numpy()[0], scans[3], rtol=1e-6)
    assert c.mode == "NORMAL" and c.scan_idx == 0  # ends one short of the recording, as the reference
