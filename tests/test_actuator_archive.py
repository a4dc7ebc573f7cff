"""The reference's own ANYmal actuator network (resources/actuator_nets/anydrive_v3_lstm.pt,
loaded at anymal.py:54) read by the build's non-executing archive reader
(legged_gym_custom_amd.actuator: zip storages + a pickletools walk; nothing unpickled or
run), and evaluated by the C oracle (lgx_oracle.c, the kernel's checker) against the torch
restatement of the archive's LSTMsea (actuator.SeaLSTM). Runs only where the reference
tree is present (the build container); nothing from the archive is stored in the repo.
CPU only."""
import os

import numpy as np
import pytest
import torch

import golden_util as G

ARCHIVE = "/root/reference/resources/actuator_nets/anydrive_v3_lstm.pt"
pytestmark = pytest.mark.skipif(not os.path.exists(ARCHIVE), reason="reference archive not present")


def test_reader_parses_the_reference_archive():
    from legged_gym_custom_amd import actuator as act
    w = act.load_sea_lstm(ARCHIVE)  # raises unless all 12 tensors are present with the reference shapes
    assert sorted(w) == sorted(act.SEA_KEYS)
    for k in act.SEA_KEYS:
        assert w[k].shape == act.SEA_SHAPES[k] and w[k].dtype == np.float32
        assert np.isfinite(w[k]).all()
    # trained, not a zero/placeholder file
    assert np.abs(w["lstm.weight_hh_l1"]).max() > 1e-3 and float(w["out_scale"][0]) != 0.0


def test_oracle_sea_torques_match_torch_on_reference_weights():
    """One actuator call (anymal.py:71-81) per joint of 64 envs: oracle torques and LSTM
    state vs SeaLSTM (torch fp32) on the reference's weights; then three chained calls."""
    import driver
    from legged_gym_custom_amd import actuator as act, model as mdl
    w = act.load_sea_lstm(ARCHIVE)
    n = 64
    cfg, m, P = G.go2_setup(n, "anymal_c_flat")
    act.fill_task_params(P, w)
    o = driver.OracleEnv(P, mdl.to_struct(m), P.num_reward_terms + P.has_termination_reward)
    a = o.a
    rng = np.random.default_rng(3)
    q0 = np.array(P.default_dof_pos[:12], np.float32)
    a["dof_state"][:, :, 0] = q0 + rng.normal(0, 0.2, (n, 12))
    a["dof_state"][:, :, 1] = rng.normal(0, 2.0, (n, 12))
    a["actions_in"][:] = rng.normal(0, 1.0, (n, 12))
    a["sea_hidden"][:] = rng.normal(0, 0.3, a["sea_hidden"].shape)
    a["sea_cell"][:] = rng.normal(0, 0.3, a["sea_cell"].shape)
    o.clip_actions()
    net = act.SeaLSTM(w)
    h = torch.from_numpy(a["sea_hidden"].copy())
    c = torch.from_numpy(a["sea_cell"].copy())
    for _ in range(3):
        x = torch.from_numpy(((a["actions"] * P.action_scale + q0) - a["dof_state"][:, :, 0]).reshape(-1))
        xin = torch.stack([x, torch.from_numpy(a["dof_state"][:, :, 1].reshape(-1))], -1)[:, None, :]
        with torch.no_grad():
            tau, (h, c) = net(xin, (h, c))
        o.compute_torques()
        np.testing.assert_allclose(a["torques"].reshape(-1), tau.numpy(), rtol=1e-4, atol=2e-4)
        np.testing.assert_allclose(a["sea_hidden"], h.numpy(), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(a["sea_cell"], c.numpy(), rtol=1e-4, atol=1e-5)
        a["dof_state"][:, :, 1] += rng.normal(0, 0.5, (n, 12)).astype(np.float32)
    assert np.abs(tau.numpy()).max() > 1.0  # the trained net produces real torques here
