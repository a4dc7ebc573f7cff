"""Host-side parameter derivation (params.build_task_params, model.load_model) against
the constants the reference computed for the golden fixture (tools/gen_golden.py):
gains, limits, default pose, noise vector (with the go2.py:120-127 slot offsets) and
the alphabetical, dt-scaled reward terms (legged_robot.py:730-754)."""
import numpy as np

import golden_util as G
from legged_gym_custom_amd import _abi


def test_task_params_match_reference_constants():
    d = G.load("go2_flat_n64.npz")
    cfg, m, P = G.go2_setup(int(d["num_envs"]))
    D = P.num_dof
    np.testing.assert_allclose(np.array(P.default_dof_pos[:D]), d["default_dof_pos"].reshape(-1), rtol=1e-6)
    np.testing.assert_allclose(np.array(P.p_gains[:D]), d["p_gains"].reshape(-1), rtol=1e-6)
    np.testing.assert_allclose(np.array(P.d_gains[:D]), d["d_gains"].reshape(-1), rtol=1e-6)
    np.testing.assert_allclose(np.array(P.torque_limits[:D]), d["torque_limits"].reshape(-1), rtol=1e-6)
    lim = np.array([[P.dof_pos_limits[i][0], P.dof_pos_limits[i][1]] for i in range(D)])
    np.testing.assert_allclose(lim, d["dof_pos_limits"].reshape(D, 2), rtol=1e-6, atol=1e-7)
    nv = np.array(P.noise_vec[:P.num_proprio])
    np.testing.assert_allclose(nv, d["noise_scale_vec"].reshape(-1)[:P.num_proprio], rtol=1e-6)


def test_reward_terms_order_and_scales():
    d = G.load("go2_flat_n64.npz")
    cfg, m, P = G.go2_setup(int(d["num_envs"]))
    inv = {v: k for k, v in _abi.REWARD_IDS.items()}
    names = [inv[P.reward_ids[i]] for i in range(P.num_reward_terms)]
    ref_names = [str(n) for n in d["reward_names"]]
    ref_scales = d["reward_scales"].astype(np.float64)
    k = [i for i, n in enumerate(ref_names) if n != "termination"]
    assert names == [ref_names[i] for i in k]
    np.testing.assert_allclose(np.array(P.reward_scales[:P.num_reward_terms]), ref_scales[k], rtol=1e-6)
    assert names == sorted(names)  # alphabetical dict order of class_to_dict
