"""liblgx.so's host backend (lgx_create(device=-1), the reference's --sim_device=cpu,
helpers.py:174-177) against the same references as the HIP kernels, on the CPU:

* post-physics replay of the three golden fixtures recorded from the reference's own tensor
  code (go2 flat, go2_parkour, anymal_c_rough): atol = rtol = 1e-5;
* the SEA actuator step against torch's fp32 nn.LSTM;
* one full env step (physics + post-physics) against the oracle's double-precision dense
  restatement, on the plane and on trimesh / heightfield terrain: atol 2e-3 on the state,
  exact on integer/bool state;
* a re-synced 200-step trajectory (integer state exact at every step, the GPU test's one-step
  float bounds) and 1000-step free-running population statistics against the oracle.

The bodies are the GPU tests' (tests/test_gpu_parity.py, test_gpu_trajectory.py,
test_gpu_terrain.py) run with device="cpu"."""
import pytest

import test_gpu_parity as T
import test_gpu_terrain as TT
import test_gpu_trajectory as TJ


@pytest.mark.parametrize("name,task", T.GOLDEN_CASES)
def test_host_post_physics_matches_reference_golden(name, task):
    T.golden_replay(name, task, "cpu")


def test_host_sea_actuator_matches_torch_lstm():
    T.sea_vs_torch("cpu")


def test_host_full_step_matches_oracle():
    T.full_step_vs_oracle("cpu")


@pytest.mark.parametrize("mesh", ["trimesh", "heightfield"])
def test_host_full_step_on_terrain_matches_oracle(mesh):
    TT.terrain_step_vs_oracle(mesh, "cpu")


def test_host_resynced_trajectory_matches_oracle():
    TJ.resynced_trajectory("cpu", 200)


def test_host_free_running_statistics():
    TJ.free_running_statistics("cpu", 1000)


def test_inconsistent_observation_config_is_refused():
    """anymal_c_flat as the reference ships it declares 48-wide observations over a 235-wide
    proprio history (the reference fails at its first compute_observations); lgx_create
    refuses it instead of writing past the observation rows."""
    import golden_util as G
    from legged_gym_custom_amd import _native, model as mdl
    cfg, m, P = G.go2_setup(8, "anymal_c_flat")
    with pytest.raises(_native.LgxError, match="num_proprio"):
        _native.NativeEnv(mdl.to_struct(m), P, -1)


def test_train_c1_on_cpu():
    """Config C1: `train.py --task=go2 --sim_device=cpu --rl_device=cpu
    --num_envs=64` — the drop-in flow (make_env -> make_alg_runner -> learn) on the host
    backend and the torch-CPU learner; two iterations, finite state, episodes reset."""
    import torch
    from legged_gym_custom_amd.envs import task_registry
    from legged_gym_custom_amd.utils.helpers import get_args
    a = get_args(["--task=go2", "--headless", "--num_envs=64", "--sim_device=cpu", "--rl_device=cpu", "--seed=1"])
    env, _ = task_registry.make_env("go2", a)
    assert env.device == "cpu" and env._native.device_index == -1
    _, tcfg = task_registry.get_cfgs("go2")
    tcfg.runner.num_steps_per_env = 8
    runner, _ = task_registry.make_alg_runner(env, args=a, train_cfg=tcfg, log_root=None)
    runner.learn(num_learning_iterations=2, init_at_random_ep_len=True)
    assert torch.isfinite(env.obs_buf).all() and torch.isfinite(env.root_states).all()
    assert int(env.episode_length_buf.max()) > 0
    assert all(torch.isfinite(p).all() for p in runner.alg.actor_critic.parameters())


@pytest.mark.parametrize("z", [(0.06, 0.16), (0.2, 0.27)])
def test_host_crowded_contacts_match_oracle(z):
    T.crowded_contacts_vs_oracle("cpu", z)


def test_host_nan_guard_resets_only_the_blown_up_env():
    T.nan_guard("cpu")


def test_host_command_curriculum_env():
    T.command_curriculum_env("cpu")
