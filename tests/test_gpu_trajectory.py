"""Multi-step parity of the HIP env step (liblgx.so) against the CPU oracle, PD torques
against the reference's golden vectors, and env-shard equivalence.

* re-synced trajectory (SURVEY.md §8c hop 2): 200 steps at N=64 with N(0,1) actions, pushes
  and resets. Before each step the oracle is loaded with the GPU's state, both take one step,
  and every field is compared: integer/bool state (reset, time-out, episode length, contact
  flags) exactly; floats within the one-step bounds below (fp32 kernel vs fp64 dense oracle,
  fixed-iteration Gauss-Seidel): root 5e-4 abs, dof / rigid-body 2e-3, contact forces
  0.25 N + 2 %, observations 2e-4, rewards 1e-5, torques 5e-3 (BOUNDS; observed maxima there).
* free-running trajectory, 1000 steps at N=128 from identical states and actions: contact
  dynamics are chaotic, so envs diverge individually; the run statistics are compared
  (bounds in the test).
* PD torques (legged_robot.py:440-478): one decimation-1 physics step from the golden
  fixture's scripted state gives the reference's `torques` to 1e-5.
* shards: two envs of N/2 with env_id_offset 0 and N/2 (num_envs_total N) reproduce one env
  of N bitwise over 50 steps (global env ids key the Philox streams, terrain types and the
  setup-time randomisation; legged_robot.py:914)."""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu

EXACT = ["reset", "time_out", "episode_length", "last_contacts"]
BOUNDS = {  # field: (atol, rtol), one step from identical inputs (observed maxima over the
    # 200 steps, r02: root 6.9e-5, dof 4.7e-4, rigid bodies 4.5e-4, contact 0.04 N, obs 2.4e-5,
    # rew 7.8e-8, torques 6.2e-4, commands 0)
    "root_states": (5e-4, 1e-4), "dof_state": (2e-3, 1e-4), "rigid_body_states": (2e-3, 1e-4),
    "contact_forces": (0.25, 2e-2), "obs": (2e-4, 1e-4), "critic": (2e-4, 1e-4), "rew": (1e-5, 1e-4),
    "torques": (5e-3, 1e-4), "commands": (1e-6, 0.0)}


def _twin(n, task="go2", push=True, decimation=None, device="cuda"):
    from native_util import Twin
    from legged_gym_custom_amd import model as mdl
    cfg, m, P = G.go2_setup(n, task)
    if not push:
        P.push_robots = 0
    if decimation is not None:
        P.decimation = decimation
    tw = Twin(P, mdl.to_struct(m), P.num_reward_terms + P.has_termination_reward, device=device)
    return cfg, P, tw


def _init(tw, P, n, rng):
    a = tw.a
    a["friction"][:] = rng.uniform(0.3, 1.2, n)
    a["mass_params"][:, 0] = rng.uniform(-1, 2, n)
    a["mass_params"][:, 1:] = rng.uniform(-0.05, 0.05, (n, 3))
    a["kp_kd"][:] = rng.uniform(0.9, 1.1, a["kp_kd"].shape)
    tw.push()
    mask = tw.torch.ones(n, dtype=tw.torch.uint8, device=tw.device)
    tw.native.reset_envs(mask, 5, 0, tw.stream())
    tw.sync()
    tw.pull()
    a["episode_length"][:] = rng.integers(0, 1000, n)  # episodes at every phase incl. time-outs
    tw.push()


def test_resynced_trajectory_matches_oracle():
    resynced_trajectory("cuda", 200)


def resynced_trajectory(device, steps):
    n = 64
    cfg, P, tw = _twin(n, device=device)
    rng = np.random.default_rng(11)
    _init(tw, P, n, rng)
    worst = {k: 0.0 for k in BOUNDS}
    nreset = 0
    for k in range(steps):
        act = rng.normal(0, 1.0, (n, 12)).astype(np.float32)
        tw.a["actions_in"][:] = act
        tw.t["actions_in"].copy_(tw.torch.from_numpy(act))
        tw.pull()
        tw.o.step(5, k + 1)
        tw.native.step(5, k + 1, tw.stream())
        tw.sync()
        a = tw.a
        for f in EXACT:
            assert np.array_equal(tw.gpu(f).astype(np.int64), a[f].astype(np.int64)), f"step {k}: {f}"
        ok = a["reset"] == 0
        nreset += int((~ok).sum())
        for f, (at, rt) in BOUNDS.items():
            g, o = tw.gpu(f), a[f]
            if f in ("contact_forces", "rew", "rigid_body_states"):  # physics of the reset step is discarded
                g, o = g[ok], o[ok]
            err = np.abs(g - o) - rt * np.abs(o)
            worst[f] = max(worst[f], float(np.max(np.abs(g - o)) if g.size else 0.0))
            assert (err <= at).all(), f"step {k}: {f} max |d| {np.max(np.abs(g - o)):.3g}"
    print("max |gpu - oracle| per field over", steps, "steps:", {k: f"{v:.2e}" for k, v in worst.items()},
          "resets:", nreset)
    assert nreset > 0


def _stats(hist):
    h = np.array(hist)  # [T, N, 4]: base z, |v_xy|, reset, |qd|
    return {"z_mean": h[:, :, 0].mean(), "v_mean": h[:, :, 1].mean(), "reset_rate": h[:, :, 2].mean(),
            "qd_mean": h[:, :, 3].mean()}


def test_free_running_trajectory_statistics():
    free_running_statistics("cuda", 1000)


def free_running_statistics(device, steps):
    n = 128
    cfg, P, tw = _twin(n, device=device)
    rng = np.random.default_rng(3)
    _init(tw, P, n, rng)
    go, gg = [], []
    for k in range(steps):
        act = np.clip(rng.normal(0, 0.5, (n, 12)), -3, 3).astype(np.float32)
        tw.a["actions_in"][:] = act
        tw.t["actions_in"].copy_(tw.torch.from_numpy(act))
        tw.o.step(9, k + 1)
        tw.native.step(9, k + 1, tw.stream())
        tw.sync()
        for rec, src in ((go, tw.a), (gg, {f: tw.gpu(f) for f in ("root_states", "reset", "dof_state")})):
            r = src["root_states"]
            rec.append(np.stack([r[:, 2], np.hypot(r[:, 7], r[:, 8]), src["reset"].astype(np.float32),
                                 np.abs(src["dof_state"][:, :, 1]).mean(1)], 1))
    so, sg = _stats(go), _stats(gg)
    print("oracle", {k: f"{v:.4f}" for k, v in so.items()}, "gpu", {k: f"{v:.4f}" for k, v in sg.items()})
    # same physics, fp32 vs fp64: the per-env trajectories decorrelate after contact events,
    # the population statistics agree
    # (r02: all four agree to 4 digits: z 0.2967 m, |v_xy| 0.174 m/s, resets 0.0010/step,
    # |qd| 1.58 rad/s)
    assert abs(sg["z_mean"] - so["z_mean"]) < 0.005
    assert abs(sg["v_mean"] - so["v_mean"]) < 0.05 * so["v_mean"] + 0.005
    assert abs(sg["qd_mean"] - so["qd_mean"]) < 0.05 * so["qd_mean"]
    assert abs(sg["reset_rate"] - so["reset_rate"]) < 0.5 * so["reset_rate"] + 1e-3
    # and the first steps, before any contact event can diverge, agree per env
    np.testing.assert_allclose(np.array(gg[:5]), np.array(go[:5]), atol=5e-3, rtol=1e-2)


@pytest.mark.parametrize("name,task", [("go2_flat_n64.npz", "go2"), ("go2_parkour_n64.npz", "go2_parkour")])
def test_pd_torques_match_golden(name, task):
    """_compute_torques on the fixture's scripted state: decimation-1 physics from that state,
    whose first (only) substep's torques are the kernel's own PD law."""
    from native_util import Twin
    from legged_gym_custom_amd import model as mdl
    d = G.load(name)
    N = int(d["num_envs"])
    cfg, m, P, terrain, _ = G.fixture_setup(d, task)
    P.decimation = 1
    tw = Twin(P, mdl.to_struct(m), P.num_reward_terms + P.has_termination_reward, terrain=terrain)
    a = tw.a
    a["friction"][:] = d["friction"]
    a["mass_params"][:] = d["mass_params"]
    a["kp_kd"][:] = d["kp_kd_multipliers"]
    a["env_origins"][:] = d["env_origins"]
    tw.push()
    checked = 0
    for step in range(G.num_steps(d)):
        S = lambda k: G.step(d, step, k)  # noqa: E731
        tw.t["actions_in"].copy_(tw.torch.from_numpy(S("actions_raw")))
        tw.t["root_states"].copy_(tw.torch.from_numpy(S("physics.root_states")))
        tw.t["dof_state"].copy_(tw.torch.from_numpy(S("physics.dof_state").reshape(N, 12, 2)))
        tw.native.step(int(d["seed"]), int(S("csc_in")) + 1, tw.stream())
        tw.sync()
        np.testing.assert_allclose(tw.gpu("torques"), S("out.torques"), atol=1e-5, rtol=1e-5,
                                   err_msg=f"step {step}")
        checked += 1
    assert checked >= 20


def _make_env(n, offset=None, total=None):
    import torch
    from legged_gym_custom_amd.envs import task_registry_configs
    from legged_gym_custom_amd.envs.go2.go2 import Go2Robot
    from legged_gym_custom_amd.utils.helpers import SimParams, class_to_dict, set_seed
    cfg, _ = task_registry_configs("go2")
    cfg.env.num_envs = n
    cfg.domain_rand.push_interval_s = 0.2  # pushes inside the window
    set_seed(0)
    dist = torch.distributed
    saved = (dist.is_initialized, dist.get_rank, dist.get_world_size)
    if offset is not None:  # stand-in for rank offset // n of a world of total // n ranks
        dist.is_initialized = lambda: True
        dist.get_rank = lambda: offset // n
        dist.get_world_size = lambda: total // n
    try:
        env = Go2Robot(cfg, SimParams(class_to_dict(cfg.sim)), 1, "cuda:0", True)
    finally:
        dist.is_initialized, dist.get_rank, dist.get_world_size = saved
    return env


def test_two_shards_reproduce_one_env():
    import torch
    n = 256
    full = _make_env(n)
    shards = [_make_env(n // 2, 0, n), _make_env(n // 2, n // 2, n)]
    for sh, off in zip(shards, (0, n // 2)):
        assert sh.env_id_offset == off and sh.num_envs_total == n
        for f in ("friction_coeffs", "privileged_mass_params", "kp_kd_multipliers", "env_origins"):
            a, b = getattr(full, f), getattr(sh, f)
            b_full = a[:, off:off + n // 2] if f == "kp_kd_multipliers" else a[off:off + n // 2]
            assert torch.equal(b_full.to(b.device), b), f
    envs = [full] + shards
    for e in envs:
        e.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    for k in range(50):
        act = torch.randn(n, 12, device="cuda", generator=g)
        full.step(act)
        shards[0].step(act[: n // 2].contiguous())
        shards[1].step(act[n // 2:].contiguous())
    torch.cuda.synchronize()
    for f in ("root_states", "obs_buf", "rew_buf", "reset_buf", "episode_length_buf", "commands", "critic_obs_buf"):
        whole = getattr(full, f)
        parts = torch.cat([getattr(s, f) for s in shards])
        assert torch.equal(whole, parts), f
