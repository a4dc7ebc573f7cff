"""Env-sharded multi-process learner on CPU with gloo, world_size 2.

Each rank holds its own envs' rollout. The only exchanges are the advantage moments
(one all-reduce of {sum a, sum a^2, n}) and, per minibatch, one all-reduce of the flat
[main | estimator | kl] gradient buffer. With equal per-rank minibatches the result must
equal ONE process learning on the union of the shards with the union minibatches
(means of means = mean of the union), and every rank must end with identical weights."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_ppo_update import N, T, _make

WORLD = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rollout(seed, n_envs):
    """Synthetic [T, n_envs, .] rollout fields + last values (seeded)."""
    g = torch.Generator().manual_seed(seed)
    alg = _make("adaptive")
    s = alg.storage
    shapes = {name: (T, n_envs) + tuple(getattr(s, name).shape[2:]) for name in
              ("observations", "privileged_observations", "critic_observations", "true_estimated_observations",
               "scan_observations", "actions", "rewards", "values", "mu", "sigma", "actions_log_prob", "dones")}
    d = {k: torch.randn(v, generator=g) for k, v in shapes.items()}
    d["sigma"] = d["sigma"].abs() + 0.5
    d["actions_log_prob"] = -d["actions_log_prob"].abs() * 5
    d["dones"] = (torch.rand(shapes["dones"], generator=g) < 0.2).byte()
    return d, torch.randn(n_envs, 1, generator=g)


def _load(alg, d, last_values):
    s = alg.storage
    for k, v in d.items():
        getattr(s, k).copy_(v)
    s.step = T
    s.compute_returns(last_values, alg.gamma, alg.lam)


def _flat_params(alg):
    return torch.cat([p.detach().reshape(-1) for p in list(alg.actor_critic.parameters()) +
                      list(alg.estimator.parameters())])


def _worker(rank, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        torch.manual_seed(0)
        alg = _make("adaptive", seed=0)  # identical init on every rank
        alg._next_perm = lambda n: torch.arange(n)
        d, lv = _rollout(100 + rank, N)
        _load(alg, d, lv)
        adv = alg.storage.advantages.clone()
        alg.update_dagger()
        _load(alg, d, lv)
        alg.update()
        out[rank] = {"adv": adv, "params": _flat_params(alg), "lr": alg.learning_rate,
                     "adapt_grads": alg.grads.segment("adaptation").clone()}
    finally:
        dist.destroy_process_group()


def _union_perm(n_local, mb):
    """Union-storage rows of minibatch i = rank 0's rows i*mb.. then rank 1's (flat row
    t*N + n of a shard -> t*2N + rank*N + n of the union)."""
    blocks = []
    for i in range(n_local * T // mb):
        for r in range(WORLD):
            f = torch.arange(i * mb, (i + 1) * mb)
            t, n = f // n_local, f % n_local
            blocks.append(t * (WORLD * n_local) + r * n_local + n)
    return torch.cat(blocks)


@pytest.fixture(scope="module")
def sharded():
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(_port(), out), nprocs=WORLD, join=True)
    return dict(out)


@pytest.fixture(scope="module")
def union():
    import test_ppo_update as tpu
    shards = [_rollout(100 + r, N) for r in range(WORLD)]
    saved = tpu.N
    tpu.N = WORLD * N
    try:
        alg = _make("adaptive", seed=0)
    finally:
        tpu.N = saved
    d = {k: torch.cat([s[0][k] for s in shards], dim=1) for k in shards[0][0]}
    lv = torch.cat([s[1] for s in shards], dim=0)
    mb = N * T // alg.num_mini_batches
    perm = _union_perm(N, mb)
    alg._next_perm = lambda n: perm
    _load(alg, d, lv)
    adv = alg.storage.advantages.clone()
    alg.update_dagger()
    _load(alg, d, lv)
    alg.update()
    return {"adv": adv, "params": _flat_params(alg), "lr": alg.learning_rate,
            "adapt_grads": alg.grads.segment("adaptation").clone()}


def test_advantages_normalised_with_global_moments(sharded, union):
    for r in range(WORLD):
        torch.testing.assert_close(sharded[r]["adv"], union["adv"][:, r * N:(r + 1) * N], rtol=1e-5, atol=1e-6)


def test_ranks_end_identical(sharded):
    assert torch.equal(sharded[0]["params"], sharded[1]["params"])
    assert sharded[0]["lr"] == sharded[1]["lr"]


def test_sharded_update_equals_union_update(sharded, union):
    torch.testing.assert_close(sharded[0]["params"], union["params"], rtol=1e-4, atol=2e-6)
    assert sharded[0]["lr"] == pytest.approx(union["lr"], rel=1e-12)
    torch.testing.assert_close(sharded[0]["adapt_grads"], union["adapt_grads"], rtol=1e-3, atol=1e-7)


def _runner_worker(rank, port, out):
    """A runner per rank (oracle env, CPU): identical initial weights (broadcast), then
    per-rank generators, so rank r's exploration noise is not rank 0's."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import cpu_env
        from legged_gym_custom_amd import model as mdl, params as prm
        from legged_gym_custom_amd.envs import task_registry_configs
        from legged_gym_custom_amd.rsl_rl.runners import OnPolicyRunner
        from legged_gym_custom_amd.utils.helpers import class_to_dict
        cfg, tcfg = task_registry_configs("go2")
        cfg.env.num_envs = 8
        m = mdl.load_model(cfg.asset.file, cfg.asset.foot_name)
        P = prm.build_task_params(cfg, m, 8)
        env = cpu_env.OracleVecEnv(cfg, m, P, mdl.to_struct(m))
        tcfg.runner.num_steps_per_env = 2
        torch.manual_seed(1)  # same seed on both ranks, as set_seed does
        r = OnPolicyRunner(env, class_to_dict(tcfg), None, device="cpu")
        o = r.env.get_observations()
        with torch.no_grad():
            a = r.alg.actor_critic.act(o, r.env.get_privileged_observations(), r.env.get_estimated_observations(),
                                       r.env.get_scan_observations())
        out[rank] = {"w": r.alg.actor_critic.actor[0].weight.detach().clone(), "noise": a - r.alg.actor_critic.action_mean}
    finally:
        dist.destroy_process_group()


def test_ranks_share_weights_but_not_noise():
    out = mp.Manager().dict()
    mp.spawn(_runner_worker, args=(_port(), out), nprocs=WORLD, join=True)
    assert torch.equal(out[0]["w"], out[1]["w"])
    assert not torch.allclose(out[0]["noise"], out[1]["noise"])


def _curriculum_run(n, steps):
    """Host-backend Go2 env (its shard under a process group) with the command curriculum,
    driven to a curriculum step; returns the ranges and this shard's commands."""
    from legged_gym_custom_amd.envs import task_registry_configs
    from legged_gym_custom_amd.envs.go2.go2 import Go2Robot
    from legged_gym_custom_amd.utils.helpers import SimParams, class_to_dict, set_seed
    cfg, _ = task_registry_configs("go2")
    cfg.env.num_envs = n
    cfg.commands.curriculum = True
    cfg.commands.ranges.lin_vel_x = [-0.3, 0.4]
    set_seed(0)
    env = Go2Robot(cfg, SimParams(class_to_dict(cfg.sim)), 1, "cpu", True)
    env.reset()
    z = torch.zeros(n, 12)
    env.common_step_counter = 999 - steps
    k = env.reward_names.index("tracking_lin_vel")
    top = env.reward_scales["tracking_lin_vel"] * env.max_episode_length
    # global envs 0..N/2: 0.95 of the episode maximum, the rest 0.7 — the global mean (0.825)
    # passes the 0.8 threshold, the second shard's own mean would not
    half = env.num_envs_total // 2
    full = torch.cat([torch.full((half,), 0.95 * top), torch.full((half,), 0.7 * top)])
    off = env.env_id_offset
    for _ in range(steps):
        env.step(z)
    env.episode_length_buf = torch.full((n,), 1000, dtype=torch.long)
    env.episode_sums_buf[:, k] = full[off:off + n]
    env.step(z)
    return env.command_ranges["lin_vel_x"], env.commands.clone()


def _curriculum_worker(rank, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        out[rank] = _curriculum_run(8, 3)
    finally:
        dist.destroy_process_group()


def test_sharded_command_curriculum_uses_global_mean():
    """go2.py:87's mean over the reset envs of ALL shards (one all-reduce of {sum, count} on the
    curriculum step): both ranks widen the range exactly when one process over the union does,
    and resample the same commands (global env ids key the draws)."""
    out = mp.Manager().dict()
    mp.spawn(_curriculum_worker, args=(_port(), out), nprocs=WORLD, join=True)
    union_range, union_cmd = _curriculum_run(8 * WORLD, 3)
    assert out[0][0] == out[1][0] == union_range == [-0.3 - 0.1, 0.4 + 0.1]
    assert torch.equal(torch.cat([out[0][1], out[1][1]]), union_cmd)
