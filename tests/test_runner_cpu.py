"""OnPolicyRunner host logic on the CPU (oracle env, torch-CPU learner): the learn loop
(DAgger at it % 20 == 0, then PPO), and checkpoints in the reference's format
(on_policy_runner.py:283-297) that load back into a fresh runner."""
import os

import torch

from legged_gym_custom_amd import model as mdl, params as prm
from legged_gym_custom_amd.envs import task_registry_configs
from legged_gym_custom_amd.rsl_rl.runners import OnPolicyRunner
from legged_gym_custom_amd.utils.helpers import class_to_dict


def _runner(log_dir, n=16, steps=4):
    import cpu_env
    cfg, tcfg = task_registry_configs("go2")
    cfg.env.num_envs = n
    m = mdl.load_model(cfg.asset.file, cfg.asset.foot_name)
    P = prm.build_task_params(cfg, m, n)
    env = cpu_env.OracleVecEnv(cfg, m, P, mdl.to_struct(m))
    tcfg.runner.num_steps_per_env = steps
    torch.manual_seed(1)
    return OnPolicyRunner(env, class_to_dict(tcfg), log_dir, device="cpu")


def test_learn_saves_reference_format_checkpoints(tmp_path):
    r = _runner(str(tmp_path))
    r.learn(2, init_at_random_ep_len=True)
    assert r.current_learning_iteration == 2
    files = sorted(os.listdir(tmp_path))
    assert "model_0.pt" in files and "model_2.pt" in files
    ck = torch.load(os.path.join(tmp_path, "model_2.pt"), weights_only=True)
    for k in ("model_state_dict", "optimizer_state_dict", "iter", "infos"):
        assert k in ck
    assert ck["iter"] == 2
    assert "actor.0.weight" in ck["model_state_dict"] and ck["model_state_dict"]["actor.0.weight"].shape == (512, 627)
    assert "adaptation_encoder_.conv_layers.0.weight" in ck["model_state_dict"]
    groups = ck["optimizer_state_dict"]["param_groups"]
    assert len(groups) == 5 and all(isinstance(g["lr"], float) for g in groups)
    # a fresh runner resumes from it
    r2 = _runner(None)
    r2.load(os.path.join(tmp_path, "model_2.pt"))
    assert r2.current_learning_iteration == 2
    for (k, a), (_, b) in zip(r.alg.actor_critic.state_dict().items(), r2.alg.actor_critic.state_dict().items()):
        assert torch.equal(a, b), k
    s1 = r.alg.optimizer.state_dict()["state"]
    s2 = r2.alg.optimizer.state_dict()["state"]
    for i in s1:
        assert torch.equal(s1[i]["exp_avg"], s2[i]["exp_avg"])
    assert r2.alg.grads.check()
    r2.learn(1)  # and keeps learning
    assert all(torch.isfinite(p).all() for p in r2.alg.actor_critic.parameters())


def test_device_episode_logging_matches_reference_deques():
    """_track_episodes (graph-capturable) == the reference's deque bookkeeping
    (on_policy_runner.py:160-170) over many steps, incl. >100 dones in one step."""
    from collections import deque
    r = OnPolicyRunner.__new__(OnPolicyRunner)
    r.device = "cpu"
    n = 300
    z = lambda *sh: torch.zeros(*sh)  # noqa: E731
    r._stats = {"cur_rew": z(n), "cur_len": z(n), "rew_ring": z(101), "len_ring": z(101),
                "ptr": torch.zeros((), dtype=torch.long), "n": torch.zeros((), dtype=torch.long), "ep_keys": None,
                "ep_sum": None, "ep_cnt": z(())}
    rewbuffer, lenbuffer = deque(maxlen=100), deque(maxlen=100)
    cur_r, cur_l = torch.zeros(n), torch.zeros(n)
    g = torch.Generator().manual_seed(0)
    ep_vals = []
    for step in range(60):
        rewards = torch.randn(n, generator=g)
        p = 0.5 if step == 7 else 0.05
        dones = torch.rand(n, generator=g) < p
        info = {"episode": {"rew_a": torch.tensor(float(step)), "rew_b": torch.tensor(2.0 * step)}}
        r._track_episodes(rewards, dones, info)
        ep_vals.append([float(step), 2.0 * step])
        cur_r += rewards
        cur_l += 1
        ids = dones.nonzero(as_tuple=False)
        rewbuffer.extend(cur_r[ids][:, 0].tolist())
        lenbuffer.extend(cur_l[ids][:, 0].tolist())
        cur_r[ids] = 0
        cur_l[ids] = 0
    rew, ln, ep = r._host_stats()
    assert rew == list(rewbuffer) and ln == list(lenbuffer)
    assert ep["rew_a"] == sum(v[0] for v in ep_vals) / 60 and ep["rew_b"] == sum(v[1] for v in ep_vals) / 60


def test_storage_holds_the_observations_the_policy_acted_on():
    """Each stored transition pairs an action with the observations it was taken on
    (ppo.py:129-153 + rollout_storage.py:87-105). The env writes its buffers in place, so
    the storage must snapshot them at act time, not after env.step; and the stored log-prob
    must equal the policy's log-prob of the stored action at the stored observations."""
    r = _runner(None, steps=4)
    seen = []
    act = r.alg.act

    def spy(obs, priv, critic, est, scan, **kw):
        seen.append([x.clone() for x in (obs, priv, critic, est, scan)])
        return act(obs, priv, critic, est, scan, **kw)

    r.alg.act = spy
    checked = []

    def check(*a, **k):
        s = r.alg.storage
        for t in range(4):
            for got, want in zip((s.observations[t], s.privileged_observations[t], s.critic_observations[t],
                                  s.true_estimated_observations[t], s.scan_observations[t]), seen[t]):
                assert torch.equal(got, want), t
            ac = r.alg.actor_critic
            with torch.no_grad():
                est = r.alg.estimator(s.observations[t])
                # iteration 0 is a DAgger iteration: the rollout acts in adaptation mode
                ac.update_distribution(s.observations[t], s.privileged_observations[t], est, s.scan_observations[t],
                                       adaptation_mode=True)
                lp = ac.get_actions_log_prob(s.actions[t])
            torch.testing.assert_close(lp, s.actions_log_prob[t].view(-1), rtol=1e-5, atol=1e-5)
        checked.append(True)
        return (0.0,) * 8

    r.alg.update_dagger = check
    r.learn(1, init_at_random_ep_len=True)
    assert checked
