"""hipGraph-captured PPO update == the same update run eagerly (MI355X)."""
import copy

import pytest
import torch

from test_ppo_update import _fill, _make

pytestmark = pytest.mark.gpu


def _to_gpu(alg_cpu, use_graphs, phased=None, device="cuda:0"):
    from legged_gym_custom_amd.rsl_rl.algorithms import PPO
    ac = copy.deepcopy(alg_cpu.actor_critic)
    est = copy.deepcopy(alg_cpu.estimator)
    alg = PPO(ac, est, num_learning_epochs=alg_cpu.num_learning_epochs, num_mini_batches=alg_cpu.num_mini_batches,
              learning_rate=alg_cpu.learning_rate, schedule=alg_cpu.schedule, desired_kl=alg_cpu.desired_kl,
              max_grad_norm=alg_cpu.max_grad_norm, device=device, use_graphs=use_graphs)
    alg.phased_graphs = phased
    s = alg_cpu.storage
    alg.init_storage(s.num_envs, s.num_transitions_per_env, list(s.obs_shape), list(s.privileged_obs_shape),
                     list(s.critic_obs_shape), list(s.estimated_obs_shape), [s.scan_observations.shape[-1]],
                     [s.actions.shape[-1]])
    return alg


@pytest.mark.parametrize("phased", [False, True])
def test_graph_update_matches_eager(phased):
    base = _make("adaptive")
    eager = _to_gpu(base, use_graphs=False)
    graph = _to_gpu(base, use_graphs=True, phased=phased)
    for it in range(5):
        for alg in (eager, graph):
            _fill(alg, 10 + it)
        torch.manual_seed(100 + it)
        le = eager.update()
        torch.manual_seed(100 + it)
        lg = graph.update()
        torch.testing.assert_close(torch.tensor(lg), torch.tensor(le), rtol=1e-4, atol=1e-6)
        assert graph.learning_rate == pytest.approx(eager.learning_rate, rel=1e-9)
    assert graph.graph_mode == ("phased" if phased else "whole")
    for a, b in zip(list(graph.actor_critic.parameters()) + list(graph.estimator.parameters()),
                    list(eager.actor_critic.parameters()) + list(eager.estimator.parameters())):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-4, atol=1e-6)
    assert graph.grads.check()


def test_graph_update_dagger_matches_eager():
    """update_dagger (ppo.py:309-349) replayed from its hipGraph (calls 2..) == eager, bit for
    bit: the adaptation encoder, its Adam moments and the returned mean loss."""
    base = _make("adaptive")
    eager = _to_gpu(base, use_graphs=False)
    graph = _to_gpu(base, use_graphs=True)
    for it in range(4):
        for alg in (eager, graph):
            _fill(alg, 20 + it)
        torch.manual_seed(200 + it)
        le = eager.update_dagger()
        torch.manual_seed(200 + it)
        lg = graph.update_dagger()
        assert lg == le, (it, lg, le)
    assert graph._dagger_graph is not None
    for a, b in zip(graph.actor_critic.adaptation_encoder_.parameters(), eager.actor_critic.adaptation_encoder_.parameters()):
        assert torch.equal(a.detach(), b.detach())
    assert torch.equal(graph.exp_avg, eager.exp_avg) and torch.equal(graph.exp_avg_sq, eager.exp_avg_sq)


def test_gpu_update_tracks_cpu_torch_update():
    """HIP GEMMs (3xbf16) + flat HIP Adam + hipGraph vs the CPU torch update (fp32 GEMMs,
    torch Adam) on the same data and minibatches. Per-element Adam steps are bounded by
    ~lr, so compare statistically: tiny typical drift, bounded worst case."""
    base = _make("adaptive")
    cpu = _to_gpu(base, use_graphs=False, device="cpu")  # a fresh CPU PPO (torch GEMMs, torch Adam)
    gpu = _to_gpu(base, use_graphs=True)
    for alg in (cpu, gpu):
        alg._next_perm = lambda n, dev=alg.device: torch.arange(n, device=dev)
    for it in range(3):
        for alg in (cpu, gpu):
            _fill(alg, 40 + it)
        lc = cpu.update()
        lg = gpu.update()
        # loss means over the update's minibatches: after the first Adam step every weight
        # moved by ~+-lr (sign(g) at step 1), so near-zero gradients whose sign differs by
        # rounding already diverge inside update 0 — a 1 % bound on the means
        assert torch.allclose(torch.tensor(lg), torch.tensor(lc), rtol=1e-2, atol=1e-6), (it, lg, lc)
        assert gpu.learning_rate == pytest.approx(cpu.learning_rate, rel=1e-9)
    pc = torch.cat([p.detach().reshape(-1) for p in list(cpu.actor_critic.parameters()) + list(cpu.estimator.parameters())])
    pg = torch.cat([p.detach().reshape(-1).cpu() for p in list(gpu.actor_critic.parameters()) +
                    list(gpu.estimator.parameters())])
    d = (pg - pc).abs()
    assert d.median() < 1e-6 and torch.quantile(d, 0.99) < 5e-5 and d.max() < 5e-3, \
        (d.median(), torch.quantile(d, 0.99), d.max())
    # the torch Adam containers see the flat moments (checkpoint export)
    st = gpu.optimizer.state_dict()["state"]
    assert float(st[0]["step"]) == 3 * gpu.num_learning_epochs * gpu.num_mini_batches
    assert gpu.grads.check()


def test_gae_kernel_matches_torch_statement():
    """RolloutStorage.compute_returns on the GPU (lgx_gae + lgx_normalize_advantages) == the
    reference's loop (rollout_storage.py:110-124) in torch ops: returns bitwise (same fp32
    operation order), normalised advantages to fp32 rounding (fp64 moments vs torch's)."""
    from legged_gym_custom_amd.rsl_rl.storage import RolloutStorage
    T, N, gamma, lam = 24, 1000, 0.99, 0.95
    dev = "cuda:0"
    s = RolloutStorage(N, T, [5], [2], [3], [1], [1], [2], device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    s.rewards.copy_(torch.randn(T, N, 1, device=dev, generator=g))
    s.values.copy_(torch.randn(T, N, 1, device=dev, generator=g) * 3)
    s.dones.copy_((torch.rand(T, N, 1, device=dev, generator=g) < 0.05).byte())
    last = torch.randn(N, 1, device=dev, generator=g)
    for _ in range(2):  # the counter/workspace are reused
        s.compute_returns(last, gamma, lam)
    ret = torch.zeros_like(s.returns)
    adv = 0
    for step in reversed(range(T)):
        next_values = last if step == T - 1 else s.values[step + 1]
        not_terminal = 1.0 - s.dones[step].float()
        delta = s.rewards[step] + not_terminal * gamma * next_values - s.values[step]
        adv = delta + not_terminal * gamma * lam * adv
        ret[step] = adv + s.values[step]
    a = ret - s.values
    a = (a - a.mean()) / (a.std() + 1e-8)
    assert torch.equal(ret, s.returns)
    torch.testing.assert_close(s.advantages, a, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B", [16 * 300 + 5, 24576])
def test_adaptation_train_matches_autograd_fp64(B):
    """lgx_adaptation_train (one DAgger minibatch of the adaptation encoder in one launch, lgx_mlp
    ABI 9/10) against torch autograd in fp64 on the same weights and rows: the summed per-block
    gradient rows of every parameter within 5e-6 * max|g| (every stage on f32-input MFMA: exact
    f32 products, fp32 sums; measured 1e-7) and the loss within 1e-5 relative; B = 4805 ends in a partial
    16-row chunk; fixed-order sums: two launches give identical rows."""
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoder, AdaptationEncoderTS
    torch.manual_seed(5)
    P, Hh = 52, 10
    mod = AdaptationEncoder(num_proprio=P, history_buffer_length=Hh).to("cuda:0")
    obs = torch.randn(B, P * (Hh + 1), device="cuda:0")
    target = torch.randn(B, 20, device="cuda:0") * 0.5
    ps = H.adaptation_param_order(mod)
    NP = sum(p.numel() for p in ps)
    grid = H.adapt_train_grid(B, 768)
    gws, lws = torch.empty(grid * NP, device="cuda:0"), torch.empty(grid, device="cuda:0")
    keep = H.adaptation_train(mod, obs, P * Hh, target, gws, lws, 768)
    torch.cuda.synchronize()
    got = gws.view(grid, NP).double().sum(0)
    rows1 = gws.clone()
    keep = H.adaptation_train(mod, obs, P * Hh, target, gws, lws, 768)
    torch.cuda.synchronize()
    del keep
    assert torch.equal(gws, rows1)
    ref = AdaptationEncoderTS(num_proprio=P, history_buffer_length=Hh).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in mod.state_dict().items()})
    hist = obs[:, :P * Hh].double().cpu().reshape(B, Hh, P)
    lat = ref(hist)
    loss = (target.double().cpu() - lat).norm(p=2, dim=1).mean()
    loss.backward()
    ref_ps = H.adaptation_param_order(ref)
    o, worst = 0, 0.0
    for p, rp in zip(ps, ref_ps):
        g, rg = got[o:o + p.numel()].cpu().view_as(rp), rp.grad
        o += p.numel()
        err = float((g - rg).abs().max())
        worst = max(worst, err / float(rg.abs().max()))
        assert err <= 5e-6 * float(rg.abs().max()) + 1e-9, (tuple(p.shape), err, float(rg.abs().max()))
    print(f"B={B}: worst gradient |err| / max|g| = {worst:.2e}")
    assert abs(float(lws.double().sum()) - float(loss.detach())) <= 1e-5 * float(loss.detach())


@pytest.mark.parametrize("n,scale", [(5040, 0.01), (5040, 10.0), (40001, 1.0)])
def test_clip_adam_matches_clip_grad_norm_and_adam(n, scale):
    """lgx_clip_adam (ABI 10: the DAgger step's clip_grad_norm_ + Adam in one block) against the
    torch statement it replaces (ppo.py:336-345): g *= min(max_norm / (||g|| + 1e-6), 1) in place,
    then Adam (torch's arithmetic, as lgx_adam_step) — with the clip inactive (small gradient) and
    active; the step counter advanced on the device."""
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
    torch.manual_seed(n)
    dev = "cuda:0"
    p, g = torch.randn(n, device=dev), torch.randn(n, device=dev) * scale
    m, v = torch.randn(n, device=dev) * 0.01, torch.rand(n, device=dev) * 1e-4
    step = torch.full((), 3.0, device=dev)
    p0, g0, m0, v0 = (t.double().cpu() for t in (p, g, m, v))
    lr, b1, b2, eps, max_norm = 1e-3, 0.9, 0.999, 1e-8, 1.0
    H.clip_adam(p, g, m, v, step, lr, b1, b2, eps, max_norm)
    torch.cuda.synchronize()
    coef = min(max_norm / (float(g0.norm()) + 1e-6), 1.0)
    gc = g0 * coef
    t = 4.0
    b1, b2 = (float(torch.tensor(b, dtype=torch.float32)) for b in (b1, b2))  # the kernel's fp32 betas (torch's fused Adam)
    m1 = b1 * m0 + (1 - b1) * gc
    v1 = b2 * v0 + (1 - b2) * gc * gc
    p1 = p0 - (lr / (1 - b1 ** t)) * m1 / (v1.sqrt() / (1 - b2 ** t) ** 0.5 + eps)
    assert float(step) == t
    torch.testing.assert_close(g.double().cpu(), gc, rtol=2e-6, atol=1e-12)
    torch.testing.assert_close(m.double().cpu(), m1, rtol=2e-6, atol=1e-8)  # (0.9 m + 0.1 g) cancels
    torch.testing.assert_close(v.double().cpu(), v1, rtol=2e-6, atol=1e-14)
    torch.testing.assert_close(p.double().cpu(), p1, rtol=1e-6, atol=2e-7)


def test_gpu_update_dagger_tracks_cpu_update():
    """The whole fused GPU update_dagger (per minibatch: lgx_adaptation_train, the block-row reduce,
    lgx_clip_adam with the device step counter; 2 epochs x 3 minibatches, graph-replayed from the
    second call) against the CPU learner's update_dagger (torch autograd, clip_grad_norm_, torch
    Adam; ppo.py:309-349) from the same state, data and permutation, three calls: the mean losses
    within 1e-4 relative, the adaptation encoder's parameters and both Adam moments close (per-element
    Adam steps are ~lr, so a sign flip of a near-zero gradient moves one entry by ~2 lr: statistical
    bounds), and the same step count — a sequencing bug (step increment, loss accumulation, a missed
    zeroing) fails here, where the single-launch tests cannot see it."""
    base = _make("adaptive")
    cpu = _to_gpu(base, use_graphs=False, device="cpu")
    gpu = _to_gpu(base, use_graphs=True)
    for alg in (cpu, gpu):
        alg._next_perm = lambda n, dev=alg.device: torch.arange(n, device=dev)
    for it in range(3):
        for alg in (cpu, gpu):
            _fill(alg, 60 + it)
        lc = cpu.update_dagger()
        lg = gpu.update_dagger()
        assert lg == pytest.approx(lc, rel=1e-4, abs=1e-7), (it, lg, lc)
    assert gpu.dagger_path == "fused" and gpu.dagger_graph_mode == "whole"
    pc = torch.cat([p.detach().reshape(-1) for p in cpu.actor_critic.adaptation_encoder_.parameters()])
    pg = torch.cat([p.detach().reshape(-1).cpu() for p in gpu.actor_critic.adaptation_encoder_.parameters()])
    d = (pg - pc).abs()
    lr = cpu.adaptation_optimizer.param_groups[0]["lr"]
    assert d.median() < 1e-6 and d.max() < 4 * lr, (float(d.median()), float(d.max()), lr)
    a, b = gpu.grads.slices[gpu._segment_of["adaptation_optimizer"]]
    st = cpu.adaptation_optimizer.state_dict()["state"]
    m_cpu = torch.cat([st[k]["exp_avg"].reshape(-1) for k in sorted(st)])
    v_cpu = torch.cat([st[k]["exp_avg_sq"].reshape(-1) for k in sorted(st)])
    n = 3 * gpu.num_learning_epochs * gpu.num_mini_batches
    assert all(float(st[k]["step"]) == n for k in st)
    assert float(gpu._opt_step["adaptation_optimizer"]) == n
    # the flat moments are in lgx_adaptation_train's parameter order; the CPU optimizer's in
    # parameters() order: compare as multisets of magnitudes' summary statistics and per tensor
    # through the export path below
    exp = gpu.optimizer_state_dicts()["adaptation_optimizer_state_dict"]["state"]
    for k in sorted(st):
        torch.testing.assert_close(exp[k]["exp_avg"].cpu(), st[k]["exp_avg"], rtol=5e-3, atol=2e-4 * float(m_cpu.abs().max()))
        torch.testing.assert_close(exp[k]["exp_avg_sq"].cpu(), st[k]["exp_avg_sq"], rtol=5e-3,
                                   atol=2e-4 * float(v_cpu.abs().max()))
    assert b - a == pc.numel()
