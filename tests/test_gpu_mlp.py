"""liblgx_mlp.so GEMMs (3 x bf16 MFMA split, fp32 accumulate) vs fp64 references.

Bound per output: |C - C64| <= 3e-5 * sum_k |A(m,k) B(k,n)| + 1e-6 — the split's
~2^-16 relative product error plus fp32 accumulation; TF32 (what the reference trains
with, train.py:39) would need ~5e-4 * sum|ab|."""
import numpy as np
import pytest
import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H

pytestmark = pytest.mark.gpu
dev = "cuda:0"


def _bound(A, B):
    return 3e-5 * (A.abs().double() @ B.abs().double()) + 1e-6


@pytest.mark.parametrize("M,N,K", [(24576, 512, 627), (1000, 13, 37), (4096, 12, 128), (77, 300, 736), (3, 1, 5)])
def test_forward_bias_elu(M, N, K):
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    x = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
    b = torch.randn(N, device=dev, generator=g)
    for elu in (False, True):
        y = H.linear_forward(x, W, b, elu)
        z = x.double() @ W.double().t() + b.double()
        ref = torch.nn.functional.elu(z) if elu else z
        err = (y.double() - ref).abs()
        assert (err <= _bound(x, W.t())).all(), float(err.max())


@pytest.mark.parametrize("M,N,K", [(24576, 627, 512), (500, 29, 64), (4096, 128, 12)])
def test_input_grad_with_elu_derivative(M, N, K):
    # dX[M,N] = dY[M,K] W[K,N] * ELU'(y_prev)
    g = torch.Generator(device=dev).manual_seed(7 * M + N)
    dy = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(K, N, device=dev, generator=g) / N ** 0.5
    y_prev = torch.nn.functional.elu(torch.randn(M, N, device=dev, generator=g) * 2)
    dx = H.linear_input_grad(dy, W, y_prev)
    d = torch.where(y_prev > 0, torch.ones_like(y_prev), y_prev + 1).double()
    ref = (dy.double() @ W.double()) * d
    err = (dx.double() - ref).abs()
    assert (err <= _bound(dy, W) * d + 1e-6).all(), float(err.max())
    dx2 = H.linear_input_grad(dy, W, None)
    assert ((dx2.double() - dy.double() @ W.double()).abs() <= _bound(dy, W)).all()


@pytest.mark.parametrize("rows,N,K", [(24576, 512, 627), (24576, 12, 128), (1000, 20, 29), (300, 64, 132),
                                       (24576, 1, 128), (1000, 13, 29), (500, 3, 64), (777, 736, 512)])
def test_weight_and_bias_grad(rows, N, K):
    g = torch.Generator(device=dev).manual_seed(rows + 3 * N)
    dy = torch.randn(rows, N, device=dev, generator=g)
    x = torch.randn(rows, K, device=dev, generator=g)
    dW, db = H.linear_weight_grad(dy, x)
    ref = dy.double().t() @ x.double()
    err = (dW.double() - ref).abs()
    assert (err <= _bound(dy.t(), x)).all(), float(err.max())
    # the bias gradient is summed in fp32 from the unsplit values: fp32 summation bound
    assert ((db.double() - dy.double().sum(0)).abs() <= 1e-6 * dy.double().abs().sum(0) + 1e-6).all()
    # deterministic (fixed split-K reduction order)
    dW2, db2 = H.linear_weight_grad(dy, x)
    assert torch.equal(dW, dW2) and torch.equal(db, db2)


def test_mlp_autograd_matches_fp64():
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import _mlp
    torch.manual_seed(0)
    net = _mlp(627, [512, 256, 128], 12, torch.nn.ELU()).to(dev)
    ref = _mlp(627, [512, 256, 128], 12, torch.nn.ELU()).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in net.state_dict().items()})
    x = torch.randn(3000, 627, device=dev, requires_grad=True)
    xr = x.detach().double().cpu().requires_grad_(True)
    y = net(x)
    yr = torch.nn.Sequential.forward(ref, xr)
    torch.testing.assert_close(y.double().cpu(), yr, rtol=1e-4, atol=1e-4)
    w = torch.randn_like(y)
    (y * w).sum().backward()
    (yr * w.double().cpu()).sum().backward()
    torch.testing.assert_close(x.grad.double().cpu(), xr.grad, rtol=1e-3, atol=1e-5)
    for (n, p), (_, pr) in zip(net.named_parameters(), ref.named_parameters()):
        scale = pr.grad.abs().max().item()
        torch.testing.assert_close(p.grad.double().cpu(), pr.grad, rtol=1e-3, atol=1e-4 * scale, msg=n)


def test_adaptation_encoder_matches_torch_fp64():
    """Channels-last conv1d-as-GEMM adaptation encoder vs the module's own torch path (fp64)."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoder
    torch.manual_seed(0)
    enc = AdaptationEncoder(num_proprio=52, history_buffer_length=10, output_dim=20).to(dev)
    ref = AdaptationEncoder(num_proprio=52, history_buffer_length=10, output_dim=20).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in enc.state_dict().items()})
    h = torch.randn(2000, 10, 52, device=dev, requires_grad=True)
    hr = h.detach().double().cpu().requires_grad_(True)
    y = enc(h)
    yr = ref(hr)  # CPU -> torch conv1d path
    torch.testing.assert_close(y.double().cpu(), yr, rtol=1e-4, atol=1e-4)
    w = torch.randn_like(y)
    (y * w).sum().backward()
    (yr * w.double().cpu()).sum().backward()
    torch.testing.assert_close(h.grad.double().cpu(), hr.grad, rtol=1e-3, atol=1e-5)
    for (n, p), (_, pr) in zip(enc.named_parameters(), ref.named_parameters()):
        scale = pr.grad.abs().max().item()
        torch.testing.assert_close(p.grad.double().cpu(), pr.grad, rtol=1e-3, atol=1e-4 * scale, msg=n)


def test_adaptation_encoder_inplace_history_bitwise():
    """ActorCritic.adaptation_encoder on obs rows without grad reads the history blocks in
    place (the per-step layer over all 11 blocks of each row): bitwise equal to the packed
    path (a contiguous copy of the history), which the grad-enabled call takes."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoder
    torch.manual_seed(0)
    enc = AdaptationEncoder(num_proprio=52, history_buffer_length=10, output_dim=20).to(dev)
    obs = torch.randn(3000, 572, device=dev)
    hist = obs[:, :-52].reshape(-1, 10, 52)
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp
    n0 = hip_mlp.ADAPT_INPLACE_CALLS
    with torch.no_grad():
        a = enc(hist)                       # in place (strided view of obs)
        assert hip_mlp.ADAPT_INPLACE_CALLS == n0 + 1, "the in-place branch did not run"
        b = enc(hist.contiguous())          # packed
    with torch.inference_mode():
        d = enc(hist)
    assert hip_mlp.ADAPT_INPLACE_CALLS == n0 + 2
    c = enc(hist)                           # grad enabled: packed path inside
    assert hip_mlp.ADAPT_INPLACE_CALLS == n0 + 2
    assert torch.equal(a, b) and torch.equal(a, c.detach()) and torch.equal(a, d)


@pytest.mark.parametrize("B", [1, 2001, 98304])
def test_adaptation_fused_forward_bitwise(B, monkeypatch):
    """lgx_adaptation_forward (the whole encoder in one launch, no gradient) == the per-layer
    launches (LGX_ADAPT_FUSED=0), bitwise, on the history read in place from obs rows and on a
    packed history; B = 1, a ragged 2001, and the update's 98,304 rows."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoder
    torch.manual_seed(7)
    enc = AdaptationEncoder(num_proprio=52, history_buffer_length=10, output_dim=20).to(dev)
    obs = torch.randn(B, 572, device=dev)
    hist = obs[:, :-52].reshape(-1, 10, 52)
    outs = {}
    for fused in (True, False):
        monkeypatch.setattr(H, "USE_ADAPT_FUSED", fused)
        with torch.no_grad():
            outs[fused] = (enc(hist), enc(hist.contiguous()))
    assert torch.equal(outs[True][0], outs[False][0]) and torch.equal(outs[True][1], outs[False][1])
    assert torch.equal(outs[True][0], outs[True][1])


@pytest.mark.parametrize("clipped", [True, False])
def test_ppo_head_matches_torch_autograd(clipped):
    """lgx_ppo_head_{forward,backward} vs the reference's loss code (ppo.py:196-262 over
    torch.distributions.Normal) differentiated by torch autograd in fp64."""
    from torch.distributions import Normal
    g = torch.Generator(device=dev).manual_seed(11)
    B, A, clip = 3000, 12, 0.2
    r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    mu, value, std = r(B, A), r(B, 1), torch.rand(A, device=dev, generator=g) + 0.3
    actions, old_mu = mu + 0.3 * r(B, A), mu + 0.1 * r(B, A)
    old_sigma = std + 0.05 * torch.rand(B, A, device=dev, generator=g)
    adv, tv, ret = r(B, 1), value + 0.3 * r(B, 1), r(B, 1)
    adv[:50] = 0.0  # surrogate ties (s1 == s2): torch.max splits the gradient
    lp_ref = Normal(mu.double(), std.double()).log_prob(actions.double()).sum(-1)
    old_logp = (lp_ref + 0.15 * r(B).double()).float().reshape(B, 1)
    old_logp[50:60, 0] = lp_ref[50:60].float()  # ratio exactly 1 (inside the clip range)

    def reference(mu, value, std):
        d = Normal(mu, mu * 0.0 + std)
        logp = d.log_prob(actions.double()).sum(-1)
        ratio = torch.exp(logp - old_logp.double().squeeze())
        a = adv.double().squeeze()
        surr = torch.max(-a * ratio, -a * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
        if clipped:
            vc = tv.double() + (value - tv.double()).clamp(-clip, clip)
            vl = torch.max((value - ret.double()).pow(2), (vc - ret.double()).pow(2)).mean()
        else:
            vl = (ret.double() - value).pow(2).mean()
        ent = d.entropy().sum(-1).mean()
        sig = d.stddev
        kl = torch.sum(torch.log(sig / old_sigma.double() + 1e-5) + (old_sigma.double() ** 2 + (old_mu.double() - mu) ** 2)
                       / (2.0 * sig ** 2) - 0.5, -1).mean()
        return surr, vl, ent, kl

    m64, v64, s64 = (t.double().requires_grad_(True) for t in (mu, value, std))
    rs, rv, re, rk = reference(m64, v64, s64)
    (rs + 0.7 * rv - 0.01 * re).backward()
    m32, v32, s32 = (t.clone().requires_grad_(True) for t in (mu, value, std))
    hs, hv, he, hk = H.ppo_head(m32, v32, s32, actions, old_logp, adv, tv, ret, old_mu, old_sigma, clip, clipped)
    (hs + 0.7 * hv - 0.01 * he).backward()
    for got, want in ((hs, rs), (hv, rv), (he, re), (hk, rk)):
        torch.testing.assert_close(got.double(), want.detach(), rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(m32.grad.double(), m64.grad, rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(v32.grad.double(), v64.grad, rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(s32.grad.double(), s64.grad, rtol=1e-4, atol=1e-7)


def test_rollout_bookkeeping_kernels_match_torch():
    """lgx_copy_batch / lgx_act_head / lgx_store_transition (the rollout step's storage
    writes, ppo.py:129-171) against the torch ops they replace."""
    import torch
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp
    g = torch.Generator(device="cuda").manual_seed(0)
    B, A = 1000, 12
    # batched copies, incl. an unaligned byte-sized entry
    srcs = [torch.randn(B, n, device="cuda", generator=g) for n in (572, 29, 736, 3, 132)]
    srcs.append(torch.randint(0, 255, (37,), device="cuda", dtype=torch.uint8, generator=g))
    dsts = [torch.empty_like(x) for x in srcs]
    hip_mlp.copy_batch(dsts, srcs)
    for d, x in zip(dsts, srcs):
        assert torch.equal(d, x)
    # action head == Normal(mean, std) sample with the same eps + log_prob
    mean = torch.randn(B, A, device="cuda", generator=g)
    std = torch.rand(A, device="cuda", generator=g) + 0.2
    eps = torch.randn(B, A, device="cuda", generator=g)
    act, mu, sig, lp = (torch.empty(B, A, device="cuda"), torch.empty(B, A, device="cuda"),
                        torch.empty(B, A, device="cuda"), torch.empty(B, 1, device="cuda"))
    hip_mlp.act_head(mean, std, eps, act, mu, sig, lp)
    want_a = mean + std * eps
    dist = torch.distributions.Normal(mean, mean * 0.0 + std)
    torch.testing.assert_close(act, want_a, rtol=0, atol=0)
    torch.testing.assert_close(mu, mean, rtol=0, atol=0)
    torch.testing.assert_close(sig, std.expand(B, A), rtol=0, atol=0)
    torch.testing.assert_close(lp.view(-1), dist.log_prob(want_a).sum(-1), rtol=1e-6, atol=1e-5)
    # eps drawn in the kernel (Philox per global env and env step, oracle/philox.py act_noise)
    import philox
    step_dev = torch.tensor([123457], dtype=torch.int64, device="cuda")
    act2 = torch.empty(B, A, device="cuda")
    hip_mlp.act_head(mean, std, None, act2, mu, sig, lp, noise=(7, step_dev, 3000))
    want_eps = philox.act_noise(7, np.arange(3000, 3000 + B), 123457, A)
    got_eps = ((act2 - mean) / std).double().cpu().numpy()
    np.testing.assert_allclose(got_eps, want_eps, atol=2e-5 * (1 + np.abs(want_eps)).max())
    dist2 = torch.distributions.Normal(mean, mean * 0.0 + std)
    torch.testing.assert_close(lp.view(-1), dist2.log_prob(act2).sum(-1), rtol=1e-6, atol=1e-5)
    # a shard: rows of global envs 3500.. are the same draws as rows 500.. above
    act3 = torch.empty(B - 500, A, device="cuda")
    hip_mlp.act_head(mean[500:].contiguous(), std, None, act3, torch.empty_like(act3), torch.empty_like(act3),
                     torch.empty(B - 500, 1, device="cuda"), noise=(7, step_dev, 3500))
    assert torch.equal(act3, act2[500:])
    # transition: r + gamma * V * time_out
    r = torch.randn(B, device="cuda", generator=g)
    v = torch.randn(B, 1, device="cuda", generator=g)
    done = torch.rand(B, device="cuda", generator=g) < 0.2
    to = done & (torch.rand(B, device="cuda", generator=g) < 0.5)
    ro, do_, vo = torch.empty(B, 1, device="cuda"), torch.empty(B, 1, device="cuda", dtype=torch.uint8), \
        torch.empty(B, 1, device="cuda")
    hip_mlp.store_transition(r, done.view(torch.uint8), to.view(torch.uint8), v.view(-1), ro.view(-1), do_.view(-1),
                             vo.view(-1), 0.99)
    want_r = r + 0.99 * torch.squeeze(v * to.unsqueeze(1).float(), 1)
    torch.testing.assert_close(ro.view(-1), want_r, rtol=0, atol=0)
    assert torch.equal(do_.view(-1).bool(), done) and torch.equal(vo, v)


def test_forward_parts_grads_only_where_needed():
    """actor(cat(obs, latent, scan, est)) as one node: the input gradient is formed for the
    latent parts only, and equals the fp64 gradient of the concatenated input there."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import _mlp
    torch.manual_seed(1)
    net = _mlp(627, [512, 256, 128], 12, torch.nn.ELU()).to(dev)
    ref = _mlp(627, [512, 256, 128], 12, torch.nn.ELU()).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in net.state_dict().items()})
    M = 2000
    obs = torch.randn(M, 572, device=dev)
    lat = torch.randn(M, 20, device=dev, requires_grad=True)
    scan = torch.randn(M, 32, device=dev, requires_grad=True)
    est = torch.randn(M, 3, device=dev)
    y = net.forward_parts((obs, lat, scan, est))
    xr = torch.cat((obs, lat, scan, est), -1).detach().double().cpu().requires_grad_(True)
    yr = torch.nn.Sequential.forward(ref, xr)
    torch.testing.assert_close(y.double().cpu(), yr, rtol=1e-4, atol=1e-4)
    w = torch.randn_like(y)
    (y * w).sum().backward()
    (yr * w.double().cpu()).sum().backward()
    torch.testing.assert_close(lat.grad.double().cpu(), xr.grad[:, 572:592], rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(scan.grad.double().cpu(), xr.grad[:, 592:624], rtol=1e-3, atol=1e-5)
    # parameter gradients sum ~M products each: cancellation needs an absolute slack
    for p, pr in zip(net.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad.double().cpu(), pr.grad, rtol=1e-3, atol=2e-3)


def test_deferred_splitk_matches_immediate_bitwise():
    """One lgx_splitk_reduce_batch over several weight-gradient GEMMs == each GEMM's own
    reduction, bit for bit (same fixed order), incl. accumulation and a shared output."""
    g = torch.Generator(device=dev).manual_seed(5)
    shapes = [(24576, 512, 627), (24576, 12, 128), (1000, 20, 29), (777, 3, 64)]
    data = [(torch.randn(r, n, device=dev, generator=g), torch.randn(r, k, device=dev, generator=g))
            for r, n, k in shapes]
    ref = []
    for dy, x in data:
        dW = torch.randn(dy.shape[1], x.shape[1], device=dev, generator=g)
        db = torch.randn(dy.shape[1], device=dev, generator=g)
        ref.append((dW.clone(), db.clone()))
    out = [(a.clone(), b.clone()) for a, b in ref]
    for (dy, x), (dW, db) in zip(data, ref):
        H.linear_weight_grad(dy, x, dW, db, accumulate=True)
        H.linear_weight_grad(dy, x, dW, db, accumulate=True)  # twice: accumulation order
    with H.deferred_splitk():
        for (dy, x), (dW, db) in zip(data, out):
            H.linear_weight_grad(dy, x, dW, db, accumulate=True)
            H.linear_weight_grad(dy, x, dW, db, accumulate=True)  # overlaps: settles the first
    for (a, b), (c, d) in zip(ref, out):
        assert torch.equal(a, c) and torch.equal(b, d)


def _wgrad_args(dy, x, dW, db, split, ws, defer):
    N, K, rows = dy.shape[1], x.shape[1], dy.shape[0]
    w = ws.data_ptr()
    return H.GemmArgs(A=dy.data_ptr(), lda=dy.stride(0), a_kcontig=0, B=x.data_ptr(), ldb=x.stride(0), b_kcontig=0,
                      C=dW.data_ptr(), ldc=dW.stride(0), M=N, N=K, K=rows, epilogue=H.EPI_ACCUM, split_k=split,
                      workspace=w, colsum=db.data_ptr(), colsum_ws=w + 4 * split * N * K, defer_reduce=int(defer))


def test_group_weight_grads_match_single_launches_bitwise():
    """deferred_weight_grads: every dW/db GEMM of a backward pass in one lgx_gemm_group launch
    (group-picked splits) == each GEMM launched alone with the same split, bit for bit; all
    four stager-mode combinations (M, N % 4 != 0) and an accumulating shared output."""
    g = torch.Generator(device=dev).manual_seed(11)
    shapes = [(24576, 512, 736), (24576, 512, 627), (24576, 256, 512), (24576, 12, 128), (24576, 1, 128),
              (24576, 20, 29), (24576, 3, 64), (24576, 64, 20)]
    data = [(torch.randn(r, n, device=dev, generator=g), torch.randn(r, k, device=dev, generator=g))
            for r, n, k in shapes]
    splits = H.pick_split_group([(n, k, r) for r, n, k in shapes])
    assert all(s >= 2 for s in splits)
    init = [(torch.randn(dy.shape[1], x.shape[1], device=dev, generator=g),
             torch.randn(dy.shape[1], device=dev, generator=g)) for dy, x in data]
    ref = [(a.clone(), b.clone()) for a, b in init]
    for (dy, x), (dW, db), s in zip(data, ref, splits):
        ws = torch.empty(s * dW.numel() + s * db.numel() + 4, device=dev)
        H._run(_wgrad_args(dy, x, dW, db, s, ws, False))
    out = [(a.clone(), b.clone()) for a, b in init]
    with H.deferred_weight_grads():
        for (dy, x), (dW, db) in zip(data, out):
            H.linear_weight_grad(dy, x, dW, db, accumulate=True)
    for (a, b), (c, d) in zip(ref, out):
        assert torch.equal(a, c) and torch.equal(b, d)
    # and against fp64
    for (dy, x), (dW0, db0), (dW, db) in zip(data, init, out):
        r = dW0.double() + dy.double().t() @ x.double()
        assert ((dW.double() - r).abs() <= _bound(dy.t(), x) + 1e-5 * dW0.abs().double()).all()
        torch.testing.assert_close(db.double(), db0.double() + dy.double().sum(0), rtol=1e-5, atol=1e-3)
    # two GEMMs into the same output: the second settles the first (accumulation order kept)
    dy, x = data[3]
    a, b = init[3][0].clone(), init[3][1].clone()
    with H.deferred_weight_grads():
        H.linear_weight_grad(dy, x, a, b, accumulate=True)
        H.linear_weight_grad(dy, x, a, b, accumulate=True)
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    torch.testing.assert_close(b.double(), init[3][1].double() + 2 * dy.double().sum(0), rtol=1e-5, atol=2e-3)


def test_group_forward_and_input_grad_match_single_launches_bitwise():
    """lgx_gemm_group of forward (bias + ELU) and of input-gradient (ELU') GEMMs of mixed
    shapes == the same GEMMs launched one by one, bit for bit."""
    g = torch.Generator(device=dev).manual_seed(12)
    fwd = [(24576, 736, 512), (24576, 29, 64), (24576, 132, 128), (24576, 572, 128), (4096, 627, 512), (333, 20, 20)]
    single, grouped, args_s, args_g = [], [], [], []
    for M, K, N in fwd:
        x = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
        b = torch.randn(N, device=dev, generator=g)
        ys, yg = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
        for y, lst in ((ys, args_s), (yg, args_g)):
            lst.append(H.GemmArgs(A=x.data_ptr(), lda=K, a_kcontig=1, B=W.data_ptr(), ldb=K, b_kcontig=1,
                                  C=y.data_ptr(), ldc=N, M=M, N=N, K=K, epilogue=H.EPI_BIAS | H.EPI_ELU,
                                  bias=b.data_ptr(), split_k=1))
        single.append((ys, x, W, b))
        grouped.append(yg)
    for a in args_s:
        H._run(a)
    H.run_group(args_g)
    for (ys, *_r), yg in zip(single, grouped):
        assert torch.equal(ys, yg)
    # input gradients: dX[M, Kin] = dY[M, N] W[N, Kin] * ELU'(y_prev), incl. Kin % 4 != 0
    dxs, dxg, args_s, args_g = [], [], [], []
    for M, Kin, N in [(24576, 512, 256), (24576, 627, 512), (24576, 64, 20), (24576, 29, 64), (4096, 128, 12)]:
        dy = torch.randn(M, N, device=dev, generator=g)
        W = torch.randn(N, Kin, device=dev, generator=g)
        yp = torch.nn.functional.elu(torch.randn(M, Kin, device=dev, generator=g))
        a, c = torch.empty(M, Kin, device=dev), torch.empty(M, Kin, device=dev)
        for o, lst in ((a, args_s), (c, args_g)):
            lst.append(H.GemmArgs(A=dy.data_ptr(), lda=N, a_kcontig=1, B=W.data_ptr(), ldb=Kin, b_kcontig=0,
                                  C=o.data_ptr(), ldc=Kin, M=M, N=Kin, K=N, epilogue=H.EPI_DELU, act=yp.data_ptr(),
                                  ld_act=Kin, split_k=1))
        dxs.append((a, dy, W, yp))
        dxg.append(c)
    for a in args_s:
        H._run(a)
    H.run_group(args_g)
    for (a, dy, W, yp), c in zip(dxs, dxg):
        assert torch.equal(a, c)
        r = (dy.double() @ W.double()) * torch.where(yp > 0, 1.0, yp.double() + 1)
        assert ((c.double() - r).abs() <= _bound(dy, W) * 2 + 1e-6).all()


def test_forward_group_matches_separate_chains_bitwise():
    """hip_mlp.forward_group (one launch per depth, one autograd node) == the chains run one
    by one: outputs, input gradients (incl. a parts input) and parameter gradients, bitwise."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import _mlp
    torch.manual_seed(3)
    act = torch.nn.ELU()
    nets = [_mlp(29, [64, 20], 20, act), _mlp(132, [128, 64], 32, act), _mlp(736, [512, 256, 128], 1, act),
            _mlp(572, [128, 64], 3, act)]
    nets = [n.to(dev) for n in nets]
    B = 3000
    g = torch.Generator(device=dev).manual_seed(4)
    xs = [torch.randn(B, d, device=dev, generator=g) for d in (29, 132, 736)]
    parts = (torch.randn(B, 520, device=dev, generator=g), torch.randn(B, 52, device=dev, generator=g,
                                                                         requires_grad=True))
    seeds = [torch.randn(B, o, device=dev, generator=g) for o in (20, 32, 1, 3)]

    def run(grouped):
        for n in nets:
            n.zero_grad(set_to_none=True)
        parts[1].grad = None
        items = [(nets[0], xs[0]), (nets[1], xs[1]), (nets[2], xs[2]), (nets[3], parts)]
        with H.deferred_weight_grads():
            outs = H.forward_group(items) if grouped else [n.forward_parts(x) if isinstance(x, tuple) else n(x)
                                                           for n, x in items]
            torch.autograd.backward(outs, seeds)
        return [o.detach().clone() for o in outs], [p.grad.clone() for n in nets for p in n.parameters()], \
            parts[1].grad.clone()

    o1, g1, d1 = run(False)
    o2, g2, d2 = run(True)
    assert all(torch.equal(a, b) for a, b in zip(o1, o2))
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))
    assert torch.equal(d1, d2)
    with torch.no_grad():
        o3 = H.forward_group([(nets[0], xs[0]), (nets[1], xs[1]), (nets[2], xs[2]), (nets[3], parts)])
    assert all(torch.equal(a, b) for a, b in zip(o1, o3))


@pytest.mark.parametrize("B", [3000, 9001])
def test_chain_launch_matches_per_depth_launches_bitwise(B, monkeypatch):
    """lgx_chain (the narrow tail layers of every chain in one launch, forward and input
    gradient; 32-row blocks at 3000 rows, 64-row blocks at 9001) == one grouped launch per
    depth (LGX_CHAIN=0): outputs, every parameter gradient and a parts input gradient,
    bitwise — the encoders (tails from depth 1), the actor / critic (from depth 2)."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import _mlp
    torch.manual_seed(11)
    act = torch.nn.ELU()
    enc = [_mlp(29, [64, 20], 20, act), _mlp(132, [128, 64], 32, act), _mlp(572, [128, 64], 3, act)]
    ac = [_mlp(627, [512, 256, 128], 12, act), _mlp(736, [512, 256, 128], 1, act)]
    enc, ac = [n.to(dev) for n in enc], [n.to(dev) for n in ac]
    g = torch.Generator(device=dev).manual_seed(12)
    xs = [torch.randn(B, d, device=dev, generator=g) for d in (29, 132, 572, 736)]
    obs = torch.randn(B, 572, device=dev, generator=g)
    seeds = [torch.randn(B, o, device=dev, generator=g) for o in (12, 1, 3)]
    calls = []
    orig = H.run_chain

    def spy(descs):
        calls.append(len(descs))
        return orig(descs)

    monkeypatch.setattr(H, "run_chain", spy)
    monkeypatch.setattr(H, "CHAIN_ROWS", 1 << 30)  # the kernel at any row count (product: <= 8192)

    def run(chain):
        monkeypatch.setattr(H, "USE_CHAIN", chain)
        for n in (*enc, *ac):
            n.zero_grad(set_to_none=True)
        with H.deferred_weight_grads():
            lat = H.forward_group([(enc[0], xs[0]), (enc[1], xs[1]), (enc[2], xs[2])])
            mu, v = H.forward_group([(ac[0], (obs, lat[0], lat[1], lat[2])), (ac[1], xs[3])])
            torch.autograd.backward([mu, v, lat[2]], seeds)
        return [t.detach().clone() for t in (*lat, mu, v)], [p.grad.clone() for n in (*enc, *ac) for p in n.parameters()]

    o1, g1 = run(False)
    assert not calls
    o2, g2 = run(True)
    assert calls == [3, 2, 2, 3]  # forward: encoders, actor/critic tails; backward: the same
    assert all(torch.equal(a, b) for a, b in zip(o1, o2))
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))
    with torch.no_grad():
        lat = H.forward_group([(enc[0], xs[0]), (enc[1], xs[1]), (enc[2], xs[2])])
    assert all(torch.equal(a, b) for a, b in zip(o1[:3], lat))


def test_forward_group_output_spans_bitwise():
    """Chains whose last layer writes into column spans of a shared buffer (the update's
    latents inside the actor input) == the same chains writing their own outputs: outputs,
    the actor's output and every gradient, bitwise; the spans hold the latents."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import _mlp
    torch.manual_seed(5)
    act = torch.nn.ELU()
    enc = [_mlp(29, [64, 20], 20, act).to(dev), _mlp(132, [128, 64], 32, act).to(dev)]
    actor = _mlp(90, [256, 128], 12, act).to(dev)
    B = 2500
    g = torch.Generator(device=dev).manual_seed(6)
    xs = [torch.randn(B, 29, device=dev, generator=g), torch.randn(B, 132, device=dev, generator=g)]
    obs, est = torch.randn(B, 35, device=dev, generator=g), torch.randn(B, 3, device=dev, generator=g)
    seed, seed_l = torch.randn(B, 12, device=dev, generator=g), torch.randn(B, 20, device=dev, generator=g)

    def run(spans):
        for n in (*enc, actor):
            n.zero_grad(set_to_none=True)
        buf = torch.full((B, 90), float("nan"), device=dev)
        buf[:, :35].copy_(obs)
        buf[:, 87:].copy_(est)
        with H.deferred_weight_grads():
            if spans:
                lat = H.forward_group([(enc[0], xs[0], None, buf[:, 35:55]), (enc[1], xs[1], None, buf[:, 55:87])])
            else:
                lat = H.forward_group([(enc[0], xs[0]), (enc[1], xs[1])])
            (mu,) = H.forward_group([(actor, (buf[:, :35], lat[0], lat[1], buf[:, 87:]), buf)])
            torch.autograd.backward([mu, lat[0]], [seed, seed_l])
        if spans:
            assert lat[0].data_ptr() == buf[:, 35:55].data_ptr()
        return [mu.detach().clone(), lat[0].detach().clone(), buf.clone()], \
            [p.grad.clone() for n in (*enc, actor) for p in n.parameters()]

    o1, g1 = run(False)
    o2, g2 = run(True)
    assert all(torch.equal(a, b) for a, b in zip(o1, o2))
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))


def test_gather_rows_matches_index_select():
    """lgx_gather_rows (one launch over the storage's buffers) == index_select, bitwise, for
    16-B (vector) and 4-B row widths."""
    g = torch.Generator(device=dev).manual_seed(21)
    rows = 5000
    srcs = [torch.randn(rows, w, device=dev, generator=g) for w in (572, 29, 736, 3, 132, 12, 1)]
    idx = torch.randperm(rows, device=dev, generator=g)[:3000]
    for a, b in zip(H.gather_rows(srcs, idx), [t.index_select(0, idx) for t in srcs]):
        assert torch.equal(a, b)
    # strided destinations: column spans of wider buffers (16-B pitch: vector path; odd
    # pitch: element path), the columns around them untouched
    for pitch in (628, 627):
        wide = torch.full((3000, pitch), -7.0, device=dev)
        outs = H.gather_rows([srcs[0], srcs[3], srcs[1]], idx, [wide[:, :572], wide[:, 624:627], None])
        assert outs[0].data_ptr() == wide.data_ptr()
        assert torch.equal(wide[:, :572], srcs[0].index_select(0, idx))
        assert torch.equal(wide[:, 624:627], srcs[3].index_select(0, idx))
        assert torch.equal(outs[2], srcs[1].index_select(0, idx))
        assert bool((wide[:, 572:624] == -7.0).all()) and bool((wide[:, 627:] == -7.0).all())


def test_transpose_batch_matches_torch():
    g = torch.Generator(device=dev).manual_seed(31)
    W = torch.randn(512, 627, device=dev, generator=g)
    mats = [W, W[:, 572:624], torch.randn(1, 128, device=dev, generator=g), torch.randn(33, 65, device=dev, generator=g)]
    for a, m in zip(H.transpose_batch(mats), mats):
        assert torch.equal(a, m.t().contiguous())


def test_fused_loss_heads_match_separate_heads_bitwise():
    """hip_mlp.loss_heads (one launch each way) == ppo_head + aux_losses: the six losses and
    the gradients of mu, value, std, the privileged latent and the estimator output."""
    g = torch.Generator(device=dev).manual_seed(41)
    B, A = 3000, 12
    r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    base = dict(actions=r(B, A), old_logp=r(B, 1), adv=r(B, 1), tv=r(B, 1), ret=r(B, 1), old_mu=r(B, A),
                old_sigma=r(B, A).abs() + 0.5, a=r(B, 20), t=r(B, 3))
    leaves = [r(B, A), r(B, 1), r(A).abs() + 0.5, r(B, 20), r(B, 3)]
    seeds = torch.tensor([1.0, 1.3, -0.01, 0.05, 1.0], device=dev)

    def run(fused, span=False):
        mu, v, std, pl, pr = [x.clone().requires_grad_(True) for x in leaves]
        if span:  # the privileged latent as a column span of a wider buffer (ld_p)
            wide = torch.zeros(B, 50, device=dev)
            wide[:, 10:30] = leaves[3]
            wide.requires_grad_(True)
            pl = wide[:, 10:30]
        b = base
        if fused:
            outs = H.loss_heads(mu, v, std, b["actions"], b["old_logp"], b["adv"], b["tv"], b["ret"], b["old_mu"],
                                b["old_sigma"], 0.2, True, pl, b["a"], pr, b["t"])
            losses = [outs[0], outs[1], outs[2], outs[4], outs[5]]
        else:
            s1, v1, e1, _k = H.ppo_head(mu, v, std, b["actions"], b["old_logp"], b["adv"], b["tv"], b["ret"],
                                        b["old_mu"], b["old_sigma"], 0.2, True)
            rg, es = H.aux_losses(pl, b["a"], pr, b["t"])
            losses = [s1, v1, e1, rg, es]
        torch.autograd.backward(losses, list(seeds.unbind()))
        dpl = wide.grad[:, 10:30] if span else pl.grad
        return [x.detach().clone() for x in losses] + [x.grad.clone() for x in (mu, v, std)] + \
            [dpl.clone(), pr.grad.clone()]

    ref = run(False)
    for x, y in zip(run(True), ref):
        assert torch.equal(x, y)
    for x, y in zip(run(True, span=True), ref):
        assert torch.equal(x, y)


def test_group_forward_on_empty_input_gives_the_bias():
    """A chain whose input has no columns (ANYmal's scan encoder: num_scan_obs = 0) — nn.Linear
    on [rows, 0] is its bias on every row — inside a grouped launch beside a normal chain."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import ScanEncoder
    torch.manual_seed(0)
    enc = ScanEncoder(num_scan_obs=0, output_dim=32, hidden_dims=[128, 64]).to(dev)
    other = ScanEncoder(num_scan_obs=20, output_dim=16, hidden_dims=[32]).to(dev)
    x0 = torch.zeros(300, 0, device=dev)
    x1 = torch.randn(300, 20, device=dev)
    with torch.no_grad():
        got0, got1 = H.forward_group([enc.group_item(x0), other.group_item(x1)])
        alone = enc(x0)  # the module's own (single-chain) forward
        ref0 = enc.scan_encoder.cpu()(torch.zeros(300, 0))
        ref1 = other.scan_encoder.cpu()(x1.cpu())
    torch.testing.assert_close(alone.cpu(), ref0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(got0.cpu(), ref0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(got1.cpu(), ref1, rtol=1e-4, atol=1e-4)


def test_empty_input_layer_gradients_match_autograd():
    """Backward through a chain whose input has no columns (ANYmal's scan encoder): the first
    layer's bias gradient is sum_rows dY (no GEMM, no split-K workspace), inside a grouped
    backward with deferred weight gradients, against nn.Linear autograd on the CPU."""
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import ScanEncoder
    torch.manual_seed(1)
    enc = ScanEncoder(num_scan_obs=0, output_dim=32, hidden_dims=[128, 64]).to(dev)
    other = ScanEncoder(num_scan_obs=20, output_dim=16, hidden_dims=[32]).to(dev)
    ref_enc = ScanEncoder(num_scan_obs=0, output_dim=32, hidden_dims=[128, 64])
    ref_other = ScanEncoder(num_scan_obs=20, output_dim=16, hidden_dims=[32])
    ref_enc.load_state_dict({k: v.cpu() for k, v in enc.state_dict().items()})
    ref_other.load_state_dict({k: v.cpu() for k, v in other.state_dict().items()})
    x0 = torch.zeros(300, 0, device=dev)
    x1 = torch.randn(300, 20, device=dev)
    w0 = torch.randn(300, 32, device=dev)
    w1 = torch.randn(300, 16, device=dev)
    for p in list(enc.parameters()) + list(other.parameters()):
        p.grad = torch.zeros_like(p)  # defined buffers (as the flat-grad views)
    with H.deferred_weight_grads():
        y0, y1 = H.forward_group([enc.group_item(x0), other.group_item(x1)])
        ((y0 * w0).sum() + (y1 * w1).sum()).backward()
    r0, r1 = ref_enc(torch.zeros(300, 0)), ref_other(x1.cpu())
    ((r0 * w0.cpu()).sum() + (r1 * w1.cpu()).sum()).backward()
    for (n, p), q in zip(list(enc.named_parameters()) + list(other.named_parameters()),
                         list(ref_enc.parameters()) + list(ref_other.parameters())):
        assert torch.isfinite(p.grad).all(), n
        torch.testing.assert_close(p.grad.cpu(), q.grad, rtol=1e-4, atol=1e-4, msg=n)
