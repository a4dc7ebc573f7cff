"""lgx_ppo_tail (the PPO minibatch optimizer tail: both grad-norm clips, the adaptive-KL
learning rate, both Adam steps, the loss sums; ppo.py:207-293 with torch.nn.utils.clip_grad_norm_
and torch.optim.Adam) against the same statement in torch fp64, on segments whose bounds are
NOT multiples of 4, so the float4 bodies, scalar heads and scalar tails of every segment run."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _reference(g, p, m, v, main, est, adapt, kl_index, max_norm, bm, em, be, ee, est_lr, desired_kl, lr, tm, te):
    g, p, m, v = (x.double().clone() for x in (g, p, m, v))
    seg = lambda r: slice(*r)  # noqa: E731
    se = g[seg(est)].square().sum()
    sm = g[seg(main)].square().sum() + g[seg(adapt)].square().sum()
    ce = min(max_norm / (math.sqrt(se) + 1e-6), 1.0)
    cm = min(max_norm / (math.sqrt(sm) + 1e-6), 1.0)
    if kl_index >= 0:
        kl = float(g[kl_index])
        if kl > desired_kl * 2.0:
            lr = max(lr / 1.5, 1e-5)
        elif desired_kl / 2.0 > kl > 0.0:
            lr = min(lr * 1.5, 1e-2)
    tm, te = tm + 1, te + 1
    for (lo, hi), c, (b1, b2), eps, rate, t in ((main, cm, bm, em, lr, tm), (est, ce, be, ee, est_lr, te)):
        gs = g[lo:hi] * c
        m[lo:hi] = b1 * m[lo:hi] + (1 - b1) * gs
        v[lo:hi] = b2 * v[lo:hi] + (1 - b2) * gs * gs
        step_size = rate / (1 - b1 ** t)
        p[lo:hi] -= step_size * m[lo:hi] / (v[lo:hi].sqrt() / math.sqrt(1 - b2 ** t) + eps)
    g[seg(adapt)] *= cm
    return g, p, m, v, lr, tm, te


@pytest.mark.parametrize("kl", [0.05, 0.001, 0.003])
def test_ppo_tail_matches_torch(kl):
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp
    dev = "cuda:0"
    gen = torch.Generator().manual_seed(7)
    n = 40_003
    main, est, adapt, kl_index = (3, 25_001), (25_001, 31_999), (32_002, 40_001), 40_001
    g = torch.randn(n, generator=gen) * 0.05
    g[kl_index] = kl
    p = torch.randn(n, generator=gen)
    m = torch.randn(n, generator=gen) * 1e-3
    v = torch.rand(n, generator=gen) * 1e-4
    max_norm, bm, em, be, ee, est_lr, desired_kl, lr, tm, te = 1.0, (0.9, 0.999), 1e-8, (0.9, 0.99), 1e-6, 2e-4, 0.01, \
        1e-3, 7.0, 3.0
    want = _reference(g, p, m, v, main, est, adapt, kl_index, max_norm, bm, em, be, ee, est_lr, desired_kl, lr, tm, te)

    gd, pd, md, vd = (x.to(dev) for x in (g, p, m, v))
    lr64 = torch.tensor([lr], dtype=torch.float64, device=dev)
    lr32 = torch.tensor([lr], dtype=torch.float32, device=dev)
    step_main = torch.tensor([tm], device=dev)
    step_est = torch.tensor([te], device=dev)
    losses = [torch.tensor([float(k + 1)], device=dev) for k in range(4)]
    sums = torch.full((4,), 10.0, device=dev)
    ws = torch.zeros(2 * 512 + 8, device=dev)
    counter = torch.zeros(1, dtype=torch.int32, device=dev)
    hip_mlp.ppo_tail(gd, pd, md, vd, main, est, adapt, kl_index, max_norm, bm, em, be, ee, est_lr, desired_kl, lr64,
                     lr32, step_main, step_est, losses, sums, ws, counter)
    torch.cuda.synchronize()

    wg, wp, wm, wv, wlr, wtm, wte = want
    torch.testing.assert_close(pd.cpu().double(), wp, rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(md.cpu().double(), wm, rtol=2e-5, atol=1e-9)
    torch.testing.assert_close(vd.cpu().double(), wv, rtol=2e-5, atol=1e-12)
    torch.testing.assert_close(gd.cpu().double(), wg, rtol=2e-5, atol=1e-9)
    # untouched outside the segments: the gap, the scalar slots around them
    for i in (0, 1, 2, 32_000, 32_001, 40_002):
        assert gd[i].item() == g[i].item() and pd[i].item() == p[i].item()
    assert lr64.item() == pytest.approx(wlr, rel=1e-12)
    assert lr32.item() == pytest.approx(wlr, rel=1e-6)
    assert step_main.item() == wtm and step_est.item() == wte
    assert sums.cpu().tolist() == [11.0, 12.0, 13.0, 14.0]
    assert counter.item() == 0
