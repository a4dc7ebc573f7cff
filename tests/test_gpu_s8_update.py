"""The PPO minibatch on the S8 GEMM core (rsl_rl/algorithms/s8_update.py) against the autograd
path on the fp32-operand GEMMs (LGX_S8_UPDATE=0), same parameters, same rollout, same permutation.

Both compute the same 3 x bf16 products of the same split values; the S8 path reads ELU'(y) from
y's hi + lo (~2^-17 relative) and sums each bias gradient per tile, then over tiles. Stated
tolerance per gradient tensor and minibatch: |g_s8 - g_ref| <= 1e-4 * max|g_ref| + 1e-8, losses
rtol 1e-5. (Against the REFERENCE rsl_rl: test_gpu_learner_golden.py, which now runs this path.)"""
import pytest
import torch

import learner_case as LC
import learner_replay as R

pytestmark = pytest.mark.gpu
dev = "cuda:0"


def _grads(case, use_s8):
    alg = R.build(case, dev, use_graphs=False)
    alg.use_s8 = use_s8
    res = {}
    R.rollout(alg, case, 1, res, False, dev)
    alg.total_updates = LC.TOTAL_UPDATES
    alg._reg_coef.fill_(alg.reg_coef())
    alg._perm.copy_(torch.from_numpy(LC.permutation(case, 1)).to(dev))
    alg._precompute()
    assert (alg._s8 is not None) == use_s8
    out = []
    for idx in alg._minibatches():
        alg._minibatch_grads(idx)
        torch.cuda.synchronize()
        out.append(({n: p.grad.detach().clone() for n, p in R.named_params(alg) if not n.startswith("adaptation")},
                    alg._head_out.clone(), alg._aux_out.clone(), alg.grads.segment("kl").clone()))
    return out


@pytest.mark.parametrize("case", list(LC.CASES))
def test_s8_minibatch_matches_autograd_path(case):
    ref = _grads(case, False)
    got = _grads(case, True)
    worst = 0.0
    for (g1, h1, a1, k1), (g0, h0, a0, k0) in zip(got, ref):
        for n, r in g0.items():
            scale = float(r.abs().max())
            err = float((g1[n] - r).abs().max())
            worst = max(worst, err / (scale + 1e-30))
            assert err <= 1e-4 * scale + 1e-8, (case, n, err, scale)
        torch.testing.assert_close(h1, h0, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(a1, a0, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(k1, k0, rtol=1e-4, atol=1e-8)
    print(f"{case}: worst |g_s8 - g_ref| / max|g_ref| = {worst:.3g}")


def test_s8_update_graph_equals_eager():
    """The hipGraph replay of the S8 update equals its eager run bit for bit (static buffers)."""
    case = "go2"
    outs = []
    for graphs in (False, True):
        alg = R.build(case, dev, use_graphs=graphs)
        res = {}
        perm = torch.from_numpy(LC.permutation(case, 1)).to(dev)
        alg._next_perm = lambda n, p=perm: p
        for it in range(3):
            R.rollout(alg, case, 1, res, False, dev)
            alg.total_updates = LC.TOTAL_UPDATES
            alg.update()
        assert alg._s8 is not None
        if graphs:
            assert alg.graph_mode == "whole"
        torch.cuda.synchronize()
        outs.append(torch.cat([p.detach().reshape(-1) for _n, p in R.named_params(alg)]))
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("graphs", [False, True])
def test_tail_writes_the_weight_split(graphs):
    """The optimizer tail's S8 copies of the updated weights (lgx_ppo_tail with the S8 table,
    include/lgx_mlp.h lgx_tail_s8_seg) equal a weight split launch of the same weights bit for
    bit, every row-major copy (the actor's segmented first layer included) and the encoders'
    fragment-packed ones, after updates whose minibatches ran no per-minibatch split."""
    from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S
    case = "go2"
    alg = R.build(case, dev, use_graphs=graphs)
    res = {}
    perm = torch.from_numpy(LC.permutation(case, 1)).to(dev)
    alg._next_perm = lambda n, p=perm: p
    for _ in range(2):
        R.rollout(alg, case, 1, res, False, dev)
        alg.total_updates = LC.TOTAL_UPDATES
        alg.update()
    s8 = alg._s8
    assert s8 is not None and s8.tail_segs is not None and s8.tail_table() is not None
    bufs = [Ws for p in s8.parts for Ws in p.Ws] + [Wp for p in s8.parts for Wp in getattr(p, "Wp", [])]
    torch.cuda.synchronize()
    got = [b.clone() for b in bufs]
    S.split(s8.wsplit)
    torch.cuda.synchronize()
    for k, (g, b) in enumerate(zip(got, bufs)):
        assert torch.equal(g, b), f"S8 copy {k} differs from the split of the updated weights"
