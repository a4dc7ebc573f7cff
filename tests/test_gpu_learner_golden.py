"""The HIP learner (grouped 3xbf16 MFMA GEMMs, fused loss heads, flat HIP Adam, hipGraph
update) against the REFERENCE rsl_rl's own outputs (tests/golden/learner_<case>.npz,
tools/gen_learner_golden.py; go2 / go2_parkour shapes at N=64, T=24, and go2_c2: C2's 4096
envs, i.e. the production 24,576-row minibatches, tile shapes and split-K picks).

Stated fp32 tolerances (the GEMMs carry ~2^-16 relative error per product, 3xbf16):
  act outputs, stored rewards, GAE returns   rtol 1e-4, atol 2e-5
  minibatch-0 gradients                      |g - g_ref| <= 2e-3 * max|g_ref| per tensor, and
                                             ||g||^2 within 1e-3 relative
  DAgger-updated adaptation encoder          atol 1e-5 (4 Adam steps of lr 2e-4 ... 20)
  losses                                     rtol 2e-3; learning rate equal (KL schedule)
  parameters after the 20-step update        Adam's first steps move a weight by +-lr whatever
                                             |g|, so near-zero gradients whose sign flips
                                             under rounding diverge by up to 2 lr per step:
                                             median |dp| <= 1e-6, 99th pct <= 5e-5,
                                             max <= 40 lr (20 steps x 2 lr)
  parameters after minibatch 0's Adam step   Adam's first step is lr * g / (|g| + eps) = +-lr:
                                             entries whose reference gradient is well above
                                             the gradient tolerance (sign determined) within
                                             1e-6; the rest (sign may flip) within 2 lr
  Adam moments after the update              exp_avg within 5e-3 * max|ref| per tensor,
                                             exp_avg_sq within 1e-2 * max|ref|

Per-minibatch pin (round 5; tools/gen_learner_golden.py PerMinibatch): the reference records,
for every one of the update's 20 minibatches, its pre-clip gradients (sampled + fp64 sums), both
clip norms and every sample's discrete decisions (ratio clip ppo.py:252, surrogate max :254,
value clip / max :258-261). The update here runs with the PPO head taking those decisions from
the record (lgx_heads_s8_args.decisions_in), so both runs follow the same branch at every sample
and the comparison is of the arithmetic alone, minibatch by minibatch:
  gradients of every minibatch               |g - g_ref| <= 2e-3 * max|g_ref| per tensor
                                             (sampled entries), sum of squares within 1e-3
  pre-clip norms (estimator; main)           rtol 1e-4
  own decisions (decisions_out)              equal to the reference's except at the samples
                                             the reference records within LC.NEAR_TIE (3e-5
                                             relative) of a clip / max boundary
  Adam moments / parameters after the update as above (5e-3 / 1e-2), every case
Free-running (no forcing), a sample whose ratio sits within ~4e-6 of 1 +- clip lands on the
other side of the clip under the GPU's fp32 rounding of its log-prob (3 x bf16 GEMMs: ~1e-5),
and that one sample moves the actor's gradients by 1-3 % of max|g| (go2_c2: minibatch 10, sample
21184, ratio 1.200002313 -> actor.4.weight 1.736e-2; minibatch 13, sample 7613, ratio
1.200004578 -> actor.6.weight 1.536e-2: tools/ref_minibatch_ties.py, which reproduces the GPU's
teacher-forced gradient errors to four digits, profiles/r05_update_decisions.txt).
Near-tie replay (round 5): the update with ONLY those near-tie samples' decisions replayed
(lgx_heads_s8_args.decisions_in bytes with bit 6 set elsewhere: every other decision is the
head's own) ends within the tight bounds (5e-3 / 1e-2) at every size — the production-size pin
of the free-running update: every decision that is not a rounding-level tie is made as the
reference makes it, and the arithmetic follows it. The fully free-running end state is held to
the tight bounds at the 384-row sizes and reported at the production sizes, where which near
ties flip depends on the last bits of mu (measured free-running: 0.067 at go2_c2 and 0.111 at
go2_parkour_c4 of max|exp_avg|; near-tie replay: 4.1e-5 at both, profiles/r05_learner_near_tie.txt).
"""
import numpy as np
import pytest
import torch

import learner_case as LC
import learner_replay as R

pytestmark = pytest.mark.gpu



@pytest.fixture(scope="module", params=list(LC.CASES))
def replay(request):
    case = request.param
    d = R.load(case)
    res, alg = R.run(case, "cuda:0")
    assert alg.graph_mode == "whole", "the update must have been captured as one hipGraph"
    # the production paths ran (no silent fallback): the S8 minibatch executor and the one-launch act
    assert alg._s8 is not None, "the update did not run on the S8 core"
    assert alg._s8act is not None, "the rollout did not run the fused act kernel"
    return case, d, res, alg


def test_gpu_rollout_act_and_returns(replay):
    case, d, res, _ = replay
    for which in (0, 1):
        for t in range(LC.T):
            for k in ("actions", "values", "logp", "mu", "sigma"):
                key = f"roll{which}.{t}.{k}"
                if key not in d:  # sampled (large case)
                    LC.compare(d, f"roll{which}.{t}", k, res[key], rtol=1e-4, atol=2e-5, stat_rtol=1e-4)
                    continue
                np.testing.assert_allclose(res[key].reshape(d[key].shape), d[key], rtol=1e-4, atol=2e-5, err_msg=key)
        for k in ("rewards", "returns", "advantages"):
            key = f"roll{which}.{k}"
            if key not in d:
                LC.compare(d, f"roll{which}", k, res[key], rtol=1e-4, atol=2e-5, stat_rtol=1e-4)
                continue
            np.testing.assert_allclose(res[key], d[key], rtol=1e-4, atol=2e-5, err_msg=key)


def test_gpu_update_dagger(replay):
    case, d, res, _ = replay
    assert res["dagger.loss"] == pytest.approx(float(d["dagger.loss"]), rel=1e-4)
    for k in d.files:
        if k.startswith("dagger.param."):
            np.testing.assert_allclose(res[k], d[k], rtol=0, atol=1e-5, err_msg=k)


def test_gpu_minibatch0_gradients(replay):
    case, d, res, _ = replay
    for n, g in res["grad0"].items():
        if f"grad0.{n}.v" not in d:
            continue
        ref = d[f"grad0.{n}.v"]
        scale = float(np.abs(ref).max()) + 1e-30
        LC.compare(d, "grad0", n, g, rtol=0, atol=2e-3 * scale, stat_rtol=1e-3)


def test_gpu_update_losses_lr_params(replay):
    case, d, res, alg = replay
    np.testing.assert_allclose(res["update.losses"], d["update.losses"], rtol=2e-3, atol=1e-6)
    assert res["update.learning_rate"] == pytest.approx(float(d["update.learning_rate"]), rel=1e-9)
    lr = LC.CASES[case]["lr"]
    diffs = []
    for n, p in res["after"].items():
        idx = LC.sample_index(n, p.size)
        diffs.append(np.abs(p.reshape(-1)[idx] - d[f"after.{n}.v"]))
    dd = np.concatenate(diffs)
    assert np.median(dd) <= 1e-6 and np.quantile(dd, 0.99) <= 5e-5 and dd.max() <= 40 * lr, \
        (np.median(dd), np.quantile(dd, 0.99), dd.max())
    assert torch.isfinite(alg.params_buf).all() and alg.grads.check()


def test_gpu_minibatch0_adam_step(replay):
    """One Adam step from identical parameters: +-lr per entry, the sign of the gradient."""
    case, d, res, _ = replay
    c = LC.CASES[case]
    flips = total = 0
    for n, p in res["mb0"].items():
        if f"mb0.{n}.v" not in d:
            continue
        lr = c["est_lr"] if n.startswith("estimator.") else c["lr"]
        idx = LC.sample_index(n, p.size)
        diff = np.abs(p.reshape(-1)[idx] - d[f"mb0.{n}.v"])
        g = np.abs(d[f"grad0.{n}.v"])
        firm = g > 4e-3 * (g.max() + 1e-30)  # twice the gradient tolerance: sign determined
        assert np.all(diff[firm] <= 1e-6), (n, diff[firm].max())
        assert np.all(diff <= 2 * lr + 1e-6), (n, diff.max())
        flips += int((diff > 1e-6).sum())
        total += diff.size
    print(f"{case}: minibatch-0 Adam step, {flips} of {total} sampled entries moved the other way (|g| ~ 0)")
    assert flips <= 0.01 * total


def _moments(case, d, res, keys, tols):
    worst = [0.0, 0.0]
    for n, m in res[keys[0]].items():
        for j, (key, tol) in enumerate(zip(keys, tols)):
            ref = d[f"{key}.{n}.v"]
            scale = float(np.abs(ref).max()) + 1e-30
            got = res[key][n].reshape(-1)[LC.sample_index(n, m.size)]
            err = float(np.abs(got - ref).max()) / scale
            worst[j] = max(worst[j], err)
            assert err <= tol, (key, n, err)
    return worst


def test_gpu_adam_moments_after_epoch0(replay):
    """Adam moments after epoch 0 (num_mini_batches minibatches: gradients still within ~1e-4 of
    the autograd path's, tools/dbg_s8_steps.py): the tight check of the update's arithmetic."""
    case, d, res, _ = replay
    w = _moments(case, d, res, ("exp_avg_e0", "exp_avg_sq_e0"), (5e-3, 1e-2))
    print(f"{case}: Adam moments after epoch 0, worst |err| / max|ref| per tensor: exp_avg {w[0]:.3g}, "
          f"exp_avg_sq {w[1]:.3g}")


def test_gpu_adam_moments_after_update(replay):
    """After all 20 minibatches, free-running. The 384-row cases within 5e-3 / 1e-2; at the
    production minibatch sizes (24,576 / 49,152 rows) near-tie clip flips (module docstring) put
    the free-running end state on another branch: there a gross-divergence guard holds it (measured
    round 5: exp_avg 0.067 / 0.111, exp_avg_sq ≈0.02 of max|ref| at go2_c2 / go2_parkour_c4; bound
    0.25 / 0.1, so a 3-10x regression of the product's own free-running path fails), and
    test_gpu_near_tie_forced_update_end_state is the tight check."""
    case, d, res, _ = replay
    large = LC.n_envs(case) >= 4096
    tols = (0.25, 0.1) if large else (5e-3, 1e-2)
    w = _moments(case, d, res, ("exp_avg", "exp_avg_sq"), tols)
    assert np.isfinite(w).all()
    print(f"{case}: free-running Adam moments, worst |err| / max|ref| per tensor: exp_avg {w[0]:.3g}, "
          f"exp_avg_sq {w[1]:.3g}")


@pytest.fixture(scope="module", params=list(LC.CASES))
def forced(request):
    case = request.param
    d = R.load(case)
    if "mb0.decisions" not in d.files:
        pytest.skip("fixture without per-minibatch records")
    res, _alg = R.run_per_minibatch(case, "cuda:0", d, force=True)
    return case, d, res


def test_gpu_every_minibatch_gradients_pinned(forced):
    """All 20 minibatches of the update, each against the reference's own gradients at that
    minibatch, with the reference's per-sample decisions replayed."""
    case, d, res = forced
    worst = []
    for k, rec in enumerate(res["mbg"]):
        w = 0.0
        for n, (v, s_, sq) in rec.items():
            key = f"mbg{k}.{n}"
            ref = d[f"{key}.v"]
            scale = float(np.abs(ref).max()) + 1e-30
            err = float(np.abs(v - ref).max()) / scale
            w = max(w, err)
            assert err <= 2e-3, (k, n, err)
            ref2 = float(d[f"{key}.sumsq"])
            assert abs(sq - ref2) <= 1e-3 * max(ref2, 1e-30) + 1e-12, (k, n, sq, ref2)
        np.testing.assert_allclose(res["norms"][k], d[f"mb{k}.norms"], rtol=1e-4, err_msg=f"minibatch {k} norms")
        worst.append(w)
    print(f"{case}: per-minibatch worst gradient error / max|g_ref|: " + " ".join(f"{w:.1e}" for w in worst))


def test_gpu_own_decisions_only_differ_at_near_ties(forced):
    """The head's OWN per-sample decisions (recorded while the reference's are replayed) equal the
    reference's at every sample except those the reference records as within NEAR_TIE of a
    boundary: the named source of the free-running divergence, and nothing else."""
    case, d, res = forced
    flips = []
    for k in range(len(res["mbg"])):
        diff = R.effective_mismatch(d[f"mb{k}.decisions"], res["dec_out"][k])
        near = set(d[f"mb{k}.near"].tolist())
        assert set(diff.tolist()) <= near, (k, sorted(set(diff.tolist()) - near)[:10])
        flips.append(len(diff))
    print(f"{case}: own-decision flips per minibatch (all at recorded near ties): {flips}")


def test_gpu_forced_update_end_state(forced):
    """With the reference's decisions, the end-of-update moments and parameters are within the
    tight bounds at every size (no branch spread)."""
    case, d, res = forced
    w = _moments(case, d, res, ("exp_avg", "exp_avg_sq"), (5e-3, 1e-2))
    lr = LC.CASES[case]["lr"]
    diffs = []
    for n, p in res["after"].items():
        idx = LC.sample_index(n, p.size)
        diffs.append(np.abs(p.reshape(-1)[idx] - d[f"after.{n}.v"]))
    dd = np.concatenate(diffs)
    assert np.median(dd) <= 1e-6 and np.quantile(dd, 0.99) <= 5e-5 and dd.max() <= 40 * lr, \
        (np.median(dd), np.quantile(dd, 0.99), dd.max())
    print(f"{case}: forced update, end-of-update moments worst |err| / max|ref|: exp_avg {w[0]:.3g}, "
          f"exp_avg_sq {w[1]:.3g}; params median {np.median(dd):.2e} max {dd.max():.2e}")


@pytest.fixture(scope="module", params=list(LC.CASES))
def near_forced(request):
    case = request.param
    d = R.load(case)
    if "mb0.decisions" not in d.files:
        pytest.skip("fixture without per-minibatch records")
    res, _alg = R.run_per_minibatch(case, "cuda:0", d, force=True, near_only=True)
    return case, d, res


def test_gpu_near_tie_forced_update_end_state(near_forced):
    """The update with only the near-tie samples' decisions replayed (every other decision the
    head's own): the end-of-update moments and parameters within the tight bounds at every size,
    and the head's own decisions equal the reference's at every sample that is not a near tie."""
    case, d, res = near_forced
    for k in range(len(res["mbg"])):
        diff = R.effective_mismatch(d[f"mb{k}.decisions"], res["dec_out"][k])
        near = set(d[f"mb{k}.near"].tolist())
        assert set(diff.tolist()) <= near, (k, sorted(set(diff.tolist()) - near)[:10])
    w = _moments(case, d, res, ("exp_avg", "exp_avg_sq"), (5e-3, 1e-2))
    lr = LC.CASES[case]["lr"]
    dd = np.concatenate([np.abs(p.reshape(-1)[LC.sample_index(n, p.size)] - d[f"after.{n}.v"])
                         for n, p in res["after"].items()])
    assert np.median(dd) <= 1e-6 and np.quantile(dd, 0.99) <= 5e-5 and dd.max() <= 40 * lr, \
        (np.median(dd), np.quantile(dd, 0.99), dd.max())
    print(f"{case}: near-tie-forced update, end-of-update moments worst |err| / max|ref|: exp_avg {w[0]:.3g}, "
          f"exp_avg_sq {w[1]:.3g}; params median {np.median(dd):.2e} max {dd.max():.2e}")
