"""The rollout's act networks in one launch (lgx_s8_act, rsl_rl/algorithms/s8_act.py) against
the grouped launches (PPO.use_fused_act False), same parameters and injected noise, over a
24-step rollout of every learner case: actions, mu, sigma, log-probs and values in the storage
(fp32: the same 3 x bf16 products; the actor's first layer sums its segmented input in a
different order: rtol 1e-5, atol 1e-5 on values of order 1), and the observation rows it writes (bit for bit). Plus: the weights are refreshed at each rollout's first step
(after an update the fused path follows the new weights), and the ABI rejects bad layouts."""
import pytest
import torch

import learner_case as LC
import learner_replay as R

pytestmark = pytest.mark.gpu
dev = "cuda:0"
FIELDS = ("actions", "mu", "sigma", "actions_log_prob", "values")
OBS_FIELDS = ("observations", "privileged_observations", "critic_observations", "true_estimated_observations",
              "scan_observations")


def _rollout(case, fused, which=1):
    alg = R.build(case, dev, use_graphs=False)
    alg.use_fused_act = fused
    R.rollout(alg, case, which, {}, False, dev)
    assert (alg._s8act is not None) == fused
    return alg, {f: getattr(alg.storage, f).clone() for f in FIELDS + OBS_FIELDS}


@pytest.mark.parametrize("case", list(LC.CASES))
def test_fused_act_matches_grouped_launches(case):
    _a, ref = _rollout(case, False)
    _b, got = _rollout(case, True)
    for f in FIELDS:
        torch.testing.assert_close(got[f], ref[f], rtol=1e-5, atol=1e-5, msg=lambda m, f=f: f"{case}.{f}: {m}")
    for f in OBS_FIELDS:  # the storage's observation rows: written by the fused kernel, copies
        assert torch.equal(got[f], ref[f]), f"{case}.{f}"


def test_fused_act_refreshes_weights_each_rollout():
    case = "go2"
    alg, _ = _rollout(case, True)
    with torch.no_grad():  # an "update": every parameter moves
        for p in alg.actor_critic.parameters():
            p.mul_(1.01).add_(0.001)
        for p in alg.estimator.parameters():
            p.mul_(1.01).add_(0.001)
    alg.storage.clear()
    R.rollout(alg, case, 2, {}, False, dev)
    got = {f: getattr(alg.storage, f).clone() for f in FIELDS}
    alg.use_fused_act = False
    alg.storage.clear()
    R.rollout(alg, case, 2, {}, False, dev)
    for f in FIELDS:
        torch.testing.assert_close(got[f], getattr(alg.storage, f), rtol=1e-5, atol=1e-5, msg=lambda m, f=f: f"{f}: {m}")


def test_act_abi_rejects_bad_layouts():
    from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S
    alg, _ = _rollout("go2", True)
    a = alg._s8act.args
    saved = a.width
    a.width = saved + 8  # not a multiple of 32
    with pytest.raises(S.S8LibError):
        S.act(a)
    a.width = saved
    saved = a.actor[1].K
    a.actor[1].K = saved + 1  # chain widths must match
    with pytest.raises(S.S8LibError):
        S.act(a)
    a.actor[1].K = saved


@pytest.mark.parametrize("drawn", [True, False])
def test_fused_act_head_matches_act_head_kernel(drawn):
    """The act head inside the fused kernel (mu from LDS) against lgx_act_head on the mu the
    same kernel writes without it: actions (and their copy), mu, sigma and log-prob bit for bit,
    with the Philox draw (the GPU rollout's) and with given eps."""
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
    alg, _ = _rollout("go2", True)
    f, s = alg._s8act, alg.storage
    obs, priv, crit, est, scan = (getattr(s, n)[3].clone() for n in OBS_FIELDS)
    mu, val = f.run(obs, priv, crit, scan)
    mu, val = mu.clone(), val.clone()
    B, A = mu.shape
    std = alg.actor_critic.std.detach()
    step = torch.tensor([7], dtype=torch.int64, device=dev)
    noise = (0x9E3779B97F4A7C15, step, 5) if drawn else None
    eps = None if drawn else torch.randn(B, A, device=dev)

    def bufs():
        return dict(actions=torch.full((B, A), 7.0, device=dev), mu=torch.full((B, A), 7.0, device=dev),
                    sigma=torch.full((B, A), 7.0, device=dev), logp=torch.full((B, 1), 7.0, device=dev),
                    actions_copy=torch.full((B, A), 7.0, device=dev))
    ref = bufs()
    H.act_head(mu, std, eps, ref["actions"], ref["mu"], ref["sigma"], ref["logp"], actions_copy=ref["actions_copy"],
               noise=noise)
    got = bufs()
    m2, v2 = f.run(obs, priv, crit, scan, head=dict(std=std, eps=eps, noise=noise, **got))
    assert m2 is None
    assert torch.equal(v2, val)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k
