"""The build's PPO/ROA learner on the CPU against the REFERENCE rsl_rl's own outputs
(tests/golden/learner_<case>.npz, recorded by tools/gen_learner_golden.py from
/root/reference/rsl_rl at the go2 / go2_parkour network shapes, N=64 envs, T=24):

  act                ppo.py:129-153, actor_critic.py:190-226
  process_env_step   ppo.py:156-171 (time-out bootstrap)
  compute_returns    rollout_storage.py:110-124
  update_dagger      ppo.py:309-349
  update             ppo.py:182-293 (minibatch-0 gradients, losses, lr, parameters and Adam
                     moments after 5 epochs x 4 minibatches, ROA coefficient 0.025)
  layouts            state_dict keys/shapes, optimizer param groups (checkpoint format)

Tolerance (fp32, stated): the CPU learner runs the same torch fp32 ops in a restructured
order (flat gradients, estimator step after the main backward, clip norms over flat
segments), so results agree to a few fp32 ulps: rtol 2e-5 on forward outputs and returns;
gradients rtol 1e-4 / atol 1e-7; parameters after 20 Adam steps atol 5e-7 (Adam moves a
weight by <= lr = 2e-4 per step; ulp-level gradient differences stay ulp-level; measured:
max |Δparam| 6.7e-8, max gradient error 3e-7 of the tensor scale)."""
import numpy as np
import pytest

import learner_case as LC
import learner_replay as R


@pytest.fixture(scope="module", params=LC.SMALL_CASES)  # (go2_c2, 4096 envs: the GPU suite)
def replay(request):
    case = request.param
    d = R.load(case)
    res, alg = R.run(case, "cpu")
    return case, d, res, alg


def test_layouts_match_reference(replay):
    case, d, res, _ = replay
    m = R.meta(d)
    for key in ("state_dict", "estimator_state_dict", "optimizer_param_groups", "adaptation_optimizer",
                "estimator_optimizer"):
        assert res["meta"][key] == m[key], key


def test_rollout_act_and_returns(replay):
    case, d, res, _ = replay
    for which in (0, 1):
        for t in range(LC.T):
            for k in ("actions", "values", "logp", "mu", "sigma"):
                key = f"roll{which}.{t}.{k}"
                np.testing.assert_allclose(res[key].reshape(d[key].shape), d[key], rtol=2e-5, atol=2e-6, err_msg=key)
        for k in ("rewards", "returns", "advantages"):
            key = f"roll{which}.{k}"
            np.testing.assert_allclose(res[key], d[key], rtol=2e-5, atol=2e-6, err_msg=key)


def test_update_dagger(replay):
    case, d, res, _ = replay
    assert res["dagger.loss"] == pytest.approx(float(d["dagger.loss"]), rel=1e-5)
    for k in d.files:
        if k.startswith("dagger.param.") or k.startswith("dagger.grad."):
            np.testing.assert_allclose(res[k], d[k], rtol=1e-4, atol=2e-6, err_msg=k)


def test_update_minibatch0_gradients(replay):
    case, d, res, _ = replay
    for n, g in res["grad0"].items():
        if f"grad0.{n}.v" in d:
            LC.compare(d, "grad0", n, g, rtol=1e-4, atol=1e-7, stat_rtol=1e-4)


def test_update_losses_lr_params_moments(replay):
    case, d, res, _ = replay
    np.testing.assert_allclose(res["update.losses"], d["update.losses"], rtol=1e-5, atol=1e-7)
    assert res["update.learning_rate"] == pytest.approx(float(d["update.learning_rate"]), rel=1e-12)
    for n, p in res["after"].items():
        LC.compare(d, "after", n, p, rtol=1e-5, atol=5e-7, stat_rtol=1e-5)
    for n, m in res["exp_avg"].items():
        LC.compare(d, "exp_avg", n, m, rtol=1e-3, atol=1e-7)
        LC.compare(d, "exp_avg_sq", n, res["exp_avg_sq"][n], rtol=1e-3, atol=1e-12)


def test_update_moments_after_epoch0(replay):
    """The Adam moments after epoch 0's last minibatch (num_mini_batches steps)."""
    case, d, res, _ = replay
    for n, m in res["exp_avg_e0"].items():
        LC.compare(d, "exp_avg_e0", n, m, rtol=1e-3, atol=1e-7)
        LC.compare(d, "exp_avg_sq_e0", n, res["exp_avg_sq_e0"][n], rtol=1e-3, atol=1e-12)


def test_update_minibatch0_adam_step(replay):
    """Parameters after minibatch 0's single Adam step (+-lr by the gradient's sign)."""
    case, d, res, _ = replay
    for n, p in res["mb0"].items():
        if f"mb0.{n}.v" in d:
            LC.compare(d, "mb0", n, p, rtol=0, atol=1e-7)
