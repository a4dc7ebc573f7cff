"""Replay of a learner fixture (tests/golden/learner_<case>.npz, recorded from the reference
rsl_rl by tools/gen_learner_golden.py) through THIS build's PPO on a given device.
Returns every quantity the fixture holds, as numpy, for the tests to compare."""
import json
from unittest import mock

import numpy as np
import torch

import golden_util as G
import learner_case as LC


def load(case):
    return G.load(f"learner_{case}.npz")


def build(case, device, use_graphs=None):
    from legged_gym_custom_amd.rsl_rl.algorithms import PPO
    from legged_gym_custom_amd.rsl_rl.modules import ActorCritic
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import MlpEstimator
    c = LC.CASES[case]
    ac = ActorCritic(num_proprio=c["P"], num_privileged_obs=c["priv"], num_critic_obs=c["critic"],
                     num_estimated_obs=c["est"], num_scan_obs=c["scan"], num_actions=c["A"],
                     history_buffer_length=c["H"], actor_hidden_dims=c["actor"], critic_hidden_dims=c["critic_h"],
                     priv_encoder_hidden_dims=c["priv_h"], scan_encoder_hidden_dims=c["scan_h"],
                     latent_encoder_output_dim=c["latent"], scan_encoder_output_dim=c["scan_out"], activation="elu",
                     init_noise_std=1.0)
    est = MlpEstimator(num_proprio=c["P"], history_buffer_length=c["H"], output_dim=c["est"],
                       hidden_dims=c["est_h"], activation="elu", use_history=True)
    w = LC.weights(case, [(k, tuple(v.shape)) for k, v in ac.state_dict().items()])
    ac.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    we = LC.weights(case, [("estimator." + k, tuple(v.shape)) for k, v in est.state_dict().items()])
    est.load_state_dict({k[len("estimator."):]: torch.from_numpy(v) for k, v in we.items()})
    alg = PPO(ac, est, num_learning_epochs=c["epochs"], num_mini_batches=c["minibatches"], clip_param=c["clip"],
              gamma=c["gamma"], lam=c["lam"], value_loss_coef=1.0, entropy_coef=c["entropy"], learning_rate=c["lr"],
              estimator_learning_rate=c["est_lr"], max_grad_norm=c["max_grad_norm"], use_clipped_value_loss=True,
              schedule=c["schedule"], desired_kl=c["desired_kl"], device=device, use_graphs=use_graphs)
    alg.init_storage(LC.n_envs(case), LC.T, [c["P"] * (c["H"] + 1)], [c["priv"]], [c["critic"]], [c["est"]], [c["scan"]],
                     [c["A"]])
    return alg


def named_params(alg):
    ac, est = alg.actor_critic, alg.estimator
    return [(k, p) for k, p in ac.named_parameters()] + [("estimator." + k, p) for k, p in est.named_parameters()]


def _np(t):
    return t.detach().float().cpu().numpy().copy()


def rollout(alg, case, which, res, adaptation_mode, device):
    pre = f"roll{which}"
    for t in range(LC.T):
        d = LC.rollout_inputs(case, which, t)
        x = {k: torch.from_numpy(v).to(device) for k, v in d.items()}
        eps = x["eps"]
        real = torch.randn_like

        def fake(t_, *a, **k):
            return eps.clone() if tuple(t_.shape) == tuple(eps.shape) else real(t_, *a, **k)

        with mock.patch("torch.randn_like", fake):
            alg.act(x["obs"], x["priv"], x["critic"], x["est"], x["scan"], adaptation_mode=adaptation_mode)
        tr = alg.transition
        res[f"{pre}.{t}.actions"] = _np(tr.actions)
        res[f"{pre}.{t}.values"] = _np(tr.values)
        res[f"{pre}.{t}.logp"] = _np(tr.actions_log_prob).reshape(-1)
        res[f"{pre}.{t}.mu"] = _np(tr.action_mean)
        res[f"{pre}.{t}.sigma"] = _np(tr.action_sigma)
        alg.process_env_step(x["rewards"], x["dones"], {"time_outs": x["time_outs"]})
    s = alg.storage
    res[f"{pre}.rewards"] = _np(s.rewards)
    alg.compute_returns(torch.from_numpy(LC.last_critic(case, which)).to(device))
    res[f"{pre}.returns"] = _np(s.returns)
    res[f"{pre}.advantages"] = _np(s.advantages)


def run(case, device, use_graphs=None):
    """The fixture's sequence on this build; returns {key: numpy} (and the algorithm)."""
    alg = build(case, device, use_graphs)
    res = {}
    rollout(alg, case, 0, res, True, device)
    perm0 = torch.from_numpy(LC.permutation(case, 0)).to(device)
    alg._next_perm = lambda n: perm0
    res["dagger.loss"] = alg.update_dagger()
    for n, p in named_params(alg):
        if n.startswith("adaptation_encoder_."):
            res[f"dagger.param.{n}"] = _np(p)
            res[f"dagger.grad.{n}"] = _np(p.grad)
    rollout(alg, case, 1, res, False, device)
    alg.total_updates = LC.TOTAL_UPDATES
    perm1 = torch.from_numpy(LC.permutation(case, 1)).to(device)
    alg._next_perm = lambda n: perm1
    # minibatch 0's gradients (before any optimizer step of this update): phase A only
    alg._reg_coef.fill_(alg.reg_coef())
    alg._perm.copy_(perm1)
    alg._precompute()
    alg._minibatch_grads(alg._minibatches()[0])
    res["grad0"] = {n: _np(p.grad) for n, p in named_params(alg)}
    # the parameters after minibatch 0's optimizer steps: snapshot at the first _minibatch_step
    # (the first update runs eagerly before any graph is captured; capture calls it again and
    # then takes no snapshot)
    mb0, e0, count = {}, {}, [0]
    step = alg._minibatch_step
    names_of = {id(p): n for n, p in named_params(alg)}

    def first_step():
        step()
        count[0] += 1
        if not mb0:
            mb0.update({n: p.detach().clone() for n, p in named_params(alg)})
        if count[0] == alg.num_mini_batches:  # the Adam moments after epoch 0 (eager update)
            for oname in ("optimizer", "estimator_optimizer"):
                opt = getattr(alg, oname)
                for grp in opt.param_groups:
                    for p in grp["params"]:
                        st = opt.state[p]
                        e0[names_of[id(p)]] = (_np(st["exp_avg"]), _np(st["exp_avg_sq"]))

    alg._minibatch_step = first_step
    mv, ms, mr, coef, me = alg.update()
    del alg._minibatch_step
    res["mb0"] = {n: _np(p) for n, p in mb0.items()}
    res["exp_avg_e0"] = {n: m for n, (m, v) in e0.items()}
    res["exp_avg_sq_e0"] = {n: v for n, (m, v) in e0.items()}
    res["update.losses"] = np.array([mv, ms, mr, coef, me])
    res["update.learning_rate"] = alg.learning_rate
    res["after"] = {n: _np(p) for n, p in named_params(alg)}
    names_of = {id(p): n for n, p in named_params(alg)}
    res["exp_avg"], res["exp_avg_sq"] = {}, {}
    for oname in ("optimizer", "estimator_optimizer"):
        opt = getattr(alg, oname)
        for grp in opt.param_groups:
            for p in grp["params"]:
                st = opt.state[p]
                res["exp_avg"][names_of[id(p)]] = _np(st["exp_avg"])
                res["exp_avg_sq"][names_of[id(p)]] = _np(st["exp_avg_sq"])
    res["meta"] = {"state_dict": [[k, list(v.shape)] for k, v in alg.actor_critic.state_dict().items()],
                   "estimator_state_dict": [[k, list(v.shape)] for k, v in alg.estimator.state_dict().items()],
                   "optimizer_param_groups": [[names_of[id(p)] for p in g["params"]] for g in alg.optimizer.param_groups],
                   "adaptation_optimizer": [names_of[id(p)] for p in alg.adaptation_optimizer.param_groups[0]["params"]],
                   "estimator_optimizer": [names_of[id(p)] for p in alg.estimator_optimizer.param_groups[0]["params"]]}
    return res, alg


def meta(d):
    return json.loads(str(d["meta_json"]))


DEC_SURR = 0x07   # decision byte: surrogate max weight (bits 0-1) + ratio in band (bit 2)
DEC_VALUE = 0x18  # value-loss max weight (bits 3-4)
DEC_VBAND = 0x20  # v - target inside the value clip band (bit 5)


def effective_mismatch(ref, got):
    """Per-sample disagreement of two decision byte arrays: every bit except the value-loss max
    weight of samples inside the value clip band, where both terms of that max are the same
    number up to rounding and give the same gradient (ppo.py:258-261)."""
    ref, got = ref.astype(np.int32), got.astype(np.int32)
    mask = np.where((ref & DEC_VBAND) != 0, DEC_SURR | DEC_VBAND, DEC_SURR | DEC_VALUE | DEC_VBAND)
    return np.flatnonzero((ref & mask) != (got & mask))


def run_per_minibatch(case, device, d, force=True, near_only=False):
    """The fixture's sequence with the update run eagerly minibatch by minibatch: with `force`, the
    PPO head takes every per-sample discrete decision (ratio clip, surrogate / value max) from
    the reference run's record (d["mb<k>.decisions"]), so the trajectory follows the reference's
    branch at every sample — with `near_only`, only at the samples the reference records within
    LC.NEAR_TIE of a boundary (all others are the head's own); the launch also records its OWN
    decisions. Returns per minibatch the
    sampled pre-clip gradients (+ fp64 sums), both pre-clip norms and the own decisions, and the
    end state (parameters, Adam moments)."""
    alg = build(case, device, use_graphs=False)
    res = {}
    rollout(alg, case, 0, res, True, device)
    perm0 = torch.from_numpy(LC.permutation(case, 0)).to(device)
    alg._next_perm = lambda n: perm0
    alg.update_dagger()
    rollout(alg, case, 1, res, False, device)
    alg.total_updates = LC.TOTAL_UPDATES
    perm1 = torch.from_numpy(LC.permutation(case, 1)).to(device)
    alg._next_perm = lambda n: perm1
    n_mb = alg.num_learning_epochs * alg.num_mini_batches
    mb = perm1.numel() // alg.num_mini_batches
    dec_in = None
    if force:
        rows = []
        for k in range(n_mb):
            dk = d[f"mb{k}.decisions"].copy()
            if near_only:  # replay only the samples within NEAR_TIE of a boundary; the rest decide freely
                keep = np.zeros(dk.size, bool)
                keep[d[f"mb{k}.near"]] = True
                dk[~keep] = 0x40
            rows.append(torch.from_numpy(dk))
        dec_in = torch.stack(rows).to(device)
    dec_out = torch.zeros(n_mb, mb, dtype=torch.uint8, device=device)
    alg._decisions = {"k": 0, "in": dec_in, "out": dec_out}
    grads, norms = [], []
    inner = alg._minibatch_grads

    def wrapped(idx):
        inner(idx)
        g = alg.grads
        rec = {}
        for n, p in named_params(alg):
            if n.startswith("adaptation"):
                continue
            flat = p.grad.detach().reshape(-1)
            sel = torch.from_numpy(LC.sample_index(n, flat.numel(), LC.SAMPLE_MB)).to(device)
            f64 = flat.double()
            rec[n] = (_np(flat[sel]), float(f64.sum()), float((f64 * f64).sum()))
        grads.append(rec)
        est = g.segment("estimator").double().norm()
        main = torch.cat([g.segment("main"), g.segment("adaptation")]).double().norm()
        norms.append((float(est), float(main)))

    alg._minibatch_grads = wrapped
    alg.update()
    del alg._minibatch_grads
    assert alg._s8 is not None and alg._decisions["k"] == n_mb, "every minibatch ran on the S8 path"
    alg._decisions = None
    res["mbg"], res["norms"], res["dec_out"] = grads, norms, dec_out.cpu().numpy()
    res["after"] = {n: _np(p) for n, p in named_params(alg)}
    names_of = {id(p): n for n, p in named_params(alg)}
    res["exp_avg"], res["exp_avg_sq"] = {}, {}
    for oname in ("optimizer", "estimator_optimizer"):
        opt = getattr(alg, oname)
        for grp in opt.param_groups:
            for p in grp["params"]:
                st = opt.state[p]
                res["exp_avg"][names_of[id(p)]] = _np(st["exp_avg"])
                res["exp_avg_sq"][names_of[id(p)]] = _np(st["exp_avg_sq"])
    return res, alg
