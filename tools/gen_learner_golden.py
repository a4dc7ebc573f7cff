#!/usr/bin/env python3
"""Learner golden-vector generator: runs the REFERENCE rsl_rl (read-only, imported from
/root/reference/rsl_rl in this container) on the deterministic inputs of
tests/learner_case.py and records its outputs as tests/golden/learner_<case>.npz.
Test infrastructure only: the reference code never travels; only the .npz data does.

Recorded per case (go2 and go2_parkour network shapes at N=64 envs; go2 at C2's 4096 envs;
T=24 steps):
  * state_dict key/shape list and the optimizers' param-group layout (meta JSON);
  * rollout A (adaptation mode) and B: per step PPO.act outputs (actions, values,
    log-probs, mean, sigma; ppo.py:129-153 / actor_critic.py:190-226) and the stored
    rewards after the time-out bootstrap (ppo.py:156-171);
  * compute_returns: returns and normalised advantages (rollout_storage.py:110-124);
  * update_dagger: the adaptation encoder after it, its Adam moments, the mean loss;
  * update: the pre-clip gradients of minibatch 0 (hooked at clip_grad_norm_), the
    parameters after minibatch 0's Adam steps (hooked at the optimizers' step), the Adam
    moments after epoch 0 (num_mini_batches steps), the returned losses, the learning rate,
    every parameter after the update and the Adam moments after it (sampled entries + fp64
    sum/sum-of-squares per tensor; learner_case.record).
Injected: the Normal sample (loc + scale * eps) and torch.randperm.

Usage:  python tools/gen_learner_golden.py  [case ...]
Run it with torch's default CPU thread count (no OMP_NUM_THREADS override): the CPU replay
test compares the first Adam step at atol 1e-7, and the CPU GEMMs' summation order follows the
thread count.
"""
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF_RSL = "/root/reference/rsl_rl"
sys.dont_write_bytecode = True
sys.path.insert(0, REF_RSL)
sys.path.append(os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = type("SummaryWriter", (), {"__init__": lambda self, *a, **k: None})
sys.modules["torch.utils.tensorboard"] = _tb

import rsl_rl  # noqa: E402
from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic  # noqa: E402
from rsl_rl.modules.support_networks import MlpEstimator  # noqa: E402

import learner_case as LC  # noqa: E402

assert os.path.realpath(rsl_rl.__file__).startswith(os.path.realpath(REF_RSL)), rsl_rl.__file__


class _Inject:
    """eps for Normal.sample and the permutation for torch.randperm."""
    eps = None
    perm = None


_orig_randperm = torch.randperm


def _sample(self, sample_shape=torch.Size()):
    with torch.no_grad():
        if _Inject.eps is None or tuple(self.loc.shape) != tuple(_Inject.eps.shape):
            return torch.normal(self.loc.expand(self._extended_shape(sample_shape)),
                                self.scale.expand(self._extended_shape(sample_shape)))
        return self.loc + self.scale * _Inject.eps


def _randperm(n, *a, **k):
    if _Inject.perm is not None and n == _Inject.perm.numel():
        return _Inject.perm.clone()
    return _orig_randperm(n, *a, **k)


torch.distributions.Normal.sample = _sample
torch.randperm = _randperm


def build(case):
    c = LC.CASES[case]
    torch.manual_seed(0)
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
              schedule=c["schedule"], desired_kl=c["desired_kl"], device="cpu")
    alg.init_storage(LC.n_envs(case), LC.T, [c["P"] * (c["H"] + 1)], [c["priv"]], [c["critic"]], [c["est"]], [c["scan"]],
                     [c["A"]])
    return alg


def rollout(alg, case, which, out, adaptation_mode):
    pre = f"roll{which}"
    sampled = LC.CASES[case].get("sampled_rollout", False)

    def put(key, arr):
        if sampled:  # (large case: sampled entries + fp64 sums, learner_case.record)
            prefix, name = key.rsplit(".", 1)
            LC.record(out, prefix, name, arr.numpy())
        else:
            out[key] = arr.numpy().copy()

    for t in range(LC.T):
        d = LC.rollout_inputs(case, which, t)
        x = {k: torch.from_numpy(v) for k, v in d.items()}
        _Inject.eps = x["eps"]
        alg.act(x["obs"], x["priv"], x["critic"], x["est"], x["scan"], adaptation_mode=adaptation_mode)
        tr = alg.transition
        put(f"{pre}.{t}.actions", tr.actions)
        put(f"{pre}.{t}.values", tr.values)
        put(f"{pre}.{t}.logp", tr.actions_log_prob)
        put(f"{pre}.{t}.mu", tr.action_mean)
        put(f"{pre}.{t}.sigma", tr.action_sigma)
        alg.process_env_step(x["rewards"], x["dones"], {"time_outs": x["time_outs"]})
        _Inject.eps = None
    s = alg.storage
    put(f"{pre}.rewards", s.rewards)
    alg.compute_returns(torch.from_numpy(LC.last_critic(case, which)))
    put(f"{pre}.returns", s.returns)
    put(f"{pre}.advantages", s.advantages)


def named_params(alg):
    ac, est = alg.actor_critic, alg.estimator
    return [(k, p) for k, p in ac.named_parameters()] + [("estimator." + k, p) for k, p in est.named_parameters()]


def adam_state(opt, names_of):
    """{param name: (exp_avg, exp_avg_sq, step)} of an optimizer."""
    res = {}
    for grp in opt.param_groups:
        for p in grp["params"]:
            st = opt.state.get(p, {})
            if "exp_avg" in st:
                res[names_of[id(p)]] = (st["exp_avg"].numpy(), st["exp_avg_sq"].numpy(), float(st["step"]))
    return res


class PerMinibatch:
    """Hooks on the reference update (ppo.py:182-293) recording every minibatch: torch.clamp
    (the ratio clamp, :252) and Tensor.clamp (v - target, :258) for the in-band bits, torch.max
    (:254 surrogate, :261 value loss) for the max weights, clip_grad_norm_ for the gradients and
    norms. Decisions are torch's gradient rules: max(x, y) gives x weight 1 / 0.5 / 0 for x > y,
    x == y, x < y; clamp passes the gradient on [min, max]."""

    def __init__(self, alg, names_of):
        self.alg, self.names_of = alg, names_of
        self.cur, self.mbs = {}, []

    def install(self):
        self._clip, self._max, self._clamp, self._tclamp = (nn.utils.clip_grad_norm_, torch.max, torch.clamp,
                                                            torch.Tensor.clamp)
        me = self

        def clip_hook(params, max_norm, *a, **k):
            params = list(params)
            est = all(me.names_of[id(p)].startswith("estimator.") for p in params)
            grads = {me.names_of[id(p)]: p.grad.detach().numpy().copy() for p in params if p.grad is not None}
            total = me._clip(params, max_norm, *a, **k)
            me.cur.setdefault("grads", {}).update(grads)
            me.cur["norm_est" if est else "norm_main"] = float(total)
            if not est:  # the minibatch's last hook call (ppo.py:275)
                me.mbs.append(me.cur)
                me.cur = {}
            return total

        def max_hook(*a, **k):
            if len(a) == 2 and isinstance(a[1], torch.Tensor) and a[0].dim() >= 1:
                x, y = a[0].detach(), a[1].detach()
                w = (x > y).to(torch.uint8) * 2 + (x == y).to(torch.uint8)
                rel = (x - y).abs() / torch.maximum(x.abs(), y.abs()).clamp_min(1e-30)
                key = "surr" if "surr_w" not in me.cur else "value"
                me.cur[key + "_w"] = w.reshape(-1).numpy().copy()
                me.cur[key + "_margin"] = torch.where(x == y, torch.ones_like(rel), rel).reshape(-1).numpy().copy()
            return me._max(*a, **k)

        def band(x, lo, hi):
            x = x.detach()
            inb = ((x >= lo) & (x <= hi)).reshape(-1).numpy().copy()
            scale = max(abs(lo), abs(hi))
            margin = (torch.minimum((x - lo).abs(), (x - hi).abs()) / scale).reshape(-1).numpy().copy()
            return inb, margin

        def clamp_hook(*a, **k):  # torch.clamp(ratio, 1 - clip, 1 + clip)
            if len(a) == 3 and not k and isinstance(a[1], float) and isinstance(a[2], float):
                me.cur["ratio_in"], me.cur["ratio_band"] = band(a[0], a[1], a[2])
            return me._clamp(*a, **k)

        def tclamp_hook(*a, **k):  # (value - target).clamp(-clip, clip)
            if len(a) == 3 and not k and isinstance(a[1], float) and isinstance(a[2], float):
                me.cur["value_in"], me.cur["value_band"] = band(a[0], a[1], a[2])
            return me._tclamp(*a, **k)

        nn.utils.clip_grad_norm_ = clip_hook
        torch.max = max_hook
        torch.clamp = clamp_hook
        torch.Tensor.clamp = tclamp_hook

    def remove(self):
        nn.utils.clip_grad_norm_, torch.max, torch.clamp, torch.Tensor.clamp = (self._clip, self._max, self._clamp,
                                                                                self._tclamp)

    def store(self, out):
        for k, m in enumerate(self.mbs):
            for n, g in m["grads"].items():
                if not n.startswith("adaptation"):
                    LC.record(out, f"mbg{k}", n, g, sample=LC.SAMPLE_MB)
            out[f"mb{k}.norms"] = np.array([m["norm_est"], m["norm_main"]], dtype=np.float64)
            dec = (m["surr_w"].astype(np.uint8) | (m["ratio_in"].astype(np.uint8) << 2) |
                   (m["value_w"].astype(np.uint8) << 3) | (m["value_in"].astype(np.uint8) << 5))
            out[f"mb{k}.decisions"] = dec
            # inside the value clip band both terms of the value max are the same number up to
            # rounding (v vs target + (v - target)) and give the same gradient: not a decision
            near = ((m["surr_margin"] < LC.NEAR_TIE) | (m["ratio_band"] < LC.NEAR_TIE) |
                    (m["value_band"] < LC.NEAR_TIE) | (~m["value_in"].astype(bool) &
                                                       (m["value_margin"] < LC.NEAR_TIE)))
            out[f"mb{k}.near"] = np.flatnonzero(near).astype(np.int32)


def main(cases):
    for case in cases:
        alg = build(case)
        out = {"case": np.array(case), "torch_version": np.array(torch.__version__), "N": LC.n_envs(case), "T": LC.T}
        names_of = {id(p): n for n, p in named_params(alg)}
        meta = {"state_dict": [[k, list(v.shape)] for k, v in alg.actor_critic.state_dict().items()],
                "estimator_state_dict": [[k, list(v.shape)] for k, v in alg.estimator.state_dict().items()],
                "optimizer_param_groups": [[names_of[id(p)] for p in g["params"]] for g in alg.optimizer.param_groups],
                "adaptation_optimizer": [names_of[id(p)] for p in alg.adaptation_optimizer.param_groups[0]["params"]],
                "estimator_optimizer": [names_of[id(p)] for p in alg.estimator_optimizer.param_groups[0]["params"]],
                "optimizer_hyper": {k: v for k, v in alg.optimizer.param_groups[0].items()
                                    if k != "params" and isinstance(v, (int, float, bool, tuple, type(None)))}}
        out["meta_json"] = np.array(json.dumps(meta))

        # ---- iteration 0: adaptation-mode rollout + DAgger (on_policy_runner.py:147, 182-183)
        rollout(alg, case, 0, out, adaptation_mode=True)
        _Inject.perm = torch.from_numpy(LC.permutation(case, 0))
        out["dagger.loss"] = np.float64(alg.update_dagger())
        _Inject.perm = None
        for n, p in named_params(alg):
            if n.startswith("adaptation_encoder_."):
                out[f"dagger.param.{n}"] = p.detach().numpy().copy()
                out[f"dagger.grad.{n}"] = p.grad.numpy().copy()  # stale: seen by the next PPO clip
        for n, (m, v, step) in adam_state(alg.adaptation_optimizer, names_of).items():
            out[f"dagger.exp_avg.{n}"] = m.copy()
            out[f"dagger.exp_avg_sq.{n}"] = v.copy()
            out["dagger.step"] = np.float64(step)

        # ---- iteration 1: rollout + PPO/ROA update
        rollout(alg, case, 1, out, adaptation_mode=False)
        alg.total_updates = LC.TOTAL_UPDATES
        grads0 = {}
        orig_clip = nn.utils.clip_grad_norm_

        def clip_hook(params, max_norm, *a, **k):
            # minibatch 0 calls it for the estimator, then for actor_critic.parameters()
            params = list(params)
            key = "est" if all(names_of[id(p)].startswith("estimator.") for p in params) else "main"
            first = key not in grads0
            if first:
                grads0[key] = {names_of[id(p)]: p.grad.detach().numpy().copy() for p in params
                               if p.grad is not None}
            total = orig_clip(params, max_norm, *a, **k)
            if first:
                grads0[key + "_norm"] = float(total)
            return total

        nn.utils.clip_grad_norm_ = clip_hook
        # the parameters after minibatch 0's optimizer steps (one Adam step each; ppo.py:228-231
        # for the estimator, :273-276 for the rest), and the Adam moments after epoch 0's last
        # minibatch (num_mini_batches steps: before the update's sensitivity to rounding builds up)
        mb0, e0, nsteps = {}, {}, {}

        def once(opt, key, oname):
            step = opt.step

            def wrapped(*a, **k):
                r = step(*a, **k)
                nsteps[key] = nsteps.get(key, 0) + 1
                if key not in mb0:
                    mb0[key] = {names_of[id(p)]: p.detach().numpy().copy() for g in opt.param_groups
                                for p in g["params"]}
                if nsteps[key] == alg.num_mini_batches:
                    e0[key] = {n: (m.copy(), v.copy()) for n, (m, v, _s) in adam_state(opt, names_of).items()}
                return r
            opt.step = wrapped

        once(alg.optimizer, "main", "optimizer")
        once(alg.estimator_optimizer, "est", "estimator_optimizer")
        # every minibatch (round 5): the pre-clip gradients (sampled + fp64 sums), both norms, the
        # surrogate / value losses and the per-sample discrete decisions (LC.DEC_* bits), with the
        # samples whose decision sits within LC.NEAR_TIE of its boundary
        per_mb = PerMinibatch(alg, names_of)
        per_mb.install()
        _Inject.perm = torch.from_numpy(LC.permutation(case, 1))
        mv, ms, mr, coef, me = alg.update()
        _Inject.perm = None
        per_mb.remove()
        nn.utils.clip_grad_norm_ = orig_clip
        del alg.optimizer.step, alg.estimator_optimizer.step
        per_mb.store(out)
        for key in ("main", "est"):
            for n, p in mb0[key].items():
                LC.record(out, "mb0", n, p)
            for n, (m, v) in e0[key].items():
                LC.record(out, "exp_avg_e0", n, m)
                LC.record(out, "exp_avg_sq_e0", n, v)
        out["update.losses"] = np.array([mv, ms, mr, coef, me], dtype=np.float64)
        out["update.learning_rate"] = np.float64(alg.learning_rate)
        out["update.grad_norm0"] = np.array([grads0["est_norm"], grads0["main_norm"]], dtype=np.float64)
        for key in ("est", "main"):
            for n, g in grads0[key].items():
                LC.record(out, "grad0", n, g)
        for n, p in named_params(alg):
            LC.record(out, "after", n, p.detach().numpy())
        steps = {}
        for oname in ("optimizer", "estimator_optimizer"):
            for n, (m, v, step) in adam_state(getattr(alg, oname), names_of).items():
                LC.record(out, "exp_avg", n, m)
                LC.record(out, "exp_avg_sq", n, v)
                steps[oname] = step
        out["update.steps"] = np.array([steps["optimizer"], steps["estimator_optimizer"]], dtype=np.float64)
        path = os.path.join(REPO, "tests", "golden", f"learner_{case}.npz")
        np.savez_compressed(path, **out)
        print(f"wrote {path}: losses {out['update.losses']}, lr {alg.learning_rate}, "
              f"{os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main(sys.argv[1:] or list(LC.CASES))
