"""Deterministic inputs of the learner fixtures (tests/golden/learner_<case>.npz).

Shared by tools/gen_learner_golden.py, which runs the REFERENCE rsl_rl
(/root/reference/rsl_rl: ActorCritic, MlpEstimator, PPO, RolloutStorage) on them, and by
tests/test_learner_golden.py / test_gpu_learner_golden.py, which run this build's PPO
on the same inputs. Everything is drawn from numpy PCG64 streams keyed by (case seed,
purpose), so the inputs are identical on every machine and never have to be stored:
the fixture holds only the reference's OUTPUTS.

Sequence recorded (the runner's first two iterations, on_policy_runner.py:143-186):
  rollout A  T steps of PPO.act(adaptation_mode=True) + process_env_step   (it 0, Q14)
  returns A  PPO.compute_returns(last critic obs)
  dagger     PPO.update_dagger()                                            (ppo.py:309-349)
  rollout B  T steps of PPO.act(adaptation_mode=False) + process_env_step
  returns B
  update     total_updates := TOTAL_UPDATES (ROA coefficient 0.025), PPO.update()  (ppo.py:182-293)
The Normal sample of act() is a + std * eps with eps injected (actor_critic.py:207), and
the minibatch permutation of each update is injected (rollout_storage.py:142).

Cases run at N=64 envs (384-row minibatches) except go2_c2: C2's exact shapes, N=4096, T=24,
so the update's minibatches are 24,576 rows as in the bench (rollout_storage.py:141) and the
HIP GEMMs take their production tile shapes, split-K picks and grids; and go2_parkour_c4: C4's,
N=8192 (49,152-row minibatches, the parkour estimator). Its per-step rollout
outputs are stored sampled (`record`) instead of whole (`sampled_rollout`).
Also recorded: the parameters after minibatch 0's optimizer steps (one Adam step each: the
tight parameter check) and the Adam moments after the update.
"""
import zlib

import numpy as np

N, T = 64, 24            # default envs per case (CASES[...]["N"] overrides), steps per rollout
TOTAL_UPDATES = 10000.0  # ppo.py:218-220: stage 0.5 of 5000..15000 -> coefficient 0.025
SAMPLE = 2048            # entries kept per large tensor (plus its fp64 sum / sum of squares)
SAMPLE_MB = 256          # per-minibatch gradients: entries kept per tensor
# a per-sample decision of the PPO head (ratio clip, surrogate / value max) whose two sides are
# within this relative margin: fp32 rounding of the log-prob (~1e-5 on a 3 x bf16 GEMM path) can
# put the sample on the other side (tools/ref_minibatch_ties.py)
NEAR_TIE = 3e-5
# decision byte (include/lgx_mlp.h lgx_heads_s8_args.decisions): surrogate max weight of the
# unclipped term x2 (bits 0-1), ratio in band (bit 2), value max weight x2 (bits 3-4), v - target
# in band (bit 5)

CASES = {
    # go2 network shapes (go2_config.py:180-200; estimator defaults support_networks.py:45) with
    # the base config's adaptive KL schedule (legged_robot_config.py:213) to cover it
    "go2": dict(seed=11, P=52, H=10, priv=29, critic=736, est=3, scan=132, A=12,
                actor=[512, 256, 128], critic_h=[512, 256, 128], priv_h=[64, 20], scan_h=[128, 64],
                est_h=[128, 64], latent=20, scan_out=32, lr=2e-4, est_lr=1e-3, schedule="adaptive",
                desired_kl=0.01, entropy=0.01, epochs=5, minibatches=4, gamma=0.99, lam=0.95, clip=0.2,
                max_grad_norm=1.0),
    # go2_parkour (go2_parkour_config.py:173-198)
    "go2_parkour": dict(seed=12, P=52, H=10, priv=29, critic=736, est=3, scan=132, A=12,
                        actor=[512, 256, 128], critic_h=[512, 256, 128], priv_h=[64, 20], scan_h=[128, 64],
                        est_h=[256, 128], latent=20, scan_out=32, lr=2e-4, est_lr=1e-4, schedule="fixed",
                        desired_kl=0.01, entropy=0.01, epochs=5, minibatches=4, gamma=0.99, lam=0.95, clip=0.2,
                        max_grad_norm=1.0),
    # C2: go2 at 4096 envs (24,576-row minibatches), the go2 train config's fixed schedule
    "go2_c2": dict(seed=13, N=4096, sampled_rollout=True, P=52, H=10, priv=29, critic=736, est=3, scan=132, A=12,
                   actor=[512, 256, 128], critic_h=[512, 256, 128], priv_h=[64, 20], scan_h=[128, 64],
                   est_h=[128, 64], latent=20, scan_out=32, lr=2e-4, est_lr=1e-3, schedule="fixed",
                   desired_kl=0.01, entropy=0.01, epochs=5, minibatches=4, gamma=0.99, lam=0.95, clip=0.2,
                   max_grad_norm=1.0),
    # C4: go2_parkour at 8192 envs (49,152-row minibatches, the [256, 128] estimator and the scan
    # encoder at their production shape; go2_parkour_config.py:229,242,256)
    "go2_parkour_c4": dict(seed=14, N=8192, sampled_rollout=True, P=52, H=10, priv=29, critic=736, est=3, scan=132,
                           A=12, actor=[512, 256, 128], critic_h=[512, 256, 128], priv_h=[64, 20], scan_h=[128, 64],
                           est_h=[256, 128], latent=20, scan_out=32, lr=2e-4, est_lr=1e-4, schedule="fixed",
                           desired_kl=0.01, entropy=0.01, epochs=5, minibatches=4, gamma=0.99, lam=0.95, clip=0.2,
                           max_grad_norm=1.0),
}
SMALL_CASES = [k for k, c in CASES.items() if c.get("N", N) <= 64]  # the CPU suite's cases


def n_envs(case):
    return CASES[case].get("N", N)


def _rng(case, *key):
    return np.random.default_rng([CASES[case]["seed"], *key])


def _key(name):
    return zlib.crc32(name.encode())


def weights(case, named_shapes):
    """{name: fp32 array} for every parameter: U(+-1/sqrt(fan_in)) like torch's Linear/Conv
    default bound, std U(0.7, 1.3) (so enforce_max_std clamps some entries)."""
    fan = {}
    for name, shape in named_shapes:
        if len(shape) >= 2:
            fan[name.rsplit(".", 1)[0]] = int(np.prod(shape[1:]))
    out = {}
    for name, shape in named_shapes:
        g = _rng(case, 1, _key(name))
        if name == "std":
            out[name] = g.uniform(0.7, 1.3, size=shape).astype(np.float32)
        else:
            b = 1.0 / np.sqrt(fan[name.rsplit(".", 1)[0]])
            out[name] = g.uniform(-b, b, size=shape).astype(np.float32)
    return out


def rollout_inputs(case, which, t):
    """Step t of rollout `which` (0 = A, 1 = B): observations, eps, rewards, dones, time_outs."""
    c = CASES[case]
    N = n_envs(case)
    g = _rng(case, 2, which, t)
    nobs = c["P"] * (c["H"] + 1)
    d = {
        "obs": g.standard_normal((N, nobs), dtype=np.float32),
        "priv": (0.5 * g.standard_normal((N, c["priv"]))).astype(np.float32),
        "critic": g.standard_normal((N, c["critic"]), dtype=np.float32),
        "est": (0.5 * g.standard_normal((N, c["est"]))).astype(np.float32),
        "scan": g.uniform(-1.0, 1.0, size=(N, c["scan"])).astype(np.float32),
        "eps": g.standard_normal((N, c["A"]), dtype=np.float32),
        "rewards": (0.5 * g.standard_normal(N)).astype(np.float32),
    }
    dones = g.random(N) < 0.08
    d["dones"] = dones
    d["time_outs"] = dones & (g.random(N) < 0.5)
    return d


def last_critic(case, which):
    c = CASES[case]
    return _rng(case, 3, which).standard_normal((n_envs(case), c["critic"]), dtype=np.float32)


def permutation(case, which):
    return _rng(case, 4, which).permutation(n_envs(case) * T).astype(np.int64)


def sample_index(name, size, sample=SAMPLE):
    """Fixed entry subset of a flattened tensor (all of it when small)."""
    if size <= sample:
        return np.arange(size, dtype=np.int64)
    return np.sort(np.random.default_rng([7, _key(name)]).choice(size, sample, replace=False)).astype(np.int64)


def record(out, prefix, name, arr, sample=SAMPLE):
    """Store a tensor's sampled entries and its full fp64 sum / sum of squares."""
    flat = np.asarray(arr, dtype=np.float32).reshape(-1)
    idx = sample_index(name, flat.size, sample)
    out[f"{prefix}.{name}.v"] = flat[idx]
    out[f"{prefix}.{name}.sum"] = np.float64(flat.astype(np.float64).sum())
    out[f"{prefix}.{name}.sumsq"] = np.float64((flat.astype(np.float64) ** 2).sum())


def compare(d, prefix, name, arr, rtol, atol, stat_rtol=None):
    """assert a tensor matches what `record` stored (sampled entries; sum/sumsq loosely)."""
    flat = np.asarray(arr, dtype=np.float32).reshape(-1)
    idx = sample_index(name, flat.size)
    np.testing.assert_allclose(flat[idx], d[f"{prefix}.{name}.v"], rtol=rtol, atol=atol, err_msg=f"{prefix}.{name}")
    if stat_rtol is not None:
        s2 = float((flat.astype(np.float64) ** 2).sum())
        ref2 = float(d[f"{prefix}.{name}.sumsq"])
        assert abs(s2 - ref2) <= stat_rtol * max(ref2, 1e-30) + 1e-12, (prefix, name, s2, ref2)
