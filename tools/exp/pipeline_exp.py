"""EXPERIMENT: does splitting the rollout's 4096 envs into two halves on two streams (the
policy GEMMs of one half overlapping the env kernel of the other) shorten a rollout step?
Two separate 2048-env go2 envs stand in for the halves; one runner's networks drive both.
Each schedule is captured as a 24-step CUDA graph and replayed (HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

torch.set_float32_matmul_precision("high")
from legged_gym_custom_amd import _abi  # noqa: E402,F401
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402


def make(n):
    a = get_args(["--task=go2", "--headless", f"--num_envs={n}", "--sim_device=cuda:0", "--rl_device=cuda:0",
                  "--seed=1"])
    env, _ = task_registry.make_env("go2", a)
    return env, a


envF, a = make(4096)
_, tcfg = task_registry.get_cfgs("go2")
runner, _ = task_registry.make_alg_runner(envF, args=a, train_cfg=tcfg, log_root=None)
ac, est = runner.alg.actor_critic, runner.alg.estimator
envA, _ = make(2048)
envB, _ = make(2048)


def policy(env):
    obs, priv, crit, scan = env.obs_buf, env.privileged_obs_buf, env.critic_obs_buf, env.scan_obs_buf
    e, s, lat = H.forward_group([est.group_item(obs), ac.scan_encoder.group_item(scan),
                                 ac.privileged_encoder_.group_item(priv)])
    mean, v = H.forward_group([(ac.actor, (obs, lat, s, e)), (ac.critic, crit)])
    env.actions_in.copy_(torch.clamp(mean, -1.0, 1.0))


def seq():
    for _ in range(24):
        policy(envF)
        envF.step(envF.actions_in)


s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
EVS = [(torch.cuda.Event(), torch.cuda.Event()) for _ in range(24)]  # alive across the capture


def pipe():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    eA = eB = None
    for k in range(24):
        with torch.cuda.stream(s1):
            policy(envA)
            if eB is not None:
                s1.wait_event(eB)
            envA.step(envA.actions_in)
            nA = EVS[k][0]
            nA.record(s1)
        with torch.cuda.stream(s2):
            policy(envB)
            if eA is not None:
                s2.wait_event(eA)
            envB.step(envB.actions_in)
            nB = EVS[k][1]
            nB.record(s2)
        eA, eB = nA, nB
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def pipe_simple():
    cur = torch.cuda.current_stream()
    for k in range(24):
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            policy(envA)
            envA.step(envA.actions_in)
        with torch.cuda.stream(s2):
            policy(envB)
            envB.step(envB.actions_in)
        cur.wait_stream(s1)
        cur.wait_stream(s2)


def pair(f1, f2):
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        f1()
    with torch.cuda.stream(s2):
        f2()
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def pipe_phased():
    """phases [env_A(k) | policy_B(k)], [env_B(k) | policy_A(k+1)], fork/join each"""
    policy(envA)
    for k in range(24):
        pair(lambda: envA.step(envA.actions_in), lambda: policy(envB))
        pair(lambda: envB.step(envB.actions_in), (lambda: policy(envA)) if k < 23 else (lambda: None))


def capture(fn):
    with torch.inference_mode():
        fn()  # warm
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.inference_mode(False), torch.no_grad(), torch.cuda.graph(g):
            fn()
    return g


def t(g, it=10):
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it / 24 * 1e3


def te(fn, it=5):
    with torch.inference_mode():
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(it):
            fn()
        e.record()
        torch.cuda.synchronize()
    return s.elapsed_time(e) / it / 24 * 1e3


for _ in range(2):
    print(f"EAGER: one batch {te(seq):.1f} us, halves w/ events {te(pipe):.1f} us, phased {te(pipe_phased):.1f} us",
          flush=True)
gs = capture(seq)
print(f"rollout step, 4096 envs as one batch: {t(gs):.1f} us", flush=True)
gq = capture(pipe_simple)
print(f"per-step fork/join halves: {t(gq):.1f} us", flush=True)
gp = capture(pipe_phased)
for _ in range(2):
    print(f"rollout step, 4096 envs: one batch {t(gs):.1f} us, two 2048-env halves phased on two streams "
          f"{t(gp):.1f} us", flush=True)
