"""Env-step kernel time vs env count on one GPU (dev tool): 1024 .. 8192 envs = 1 .. 8 waves
per SIMD (one residency round up to 4096). python tools/env_scaling.py
NS="4096" restricts the env counts; LGX_LIB=<path> times another build of liblgx.so."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

for n in [int(x) for x in os.environ.get("NS", "1024 2048 3072 4096 6144 8192").split()]:
    a = get_args(["--task=go2", "--headless", f"--num_envs={n}", "--sim_device=cuda:0", "--rl_device=cuda:0",
                  "--seed=1"])
    env, _ = task_registry.make_env("go2", a)
    g = torch.Generator(device="cuda:0").manual_seed(1234)
    K = int(os.environ.get("K", "30"))
    acts = torch.clamp(torch.randn(K + 5, n, 12, device="cuda:0", generator=g), -3.14, 3.14)
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for i in range(K + 5):
        env.actions_in.copy_(acts[i])
        env.common_step_counter += 1
        if i >= 5:
            ev[i - 5][0].record(st)
        env._native.step(env.seed, env.common_step_counter, st.cuda_stream)
        if i >= 5:
            ev[i - 5][1].record(st)
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) * 1e3 for s, e in ev)
    print(f"N={n:5d} waves/SIMD={n / 1024:.0f}: median {ts[len(ts) // 2]:7.1f} us  min {ts[0]:7.1f} us  "
          f"per env {ts[len(ts) // 2] / n * 1e3:6.1f} ns", flush=True)
    del env
