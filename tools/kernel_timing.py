"""Time the env-step kernel under parameter variants (dev tool): solver iterations,
decimation, post-physics only. Prints avg µs per launch at N envs."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from legged_gym_custom_amd import _native  # noqa: E402
from legged_gym_custom_amd.envs import task_registry  # noqa: E402
from legged_gym_custom_amd.utils.helpers import get_args  # noqa: E402

N = int(os.environ.get("N", "4096"))
args = get_args(["--task=go2", "--headless", f"--num_envs={N}", "--sim_device=cuda:0", "--rl_device=cuda:0"])
env, _ = task_registry.make_env("go2", args)
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
for _ in range(20):
    env.step(torch.randn(N, 12, device="cuda", generator=g).clamp(-3, 3))
torch.cuda.synchronize()
stream = torch.cuda.current_stream().cuda_stream


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def variant(**kw):
    P = copy.copy(env.task_params)
    for k, v in kw.items():
        setattr(P, k, v)
    ne = _native.NativeEnv(env._native.model, P, 0)
    ne.bind(env._native._keep)
    return ne


base = env._native
cnt = [env.common_step_counter]


def run(ne, post=False):
    def f():
        cnt[0] += 1
        (ne.post_physics if post else ne.step)(1, cnt[0], stream)
    return f


print(f"N={N}")
print(f"full step (iters={env.task_params.solver_iterations}, decim 4): {timeit(run(base)):.1f} us")
for it in (0, 1, 4):
    print(f"solver_iterations={it}: {timeit(run(variant(solver_iterations=it))):.1f} us")
print(f"decimation=1: {timeit(run(variant(decimation=1))):.1f} us")
print(f"post-physics only: {timeit(run(base, post=True)):.1f} us")
cf = env.contact_forces.reshape(N, -1, 3).norm(dim=-1)
nb = (cf > 1e-6).sum(dim=1).float()
print("bodies in contact per env: mean %.2f p50 %.0f p90 %.0f max %.0f" % (
    nb.mean().item(), nb.median().item(), torch.quantile(nb, 0.9).item(), nb.max().item()))
