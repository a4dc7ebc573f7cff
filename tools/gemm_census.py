"""Every learner/rollout GEMM launch of one runner iteration with its shapes and HIP-event
time (dev tool; eager mode, so launch gaps are not representative — the kernel times are).
python tools/gemm_census.py [task] [num_envs]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "go2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    torch.set_float32_matmul_precision("high")
    from legged_gym_custom_amd import _abi  # noqa: F401
    from legged_gym_custom_amd.envs import task_registry
    from legged_gym_custom_amd.utils.helpers import get_args
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
    a = get_args([f"--task={task}", "--headless", f"--num_envs={n}", "--sim_device=cuda:0", "--rl_device=cuda:0",
                  "--seed=1"])
    env, _ = task_registry.make_env(task, a)
    _, tcfg = task_registry.get_cfgs(task)
    runner, _ = task_registry.make_alg_runner(env, args=a, train_cfg=tcfg, log_root=None)
    runner.use_graphs = False
    runner.alg.use_graphs = False
    rec = []
    on = [False]
    orig_group, orig_run = H.run_group, H._run

    def desc(g):
        return (g.M, g.N, g.K, g.a_kcontig, g.b_kcontig, g.split_k)

    def run_group(args):
        if not on[0]:
            return orig_group(args)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        orig_group(args)
        e.record()
        rec.append(("group", tuple(desc(g) for g in args), s, e))

    def run(args):
        if not on[0]:
            return orig_run(args)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        orig_run(args)
        e.record()
        rec.append(("single", (desc(args),), s, e))

    H.run_group, H._run = run_group, run
    runner.learn(2, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    on[0] = True
    runner.learn(1)
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for kind, d, s, e in rec:
        k = (kind, d)
        agg[k][0] += 1
        agg[k][1] += s.elapsed_time(e) * 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"{len(rec)} GEMM launches, {tot / 1e3:.2f} ms (HIP events, eager)")
    for (kind, d), (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        fl = sum(2 * m * nn * kk for (m, nn, kk, *_r) in d) * 3
        print(f"{us / 1e3:7.3f} ms {c:4d} x {us / c:7.1f} us {fl / (us / c) / 1e6:6.0f} TF-bf16 {kind:6s} "
              + " ".join(f"{m}x{nn}x{kk}{'' if ak else 'a'}{'' if bk else 'b'}{f'/s{sp}' if sp > 1 else ''}"
                         for (m, nn, kk, ak, bk, sp) in d))


if __name__ == "__main__":
    main()
