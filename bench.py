#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: env-steps/sec (whole node), Go2 flat, 4096 envs per GPU.

One "step" = one rsl_rl learning iteration of the drop-in runner on synthetic Go2 flat
terrain: 24 env steps (policy act + fused HIP env step + storage + the per-step episode
bookkeeping train.py's runner does, on_policy_runner.py:160-170) + GAE + the PPO/ROA update
(5 epochs x 4 minibatches) — i.e. Perf/total_fps of on_policy_runner.py:219.
value = num_envs x 24 x world_size x K / (max over ranks of the timed K iterations), the MEDIAN
of 3 windows of K iterations each (`windows` lists all three, with the GPU shader clock read
after each); `value_no_episode_tracking` is one window of the same loop without the bookkeeping.
The windows avoid the runner's DAgger iterations (it % 20 == 0, on_policy_runner.py:147) when
W + K <= 18.

Also reported: `roofline` of the env-step kernel (algorithmic bytes per launch over its
HIP-event-timed duration vs 8 TB/s HBM; the kernel is not HBM-bound: `roofline_valu` gives
its VALU issue utilisation and wait fraction from the committed PMC profile), `roofline_learner`, and
`cpu_baseline`: the same framework on the host (--sim_device=cpu --rl_device=cpu: liblgx.so's
host backend, OpenMP over envs, + the torch-CPU learner) at the same shape (one iteration),
rank 0 at N=1 only.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--num_envs 4096]
  N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "env-steps/sec (whole node), Go2 4096 envs, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0


def env_bytes_per_env_step(P, num_bodies, ks):
    """Algorithmic HBM bytes one env moves per lgx_step (DESIGN.md 'Roofline'):
    every per-env row the kernel must read and write once (4-B words; int64 = 8 B;
    bool = 1 B)."""
    D, A, H, Pp = P.num_dof, P.num_actions, P.history_len, P.num_proprio
    f = 4
    rd = f * (A + 2 * D + 2 * D + D + 13 + 4 + 1 + 4 + 1 + 4 + A + D + 4 + ks + H * Pp) + 8 + 4
    wr = f * (A + num_bodies * 13 + num_bodies * 3 + D + ks + 1 + P.num_obs + P.num_critic + P.num_priv +
              P.num_est + P.num_scan + H * Pp + A + 2 * D + 2 * D + 6 + 3 + 9 + 13 + 4 + 4 + 4 + 8 +
              P.num_height_points) + 8 + 2 + 4
    return rd + wr


MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 (MI355X_MICROARCH.md); 3xbf16 = 3 MFMA products per fp32 MAC


def sclk_mhz():
    """The current shader clock (MHz) of the busiest GPU on this node, from the driver's sysfs
    DPM table (the line marked '*'); None where it cannot be read."""
    import glob
    best = None
    for f in glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk"):
        try:
            for line in open(f):
                if line.rstrip().endswith("*"):
                    mhz = int(line.split(":")[1].strip().lower().split("mhz")[0])
                    best = mhz if best is None else max(best, mhz)
        except (OSError, ValueError, IndexError):
            pass
    return best


def learner_gemm_roofline(dev, rows=24576, reps=10):
    """The update's weight-gradient group — every dW of one go2 minibatch backward in ONE
    lgx_s8_gemm_group launch on pre-split (S8) operands, plus its split-K reduction launch —
    timed with HIP events on its stream: MFMA rate = 3 bf16 products x 2 x rows x sum(in x out)
    / time; HBM = the operands (4 B per element, S8 as fp32) read once."""
    from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S
    layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (512, 256), (256, 128), (128, 1),
              (29, 64), (64, 20), (20, 20), (132, 128), (128, 64), (64, 32), (572, 128), (128, 64), (64, 3)]
    g = torch.Generator(device=dev).manual_seed(7)
    data = [(S.to_s8(torch.randn(rows, o, device=dev, generator=g)), S.to_s8(torch.randn(rows, i, device=dev, generator=g)),
             torch.zeros(o, i, device=dev)) for i, o in layers]
    splits = S.pick_split([(o, i, rows) for i, o in layers])
    ws = torch.empty(sum(s * i * o for s, (i, o) in zip(splits, layers)), device=dev)
    args, red, off = [], [], 0
    for (dy, x, dW), s, (i, o) in zip(data, splits, layers):
        w = ws.data_ptr() + 4 * off
        args.append(S.GemmArgs(A=dy.data_ptr(), lda=dy.shape[1], B=x.data_ptr(), ldb=x.shape[1], M=o, N=i, K=rows,
                               C32=w, ldc32=i, split=s))
        red.append(S.flat_reduce(w, o * i, dW.data_ptr(), o * i, s))
        off += s * o * i

    def once():
        S.gemm_group(args, S.DW)
        S.reduce(red)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            once()
    torch.cuda.current_stream(dev).wait_stream(side)
    graph = torch.cuda.CUDAGraph()  # replayed: device time only, no host launch gaps
    with torch.cuda.graph(graph):
        for _ in range(reps):
            once()
    stream = torch.cuda.current_stream(dev)
    # the median of 7 timed replays after 2 untimed ones: a single replay right after the
    # training loop read 360-366 us where the warm median reads 304 (tools/dw_cache_probe.py,
    # profiles/r03_dw_experiments.txt; the in-runner rocprofv3 average is 299 us)
    ts = []
    for i in range(9):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        s.record(stream)
        graph.replay()
        e.record(stream)
        torch.cuda.synchronize(dev)
        if i >= 2:
            ts.append(s.elapsed_time(e))
    t = sorted(ts)[len(ts) // 2] / reps * 1e-3
    flop = 2.0 * rows * sum(i * o for i, o in layers)
    achieved = 3 * flop / t / 1e12
    # algorithmic HBM bytes: every activation (X) and output gradient (dY) of the minibatch
    # read once (4 B per element: bf16 hi + lo), every dW written once
    nbytes = 4.0 * rows * sum(i + o for i, o in layers) + 4.0 * sum(i * o for i, o in layers)
    gbs = nbytes / t / 1e9
    # the binding roofline is the larger of the two ideal times (here HBM: 657 MB at 8 TB/s
    # = 82 us vs 168 bf16 GFLOP at 2.5 PF/s = 67 us)
    t_hbm, t_mfma = nbytes / (HBM_PEAK_GBS * 1e9), 3 * flop / (MFMA_BF16_PEAK_TFLOPS * 1e12)
    mfma = {"achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "fp32_equivalent_tflops": round(flop / t / 1e12, 1),
            "note": "3xbf16 split: 3 bf16 MFMA products per fp32 multiply-add"}
    hbm = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
           "algorithmic_bytes": int(nbytes)}
    top = dict(hbm if t_hbm >= t_mfma else mfma)
    top.pop("note", None)
    return {"bound": "hbm" if t_hbm >= t_mfma else "mfma",
            "kernel": "lgxs::s8_gemm_kernel<2, 2> + s8_reduce_kernel",
            "workload": f"all 17 weight gradients of one go2 minibatch ({rows} rows)", **top,
            "us_per_launch": round(t * 1e6, 1), "ideal_us": {"hbm": round(t_hbm * 1e6, 1), "mfma": round(t_mfma * 1e6, 1)},
            "hbm": hbm, "mfma": mfma}


def committed_traffic(num_envs):
    """Env-step kernel HBM bytes per launch from the newest committed PMC profile
    (profiles/<round>_env_traffic.json, made by tools/gpu/pmc_env.sh: FETCH_SIZE and
    WRITE_SIZE from separate --pmc passes, corrected by the dword-access calibration), when
    it was measured on this workload size."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_env_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    if "traffic_bytes_per_launch" not in d or f"{num_envs} envs" not in d.get("workload", ""):
        return None, None
    return d["traffic_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def committed_valu(num_envs):
    """VALU issue utilisation of the env-step kernel from the newest committed PMC profile
    (profiles/<round>_env_kernel_pmc.txt): on CDNA4 a wave64 VALU instruction issues over 2
    cycles (SIMD-32; MI355X_MICROARCH.md), so utilisation = 2 x SQ_INSTS_VALU / (1024 SIMDs x
    kernel cycles), kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs. Beside it the wait fraction
    (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and LDS instructions per env step: the kernel is
    latency-bound (LDS round trips of the LDS-resident per-env state, DPP/readlane chains)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_env_kernel_pmc.txt")))
    if not files:
        return None
    vals = {}
    kname = "lgx::env_step_kernel"
    for line in open(files[-1]):
        if "kernel void " in line:  # the header names the profiled instance
            kname = line.split("kernel void ", 1)[1].split("(", 1)[0].strip()
        f = line.split()
        if len(f) == 2 and f[0].isupper():
            try:
                vals[f[0]] = float(f[1])
            except ValueError:
                pass
    if not {"SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"} <= set(vals):
        return None
    cyc = vals["GRBM_GUI_ACTIVE"] / 8
    used = 2 * vals["SQ_INSTS_VALU"]
    cap = 1024 * cyc
    out = {"bound": "valu", "kernel": kname,
           "achieved": round(used / 1e6, 1), "peak": round(cap / 1e6, 1), "unit": "M VALU issue cycles per launch",
           "frac": round(used / cap, 4), "valu_instructions_per_env_step": round(vals["SQ_INSTS_VALU"] / num_envs),
           "source": os.path.relpath(files[-1], ROOT)}
    if {"SQ_WAIT_ANY", "SQ_WAVE_CYCLES"} <= set(vals):
        out["wait_fraction"] = round(vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"], 3)
    if "SQ_INSTS_LDS" in vals:
        out["lds_instructions_per_env_step"] = round(vals["SQ_INSTS_LDS"] / num_envs)
    out["note"] = ("VALU pipe partly busy; the waves wait on LDS / memory (wait_fraction) and on dependent "
                   "DPP / readlane chains: latency-bound (4096 envs fill one wave slot each: 2 waves per SIMD "
                   "at two envs per wavefront, DESIGN.md 4.1)")
    return out


LIB_OVERRIDES = ("LGX_LIB", "LGX_MLP_LIB", "LGX_S8_LIB")


def refuse_overrides():
    """The bench measures the in-tree product libraries only: a library-path override (dev builds)
    is refused, not recorded."""
    bad = [k for k in LIB_OVERRIDES if os.environ.get(k)]
    if bad:
        sys.exit(f"bench.py: refusing to run with library override(s) {bad}: the bench measures the in-tree "
                 f"legged_gym_custom_amd/lib/*.so only")


def loaded_binaries():
    """The native libraries this process actually mapped (from /proc/self/maps), each with its
    path and sha256: which binaries produced the line."""
    import hashlib
    paths = set()
    try:
        for line in open("/proc/self/maps"):
            f = line.split()
            if len(f) >= 6 and f[-1].endswith(".so") and "liblgx" in os.path.basename(f[-1]):
                paths.add(f[-1])
    except OSError:
        return None
    out = {}
    for pth in sorted(paths):
        h = hashlib.sha256()
        with open(pth, "rb") as fh:
            for chunk in iter(lambda: fh.read(1 << 20), b""):
                h.update(chunk)
        out[os.path.basename(pth)] = {"path": os.path.relpath(pth, ROOT) if pth.startswith(ROOT) else pth,
                                      "sha256": h.hexdigest()}
    return out


def cpu_baseline(num_envs=4096, iters=3, steps_per_env=24):
    """The same framework on the host: `--sim_device=cpu --rl_device=cpu` (helpers.py:174-177)
    — liblgx.so's host backend (OpenMP over envs) for the env step and the torch-CPU rsl_rl
    learner, through the same task registry and runner, at the benchmark's shape (C2: 4096 envs
    x 24 steps): a warm-up iteration, then `iters` timed PPO iterations, reported as the median
    (SURVEY.md §8d), on the host threads this process may use (OMP_NUM_THREADS: 16 per GPU on
    the GPU box, whose `nproc` counts the whole shared machine; both are recorded)."""
    from legged_gym_custom_amd.envs import task_registry
    from legged_gym_custom_amd.utils.helpers import get_args
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    a = get_args(["--task=go2", "--headless", f"--num_envs={num_envs}", "--sim_device=cpu", "--rl_device=cpu",
                  "--seed=1"])
    env, _ = task_registry.make_env("go2", a)
    _, tcfg = task_registry.get_cfgs("go2")
    tcfg.runner.num_steps_per_env = steps_per_env
    runner, _ = task_registry.make_alg_runner(env, args=a, train_cfg=tcfg, log_root=None)
    runner.learn(1, init_at_random_ep_len=True)  # warm-up (also a DAgger iteration: it=0)
    times, perfs = [], []
    for _ in range(iters):
        t0 = time.time()
        runner.learn(1)
        times.append(time.time() - t0)
        perfs.append(dict(runner.last_perf))
    order = sorted(range(iters), key=lambda i: times[i])
    mid = order[iters // 2]
    dt, perf = times[mid], perfs[mid]
    return {"value": round(num_envs * steps_per_env / dt, 1), "unit": "env-steps/s", "cores": threads,
            "nproc": os.cpu_count(), "kind": "port",
            "sample": f"median of {iters} PPO iterations of Go2 flat at {num_envs} envs x {steps_per_env} steps on "
                      f"the host (--sim_device=cpu --rl_device=cpu): liblgx.so host-backend env step (OpenMP) + "
                      f"torch-CPU learner, {threads} threads",
            "seconds": [round(t, 2) for t in times], "collection_s": round(perf.get("collection_time", 0.0), 3),
            "learn_s": round(perf.get("learn_time", 0.0), 3)}


def rollout_only(args, runner, env, dev, world, rank, barrier):
    """C3: ANYmal-C rough trimesh + height scan, the env step plus the actor /
    critic / encoder forward in privileged-latent mode, 24 steps per iteration as the runner's
    (graph-replayed) rollout; no update — the reference's ANYmal learner cannot run (its
    train config lacks the runner keys, Q16, and AdaptationEncoder needs history 10, Q17)."""
    steps = runner.num_steps_per_env
    runner._obs = [env.get_observations().to(dev), env.get_privileged_observations().to(dev),
                   env.get_critic_observations().to(dev), env.get_estimated_observations().to(dev),
                   env.get_scan_observations().to(dev)]

    def iters(n):
        for _ in range(n):
            with torch.inference_mode():
                runner._rollout(False, False)
            runner.alg.storage.clear()
            runner._capture_rollout(False)

    iters(args.warmup + 1)  # (the first eager rollout, then the capture)
    barrier()
    t0 = time.time()
    iters(args.steps)
    barrier()
    el = time.time() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    # env kernel alone (HIP events on the launch stream)
    stream = torch.cuda.current_stream(dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    n_k = args.kernel_iters
    acts = torch.randn(n_k, env.num_envs, env.num_actions, device=dev, generator=g)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_k)]
    for i in range(n_k):
        env.actions_in.copy_(acts[i])
        env.common_step_counter += 1
        evs[i][0].record(stream)
        env._native.step(env.seed, env.common_step_counter, stream.cuda_stream)
        evs[i][1].record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = sorted(a.elapsed_time(b) for a, b in evs)
    kern_avg = sum(kern_ms) / len(kern_ms)
    if rank == 0:
        total = args.num_envs * steps * world * args.steps
        print(json.dumps({
            "metric": f"env-steps/sec, {args.task} {args.num_envs} envs per GPU (env step + actor forward, "
                      f"privileged latent)", "value": round(total / el, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic ({args.task}: generated rough trimesh, random-init networks and SEA-LSTM weights, "
                    f"seed 1)",
            "config": {"workload": f"{args.task} rollout: {steps} x (act in privileged-latent mode + env step)",
                       "num_envs_per_gpu": args.num_envs, "num_steps_per_env": steps,
                       "global_envs": args.num_envs * world, "parallelism": f"env-sharded dp{world}"},
            "env_kernel": {"avg_us": round(kern_avg * 1e3, 2), "min_us": round(kern_ms[0] * 1e3, 2),
                           "env_steps_per_s": round(env.num_envs / (kern_avg * 1e-3), 1)}}))
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--num_envs", type=int, default=4096)
    ap.add_argument("--no_cpu_baseline", action="store_true")
    ap.add_argument("--kernel_iters", type=int, default=50)
    ap.add_argument("--task", default="go2", help="go2 (the BASELINE metric) | go2_parkour (C4) | anymal_c_rough "
                                                  "(C3: rollout only)")
    args = ap.parse_args()
    refuse_overrides()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LGX_DIST_BACKEND=gloo: rehearsal of the N>1 path with several ranks on one GPU
    # (correctness only; RCCL needs one GPU per rank)
    backend = os.environ.get("LGX_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    dev = f"cuda:{local}"
    # the reference's own training precision (legged_gym/scripts/train.py:39): fp32
    # storage, hipBLASLt's reduced-precision fp32 GEMM path allowed
    torch.set_float32_matmul_precision("high")

    from legged_gym_custom_amd import _abi
    from legged_gym_custom_amd.envs import task_registry
    from legged_gym_custom_amd.utils.helpers import get_args
    a = get_args([f"--task={args.task}", "--headless", f"--num_envs={args.num_envs}", f"--sim_device={dev}",
                  f"--rl_device={dev}", "--seed=1"])
    env_cfg = None
    if args.task.startswith("anymal"):
        # the reference's trained actuator archive does not ship with this build:
        # a synthetic SEA-LSTM archive of the same layout, written here
        import tempfile
        from legged_gym_custom_amd import actuator as act
        env_cfg, _ = task_registry.get_cfgs(args.task)
        sea = os.path.join(tempfile.mkdtemp(prefix="lgx_sea_"), "sea.pt")
        act.save_sea_archive(act.random_sea_weights(1, scale=0.3), sea)
        env_cfg.control.actuator_net_file = sea
    env, env_cfg = task_registry.make_env(args.task, a, env_cfg=env_cfg)
    _, train_cfg = task_registry.get_cfgs(args.task)
    runner, _ = task_registry.make_alg_runner(env, args=a, train_cfg=train_cfg, log_root=None)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def timed(track):
        """W warm-up + K timed iterations (barrier + synchronize both sides, max over ranks)."""
        runner.track_episodes = track
        runner.learn(num_learning_iterations=args.warmup, init_at_random_ep_len=True)
        barrier()
        t0 = time.time()
        runner.learn(num_learning_iterations=args.steps)
        barrier()
        el = time.time() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = t.item()
        return el, dict(runner.last_perf)

    if args.task.startswith("anymal"):
        return rollout_only(args, runner, env, dev, world, rank, barrier)
    elapsed_nt, perf_nt = timed(False)  # iterations 0..W-1 warm-up (0 is a DAgger iteration), then W..W+K-1
    # the headline, as train.py runs it: 3 windows, each W warm-up + K timed iterations starting
    # right after a DAgger iteration (it % 20 == 0, on_policy_runner.py:147), so none is inside
    steps_per_iter = train_cfg.runner.num_steps_per_env
    total_env_steps = args.num_envs * steps_per_iter * world * args.steps
    windows = []
    for w in range(3):
        runner.current_learning_iteration = 20 * (w + 1) + 1
        el_w, perf_w = timed(True)
        windows.append((el_w, perf_w, sclk_mhz()))
    order = sorted(range(3), key=lambda i: windows[i][0])
    elapsed, perf, _clk = windows[order[1]]
    value = total_env_steps / elapsed

    # ---- env-step kernel alone (HIP events on the launch stream) -> roofline
    g = torch.Generator(device=dev).manual_seed(1234)
    acts = torch.clamp(torch.randn(args.kernel_iters, env.num_envs, env.num_actions, device=dev, generator=g), -3.14, 3.14)
    for i in range(3):
        env.step(acts[i])
    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.kernel_iters)]
    env.actions_in.copy_(acts[0])
    for i in range(args.kernel_iters):
        env.actions_in.copy_(acts[i])
        env.common_step_counter += 1
        evs[i][0].record(stream)
        env._native.step(env.seed, env.common_step_counter, stream.cuda_stream)
        evs[i][1].record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = sorted(s.elapsed_time(e) for s, e in evs)
    kern_avg_ms = sum(kern_ms) / len(kern_ms)
    ks = len(env._episode_keys)
    bpe = env_bytes_per_env_step(env.task_params, env.num_bodies, ks)
    launch_bytes = bpe * env.num_envs
    achieved = launch_bytes / (kern_avg_ms * 1e-3) / 1e9
    traffic, traffic_src = committed_traffic(args.num_envs) if args.task == "go2" else (None, None)

    if rank == 0:
        terrain = env.cfg.terrain.mesh_type in ("heightfield", "trimesh")
        # two envs per wavefront (EPW 2) by default on the plane with an even env count (lgx_env.hip launch_step)
        actnet = bool(getattr(env.cfg.control, "use_actuator_network", False))
        epw = 2 if (env.num_envs % 2 == 0 and not actnet and not terrain) else 1
        kname = f"lgx::env_step_kernel<true, {'true' if terrain else 'false'}, {'true' if actnet else 'false'}, {epw}>"
        data = ("synthetic (Go2 flat terrain, random-init ActorCritic/estimator, seed 1)" if args.task == "go2" else
                f"synthetic ({args.task}: generated terrain, random-init ActorCritic/estimator, seed 1)")
        out = {
            "metric": METRIC if args.task == "go2" else f"env-steps/sec, {args.task} {args.num_envs} envs per GPU", "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": data,
            "config": {"workload": f"{args.task}, rsl_rl PPO/ROA iteration (24 env steps + 5x4 minibatch update)",
                       "num_envs_per_gpu": args.num_envs, "num_steps_per_env": steps_per_iter,
                       "global_envs": args.num_envs * world, "parallelism": f"env-sharded dp{world}"},
            "value_no_episode_tracking": round(total_env_steps / elapsed_nt, 1),
            "windows": [{"value": round(total_env_steps / el, 1), "ms_per_step": round(el / args.steps * 1e3, 3),
                         "sclk_mhz": clk} for el, _p, clk in windows],
            "window_spread": round((max(w[0] for w in windows) - min(w[0] for w in windows)) / elapsed, 4),
            # which code paths the timed iterations ran (no silent fallback: ppo.py / s8_*.py raise
            # on a missing library; these say which of the built paths were selected)
            "paths": {"learner": "s8" if runner.alg._s8 is not None else "autograd",
                      "act": "fused" if runner.alg._s8act is not None else "grouped",
                      "graph_mode": runner.alg.graph_mode,
                      "dagger": runner.alg.dagger_path, "dagger_graph_mode": runner.alg.dagger_graph_mode,
                      "rollout_graphs": sorted(str(k) for k in runner._graphs)},
            # the native libraries that ran (mapped by this process) and any LGX_* variables set
            "binaries": loaded_binaries(),
            "env_overrides": {k: v for k, v in sorted(os.environ.items()) if k.startswith("LGX_")},
            "collection_s": round(perf.get("collection_time", 0.0), 4),
            "learn_s": round(perf.get("learn_time", 0.0), 4),
            "env_kernel": {"avg_us": round(kern_avg_ms * 1e3, 2), "min_us": round(kern_ms[0] * 1e3, 2),
                           "env_steps_per_s": round(env.num_envs / (kern_avg_ms * 1e-3), 1)},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "bytes_per_env_step": bpe, "bytes_per_launch": launch_bytes,
                         "traffic": None if traffic is None else round(traffic), "traffic_source": traffic_src,
                         "note": "the kernel's algorithmic bytes vs HBM peak, as north_star asks; it is bound by "
                                 "per-env latency (LDS round trips, dependent lane exchanges), not HBM (roofline_valu, "
                                 "DESIGN.md 4.1)"},
        }
        if args.task == "go2" and args.num_envs == 4096:
            out["roofline_valu"] = committed_valu(args.num_envs)
        if args.task == "go2":
            out["roofline_learner"] = learner_gemm_roofline(dev)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
