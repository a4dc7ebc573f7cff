"""Per-phase cycle counts of the env-step kernel (dev tool).

`python tools/phase_clock.py --build` (CPU container) compiles lib/liblgx_prof.so with
-DLGX_PHASE_CLOCK; on the GPU box `python tools/phase_clock.py` runs the Go2 bench
workload through it and prints, per phase, the mean/p50/p90 s_memtime cycles one env's
wave spends there (summed over the 4 substeps), and the share of the wave's total.
Env vars: TASK (go2), N (4096), K (10 timed steps), STATE=crowded (tilted robots at the ground
before every step: many contacts)."""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "legged_gym_custom_amd", "lib")
PROF = os.environ.get("PROF_LIB") or os.path.join(LIBDIR, "liblgx_prof.so")
sys.path.insert(0, ROOT)
PHASES = ["load", "pd", "kinematics", "dynamics", "free_vel", "detect+rows", "row_solves", "A_build", "pgs",
          "u_update", "forces+integrate", "final_kin+writes", "uniforms", "post_scalar", "heights+rewards",
          "reset+obs+writes"]


def build():
    from legged_gym_custom_amd import build_native
    build_native.build_env_variant(PROF, ["-DLGX_PHASE_CLOCK"] + os.environ.get("EXTRA", "").split())


def run():
    os.environ["LGX_LIB"] = PROF
    sys.path.insert(0, ROOT)
    import torch
    from legged_gym_custom_amd import _native
    from legged_gym_custom_amd.envs import task_registry
    from legged_gym_custom_amd.utils.helpers import get_args
    task = os.environ.get("TASK", "go2")
    n = int(os.environ.get("N", "4096"))
    k = int(os.environ.get("K", "10"))
    a = get_args([f"--task={task}", "--headless", f"--num_envs={n}", "--sim_device=cuda:0", "--rl_device=cuda:0",
                  "--seed=1"])
    env_cfg, _ = task_registry.get_cfgs(task)
    if task.startswith("anymal"):
        import tempfile
        from legged_gym_custom_amd import actuator as act
        path = os.path.join(tempfile.mkdtemp(), "sea.pt")
        act.save_sea_archive(act.random_sea_weights(1, scale=0.3), path)
        env_cfg.control.actuator_net_file = path
    env, _ = task_registry.make_env(task, a, env_cfg)
    L = _native.lib()
    L.lgx_debug_phase_buffer.argtypes = [C.c_void_p]
    buf = torch.zeros(n, 20, dtype=torch.int32, device="cuda:0")
    g = torch.Generator(device="cuda:0").manual_seed(1234)
    stream = torch.cuda.current_stream()
    acc = torch.zeros(n, 20, dtype=torch.float64, device="cuda:0")
    rows = []
    per_step = []
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = 0.0
    for i in range(20 + k):
        if i == 20:
            assert L.lgx_debug_phase_buffer(C.c_void_p(buf.data_ptr())) == 0
        env.actions_in.copy_(torch.clamp(torch.randn(n, env.num_actions, device="cuda:0", generator=g), -3.14, 3.14))
        if os.environ.get("STATE") in ("crowded", "tilted"):  # tilted robots at the ground (many contacts)
            ax = torch.randn(n, 3, device="cuda:0", generator=g)
            ax[:, 2] *= 0.2
            ax /= ax.norm(dim=1, keepdim=True)
            ang = 0.2 + 1.2 * torch.rand(n, device="cuda:0", generator=g)
            env.root_states[:, 3:6] = ax * torch.sin(ang / 2)[:, None]
            env.root_states[:, 6] = torch.cos(ang / 2)
            z0, z1 = (0.06, 0.16) if os.environ["STATE"] == "crowded" else (0.13, 0.19)
            env.root_states[:, 2] = z0 + (z1 - z0) * torch.rand(n, device="cuda:0", generator=g)
            env.root_states[:, 7:13] = 0.2 * torch.randn(n, 6, device="cuda:0", generator=g)
        env.common_step_counter += 1
        if i >= 20:
            s.record()
        env._native.step(env.seed, env.common_step_counter, stream.cuda_stream)
        if i >= 20:
            e.record()
            torch.cuda.synchronize()
            ms += s.elapsed_time(e)
            cyc = buf.double().remainder(2 ** 32)
            acc[:, :18] += cyc[:, :18]
            rows.append(buf[:, 16].clone())
            wt = cyc[:, :16].sum(dim=1)
            j = int(wt.argmax())
            per_step.append((s.elapsed_time(e) * 1e3, float(wt.median()), float(wt.max()), int(buf[j, 16]),
                             int(buf[j, 17]), float(torch.quantile(wt, 0.999))))
    # the last step's slowest waves against the median: phases and where they ran
    last = buf.double().remainder(2 ** 32)
    wt = last[:, :16].sum(dim=1)
    order = torch.argsort(wt)
    med = order[n // 2]
    hw = buf[:, 18].long() & 0xffffffff
    xcc = buf[:, 19].long() & 0xf

    def where(i):
        h = int(hw[i])
        return f"xcc {int(xcc[i])} se {(h >> 13) & 7} cu {(h >> 8) & 15} simd {(h >> 4) & 3} wave {h & 15}"
    print("last step, slowest envs vs the median env (cycles per phase):")
    print("  median env", int(med), where(int(med)), " ".join(f"{PHASES[j]}={int(last[med, j])}" for j in range(16)))
    for i in order[-6:].tolist():
        print("  env", i, where(i), f"total {int(wt[i])}:", " ".join(f"{PHASES[j]}={int(last[i, j])}" for j in range(16)))
    import collections
    slow = order[-max(1, n // 100):].tolist()
    print("  slowest 1 % by xcc:", dict(collections.Counter(int(xcc[i]) for i in slow)),
          "by simd:", dict(collections.Counter((int(hw[i]) >> 4) & 3 for i in slow)),
          "by wave slot:", dict(collections.Counter(int(hw[i]) & 15 for i in slow)))
    acc /= k
    tot = acc[:, :16].sum(dim=1)
    r = torch.stack(rows).float()
    print("constraint rows per env step (max over substeps): mean %.1f p50 %.0f p90 %.0f p99 %.0f max %.0f; "
          "wide-path (> AMAX rows) substeps: %.2f %%" % (r.mean(), r.median(), torch.quantile(r, 0.9),
                                                         torch.quantile(r, 0.99), r.max(), acc[:, 17].mean() / 4 * 100))
    print("per step: kernel us | wave cycles p50 / p99.9 / max | slowest env: rows, wide substeps")
    for us, med, p999, mx, rw, wide in [(a_, b_, f_, c_, d_, e_) for a_, b_, c_, d_, e_, f_ in per_step]:
        print(f"  {us:7.1f} | {med:8.0f} {p999:8.0f} {mx:8.0f} | {rw:3d} {wide:2d}")
    print(f"task {task} N={n}: kernel {ms / k * 1e3:.1f} us/launch; wave total cycles mean {tot.mean():.0f} "
          f"p50 {tot.median():.0f} p90 {torch.quantile(tot, 0.9):.0f} (s_memtime clock)")
    print(f"{'phase':18s} {'mean':>9s} {'p50':>9s} {'p90':>9s} {'share':>6s}")
    for j, name in enumerate(PHASES):
        c = acc[:, j]
        print(f"{name:18s} {c.mean():9.0f} {c.median():9.0f} {torch.quantile(c, 0.9):9.0f} {c.mean() / tot.mean():6.1%}")


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    else:
        run()
