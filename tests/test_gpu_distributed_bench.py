"""The N>1 path as the driver runs it, rehearsed on ONE MI355X.

1. bench.py under `python -m torch.distributed.run --nproc-per-node 2` with LGX_DIST_BACKEND=gloo
   (two ranks on cuda:0: RCCL refuses two ranks on one device; the driver's 8-GPU run uses RCCL):
   init_process_group / device selection / barrier + max-over-ranks timing / rank-0 JSON line,
   the phased update graphs (the per-minibatch gradient all-reduce of ppo.py:273-276 between graph
   A and graph B) and the phased DAgger graphs (iteration 0).
2. update_dagger at world size 2 (phased graphs: graph A, the host all-reduce of the adaptation
   segment, graph B = mean + clip + Adam; ppo.py:309-349) replayed three times, both ranks on the
   same rows, against one process's eager update_dagger on those rows: an all-reduce of two equal
   fp32 gradients halved is exact, so the ranks must equal the single process bit for bit."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_gloo_line():
    env = dict(os.environ, LGX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("LGX_LIB", "LGX_MLP_LIB", "LGX_S8_LIB"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--no_cpu_baseline", "--kernel_iters", "5"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]  # rank 0 only
    d = json.loads(lines[0])
    print({k: d[k] for k in ("value", "ms_per_step", "n_gpus")}, d["paths"])
    assert d["n_gpus"] == 2 and d["config"]["global_envs"] == 8192
    assert d["value"] > 0 and d["value"] == d["value"] and d["value"] != float("inf")
    assert d["paths"]["graph_mode"] == "phased"
    assert d["paths"]["dagger"] == "fused" and d["paths"]["dagger_graph_mode"] == "phased"
    assert set(d["binaries"]) >= {"liblgx.so", "liblgx_mlp.so", "liblgx_s8.so"}
    assert all(b["path"].startswith("legged_gym_custom_amd/lib/") for b in d["binaries"].values())


def _dagger_run(use_graphs, n_calls):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_learner import _to_gpu
    from test_ppo_update import _fill, _make
    alg = _to_gpu(_make("adaptive"), use_graphs=use_graphs)
    alg._next_perm = lambda n: torch.arange(n, device="cuda:0")
    losses = []
    for it in range(n_calls):
        _fill(alg, 80 + it)
        losses.append(alg.update_dagger())
    torch.cuda.synchronize()
    a, b = alg.grads.slices[alg._segment_of["adaptation_optimizer"]]
    return {"losses": losses, "params": alg.params_buf[a:b].cpu().clone(), "m": alg.exp_avg[a:b].cpu().clone(),
            "v": alg.exp_avg_sq[a:b].cpu().clone(), "path": alg.dagger_path, "mode": alg.dagger_graph_mode}


def _dagger_worker(rank, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        out[rank] = _dagger_run(True, 3)
    finally:
        dist.destroy_process_group()


def test_dagger_phased_graphs_two_ranks_equal_single_process():
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_dagger_worker, args=(_port(), out), nprocs=2, join=True, start_method="spawn")
    ref = _dagger_run(False, 3)
    r0, r1 = out[0], out[1]
    assert r0["path"] == "fused" and r0["mode"] == "phased"
    for r in (r0, r1):
        assert r["losses"] == ref["losses"], (r["losses"], ref["losses"])
        for k in ("params", "m", "v"):
            assert torch.equal(r[k], ref[k]), k
