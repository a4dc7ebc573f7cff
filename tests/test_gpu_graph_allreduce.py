"""The world-size > 1 update with its gradient all-reduce RECORDED in the one update hipGraph
(RCCL: the "nccl" backend), on ONE GPU: a world-size-1 RCCL group with the distributed path
forced on (PPO.allreduce_always), so every minibatch runs the all-reduce of [main | estimator |
kl] between its backward and its optimizer tail (ppo.py:273-276) — eagerly in one run, inside the
captured graph in the other. Graph == eager, bit for bit, over three updates; with
LGX_GRAPH_ALLREDUCE=1 the graph mode is "whole" (no per-minibatch replays around host-issued
collectives; without it, the default, "phased")."""
import os
import queue
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, out):
    sys.path.insert(0, HERE)
    # the in-graph collective is opt-in (LGX_GRAPH_ALLREDUCE; phased graphs are the default at
    # world size > 1): set before the learner is imported in this spawned process
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LGX_GRAPH_ALLREDUCE="1")
    import torch.distributed as dist
    import learner_case as LC
    import learner_replay as R
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    res = {}
    try:
        for graphs in (False, True):
            alg = R.build("go2", "cuda:0", use_graphs=graphs)
            alg.allreduce_always = True
            perm = torch.from_numpy(LC.permutation("go2", 1)).to("cuda:0")
            alg._next_perm = lambda n, p=perm: p
            scratch = {}
            for _ in range(3):
                R.rollout(alg, "go2", 1, scratch, False, "cuda:0")
                alg.total_updates = LC.TOTAL_UPDATES
                alg.update()
            torch.cuda.synchronize()
            res[graphs] = (torch.cat([p.detach().reshape(-1) for _n, p in R.named_params(alg)]).cpu(),
                           alg.graph_mode, float(alg._lr64))
    finally:
        dist.destroy_process_group()
    out.put({k: (v[0].numpy(), v[1], v[2]) for k, v in res.items()})


def test_update_graph_records_the_rccl_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, _port(), q))
    p.start()
    res = None
    for _ in range(320):  # the child reports or dies; never wait on a dead one
        try:
            res = q.get(timeout=0.5)
            break
        except queue.Empty:
            if not p.is_alive():
                break
    p.join(timeout=60)
    assert res is not None and p.exitcode == 0, p.exitcode
    (w_eager, mode_eager, lr_eager), (w_graph, mode_graph, lr_graph) = res[False], res[True]
    assert mode_graph == "whole", mode_graph
    assert lr_graph == lr_eager
    assert (w_graph == w_eager).all()
