"""lgx_s8_chain on the go2 update's encoder chains (scan 132-128-64-32, privileged 29-64-20,
24,576 rows): HIP-event time per launch, the product library and build variants interleaved,
against the same layers as three grouped levels (dev tool).
Usage: PYTHONPATH=.:tests:tools python tools/chain_bench.py [variant.so ...]"""
import json
import sys

import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S
from s8_bench import timeit_many

dev = "cuda:0"
PACKED = 1


def main(rows=24576):
    g = torch.Generator(device="cpu").manual_seed(0)
    keep, chains, levels, rowW = [], [], [[], [], []], []
    for w in ([132, 128, 64, 32], [29, 64, 20]):
        x = S.to_s8_torch(torch.randn(rows, w[0], generator=g).to(dev))
        c = S.ChainArgs(A=x.data_ptr(), lda=x.shape[1], rows=rows, nlayers=len(w) - 1)
        A, lda = x, x.shape[1]
        keep.append(x)
        for l, (k, n) in enumerate(zip(w[:-1], w[1:])):
            W = (torch.randn(n, k, generator=g) * 0.2).to(dev)
            Ws, Wp = S.to_s8_torch(W), S.packed_empty(n, k, dev)
            S.split([S.split_packed_job(W, Wp)])
            b = torch.randn(n, generator=g).to(dev)
            out = S.empty(rows, n, dev)
            keep += [Ws, Wp, b, out]
            L = c.layers[l]
            L.W, L.ldw, L.bias, L.K, L.N, L.elu = Ws.data_ptr(), Ws.shape[1], b.data_ptr(), k, n, 1
            L.C, L.ldc = out.data_ptr(), out.shape[1]
            rowW.append((L, Ws.data_ptr()))
            if PACKED:
                L.W, L.packed = Wp.data_ptr(), 1
            levels[l].append(S.GemmArgs(A=A.data_ptr(), lda=lda, B=Ws.data_ptr(), ldb=Ws.shape[1], M=rows, N=n, K=k,
                                        epilogue=S.EPI_BIAS | S.EPI_ELU, C=out.data_ptr(), ldc=out.shape[1],
                                        bias=b.data_ptr()))
            A, lda = out, out.shape[1]
        chains.append(c)
    libs = {"product": S.lib()}
    for v in sys.argv[1:]:
        libs[v.split("/")[-1]] = S.load(v)
    fns = {k: (lambda L=L: S.chain(chains, L)) for k, L in libs.items()}
    fns["levels"] = lambda: [S.gemm_group(lv, S.FWD) for lv in levels if lv]
    print(json.dumps(timeit_many(fns, n=20, rounds=5)))
    for L, w in rowW:  # the same chains on row-layout weights
        L.W, L.packed = w, 0
    print("row-layout weights", json.dumps(timeit_many({"product": lambda: S.chain(chains)}, n=20, rounds=3)))


if __name__ == "__main__":
    main()
