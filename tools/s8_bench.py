"""S8 GEMM core vs the fp32-operand GEMMs (lgx_mlp) on the go2 update shapes (24,576 rows):
the weight-gradient group of all 17 layers, and the forward / input-gradient launches per
depth. HIP-event averages over back-to-back launches (median of rounds) — dev tool.
--variants a.so b.so ...: build variants of liblgx_s8 timed in the same process (interleaved)."""
import argparse
import json
import statistics

import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S

CHAINS = {  # go2: (in, out) per layer
    "actor": [(627, 512), (512, 256), (256, 128), (128, 12)],
    "critic": [(736, 512), (512, 256), (256, 128), (128, 1)],
    "est": [(572, 128), (128, 64), (64, 3)],
    "scan": [(132, 128), (128, 64), (64, 32)],
    "priv": [(29, 64), (64, 20), (20, 20)],
}


def timeit_many(fns, n=20, rounds=5):
    """{name: (median, min)} with the variants interleaved per round (one process, one device)."""
    for fn in fns.values():
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    res = {k: [] for k in fns}
    for _ in range(rounds):
        for k, fn in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(n):
                fn()
            b.record()
            b.synchronize()
            res[k].append(a.elapsed_time(b) * 1000 / n)
    return {k: (round(statistics.median(v), 2), round(min(v), 2)) for k, v in res.items()}


def timeit(fn, n=20, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            fn()
        b.record()
        b.synchronize()
        res.append(a.elapsed_time(b) * 1000 / n)
    return statistics.median(res), min(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=24576)
    ap.add_argument("--out", default=None)
    ap.add_argument("--variants", nargs="*", default=[])
    a = ap.parse_args()
    dev = "cuda:0"
    R = a.rows
    g = torch.Generator(device="cpu").manual_seed(0)
    layers = [(c, i, fi, fo) for c, ls in CHAINS.items() for i, (fi, fo) in enumerate(ls)]
    X = {(c, i): torch.randn(R, fi, generator=g).to(dev) for c, i, fi, fo in layers}
    DY = {(c, i): torch.randn(R, fo, generator=g).to(dev) * 0.01 for c, i, fi, fo in layers}
    W = {(c, i): (torch.randn(fo, fi, generator=g) * 0.05).to(dev) for c, i, fi, fo in layers}
    Bs = {(c, i): torch.randn(fo, generator=g).to(dev) for c, i, fi, fo in layers}
    Xs = {k: S.to_s8(v) for k, v in X.items()}
    DYs = {k: S.to_s8(v) for k, v in DY.items()}
    Ws = {k: S.to_s8(v) for k, v in W.items()}
    torch.cuda.synchronize()
    out = {}

    # ---- weight-gradient group
    shapes = [(fo, fi, R) for c, i, fi, fo in layers]
    splits = S.pick_split(shapes)
    ws = [torch.empty(s, fo, fi, device=dev) for s, (fo, fi, _r) in zip(splits, shapes)]
    dW = [torch.zeros(fo, fi, device=dev) for (fo, fi, _r) in shapes]
    dargs = [S.GemmArgs(A=DYs[(c, i)].data_ptr(), lda=DYs[(c, i)].shape[1], B=Xs[(c, i)].data_ptr(),
                        ldb=Xs[(c, i)].shape[1], M=fo, N=fi, K=R, C32=w.data_ptr(), ldc32=fi, split=s)
             for (c, i, fi, fo), w, s in zip(layers, ws, splits)]
    rjobs = [S.flat_reduce(w.data_ptr(), fo * fi, d.data_ptr(), fo * fi, s)
             for w, d, s, (fo, fi, _r) in zip(ws, dW, splits, shapes)]
    libs = {"product": S.lib()}
    for v in a.variants:
        libs[v.split("/")[-1]] = S.load(v)
    out["dw_group_us"] = timeit_many({k: (lambda L=L: S.gemm_group(dargs, S.DW, L)) for k, L in libs.items()})
    out["s8_dw_reduce_us"] = timeit(lambda: S.reduce(rjobs))
    ws8 = [torch.empty(8, fo, fi, device=dev) for (fo, fi, _r) in shapes]
    dargs8 = [S.GemmArgs(A=DYs[(c, i)].data_ptr(), lda=DYs[(c, i)].shape[1], B=Xs[(c, i)].data_ptr(),
                         ldb=Xs[(c, i)].shape[1], M=fo, N=fi, K=R, C32=w.data_ptr(), ldc32=fi, split=8)
              for (c, i, fi, fo), w in zip(layers, ws8)]
    out["dw_group_split8_us"] = timeit_many({k: (lambda L=L: S.gemm_group(dargs8, S.DW, L)) for k, L in libs.items()})
    own = {}  # each variant at the split its own lgx_s8_pick_split chooses
    for k, L in libs.items():
        sp = S.pick_split(shapes, L)
        wk = [torch.empty(q, fo, fi, device=dev) for q, (fo, fi, _r) in zip(sp, shapes)]
        ak = [S.GemmArgs(A=DYs[(c, i)].data_ptr(), lda=DYs[(c, i)].shape[1], B=Xs[(c, i)].data_ptr(),
                         ldb=Xs[(c, i)].shape[1], M=fo, N=fi, K=R, C32=w.data_ptr(), ldc32=fi, split=q)
              for (c, i, fi, fo), w, q in zip(layers, wk, sp)]
        rk = [S.flat_reduce(w.data_ptr(), fo * fi, d.data_ptr(), fo * fi, q)
              for w, d, q, (fo, fi, _r) in zip(wk, dW, sp, shapes)]
        own[k] = (lambda L=L, ak=ak, rk=rk, wk=wk: (S.gemm_group(ak, S.DW, L), S.reduce(rk, L)))
        out[f"s8_splits_{k}"] = sp
    out["dw_group_plus_reduce_own_split_us"] = timeit_many(own)
    ref_ws = None
    for k, L in libs.items():  # every variant computes the same partials (same MFMA order)
        for w in ws:
            w.fill_(float("nan"))
        S.gemm_group(dargs, S.DW, L)
        torch.cuda.synchronize()
        cur = [w.clone() for w in ws]
        if ref_ws is None:
            ref_ws = cur
        out[f"dw_bitwise_equal_{k}"] = all(torch.equal(x, y) for x, y in zip(cur, ref_ws))
    out["s8_splits"] = splits
    # correctness spot check vs fp32-operand path
    S.gemm_group(dargs, S.DW)
    S.reduce(rjobs)
    dW_old = [torch.zeros(fo, fi, device=dev) for (fo, fi, _r) in shapes]
    db_old = [torch.zeros(fo, device=dev) for (fo, fi, _r) in shapes]

    def old_dw():
        with H.deferred_weight_grads():
            for (c, i, fi, fo), d, b in zip(layers, dW_old, db_old):
                H.linear_weight_grad(DY[(c, i)], X[(c, i)], d, b, accumulate=False)
    old_dw()
    torch.cuda.synchronize()
    out["dw_max_rel_diff"] = max(float((x - y).abs().max() / (y.abs().max() + 1e-30)) for x, y in zip(dW, dW_old))
    out["old_dw_group_plus_reduce_us"] = timeit(old_dw)

    # ---- forward and input-gradient launches per depth
    depth = max(len(v) for v in CHAINS.values())
    for d in range(depth):
        fa, ga, fo_old, go_old = [], [], [], []
        for c, ls in CHAINS.items():
            if d >= len(ls):
                continue
            fi, fo = ls[d]
            k = (c, d)
            y = S.empty(R, fo, dev)
            fa.append(S.GemmArgs(A=Xs[k].data_ptr(), lda=Xs[k].shape[1], B=Ws[k].data_ptr(), ldb=Ws[k].shape[1],
                                 M=R, N=fo, K=fi, epilogue=S.EPI_BIAS | S.EPI_ELU, C=y.data_ptr(), ldc=y.shape[1],
                                 bias=Bs[k].data_ptr()))
            y32 = torch.empty(R, fo, device=dev)
            fo_old.append(H._fwd_args(X[k], W[k], Bs[k], True, y32))
            if d > 0:
                dx = S.empty(R, fi, dev)
                ga.append(S.GemmArgs(A=DYs[k].data_ptr(), lda=DYs[k].shape[1], B=Ws[k].data_ptr(), ldb=Ws[k].shape[1],
                                     M=R, N=fi, K=fo, epilogue=S.EPI_DELU, C=dx.data_ptr(), ldc=dx.shape[1],
                                     act=Xs[k].data_ptr(), ld_act=Xs[k].shape[1]))
                dx32 = torch.empty(R, fi, device=dev)
                Wt = W[k].t().contiguous()
                go_old.append(H._dxt_args(DY[k], Wt, X[k], dx32))
        out[f"fwd_d{d}_us"] = timeit_many({k: (lambda L=L: S.gemm_group(fa, S.FWD, L)) for k, L in libs.items()})
        out[f"old_fwd_d{d}_us"] = timeit(lambda: H.run_group(fo_old))
        if ga:
            out[f"dx_d{d}_us"] = timeit_many({k: (lambda L=L: S.gemm_group(ga, S.DX, L)) for k, L in libs.items()})
            out[f"old_dx_d{d}_us"] = timeit(lambda: H.run_group(go_old))
    line = json.dumps(out)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
