"""Single-problem timings of the S8 GEMM kinds (dev tool): each problem alone in a launch, the
product library and build variants interleaved in one process (HIP events, median of rounds),
with fp32-equivalent TFLOP/s. Usage: PYTHONPATH=. python tools/s8_one.py [variant.so ...]"""
import json
import sys

import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S
from s8_bench import timeit_many  # noqa: E402  (tools/ on sys.path via PYTHONPATH=.:tools)

dev = "cuda:0"
R = 24576
PROBS = [("fwd", R, 512, 736), ("fwd", R, 256, 512), ("fwd", R, 1024, 1024), ("dx", R, 512, 256),
         ("dx", R, 512, 512), ("dw", 512, 736, R), ("dw", 512, 640, R), ("dw", 256, 512, R), ("dw", 1024, 1024, R)]


def main():
    libs = {"product": S.lib()}
    for v in sys.argv[1:]:
        libs[v.split("/")[-1]] = S.load(v)
    g = torch.Generator(device="cpu").manual_seed(0)
    out = {}
    for kind, M, N, K in PROBS:
        fns = {}
        if kind == "fwd":
            A = S.to_s8(torch.randn(M, K, generator=g).to(dev))
            B = S.to_s8((torch.randn(N, K, generator=g) * 0.05).to(dev))
            C = S.empty(M, N, dev)
            bias = torch.zeros(N, device=dev)
            args = [S.GemmArgs(A=A.data_ptr(), lda=A.shape[1], B=B.data_ptr(), ldb=B.shape[1], M=M, N=N, K=K,
                               epilogue=S.EPI_BIAS | S.EPI_ELU, C=C.data_ptr(), ldc=C.shape[1], bias=bias.data_ptr())]
            for k, L in libs.items():
                fns[k] = (lambda L=L, a=args: S.gemm_group(a, S.FWD, L))
        elif kind == "dx":  # dy [M, K], W [K, N] (S8 rows = K), act [M, N]
            A = S.to_s8(torch.randn(M, K, generator=g).to(dev))
            B = S.to_s8((torch.randn(K, N, generator=g) * 0.05).to(dev))
            act = S.to_s8(torch.randn(M, N, generator=g).to(dev))
            C = S.empty(M, N, dev)
            args = [S.GemmArgs(A=A.data_ptr(), lda=A.shape[1], B=B.data_ptr(), ldb=B.shape[1], M=M, N=N, K=K,
                               epilogue=S.EPI_DELU, C=C.data_ptr(), ldc=C.shape[1], act=act.data_ptr(),
                               ld_act=act.shape[1])]
            for k, L in libs.items():
                fns[k] = (lambda L=L, a=args: S.gemm_group(a, S.DX, L))
        else:  # dW [M, N] = dy[K, M]^T x[K, N]
            A = S.to_s8(torch.randn(K, M, generator=g).to(dev))
            B = S.to_s8(torch.randn(K, N, generator=g).to(dev))
            for k, L in libs.items():
                sp = S.pick_split([(M, N, K)], L)[0]
                ws = torch.empty(sp, M, N, device=dev)
                args = [S.GemmArgs(A=A.data_ptr(), lda=A.shape[1], B=B.data_ptr(), ldb=B.shape[1], M=M, N=N, K=K,
                                   C32=ws.data_ptr(), ldc32=N, split=sp)]
                fns[k] = (lambda L=L, a=args, ws=ws: S.gemm_group(a, S.DW, L))
                out[f"split_{kind}_{M}x{N}x{K}_{k}"] = sp
        t = timeit_many(fns)
        flops = 2.0 * M * N * K
        out[f"{kind}_{M}x{N}x{K}"] = {k: (v[0], round(flops / v[0] / 1e6, 1)) for k, v in t.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
