"""Per-block cycle accounts of the S8 GEMM (dev tool, GPU): a -DLGX_S8_CLOCK build of the library
(exp/s8_clock.so: hipcc ... -DLGX_S8_CLOCK -shared lgx_s8.hip lgx_act.hip lgx_s8chain.hip) runs
single problems; waves 0 and NW-1 of every block report the K loop's DMA wait, barrier and
issue + compute cycles per K step and the epilogue's (lgx_s8.hip g_s8clk). The "-solo" problems
have one block per CU (no co-resident block's MFMAs).
Usage: PYTHONPATH=.:tools python tools/s8_clock.py exp/s8_clock.so [...]"""
import ctypes as C
import sys

import numpy as np
import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S

dev = "cuda:0"
R = 24576
PROBS = [("fwd", R, 512, 736), ("fwd-noelu", R, 512, 736), ("fwd", R, 1024, 1024), ("dx", R, 512, 256),
         ("dx-nodelu", R, 512, 256), ("fwd-solo", 16384, 128, 736), ("fwd-solo-noelu", 16384, 128, 736),
         ("dx-solo", 16384, 128, 256)]


def problem(kind, M, N, K, L, g):
    if kind.startswith("fwd"):
        A = S.to_s8(torch.randn(M, K, generator=g).to(dev))
        B = S.to_s8((torch.randn(N, K, generator=g) * 0.05).to(dev))
        Cb = S.empty(M, N, dev)
        bias = torch.zeros(N, device=dev)
        keep = (A, B, Cb, bias)
        args = [S.GemmArgs(A=A.data_ptr(), lda=A.shape[1], B=B.data_ptr(), ldb=B.shape[1], M=M, N=N, K=K,
                           epilogue=S.EPI_BIAS | (0 if "noelu" in kind else S.EPI_ELU), C=Cb.data_ptr(), ldc=Cb.shape[1], bias=bias.data_ptr())]
        return keep, (lambda: S.gemm_group(args, S.FWD, L))
    if kind.startswith("dx"):
        A = S.to_s8(torch.randn(M, K, generator=g).to(dev))
        B = S.to_s8((torch.randn(K, N, generator=g) * 0.05).to(dev))
        act = S.to_s8(torch.randn(M, N, generator=g).to(dev))
        Cb = S.empty(M, N, dev)
        keep = (A, B, act, Cb)
        args = [S.GemmArgs(A=A.data_ptr(), lda=A.shape[1], B=B.data_ptr(), ldb=B.shape[1], M=M, N=N, K=K,
                           epilogue=0 if "nodelu" in kind else S.EPI_DELU, C=Cb.data_ptr(), ldc=Cb.shape[1], act=act.data_ptr(),
                           ld_act=act.shape[1])]
        return keep, (lambda: S.gemm_group(args, S.DX, L))
    A = S.to_s8(torch.randn(K, M, generator=g).to(dev))
    B = S.to_s8(torch.randn(K, N, generator=g).to(dev))
    sp = S.pick_split([(M, N, K)], L)[0]
    ws = torch.empty(sp, M, N, device=dev)
    keep = (A, B, ws)
    args = [S.GemmArgs(A=A.data_ptr(), lda=A.shape[1], B=B.data_ptr(), ldb=B.shape[1], M=M, N=N, K=K,
                       C32=ws.data_ptr(), ldc32=N, split=sp)]
    return keep, (lambda: S.gemm_group(args, S.DW, L))


def main():
    g = torch.Generator(device="cpu").manual_seed(0)
    for path in sys.argv[1:]:
        L = S.load(path)
        L.lgx_s8_set_clock.argtypes = [C.c_void_p]
        buf = torch.zeros(24 * 40000, dtype=torch.int32, device=dev)
        for kind, M, N, K in PROBS:
            keep, fn = problem(kind, M, N, K, L, g)
            for _ in range(3):
                fn()
            buf.zero_()
            torch.cuda.synchronize()
            assert L.lgx_s8_set_clock(buf.data_ptr()) == 0
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            L.lgx_s8_set_clock(None)
            us = a.elapsed_time(b) * 1000
            d = buf.view(-1, 2, 12).cpu().numpy().astype(np.int64)
            live = d[:, 0, 4] > 0
            d = d[live]
            nk = d[:, 0, 5].astype(np.float64)
            tot = d[:, :, 4].astype(np.float64)
            print(f"== {path.split('/')[-1]} {kind} {M}x{N}x{K}: {us:.1f} us, {len(d)} blocks, "
                  f"K steps {int(nk.min())}-{int(nk.max())}")
            for w, name in ((0, "wave 0"), (1, "last wave")):
                per = lambda c: d[:, w, c].astype(np.float64) / nk  # noqa: E731
                print(f"  {name}: per K step  wait {per(0).mean():7.0f}  barrier {per(1).mean():7.0f}  "
                      f"issue+compute {per(2).mean():7.0f}   epilogue/tile "
                      f"{(d[:, w, 3] / np.maximum(d[:, w, 7], 1)).mean():6.0f}  tiles/block {np.maximum(d[:, w, 7], 1).mean():4.2f}  "
                      f"block total {tot[:, w].mean():9.0f} (p10 {np.percentile(tot[:, w], 10):9.0f}, "
                      f"max {tot[:, w].max():9.0f})")
            del keep


if __name__ == "__main__":
    main()
