"""The S8 GEMM core (liblgx_s8.so, include/lgx_s8.h) against fp64 references.

Operands are S8 (bf16 hi/lo planes): the reference multiplies the SAME split values (hi + lo)
in fp64, so what remains is the dropped lo*lo term (<= 2^-16 |a b|) and fp32 accumulation:
    |C - C_ref| <= 2e-5 * sum_k |a_k b_k| + 1e-6          (stated tolerance, per element)
Epilogues (bias + ELU; ELU' from an S8 y_prev; addend; zero pads; column sums) are checked
against torch fp64 on the same values; the fp32 -> S8 split against torch's bf16 rounding
(bit-exact)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda:0"


@pytest.fixture(scope="module")
def S():
    from legged_gym_custom_amd.rsl_rl.modules import hip_s8
    hip_s8.lib()
    return hip_s8


def _bound(a, b):
    return 2e-5 * (a.abs() @ b.abs()) + 1e-6


def _s8(S, x, ld=None, rows_pad=None):
    return S.to_s8_torch(x, ld=ld, rows_pad=rows_pad)


def test_split_matches_torch_bf16_rounding_and_colsums(S):
    g = torch.Generator(device="cpu").manual_seed(0)
    for rows, cols in ((1, 1), (300, 13), (513, 64), (64, 627)):
        x = (torch.randn(rows, cols, generator=g) * torch.logspace(-6, 3, cols)).to(dev)
        buf = S.empty(rows, cols, dev)
        cs = torch.zeros((rows + S.SPLIT_ROWS - 1) // S.SPLIT_ROWS, cols, device=dev) if cols <= 64 else None
        S.split([S.split_job(x, buf.data_ptr(), buf.shape[1], colsum_ws=cs)])
        torch.cuda.synchronize()
        ref = S.to_s8_torch(x)
        assert torch.equal(buf, ref), (rows, cols)
        if cs is not None:
            blocks = [x[i:i + S.SPLIT_ROWS].double().sum(0) for i in range(0, rows, S.SPLIT_ROWS)]
            torch.testing.assert_close(cs.double(), torch.stack(blocks), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (300, 200, 72), (24576 // 8, 627, 512), (129, 12, 128), (257, 130, 33)])
def test_forward_bias_elu(S, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(dev)
    W = (torch.randn(N, K, generator=g) * 0.1).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    xs, Ws = _s8(S, x), _s8(S, W)
    xv, Wv = S.from_s8(xs, M, K).double(), S.from_s8(Ws, N, K).double()
    out = S.empty(M, N, dev)
    y32 = torch.full((M, N + 3), float("nan"), device=dev)
    cs = torch.zeros((M + S.TILE_M - 1) // S.TILE_M, N, device=dev)
    S.gemm_group([S.GemmArgs(A=xs.data_ptr(), lda=xs.shape[1], B=Ws.data_ptr(), ldb=Ws.shape[1], M=M, N=N, K=K,
                             epilogue=S.EPI_BIAS | S.EPI_ELU, C=out.data_ptr(), ldc=out.shape[1], C32=y32.data_ptr(),
                             ldc32=y32.stride(0), bias=b.data_ptr(), colsum_ws=cs.data_ptr())], S.FWD)
    torch.cuda.synchronize()
    z = xv @ Wv.t() + b.double()
    ref = torch.nn.functional.elu(z)
    bound = _bound(xv, Wv.t()) * 1.5 + 1e-6  # ELU' <= 1; its polynomial ~1e-8
    y = y32[:, :N].double()
    assert (y - ref).abs().le(bound).all(), float((y - ref).abs().max())
    assert torch.isnan(y32[:, N:]).all()  # nothing past N in the fp32 copy
    # the S8 output is the split of the fp32 output, pads zero
    assert torch.equal(out, S.to_s8_torch(y32[:, :N].contiguous(), ld=out.shape[1], rows_pad=out.shape[0]))
    blocks = torch.stack([y32[i:i + S.TILE_M, :N].double().sum(0) for i in range(0, M, S.TILE_M)])
    torch.testing.assert_close(cs.double(), blocks, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,N,K", [(300, 512, 256), (200, 627, 512), (64, 55, 512), (130, 128, 12), (33, 20, 1)])
def test_input_grad_delu_addend(S, M, N, K):
    """dX[m][n] = (sum_k dY[m][k] W[k][n]) * ELU'(y_prev) + addend (n < add_cols); W read TR."""
    g = torch.Generator(device="cpu").manual_seed(7 * M + N + K)
    dy = torch.randn(M, K, generator=g).to(dev)
    W = (torch.randn(K, N, generator=g) * 0.1).to(dev)
    yp = torch.nn.functional.elu(torch.randn(M, N, generator=g)).to(dev)
    add = torch.randn(M, 17, generator=g).to(dev)
    dys, Ws, yps = _s8(S, dy), _s8(S, W), _s8(S, yp)
    dyv, Wv, ypv = S.from_s8(dys, M, K).double(), S.from_s8(Ws, K, N).double(), S.from_s8(yps, M, N).double()
    out = S.empty(M, N, dev)
    cs = torch.zeros((M + S.TILE_M - 1) // S.TILE_M, N, device=dev)
    S.gemm_group([S.GemmArgs(A=dys.data_ptr(), lda=dys.shape[1], B=Ws.data_ptr(), ldb=Ws.shape[1], M=M, N=N, K=K,
                             epilogue=S.EPI_DELU, C=out.data_ptr(), ldc=out.shape[1], act=yps.data_ptr(),
                             ld_act=yps.shape[1], addend=add.data_ptr(), ld_add=add.stride(0), add_cols=17,
                             colsum_ws=cs.data_ptr())], S.DX)
    torch.cuda.synchronize()
    d = torch.where(ypv > 0, torch.ones_like(ypv), ypv + 1.0)
    ref = (dyv @ Wv) * d
    ref[:, :17] += add.double()[:, :min(17, N)] if N >= 17 else add.double()[:, :N]
    got = S.from_s8(out, M, N).double()
    bound = _bound(dyv, Wv) + 1e-5 * ref.abs() + 1e-6  # + the S8 output's own split (2^-17)
    assert (got - ref).abs().le(bound).all(), float((got - ref).abs().max())
    # the pad columns of the output's last group stay zero
    hi, lo = S.planes(out, M, out.shape[1])
    assert (hi[:, N:] == 0).all() and (lo[:, N:] == 0).all()
    blocks = torch.stack([got[i:i + S.TILE_M].sum(0) for i in range(0, M, S.TILE_M)])
    torch.testing.assert_close(cs.double(), blocks, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("rows,M,N,split", [(384, 12, 128, 1), (4096, 512, 627, 4), (2048, 20, 29, 3),
                                             (1024, 130, 257, 2)])
def test_weight_grad_split_k(S, rows, M, N, split):
    """dW[m][n] = sum_r dY[r][m] X[r][n]: both operands TR; split-K partials + lgx_s8_reduce."""
    g = torch.Generator(device="cpu").manual_seed(rows + M + N)
    dy = torch.randn(rows, M, generator=g).to(dev)
    x = torch.randn(rows, N, generator=g).to(dev)
    dys, xs = _s8(S, dy), _s8(S, x)
    dyv, xv = S.from_s8(dys, rows, M).double(), S.from_s8(xs, rows, N).double()
    ref = dyv.t() @ xv
    bound = _bound(dyv.t(), xv)
    if split == 1:
        out = torch.full((M, N), 0.5, device=dev)
        S.gemm_group([S.GemmArgs(A=dys.data_ptr(), lda=dys.shape[1], B=xs.data_ptr(), ldb=xs.shape[1], M=M, N=N, K=rows,
                                 epilogue=S.EPI_ACCUM, C32=out.data_ptr(), ldc32=N, split=1)], S.DW)
        torch.cuda.synchronize()
        assert ((out.double() - 0.5) - ref).abs().le(bound + 1e-6).all()
        return
    ws = torch.empty(split, M, N, device=dev)
    S.gemm_group([S.GemmArgs(A=dys.data_ptr(), lda=dys.shape[1], B=xs.data_ptr(), ldb=xs.shape[1], M=M, N=N, K=rows,
                             C32=ws.data_ptr(), ldc32=N, split=split)], S.DW)
    out = torch.full((M, N), 0.25, device=dev)
    S.reduce([S.flat_reduce(ws.data_ptr(), M * N, out.data_ptr(), M * N, split, accumulate=1)])
    torch.cuda.synchronize()
    assert ((out.double() - 0.25) - ref).abs().le(bound + 1e-6).all(), float(((out.double() - 0.25) - ref).abs().max())


def _tail_buffer(rows, ld):
    """An S8 buffer [rows, ld] ending exactly at the end of its own 2 MiB allocation (the caching
    allocator gives a 2 MiB request its own segment): a read past its last row leaves the segment."""
    n = 1 << 19  # int32 words = 2 MiB
    assert rows * ld <= n
    flat = torch.zeros(n, dtype=torch.int32, device=dev)
    return flat, flat[n - rows * ld:].view(rows, ld)


def test_column_span_operands_at_allocation_end(S):
    """Regression test for the round-4 fault (gpurun_out/s8_update_tests.log:70, "illegal memory
    access" under test_gpu_learner.py): TR-mode operand offsets were clamped to the row PITCH, so
    an operand that is a column span of a wider row (the actor's latent columns, the encoders'
    last-layer gradients) read up to its column offset past the buffer's last row. Every operand
    here is a column span (offset 64, width 40, pitch 128) of a buffer flush against the end of
    its allocation; FWD, DX and DW against fp64 (lgx_s8.hip Op::offsets clamps to the span)."""
    g = torch.Generator(device="cpu").manual_seed(11)
    c0, w, ld = 64, 40, 128
    rows, K = 1024, 512
    # DX: dX = dY W[:, span] with W [K, ld] read TR (k = source row), span at column c0
    W = (torch.randn(K, ld, generator=g) * 0.1).to(dev)
    _keep_w, Wb = _tail_buffer(K, ld)
    Wb.copy_(_s8(S, W, ld=ld))
    dy = torch.randn(rows, K, generator=g).to(dev)
    dys = _s8(S, dy)
    out = S.empty(rows, w, dev)
    S.gemm_group([S.GemmArgs(A=dys.data_ptr(), lda=dys.shape[1], B=S.group_ptr(Wb, c0), ldb=ld, M=rows, N=w, K=K,
                             C=out.data_ptr(), ldc=out.shape[1])], S.DX)
    # DW: dW = dY[:, span]^T X[:, span], both TR column spans of tail buffers (K = rows)
    A = torch.randn(rows, ld, generator=g).to(dev)
    X = torch.randn(rows, ld, generator=g).to(dev)
    _keep_a, Ab = _tail_buffer(rows, ld)
    _keep_x, Xb = _tail_buffer(rows, ld)
    Ab.copy_(_s8(S, A, ld=ld))
    Xb.copy_(_s8(S, X, ld=ld))
    dw = torch.zeros(w, w, device=dev)
    S.gemm_group([S.GemmArgs(A=S.group_ptr(Ab, c0), lda=ld, B=S.group_ptr(Xb, c0), ldb=ld, M=w, N=w, K=rows,
                             epilogue=S.EPI_ACCUM, C32=dw.data_ptr(), ldc32=w, split=1)], S.DW)
    # FWD: Y = X[:, c0:] V^T with the input a ROW-mode column span (the last 64 columns: whole
    # K steps) of a tail buffer
    kf = ld - c0
    V = (torch.randn(24, kf, generator=g) * 0.1).to(dev)
    Vs = _s8(S, V)
    y = torch.full((rows, 24), float("nan"), device=dev)
    S.gemm_group([S.GemmArgs(A=S.group_ptr(Xb, c0), lda=ld, B=Vs.data_ptr(), ldb=Vs.shape[1], M=rows, N=24, K=kf,
                             C32=y.data_ptr(), ldc32=24)], S.FWD)
    torch.cuda.synchronize()
    Wv = S.from_s8(Wb, K, ld).double()[:, c0:c0 + w]
    dyv = S.from_s8(dys, rows, K).double()
    ref = dyv @ Wv
    got = S.from_s8(out, rows, w).double()
    assert (got - ref).abs().le(_bound(dyv, Wv) + 1e-5 * ref.abs() + 1e-6).all(), float((got - ref).abs().max())
    Av = S.from_s8(Ab, rows, ld).double()[:, c0:c0 + w]
    Xv = S.from_s8(Xb, rows, ld).double()[:, c0:c0 + w]
    ref = Av.t() @ Xv
    assert (dw.double() - ref).abs().le(_bound(Av.t(), Xv) + 1e-6).all(), float((dw.double() - ref).abs().max())
    Vv = S.from_s8(Vs, 24, kf).double()
    Xf = S.from_s8(Xb, rows, ld).double()[:, c0:]
    ref = Xf @ Vv.t()
    assert (y.double() - ref).abs().le(_bound(Xf, Vv.t()) + 1e-6).all(), float((y.double() - ref).abs().max())


def test_grouped_launch_equals_single_launches(S):
    """Several problems in one launch give the single launches' results bit for bit."""
    g = torch.Generator(device="cpu").manual_seed(3)
    rows = 1024
    probs, bufs = [], []
    for (M, N) in ((512, 627), (12, 128), (20, 29), (128, 256)):
        dy = _s8(S, torch.randn(rows, M, generator=g).to(dev))
        x = _s8(S, torch.randn(rows, N, generator=g).to(dev))
        bufs.append((dy, x, M, N))
    outs_g = [torch.zeros(M, N, device=dev) for (_d, _x, M, N) in bufs]
    args = [S.GemmArgs(A=d.data_ptr(), lda=d.shape[1], B=x.data_ptr(), ldb=x.shape[1], M=M, N=N, K=rows,
                       C32=o.data_ptr(), ldc32=N, split=1) for (d, x, M, N), o in zip(bufs, outs_g)]
    S.gemm_group(args, S.DW)
    outs_s = [torch.zeros(M, N, device=dev) for (_d, _x, M, N) in bufs]
    for (d, x, M, N), o in zip(bufs, outs_s):
        S.gemm_group([S.GemmArgs(A=d.data_ptr(), lda=d.shape[1], B=x.data_ptr(), ldb=x.shape[1], M=M, N=N, K=rows,
                                 C32=o.data_ptr(), ldc32=N, split=1)], S.DW)
    torch.cuda.synchronize()
    for a, b in zip(outs_g, outs_s):
        assert torch.equal(a, b)


def test_rejects_bad_arguments(S):
    import ctypes as C
    L = S.lib()
    a = S.GemmArgs(M=-1, N=1, K=1)
    assert L.lgx_s8_gemm_group(C.byref(a), 1, S.FWD, None) < 0
    a = S.GemmArgs(A=16, B=16, lda=12, ldb=32, M=4, N=4, K=4, C=16, ldc=32)
    assert L.lgx_s8_gemm_group(C.byref(a), 1, S.FWD, None) < 0 and b"multiples of 8" in L.lgx_s8_last_error()
    a = S.GemmArgs(A=16, B=16, lda=8, ldb=32, M=4, N=4, K=40, C=16, ldc=32)
    assert L.lgx_s8_gemm_group(C.byref(a), 1, S.FWD, None) < 0 and b"pitch" in L.lgx_s8_last_error()
    np.testing.assert_array_equal(S.pick_split([(512, 627, 24576)] * 2), [S.pick_split([(512, 627, 24576)] * 2)[0]] * 2)


def test_gather_split_and_span_reduce(S):
    """lgx_s8_split with a row permutation (the update's minibatch gather) and lgx_s8_reduce over
    2-D column spans (a weight whose input columns sit elsewhere in S8 space)."""
    g = torch.Generator(device="cpu").manual_seed(11)
    src = torch.randn(3000, 100, generator=g).to(dev)
    idx = torch.randperm(3000, generator=g)[:1000].to(dev)
    buf = S.empty(1000, 100, dev)
    S.split([S.split_job(src, buf.data_ptr(), buf.shape[1], idx=idx, rows=1000)])
    ws = torch.randn(3, 20, 64, generator=g).to(dev)
    out = torch.full((20, 50), 7.0, device=dev)
    S.reduce([S.ReduceArgs(ws=ws.data_ptr() + 4 * 10, stride=20 * 64, ld_ws=64, out=out.data_ptr() + 4 * 5, ld_out=50,
                           rows=20, cols=40, nsplit=3, accumulate=0)])
    torch.cuda.synchronize()
    assert torch.equal(buf, S.to_s8_torch(src[idx]))
    ref = torch.full((20, 50), 7.0, device=dev)
    ref[:, 5:45] = ws[0, :, 10:50] + ws[1, :, 10:50] + ws[2, :, 10:50]
    assert torch.equal(out, ref)


def test_loss_heads_fused_equals_forward_plus_backward(S):
    """lgx_loss_heads_fused (one launch) == lgx_loss_heads_forward + lgx_loss_heads_backward on
    the same arguments: the six losses, dstd, the latent gradient and the fp32 dmu / dvalue / de
    bit for bit; its S8 outputs are the exact split of those fp32 gradients, and its column
    sums are the 256-row block sums (fp32, fixed order: 1e-5)."""
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
    g = torch.Generator(device=dev).manual_seed(43)
    B, A, L, E = 3000, 12, 20, 3
    r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    mu, value, std = r(B, A), r(B, 1), r(A).abs() + 0.5
    actions, old_logp, adv, tv, ret = r(B, A), r(B, 1), r(B, 1), r(B, 1), r(B, 1)
    old_mu, old_sigma = r(B, A), r(B, A).abs() + 0.5
    p_lat, a_lat, pred, t_est = r(B, L), r(B, L), r(B, E), r(B, E)
    seeds = torch.tensor([1.0, 1.3, -0.01, 0.05, 1.0], device=dev)
    nblk = (B + 255) // 256

    def args(ws, wsa, out, out_aux, dmu, dvalue, dstd, dp, de, cnt, cnta):
        h = H.HeadArgs(mu=mu.data_ptr(), value=value.data_ptr(), std=std.data_ptr(), actions=actions.data_ptr(),
                       old_logp=old_logp.data_ptr(), adv=adv.data_ptr(), target_values=tv.data_ptr(),
                       returns=ret.data_ptr(), old_mu=old_mu.data_ptr(), old_sigma=old_sigma.data_ptr(), B=B, A=A,
                       clip=0.2, clipped_value=1, out=out.data_ptr(), g=seeds.data_ptr(),
                       dmu=None if dmu is None else dmu.data_ptr(), dvalue=None if dvalue is None else dvalue.data_ptr(),
                       dstd=dstd.data_ptr(), ws=ws.data_ptr(), counter=cnt.data_ptr(), accumulate_dstd=0)
        x = H.AuxArgs(p=p_lat.data_ptr(), a=a_lat.data_ptr(), L=L, e=pred.data_ptr(), t=t_est.data_ptr(), E=E, B=B,
                      out=out_aux.data_ptr(), g=seeds.data_ptr() + 12, dp=dp.data_ptr(),
                      de=None if de is None else de.data_ptr(), ws=wsa.data_ptr(), counter=cnta.data_ptr(), ld_p=L)
        return h, x

    def bufs():
        z = lambda *s: torch.full(s, float("nan"), device=dev)  # noqa: E731
        return dict(ws=torch.zeros(19 * nblk, device=dev), wsa=torch.zeros(2 * nblk, device=dev), out=z(8),
                    out_aux=z(2), dmu=z(B, A), dvalue=z(B), dstd=z(A), dp=z(B, L), de=z(B, E),
                    cnt=torch.zeros(1, dtype=torch.int32, device=dev), cnta=torch.zeros(1, dtype=torch.int32, device=dev))
    ref = bufs()
    h, x = args(**ref)
    H._check(H.lib().lgx_loss_heads_forward(H.C.byref(h), H.C.byref(x), H._stream()), "fwd")
    H._check(H.lib().lgx_loss_heads_backward(H.C.byref(h), H.C.byref(x), H._stream()), "bwd")
    got = bufs()
    dmu8, dv8, de8 = S.empty(B, A, dev), S.empty(B, 1, dev), S.empty(B, E, dev)
    cs_mu, cs_v, cs_e = (torch.full((nblk, n), float("nan"), device=dev) for n in (A, 1, E))
    s8 = H.HeadsS8Args(dmu_s8=dmu8.data_ptr(), ld_dmu=dmu8.shape[1], dmu_cs=cs_mu.data_ptr(), dvalue_s8=dv8.data_ptr(),
                       ld_dvalue=dv8.shape[1], dvalue_cs=cs_v.data_ptr(), de_s8=de8.data_ptr(), ld_de=de8.shape[1],
                       de_cs=cs_e.data_ptr())
    h, x = args(**got)
    H._check(H.lib().lgx_loss_heads_fused(H.C.byref(h), H.C.byref(x), H.C.byref(s8), H._stream()), "fused")
    torch.cuda.synchronize()
    for k in ("out", "out_aux", "dmu", "dvalue", "dstd", "dp", "de"):
        if k == "out":
            idx = [0, 1, 2, 3]
            assert torch.equal(got[k][idx], ref[k][idx]), k
        else:
            assert torch.equal(got[k], ref[k]), k
    assert torch.equal(dmu8, S.to_s8_torch(ref["dmu"], ld=dmu8.shape[1], rows_pad=dmu8.shape[0]))
    assert torch.equal(dv8, S.to_s8_torch(ref["dvalue"].view(B, 1), ld=dv8.shape[1], rows_pad=dv8.shape[0]))
    assert torch.equal(de8, S.to_s8_torch(ref["de"], ld=de8.shape[1], rows_pad=de8.shape[0]))
    for cs, full in ((cs_mu, ref["dmu"]), (cs_v, ref["dvalue"].view(B, 1)), (cs_e, ref["de"])):
        blocks = torch.stack([full[i:i + 256].double().sum(0) for i in range(0, B, 256)])
        torch.testing.assert_close(cs.double(), blocks, rtol=1e-5, atol=1e-6)


def _pack_ref(Ws, N, K):
    """Fragment packing of an S8 weight buffer in torch (lgx_s8_chain_layer.packed)."""
    T, st = (N + 15) // 16, (K + 31) // 32
    r, ld = Ws.shape
    b = torch.zeros(T * 16, st * 32 // 8, 2, 8, dtype=torch.bfloat16, device=Ws.device)
    src = Ws.view(torch.bfloat16).view(r, ld // 8, 2, 8)
    g = min(st * 4, ld // 8)
    b[:N, :g] = src[:N, :g]
    # [tile, fr, step, fc, 2, 8] -> [tile, step, 2, fc, fr, 8]
    b = b.view(T, 16, st, 4, 2, 8).permute(0, 2, 4, 3, 1, 5).contiguous()
    return b.view(-1).view(torch.int32)


def test_split_packed_matches_reference(S):
    g = torch.Generator(device="cpu").manual_seed(5)
    for N, K in ((128, 132), (20, 64), (64, 29), (33, 200)):
        W = torch.randn(N, K, generator=g).to(dev)
        Wp = S.packed_empty(N, K, dev)
        S.split([S.split_packed_job(W, Wp)])
        torch.cuda.synchronize()
        assert torch.equal(Wp, _pack_ref(S.to_s8_torch(W), N, K)), (N, K)


@pytest.mark.parametrize("rows,packed", [(1000, 0), (1000, 1), (24576, 1)])
def test_chain_fwd_equals_grouped_levels(S, rows, packed):
    """lgx_s8_chain (the privileged / scan encoders' forward in one launch) against the same
    layers as one grouped FWD launch each: S8 outputs (hidden layers, the last one at a column
    offset of a wider buffer, pads zero), the fp32 copy, bit for bit."""
    g = torch.Generator(device="cpu").manual_seed(rows)
    shapes = {"scan": [132, 128, 64, 32], "priv": [29, 64, 20]}
    wide = S.empty(rows, 96, dev)  # the last layers' outputs: columns 0 (scan) and 40 (priv)
    wide_ref = S.empty(rows, 96, dev)
    chains, outs = [], {}
    for name, col in (("scan", 0), ("priv", 40)):
        w = shapes[name]
        x = S.to_s8_torch(torch.randn(rows, w[0], generator=g).to(dev))
        W32 = [(torch.randn(n, k, generator=g) * 0.2).to(dev) for k, n in zip(w[:-1], w[1:])]
        Ws = [S.to_s8_torch(W) for W in W32]
        Wp = [S.packed_empty(W.shape[0], W.shape[1], dev) for W in W32]
        S.split([S.split_packed_job(W, P) for W, P in zip(W32, Wp)])
        bs = [torch.randn(n, generator=g).to(dev) for n in w[1:]]
        hid = [S.empty(rows, n, dev) for n in w[1:-1]]
        hid_ref = [S.empty(rows, n, dev) for n in w[1:-1]]
        y32, y32_ref = torch.full((rows, w[-1]), float("nan"), device=dev), torch.full((rows, w[-1]), 7.0, device=dev)
        c = S.ChainArgs(A=x.data_ptr(), lda=x.shape[1], rows=rows, nlayers=len(w) - 1)
        A, lda = x, x.shape[1]
        for l, (k, n) in enumerate(zip(w[:-1], w[1:])):
            last = l == len(w) - 2
            L = c.layers[l]
            L.W, L.ldw, L.bias, L.K, L.N, L.elu = Ws[l].data_ptr(), Ws[l].shape[1], bs[l].data_ptr(), k, n, int(not last)
            if packed:
                L.W, L.packed = Wp[l].data_ptr(), 1
            if last:
                L.C, L.ldc, L.C32, L.ldc32 = S.group_ptr(wide, col), wide.shape[1], y32.data_ptr(), n
                ref_c, ref_ldc = S.group_ptr(wide_ref, col), wide_ref.shape[1]
            else:
                L.C, L.ldc = hid[l].data_ptr(), hid[l].shape[1]
                ref_c, ref_ldc = hid_ref[l].data_ptr(), hid_ref[l].shape[1]
            S.gemm_group([S.GemmArgs(A=A.data_ptr(), lda=lda, B=Ws[l].data_ptr(), ldb=Ws[l].shape[1], M=rows, N=n, K=k,
                                     epilogue=S.EPI_BIAS | (0 if last else S.EPI_ELU), C=ref_c, ldc=ref_ldc,
                                     C32=y32_ref.data_ptr() if last else None, ldc32=n if last else 0,
                                     bias=bs[l].data_ptr())], S.FWD)
            if not last:
                A, lda = hid_ref[l], hid_ref[l].shape[1]
        chains.append(c)
        outs[name] = (hid, hid_ref, y32, y32_ref, x, Ws, Wp, bs)  # (the chain reads x, Ws, bs at launch)
    S.chain(chains)
    torch.cuda.synchronize()
    for name, (hid, hid_ref, y32, y32_ref, *_keep) in outs.items():
        for h, hr in zip(hid, hid_ref):
            assert torch.equal(h, hr), name
        assert torch.equal(y32, y32_ref), name
    assert torch.equal(wide, wide_ref)


def test_chain_fwd_rejects_bad_arguments(S):
    x = S.empty(64, 40, dev)
    W = S.empty(16, 40, dev)
    c = S.ChainArgs(A=x.data_ptr(), lda=x.shape[1], rows=64, nlayers=2)
    c.layers[0] = S.ChainLayer(W=W.data_ptr(), ldw=W.shape[1], K=40, N=16)
    c.layers[1] = S.ChainLayer(W=W.data_ptr(), ldw=W.shape[1], K=40, N=16)  # K != previous N
    with pytest.raises(S.S8LibError, match="K_l"):
        S.chain([c])
    c.nlayers = 1
    c.layers[0].K = 300  # wider than the chain's image
    with pytest.raises(S.S8LibError):
        S.chain([c])


@pytest.mark.parametrize("rows", [1000, 24576])
def test_chain_input_grads_equal_grouped_levels(S, rows):
    """The encoders' input gradients as one chain launch (elu = 2: times ELU'(y), W^T
    fragment-packed by a transposed split, column sums per 32-row block) against one grouped DX
    launch per layer: S8 outputs bit for bit; the column totals (the bias gradients, summed in
    another order) to fp32 rounding. The inputs are column spans of one wider buffer (the
    update's dlat: privileged latent at 0, scan latent at 24): the chain reads zeros past K."""
    g = torch.Generator(device="cpu").manual_seed(rows + 1)
    dlat32 = torch.zeros(rows, 64, device=dev)
    dlat32[:, :20] = torch.randn(rows, 20, generator=g).to(dev)
    dlat32[:, 24:56] = torch.randn(rows, 32, generator=g).to(dev)
    dlat = S.to_s8_torch(dlat32)
    chains, checks, keep = [], [], []
    for c0, widths in ((24, [32, 64, 128]), (0, [20, 64])):  # scan (layers 2, 1), privileged (layer 1)
        c = S.ChainArgs(A=S.group_ptr(dlat, c0), lda=dlat.shape[1], rows=rows, nlayers=len(widths) - 1)
        A, lda = S.group_ptr(dlat, c0), dlat.shape[1]
        for q, (k, n) in enumerate(zip(widths[:-1], widths[1:])):
            W = (torch.randn(k, n, generator=g) * 0.2).to(dev)  # the forward weight [out k][in n]
            y = S.to_s8_torch(torch.nn.functional.elu(torch.randn(rows, n, generator=g)).to(dev))
            WpT = S.packed_empty(n, k, dev)
            S.split([S.split_packed_job(W, WpT, transpose=True)])
            Ws = S.to_s8_torch(W)
            out, out_ref = S.empty(rows, n, dev), S.empty(rows, n, dev)
            cs = torch.full(((rows + 31) // 32, n), float("nan"), device=dev)
            cs_ref = torch.zeros((rows + S.TILE_M - 1) // S.TILE_M, n, device=dev)
            L = c.layers[q]
            L.W, L.packed, L.K, L.N, L.elu = WpT.data_ptr(), 1, k, n, 2
            L.act, L.ld_act, L.C, L.ldc, L.colsum_ws = y.data_ptr(), y.shape[1], out.data_ptr(), out.shape[1], cs.data_ptr()
            S.gemm_group([S.GemmArgs(A=A, lda=lda, B=Ws.data_ptr(), ldb=Ws.shape[1], M=rows, N=n, K=k,
                                     epilogue=S.EPI_DELU, C=out_ref.data_ptr(), ldc=out_ref.shape[1], act=y.data_ptr(),
                                     ld_act=y.shape[1], colsum_ws=cs_ref.data_ptr())], S.DX)
            A, lda = out_ref.data_ptr(), out_ref.shape[1]
            keep += [W, y, WpT, Ws]
            checks.append((out, out_ref, cs, cs_ref))
        chains.append(c)
    S.chain(chains)
    torch.cuda.synchronize()
    for out, out_ref, cs, cs_ref in checks:
        assert torch.equal(out, out_ref)
        torch.testing.assert_close(cs.double().sum(0), cs_ref.double().sum(0), rtol=1e-5, atol=1e-4)


def test_chain_rejects_partial_column_sums(S):
    x = S.empty(256, 64, dev)
    W = S.packed_empty(64, 64, dev)
    cs = torch.zeros(2, 64, device=dev)
    c = S.ChainArgs(A=x.data_ptr(), lda=x.shape[1], rows=256, nlayers=2)
    c.layers[0] = S.ChainLayer(W=W.data_ptr(), packed=1, K=64, N=64, colsum_ws=cs.data_ptr())
    c.layers[1] = S.ChainLayer(W=W.data_ptr(), packed=1, K=64, N=64)  # no column sums here
    with pytest.raises(S.S8LibError, match="column sums"):
        S.chain([c])


def test_reduce_long_sums_one_wave_per_output(S):
    """Reduce jobs with many partials (the bias gradients: one per 128-row tile) run one wave per
    output; mixed in one launch with per-thread jobs, against fp64 sums; deterministic."""
    g = torch.Generator(device="cpu").manual_seed(9)
    jobs, refs = [], []
    for nsplit, n in ((192, 128), (768, 64), (3, 1000), (65, 20), (96, 1)):
        ws = torch.randn(nsplit, n, generator=g).to(dev)
        out = torch.full((n,), 5.0, device=dev)
        jobs.append(S.flat_reduce(ws.data_ptr(), n, out.data_ptr(), n, nsplit))
        refs.append((ws, out))
    S.reduce(jobs)
    torch.cuda.synchronize()
    first = [o.clone() for _, o in refs]
    for ws, out in refs:
        torch.testing.assert_close(out.double(), ws.double().sum(0), rtol=1e-5, atol=1e-5)
    S.reduce(jobs)
    torch.cuda.synchronize()
    assert all(torch.equal(a, o) for a, (_, o) in zip(first, refs))


@pytest.mark.parametrize("B,H,Hc", [(3000, 128, 128), (777, 64, 256)])
def test_loss_heads_tail_equals_last_layers_and_fused_heads(S, B, H, Hc):
    """lgx_loss_heads_tail (the actor's / critic's last layers fused around the PPO head, lgx_mlp
    ABI 9) against its parts: mu = y W^T + b and value = y_c W_c^T + b_c against fp64 on the
    same S8 values (|err| <= 1e-5 sum|y w| + 1e-6); lgx_loss_heads_fused fed those mu / value
    gives the same per-row gradients (dmu, dvalue, their S8 splits, the latent and estimator
    gradients) bit for bit, and the per-block rows it leaves in ws sum to the same losses and dstd
    to fp32 rounding (another block partition);
    the hidden layers' input gradients (dmu W) * ELU'(y) and (dvalue W_c) * ELU'(y_c) against
    fp64 and their 32-row column sums."""
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H_
    g = torch.Generator(device=dev).manual_seed(B + H)
    A, L, E = 12, 20, 3
    r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    y8 = S.to_s8_torch(torch.nn.functional.elu(r(B, H)))
    yc8 = S.to_s8_torch(torch.nn.functional.elu(r(B, Hc)))
    yv, ycv = S.from_s8(y8, B, H).double(), S.from_s8(yc8, B, Hc).double()
    W, b, Wc, bc = 0.1 * r(A, H), r(A), 0.1 * r(1, Hc), r(1)
    std = r(A).abs() + 0.5
    actions, old_logp, adv, tv, ret = r(B, A), r(B, 1), r(B, 1), r(B, 1), r(B, 1)
    old_mu, old_sigma = r(B, A), r(B, A).abs() + 0.5
    p_lat, a_lat, pred, t_est = r(B, L), r(B, L), r(B, E), r(B, E)
    seeds = torch.tensor([1.0, 1.3, -0.01, 0.05, 1.0], device=dev)
    nt, nblk = (B + 31) // 32, (B + 255) // 256
    z = lambda *s: torch.full(s, float("nan"), device=dev)  # noqa: E731

    def run(tail, mu=None, value=None):
        o = dict(ws=torch.zeros(19 * nt, device=dev), wsa=torch.zeros(2 * nt, device=dev), out=z(8), out_aux=z(2),
                 dmu=z(B, A), dvalue=z(B), dstd=z(A), dp=z(B, L), de=z(B, E),
                 cnt=torch.zeros(1, dtype=torch.int32, device=dev), cnta=torch.zeros(1, dtype=torch.int32, device=dev),
                 dmu8=S.empty(B, A, dev), dv8=S.empty(B, 1, dev), de8=S.empty(B, E, dev),
                 cs_mu=z(nt if tail else nblk, A), cs_v=z(nt if tail else nblk, 1), cs_e=z(nblk, E),
                 mu=z(B, A) if mu is None else mu, value=z(B, 1) if value is None else value)
        h = H_.HeadArgs(mu=o["mu"].data_ptr(), value=o["value"].data_ptr(), std=std.data_ptr(),
                        actions=actions.data_ptr(), old_logp=old_logp.data_ptr(), adv=adv.data_ptr(),
                        target_values=tv.data_ptr(), returns=ret.data_ptr(), old_mu=old_mu.data_ptr(),
                        old_sigma=old_sigma.data_ptr(), B=B, A=A, clip=0.2, clipped_value=1, out=o["out"].data_ptr(),
                        g=seeds.data_ptr(), dmu=o["dmu"].data_ptr(), dvalue=o["dvalue"].data_ptr(),
                        dstd=o["dstd"].data_ptr(), ws=o["ws"].data_ptr(), counter=o["cnt"].data_ptr(),
                        accumulate_dstd=0)
        x = H_.AuxArgs(p=p_lat.data_ptr(), a=a_lat.data_ptr(), L=L, e=pred.data_ptr(), t=t_est.data_ptr(), E=E, B=B,
                       out=o["out_aux"].data_ptr(), g=seeds.data_ptr() + 12, dp=o["dp"].data_ptr(),
                       de=o["de"].data_ptr(), ws=o["wsa"].data_ptr(), counter=o["cnta"].data_ptr(), ld_p=L)
        s8 = H_.HeadsS8Args(dmu_s8=o["dmu8"].data_ptr(), ld_dmu=o["dmu8"].shape[1], dmu_cs=o["cs_mu"].data_ptr(),
                            dvalue_s8=o["dv8"].data_ptr(), ld_dvalue=o["dv8"].shape[1], dvalue_cs=o["cs_v"].data_ptr(),
                            de_s8=o["de8"].data_ptr(), ld_de=o["de8"].shape[1], de_cs=o["cs_e"].data_ptr())
        if tail:
            o.update(dy8=S.empty(B, H, dev), dyc8=S.empty(B, Hc, dev), cs_y=z(nt, H), cs_yc=z(nt, Hc))
            t = H_.HeadsTailArgs(y=y8.data_ptr(), ld_y=y8.shape[1], W=W.data_ptr(), b=b.data_ptr(),
                                 dy=o["dy8"].data_ptr(), ld_dy=o["dy8"].shape[1], dy_cs=o["cs_y"].data_ptr(),
                                 yc=yc8.data_ptr(), ld_yc=yc8.shape[1], Wc=Wc.data_ptr(), bc=bc.data_ptr(),
                                 dyc=o["dyc8"].data_ptr(), ld_dyc=o["dyc8"].shape[1], dyc_cs=o["cs_yc"].data_ptr(),
                                 mu_out=o["mu"].data_ptr(), value_out=o["value"].data_ptr(), H=H, Hc=Hc)
            H_._check(H_.lib().lgx_loss_heads_tail(H_.C.byref(h), H_.C.byref(x), H_.C.byref(s8), H_.C.byref(t),
                                                   H_._stream()), "tail")
        else:
            H_._check(H_.lib().lgx_loss_heads_fused(H_.C.byref(h), H_.C.byref(x), H_.C.byref(s8), H_._stream()),
                      "fused")
        torch.cuda.synchronize()
        return o

    got = run(True)
    mu_ref = yv @ W.double().t() + b.double()
    v_ref = ycv @ Wc.double().t() + bc.double()
    assert (got["mu"].double() - mu_ref).abs().le(1e-5 * (yv.abs() @ W.double().abs().t()) + 1e-6).all()
    assert (got["value"].double() - v_ref).abs().le(1e-5 * (ycv.abs() @ Wc.double().abs().t()) + 1e-6).all()
    ref = run(False, mu=got["mu"].clone(), value=got["value"].clone())
    for k in ("dmu", "dvalue", "dp", "de", "dmu8", "dv8", "de8", "cs_e", "out_aux"):
        assert torch.equal(got[k], ref[k]), k
    # the head's totals are the caller's flat sums of the per-block rows (no last-block pass)
    rows = got["ws"].view(-1, 19)[:nt].double()
    assert torch.equal(got["out"][2], ref["out"][2])  # the entropy, written by block 0
    torch.testing.assert_close(rows[:, :3].sum(0), ref["out"][[0, 1, 3]].double(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rows[:, 3:3 + A].sum(0), ref["dstd"].double(), rtol=1e-5, atol=1e-6)
    dmu, dv = got["dmu"].double(), got["dvalue"].double().view(B, 1)
    for dy8, yy, WW, dd, cs, n in ((got["dy8"], yv, W, dmu, got["cs_y"], H), (got["dyc8"], ycv, Wc, dv, got["cs_yc"], Hc)):
        ref_dy = (dd @ WW.double()) * torch.where(yy > 0, torch.ones_like(yy), yy + 1.0)
        got_dy = S.from_s8(dy8, B, n).double()
        bound = 1e-5 * ((dd.abs() @ WW.double().abs()) * (yy.abs() + 1)) + 1e-6
        assert (got_dy - ref_dy).abs().le(bound).all(), float((got_dy - ref_dy).abs().max())
        blocks = torch.stack([ref_dy[i:i + 32].sum(0) for i in range(0, B, 32)])
        torch.testing.assert_close(cs.double(), blocks, rtol=1e-4, atol=1e-5)
    for cs, full in ((got["cs_mu"], dmu), (got["cs_v"], dv)):
        blocks = torch.stack([full[i:i + 32].sum(0) for i in range(0, B, 32)])
        torch.testing.assert_close(cs.double(), blocks, rtol=1e-5, atol=1e-6)
