"""ctypes binding of liblgx_s8.so (include/lgx_s8.h): the learner's GEMM core on pre-split
(S8) operands — forward, input-gradient and weight-gradient GEMMs whose operands are stored as
bf16 hi/lo planes (interleaved per 8 columns) by the kernels that produce them.

S8 buffers are torch int32 tensors [rows_pad, ld] (4 bytes per logical fp32 element):
ld = round_up(cols, 64), rows_pad = round_up(rows, 64) (the GEMMs' K step is 32 or 64), allocated
zeroed (pad rows/columns stay zero: the GEMMs rely on it, see the header's operand contract)."""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("LGX_S8_LIB") or os.path.join(os.path.dirname(os.path.dirname(_HERE)), "lib", "liblgx_s8.so")  # env: A/B builds
_lib = None

ABI_VERSION = 4
FWD, DX, DW = 0, 1, 2
EPI_BIAS, EPI_ELU, EPI_DELU, EPI_ACCUM = 1, 2, 4, 8
GROUP_MAX = 20
BATCH_MAX = 48
TILE_M = 64  # rows of one FWD / DX column-sum partial (lgx_s8.h LGX_S8_TILE_M)
SPLIT_ROWS = 256
EXPORTED = ("lgx_s8_abi_version", "lgx_s8_sizeof_gemm_args", "lgx_s8_last_error", "lgx_s8_gemm_group",
            "lgx_s8_pick_split", "lgx_s8_split", "lgx_s8_reduce", "lgx_s8_act", "lgx_s8_act_last_error",
            "lgx_s8_sizeof_act_args", "lgx_s8_act_pack", "lgx_s8_sizeof_act_pack_args", "lgx_s8_chain",
            "lgx_s8_sizeof_chain_args")
CHAIN_MAX, CHAIN_MAXL, CHAIN_MAXW = 4, 3, 256
ACT_ROWS, ACT_MAXIN, ACT_MAXH, ACT_MAXENC, ACT_MAXL = 32, 640, 512, 256, 6

vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64


class GemmArgs(C.Structure):
    _fields_ = [("A", vp), ("lda", i64), ("B", vp), ("ldb", i64), ("M", i32), ("N", i32), ("K", i32),
                ("epilogue", i32), ("C", vp), ("ldc", i64), ("C32", vp), ("ldc32", i64), ("bias", vp),
                ("act", vp), ("ld_act", i64), ("addend", vp), ("ld_add", i64), ("add_cols", i32),
                ("colsum_ws", vp), ("split", i32), ("pad0", i32)]


class SplitArgs(C.Structure):
    _fields_ = [("src", vp), ("ld_src", i64), ("dst", vp), ("ld_dst", i64), ("rows", i32), ("cols", i32),
                ("colsum_ws", vp), ("idx", vp), ("packed_steps", i32), ("transpose", i32)]


class ReduceArgs(C.Structure):
    _fields_ = [("ws", vp), ("stride", i64), ("ld_ws", i64), ("out", vp), ("ld_out", i64), ("rows", i32),
                ("cols", i32), ("nsplit", i32), ("accumulate", i32)]


class ActLayer(C.Structure):
    _fields_ = [("W", vp), ("ldw", i64), ("b", vp), ("K", i32), ("N", i32), ("elu", i32), ("pad0", i32)]


class ActPackArgs(C.Structure):
    _fields_ = [("W", vp), ("ld", i64), ("dst", vp), ("N", i32), ("steps", i32), ("nspans", i32),
                ("span_c0", i32 * 4), ("span_p0", i32 * 4), ("span_w", i32 * 4)]


class ActArgs(C.Structure):
    _fields_ = [("B", i32), ("width", i32), ("obs", vp), ("ld_obs", i64), ("n_obs", i32), ("priv_obs", vp),
                ("ld_priv", i64), ("n_priv_in", i32), ("scan_obs", vp), ("ld_scan", i64), ("n_scan_in", i32),
                ("critic_obs", vp), ("ld_critic", i64), ("n_critic_in", i32), ("est_c0", i32), ("seg", i32 * 4),
                ("est", ActLayer * 6), ("scan", ActLayer * 6), ("priv", ActLayer * 6), ("actor", ActLayer * 6),
                ("critic", ActLayer * 6), ("n_est", i32), ("n_scan", i32), ("n_priv", i32), ("n_actor", i32),
                ("n_critic", i32), ("mu", vp), ("ld_mu", i64), ("value", vp), ("obs_st", vp), ("priv_st", vp),
                ("scan_st", vp), ("critic_st", vp), ("est_st", vp), ("est_obs", vp), ("ld_est", i64),
                ("n_est_obs", i32), ("pad1", i32), ("part_src", vp * 3), ("part_ld", i64 * 3), ("part_w", i32 * 3),
                ("nets", i32), ("std", vp), ("eps", vp), ("actions", vp), ("mu_st", vp), ("sigma_st", vp),
                ("logp_st", vp), ("actions_copy", vp), ("step_dev", vp), ("seed", C.c_uint64), ("env_offset", i64)]


class ChainLayer(C.Structure):
    _fields_ = [("W", vp), ("ldw", i64), ("bias", vp), ("C", vp), ("ldc", i64), ("C32", vp), ("ldc32", i64),
                ("act", vp), ("ld_act", i64), ("colsum_ws", vp), ("K", i32), ("N", i32), ("elu", i32), ("packed", i32)]


class ChainArgs(C.Structure):
    _fields_ = [("A", vp), ("lda", i64), ("rows", i32), ("nlayers", i32), ("layers", ChainLayer * 3)]


def flat_reduce(ws, stride, out, n, nsplit, accumulate=0):
    """ReduceArgs for out[i] (+)= sum_s ws[s * stride + i], i < n (raw addresses)."""
    return ReduceArgs(ws=ws, stride=stride, ld_ws=n, out=out, ld_out=n, rows=1, cols=n, nsplit=nsplit,
                      accumulate=accumulate)


class S8LibError(RuntimeError):
    pass


def load(path=_LIB_PATH):
    """A liblgx_s8 handle (the product library by default; dev tools load build variants)."""
    if not os.path.exists(path):
        raise S8LibError(f"liblgx_s8.so not built ({path}); run `python -m legged_gym_custom_amd.build_native`")
    L = C.CDLL(path)
    L.lgx_s8_abi_version.restype = i32
    L.lgx_s8_sizeof_gemm_args.restype = i32
    L.lgx_s8_last_error.restype = C.c_char_p
    L.lgx_s8_gemm_group.argtypes = [vp, i32, i32, vp]
    L.lgx_s8_gemm_group.restype = i32
    L.lgx_s8_pick_split.argtypes = [vp, vp, vp, i32, vp]
    L.lgx_s8_pick_split.restype = i32
    for fn in ("lgx_s8_split", "lgx_s8_reduce"):
        getattr(L, fn).argtypes = [vp, i32, vp]
        getattr(L, fn).restype = i32
    L.lgx_s8_act.argtypes = [vp, vp]
    L.lgx_s8_act.restype = i32
    L.lgx_s8_act_last_error.restype = C.c_char_p
    L.lgx_s8_sizeof_act_args.restype = i32
    L.lgx_s8_act_pack.argtypes = [vp, i32, vp]
    L.lgx_s8_act_pack.restype = i32
    L.lgx_s8_sizeof_act_pack_args.restype = i32
    L.lgx_s8_chain.argtypes = [vp, i32, vp]
    L.lgx_s8_chain.restype = i32
    L.lgx_s8_sizeof_chain_args.restype = i32
    if L.lgx_s8_abi_version() != ABI_VERSION:
        raise S8LibError("liblgx_s8 ABI version mismatch; rebuild")
    if L.lgx_s8_sizeof_gemm_args() != C.sizeof(GemmArgs):
        raise S8LibError(f"lgx_s8_gemm_args layout mismatch: C {L.lgx_s8_sizeof_gemm_args()} vs ctypes "
                         f"{C.sizeof(GemmArgs)}")
    if L.lgx_s8_sizeof_act_pack_args() != C.sizeof(ActPackArgs):
        raise S8LibError("lgx_s8_act_pack_args layout mismatch")
    if L.lgx_s8_sizeof_chain_args() != C.sizeof(ChainArgs):
        raise S8LibError("lgx_s8_chain_args layout mismatch")
    if L.lgx_s8_sizeof_act_args() != C.sizeof(ActArgs):
        raise S8LibError(f"lgx_s8_act_args layout mismatch: C {L.lgx_s8_sizeof_act_args()} vs ctypes "
                         f"{C.sizeof(ActArgs)}")
    return L


def lib():
    global _lib
    if _lib is None:
        _lib = load()
    return _lib


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise S8LibError(f"{what}: " + lib().lgx_s8_last_error().decode())


def _ptr(t):
    return None if t is None else t.data_ptr()


def rup(x, m):
    return (x + m - 1) // m * m


# ------------------------------------------------------------------ S8 buffers
def empty(rows, cols, device, ld=None):
    """A zeroed S8 buffer for a logical [rows, cols] fp32 matrix (int32 storage)."""
    ld = rup(max(cols, 1), 64) if ld is None else ld
    return torch.zeros(rup(max(rows, 1), 64), ld, dtype=torch.int32, device=device)


def group_ptr(buf, col):
    """Address of S8 column `col` (a multiple of 8) of row 0."""
    if col % 8:
        raise S8LibError("S8 column offsets are multiples of 8")
    return buf.data_ptr() + 4 * col


def to_s8_torch(x, ld=None, rows_pad=None):
    """Reference split in torch (tests): x [rows, cols] fp32 -> S8 int32 [rows_pad, ld]."""
    rows, cols = x.shape
    ld = rup(cols, 64) if ld is None else ld
    rows_pad = rup(rows, 64) if rows_pad is None else rows_pad
    xp = torch.zeros(rows_pad, ld, dtype=torch.float32, device=x.device)
    xp[:rows, :cols] = x
    hi = xp.to(torch.bfloat16)
    lo = (xp - hi.float()).to(torch.bfloat16)
    g = torch.stack([hi.view(rows_pad, ld // 8, 8), lo.view(rows_pad, ld // 8, 8)], dim=2)  # [r, G, 2, 8]
    return g.reshape(rows_pad, ld * 2).view(torch.int32).contiguous()


def from_s8(buf, rows, cols, col0=0):
    """hi + lo of an S8 buffer's [rows, cols] span starting at column col0 (fp32)."""
    r, ld = buf.shape
    b = buf.view(torch.bfloat16).view(r, ld // 8, 2, 8).float()
    x = (b[:, :, 0, :] + b[:, :, 1, :]).reshape(r, ld)
    return x[:rows, col0:col0 + cols]


def planes(buf, rows, cols, col0=0):
    """(hi, lo) fp32 views of the bf16 planes of an S8 span (tests)."""
    r, ld = buf.shape
    b = buf.view(torch.bfloat16).view(r, ld // 8, 2, 8).float()
    hi = b[:, :, 0, :].reshape(r, ld)[:rows, col0:col0 + cols]
    lo = b[:, :, 1, :].reshape(r, ld)[:rows, col0:col0 + cols]
    return hi, lo


# ------------------------------------------------------------------ launches
def gemm_group(args, kind, L=None):
    L = lib() if L is None else L
    for i in range(0, len(args), GROUP_MAX):
        chunk = args[i:i + GROUP_MAX]
        arr = (GemmArgs * len(chunk))(*chunk)
        _check(L.lgx_s8_gemm_group(arr, len(chunk), kind, _stream()), "lgx_s8_gemm_group")


def pick_split(shapes, L=None):
    n = len(shapes)
    Iv = C.c_int32 * n
    Ms, Ns, Ks, out = Iv(*[s[0] for s in shapes]), Iv(*[s[1] for s in shapes]), Iv(*[s[2] for s in shapes]), Iv()
    _check((L or lib()).lgx_s8_pick_split(Ms, Ns, Ks, n, out), "lgx_s8_pick_split")
    return list(out)


def split(jobs):
    """jobs: [SplitArgs]."""
    for i in range(0, len(jobs), BATCH_MAX):
        chunk = jobs[i:i + BATCH_MAX]
        arr = (SplitArgs * len(chunk))(*chunk)
        _check(lib().lgx_s8_split(arr, len(chunk), _stream()), "lgx_s8_split")


def reduce(jobs, L=None):
    """jobs: [ReduceArgs]."""
    L = lib() if L is None else L
    for i in range(0, len(jobs), BATCH_MAX):
        chunk = jobs[i:i + BATCH_MAX]
        arr = (ReduceArgs * len(chunk))(*chunk)
        _check(L.lgx_s8_reduce(arr, len(chunk), _stream()), "lgx_s8_reduce")


def chain(chains, L=None):
    """lgx_s8_chain: up to CHAIN_MAX narrow forward chains in one launch ([ChainArgs])."""
    L = lib() if L is None else L
    arr = (ChainArgs * len(chains))(*chains)
    _check(L.lgx_s8_chain(arr, len(chains), _stream()), "lgx_s8_chain")


def act(args, L=None):
    """lgx_s8_act: the rollout's act networks in one launch (ActArgs)."""
    L = lib() if L is None else L
    if L.lgx_s8_act(C.byref(args), _stream()) != 0:
        raise S8LibError("lgx_s8_act: " + L.lgx_s8_act_last_error().decode())


def act_pack(jobs, L=None):
    """lgx_s8_act_pack: fp32 weights -> the act kernel's packed S8 fragments ([ActPackArgs])."""
    L = lib() if L is None else L
    for i in range(0, len(jobs), BATCH_MAX):
        chunk = jobs[i:i + BATCH_MAX]
        arr = (ActPackArgs * len(chunk))(*chunk)
        if L.lgx_s8_act_pack(arr, len(chunk), _stream()) != 0:
            raise S8LibError("lgx_s8_act_pack: " + L.lgx_s8_act_last_error().decode())


def packed_empty(N, K, device):
    """A zeroed fragment-packed S8 weight buffer for [N, K] (lgx_s8_chain_layer.packed)."""
    return torch.zeros((N + 15) // 16 * ((K + 31) // 32) * 512, dtype=torch.int32, device=device)


def split_packed_job(W, dst, transpose=False):
    """SplitArgs: fp32 weight [N, K] -> its fragment-packed S8 copy (packed_empty(N, K)), or with
    transpose its transpose's (packed_empty(K, N): an input-gradient chain's B operand)."""
    if W.stride(1) != 1 or W.dtype != torch.float32:
        raise S8LibError("split: fp32 with unit column stride")
    rows, cols = (W.shape[1], W.shape[0]) if transpose else W.shape
    return SplitArgs(src=W.data_ptr(), ld_src=W.stride(0), dst=dst.data_ptr(), ld_dst=0, rows=rows, cols=cols,
                     packed_steps=(cols + 31) // 32, transpose=int(transpose))


def split_job(src, dst_ptr, ld_dst, colsum_ws=None, idx=None, rows=None):
    """SplitArgs for an fp32 [rows, cols] view (unit column stride) into S8 at dst_ptr; with idx
    (int64 [rows]) dst row r is src row idx[r]."""
    if src.stride(1) != 1 or src.dtype != torch.float32:
        raise S8LibError("split: fp32 with unit column stride")
    if idx is not None and (idx.dtype != torch.int64 or not idx.is_contiguous()):
        raise S8LibError("split: idx must be contiguous int64")
    return SplitArgs(src=src.data_ptr(), ld_src=src.stride(0), dst=dst_ptr, ld_dst=ld_dst,
                     rows=src.shape[0] if rows is None else rows, cols=src.shape[1], colsum_ws=_ptr(colsum_ws),
                     idx=_ptr(idx))


def to_s8(x, buf=None):
    """x [rows, cols] fp32 (device) -> S8 buffer via lgx_s8_split."""
    if buf is None:
        buf = empty(x.shape[0], x.shape[1], x.device)
    split([split_job(x, buf.data_ptr(), buf.shape[1])])
    return buf
