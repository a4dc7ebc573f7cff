"""HIP MLP: the rsl_rl networks' Linear/ELU chains on liblgx_mlp.so (include/lgx_mlp.h).

`HipMLP` is an nn.Sequential with the reference's exact children ([Linear, act]*, Linear —
rsl_rl/modules/actor_critic.py:64-87, support_networks.py:22-33,60-70,100-112), so
state_dict keys (`actor.0.weight`, ...) and TorchScript-exported layouts are unchanged.
On a HIP device its forward is ONE autograd node for the whole chain:
  forward   per layer  Y = ELU(X W^T + b)          bias + ELU fused in the GEMM epilogue
  backward  per layer  dW, db = dY^T X, sum dY      split-K GEMM, bias grad in the same pass
                       dX = (dY W) * ELU'(X)        ELU' of the previous layer fused
so only each layer's output is kept (ELU'(z) = y > 0 ? 1 : y + 1 from the output y).
On the CPU (the host-side baseline learner) it is the plain nn.Sequential. On a HIP
device a missing liblgx_mlp.so raises: there is no silent torch fallback.
"""
import ctypes as C
import os

import torch
import torch.nn as nn

_LIB_PATH = os.environ.get("LGX_MLP_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "lib", "liblgx_mlp.so")
_lib = None
ABI_VERSION = 11
EPI_BIAS, EPI_ELU, EPI_DELU, EPI_ACCUM = 1, 2, 4, 8
EXPORTED = ["lgx_mlp_abi_version", "lgx_mlp_sizeof_gemm_args", "lgx_mlp_pick_split", "lgx_gemm",
            "lgx_mlp_last_error", "lgx_adam_step", "lgx_ppo_head_forward", "lgx_ppo_head_backward",
            "lgx_copy_batch", "lgx_act_head", "lgx_store_transition", "lgx_splitk_reduce_batch",
            "lgx_aux_loss_forward", "lgx_aux_loss_backward", "lgx_ppo_tail", "lgx_gemm_group",
            "lgx_mlp_pick_split_group", "lgx_gae", "lgx_normalize_advantages",
            "lgx_gather_rows", "lgx_transpose_batch", "lgx_loss_heads_forward", "lgx_loss_heads_backward",
            "lgx_track_episodes", "lgx_chain", "lgx_adaptation_forward", "lgx_loss_heads_fused",
            "lgx_loss_heads_tail", "lgx_adaptation_train", "lgx_clip_adam", "lgx_post_step"]
TAIL_MAX_LOSSES = 8
TAIL_S8_MAX = 32
# dev knob: LGX_TAIL_S8=0 keeps the per-minibatch weight split launch (the optimizer tail then
# writes no S8 copies)
TAIL_S8 = os.environ.get("LGX_TAIL_S8", "1") != "0"
COPY_MAX = 16
SPLITK_MAX = 24
GROUP_MAX = 20
TRANSPOSE_MAX = 24
CHAIN_MAX, CHAIN_MAXL, CHAIN_MAXW = 4, 3, 256
# lgx_chain serves batches of at most CHAIN_ROWS rows (the rollout's 4096-row act pass): at the
# update's 24,576 rows one grouped launch per depth measured faster (profiles/r03_chain.txt).
# Dev knobs: LGX_CHAIN=0 (never chain), LGX_CHAIN_ROWS (the row limit).
USE_CHAIN = os.environ.get("LGX_CHAIN", "1") != "0"
# dev knob: LGX_ADAPT_FUSED=0 runs the no-gradient adaptation encoder as per-layer launches
USE_ADAPT_FUSED = os.environ.get("LGX_ADAPT_FUSED", "1") != "0"
CHAIN_ROWS = int(os.environ.get("LGX_CHAIN_ROWS", "8192"))


class GemmArgs(C.Structure):
    """Mirror of lgx_gemm_args (include/lgx_mlp.h)."""
    _fields_ = [("A", C.c_void_p), ("lda", C.c_int64), ("a_kcontig", C.c_int32),
                ("B", C.c_void_p), ("ldb", C.c_int64), ("b_kcontig", C.c_int32),
                ("C", C.c_void_p), ("ldc", C.c_int64),
                ("M", C.c_int32), ("N", C.c_int32), ("K", C.c_int32), ("epilogue", C.c_int32),
                ("bias", C.c_void_p), ("act", C.c_void_p), ("ld_act", C.c_int64),
                ("split_k", C.c_int32), ("workspace", C.c_void_p), ("colsum", C.c_void_p),
                ("colsum_ws", C.c_void_p), ("defer_reduce", C.c_int32)]


class SplitkDesc(C.Structure):
    """Mirror of lgx_splitk_desc."""
    _fields_ = [("ws", C.c_void_p), ("colsum_ws", C.c_void_p), ("C", C.c_void_p), ("ldc", C.c_int64),
                ("colsum", C.c_void_p), ("M", C.c_int32), ("N", C.c_int32), ("split", C.c_int32),
                ("epilogue", C.c_int32)]


class HeadArgs(C.Structure):
    """Mirror of lgx_ppo_head_args (include/lgx_mlp.h)."""
    _fields_ = [(n, C.c_void_p) for n in ("mu", "value", "std", "actions", "old_logp", "adv", "target_values",
                                          "returns", "old_mu", "old_sigma")] + \
               [("B", C.c_int32), ("A", C.c_int32), ("clip", C.c_float), ("clipped_value", C.c_int32),
                ("out", C.c_void_p), ("g", C.c_void_p), ("dmu", C.c_void_p), ("dvalue", C.c_void_p),
                ("dstd", C.c_void_p), ("ws", C.c_void_p), ("counter", C.c_void_p), ("kl_dst", C.c_void_p),
                ("accumulate_dstd", C.c_int32)]


class AuxArgs(C.Structure):
    """Mirror of lgx_aux_loss_args."""
    _fields_ = [("p", C.c_void_p), ("a", C.c_void_p), ("L", C.c_int32), ("e", C.c_void_p), ("t", C.c_void_p),
                ("E", C.c_int32), ("B", C.c_int32), ("out", C.c_void_p), ("g", C.c_void_p), ("dp", C.c_void_p),
                ("de", C.c_void_p), ("ws", C.c_void_p), ("counter", C.c_void_p), ("ld_p", C.c_int64)]


class HeadsS8Args(C.Structure):
    """Mirror of lgx_heads_s8_args (pitches in S8 elements)."""
    _fields_ = [("dmu_s8", C.c_void_p), ("ld_dmu", C.c_int64), ("dmu_cs", C.c_void_p),
                ("dvalue_s8", C.c_void_p), ("ld_dvalue", C.c_int64), ("dvalue_cs", C.c_void_p),
                ("de_s8", C.c_void_p), ("ld_de", C.c_int64), ("de_cs", C.c_void_p),
                ("decisions_in", C.c_void_p), ("decisions_out", C.c_void_p)]


class HeadsTailArgs(C.Structure):
    """Mirror of lgx_heads_tail_args (ABI 9: the actor's / critic's last layers fused around the
    PPO head; pitches in S8 elements)."""
    _fields_ = [("y", C.c_void_p), ("ld_y", C.c_int64), ("W", C.c_void_p), ("b", C.c_void_p),
                ("dy", C.c_void_p), ("ld_dy", C.c_int64), ("dy_cs", C.c_void_p),
                ("yc", C.c_void_p), ("ld_yc", C.c_int64), ("Wc", C.c_void_p), ("bc", C.c_void_p),
                ("dyc", C.c_void_p), ("ld_dyc", C.c_int64), ("dyc_cs", C.c_void_p),
                ("mu_out", C.c_void_p), ("value_out", C.c_void_p), ("H", C.c_int32), ("Hc", C.c_int32)]


HEADS_TAIL_ROWS = 32  # LGX_HEADS_TAIL_ROWS: rows of one column-sum partial of lgx_loss_heads_tail


class TailArgs(C.Structure):
    """Mirror of lgx_ppo_tail_args."""
    _fields_ = [(n, C.c_void_p) for n in ("grads", "params", "exp_avg", "exp_avg_sq")] + \
               [(n, C.c_int64) for n in ("main_lo", "main_hi", "est_lo", "est_hi", "adapt_lo", "adapt_hi",
                                         "kl_index")] + \
               [(n, C.c_float) for n in ("max_norm", "b1_main", "b2_main", "eps_main", "b1_est", "b2_est", "eps_est",
                                         "est_lr")] + \
               [("desired_kl", C.c_double), ("lr64", C.c_void_p), ("lr32", C.c_void_p), ("step_main", C.c_void_p),
                ("step_est", C.c_void_p), ("loss_ptrs", C.c_void_p * TAIL_MAX_LOSSES), ("sums", C.c_void_p),
                ("nloss", C.c_int32), ("ws", C.c_void_p), ("counter", C.c_void_p), ("s8", C.c_void_p),
                ("n_s8", C.c_int32)]


class TailS8Seg(C.Structure):
    """Mirror of lgx_tail_s8_seg."""
    _fields_ = [("p0", C.c_int64), ("N", C.c_int32), ("K", C.c_int32), ("c0", C.c_int32), ("w", C.c_int32),
                ("dst", C.c_void_p), ("ld", C.c_int32), ("packed", C.c_int32)]


def tail_s8_table(segs):
    """[(p0, N, K, c0, w, dst, ld, packed)] -> the host table lgx_ppo_tail reads (sorted by p0,
    a weight's entries consecutive)."""
    segs = sorted(segs, key=lambda q: q[0])
    return (TailS8Seg * len(segs))(*[TailS8Seg(*q) for q in segs])


class CopyDesc(C.Structure):
    """Mirror of lgx_copy_desc."""
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("nbytes", C.c_int64), ("dst_stride", C.c_int64)]


class ActHeadArgs(C.Structure):
    """Mirror of lgx_act_head_args."""
    _fields_ = [(n, C.c_void_p) for n in ("mean", "std", "eps", "actions", "mu", "sigma", "logp")] + \
               [("B", C.c_int32), ("A", C.c_int32), ("actions_copy", C.c_void_p), ("step_dev", C.c_void_p),
                ("seed", C.c_uint64), ("env_offset", C.c_int64)]


class TransitionArgs(C.Structure):
    """Mirror of lgx_transition_args."""
    _fields_ = [(n, C.c_void_p) for n in ("rewards", "dones", "time_outs", "values", "rewards_out", "dones_out",
                                          "values_out")] + [("gamma", C.c_float), ("B", C.c_int32)]


class TrackArgs(C.Structure):
    """Mirror of lgx_track_args."""
    _fields_ = [(n, C.c_void_p) for n in ("rewards", "dones", "cur_rew", "cur_len", "rew_ring", "len_ring", "ptr",
                                          "n", "ep_a", "ep_b", "ep_sum", "ep_cnt")] + \
        [("N", C.c_int32), ("na", C.c_int32), ("nb", C.c_int32)]


class TransposeDesc(C.Structure):
    """Mirror of lgx_transpose_desc."""
    _fields_ = [("src", C.c_void_p), ("ld", C.c_int64), ("rows", C.c_int32), ("cols", C.c_int32),
                ("dst", C.c_void_p)]


class ChainLayer(C.Structure):
    """Mirror of lgx_chain_layer."""
    _fields_ = [("B", C.c_void_p), ("ldb", C.c_int64), ("C", C.c_void_p), ("ldc", C.c_int64),
                ("K", C.c_int32), ("N", C.c_int32), ("epilogue", C.c_int32), ("bias", C.c_void_p),
                ("act", C.c_void_p), ("ld_act", C.c_int64)]


class ChainDesc(C.Structure):
    """Mirror of lgx_chain_desc."""
    _fields_ = [("A", C.c_void_p), ("lda", C.c_int64), ("rows", C.c_int32), ("nlayers", C.c_int32),
                ("layers", ChainLayer * CHAIN_MAXL)]


class AdaptArgs(C.Structure):
    """Mirror of lgx_adapt_args."""
    _fields_ = [("x", C.c_void_p), ("ldx", C.c_int64), ("B", C.c_int32), ("H", C.c_int32), ("P", C.c_int32),
                ("w0", C.c_void_p), ("b0", C.c_void_p), ("C1", C.c_int32),
                ("w1", C.c_void_p), ("b1", C.c_void_p), ("C2", C.c_int32), ("k1", C.c_int32), ("s1", C.c_int32),
                ("w2", C.c_void_p), ("b2", C.c_void_p), ("C3", C.c_int32), ("k2", C.c_int32), ("s2", C.c_int32),
                ("wf", C.c_void_p), ("bf", C.c_void_p), ("NO", C.c_int32),
                ("out", C.c_void_p), ("ldo", C.c_int64)]


class AdaptTrainArgs(C.Structure):
    """Mirror of lgx_adapt_train_args (ABI 9)."""
    _fields_ = [("f", AdaptArgs), ("target", C.c_void_p), ("ldt", C.c_int64), ("gws", C.c_void_p),
                ("loss_ws", C.c_void_p), ("blocks", C.c_int32)]


ADAPT_TRAIN_ROWS = 16  # rows per chunk of lgx_adaptation_train (lgx_mlp.hip ATR)


def adapt_train_grid(rows, blocks):
    """lgx_adaptation_train's grid for `rows` rows and a `blocks` budget (its partial rows)."""
    nchunk = (rows + ADAPT_TRAIN_ROWS - 1) // ADAPT_TRAIN_ROWS
    chunks = (nchunk + blocks - 1) // blocks
    return (nchunk + chunks - 1) // chunks


def adaptation_train_supported(mod, P):
    """Whether lgx_adaptation_train's tiling covers this encoder (the checks of its C entry point:
    16-row chunks, <= 4 positions after each convolution, the per-wave weight-gradient tiles, the
    fc_encoder fragment in registers, 80 KB of LDS)."""
    H = mod.history_buffer_length
    C1, C2, C3, k1, s1, k2, s2, L1, L2 = _conv_dims(mod, H)
    NO = mod.fc_final[0].weight.shape[0]
    r4 = lambda v: (v + 3) // 4 * 4
    tiles = lambda m, n: ((m + 15) // 16) * ((n + 15) // 16)
    Y0P = C1 | 1
    if L1 < 1 or L2 < 1 or L1 > 4 or L2 > 4 or 4 % ((C1 + 15) // 16) or (P + 3) // 4 > 16:
        return False
    if ADAPT_TRAIN_ROWS * H * P > 36 * 256 or ADAPT_TRAIN_ROWS * NO > 2 * 256:
        return False
    if tiles(C1, P + 1) > 8 or tiles(C2, k1 * Y0P + 1) > 16 or tiles(C3, k2 * C2 + 1) > 4 or \
            tiles(NO, L2 * C3 + 1) > 4:
        return False
    regions = [16 * H * P, 16 * H * Y0P, 16 * L1 * C2, 16 * r4(L2 * C3), 16 * NO, 16 * NO,
               r4(C2) * r4(k1 * Y0P), r4(C3) * r4(k2 * C2), r4(NO) * r4(L2 * C3), C1 + C2 + C3 + NO, 8]
    return 4 * sum(r4(r) for r in regions) <= 80 * 1024


def adaptation_param_order(mod):
    """The adaptation encoder's parameters in lgx_adaptation_train's flat gradient order."""
    return [mod.fc_encoder[0].weight, mod.fc_encoder[0].bias, mod.conv_layers[0].weight, mod.conv_layers[0].bias,
            mod.conv_layers[2].weight, mod.conv_layers[2].bias, mod.fc_final[0].weight, mod.fc_final[0].bias]


def adaptation_train(mod, obs_rows, hist_cols, target, gws, loss_ws, blocks):
    """One DAgger minibatch's forward + loss + backward of the adaptation encoder in ONE launch
    (lgx_adaptation_train): obs_rows [B, >= hist_cols] fp32 (the history = its first hist_cols
    columns, read in place), target [B, NO] (the privileged latent). Writes the per-block gradient
    rows gws [grid, NP] and loss rows loss_ws [grid] (adapt_train_grid)."""
    Bn = obs_rows.shape[0]
    H = mod.history_buffer_length
    P = hist_cols // H
    C1, C2, C3, k1, s1, k2, s2, L1, L2 = _conv_dims(mod, H)
    f_w = mod.fc_final[0].weight
    if L2 * C3 != f_w.shape[1] or obs_rows.stride(1) != 1 or target.stride(1) != 1:
        raise MlpLibError("adaptation_train: layout outside the fused kernel's limits")
    fc_w, fc_b = mod.fc_encoder[0].weight, mod.fc_encoder[0].bias
    W1, W2, Wf = _conv_w(mod.conv_layers[0].weight), _conv_w(mod.conv_layers[2].weight), _final_w(f_w, C3, L2)
    f = AdaptArgs(x=obs_rows.data_ptr(), ldx=obs_rows.stride(0), B=Bn, H=H, P=P, w0=_ptr(fc_w), b0=_ptr(fc_b), C1=C1,
                  w1=_ptr(W1), b1=_ptr(mod.conv_layers[0].bias), C2=C2, k1=k1, s1=s1, w2=_ptr(W2),
                  b2=_ptr(mod.conv_layers[2].bias), C3=C3, k2=k2, s2=s2, wf=_ptr(Wf), bf=_ptr(mod.fc_final[0].bias),
                  NO=f_w.shape[0], out=None, ldo=0)
    t = AdaptTrainArgs(f=f, target=target.data_ptr(), ldt=target.stride(0), gws=gws.data_ptr(),
                       loss_ws=loss_ws.data_ptr(), blocks=blocks)
    _check(lib().lgx_adaptation_train(C.byref(t), _stream()), "lgx_adaptation_train")
    return (W1, W2, Wf)  # keep the re-laid weights alive until the launch has run (stream order)


class GaeArgs(C.Structure):
    """Mirror of lgx_gae_args."""
    _fields_ = [(n, C.c_void_p) for n in ("rewards", "dones", "values", "last_values", "returns", "advantages")] + \
               [("T", C.c_int32), ("N", C.c_int32), ("gamma", C.c_float), ("lam", C.c_float)] + \
               [(n, C.c_void_p) for n in ("moments", "ws", "counter")]


class MlpLibError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise MlpLibError(f"liblgx_mlp.so not built ({_LIB_PATH}); run `python -m legged_gym_custom_amd.build_native`")
    L = C.CDLL(_LIB_PATH)
    L.lgx_mlp_abi_version.restype = C.c_int32
    L.lgx_mlp_pick_split.argtypes = [C.c_int32, C.c_int32, C.c_int32]
    L.lgx_mlp_pick_split.restype = C.c_int32
    L.lgx_gemm.argtypes = [C.c_void_p, C.c_void_p]
    L.lgx_gemm.restype = C.c_int32
    L.lgx_mlp_last_error.restype = C.c_char_p
    vp, f32 = C.c_void_p, C.c_float
    L.lgx_ppo_head_forward.argtypes = [vp, vp]
    L.lgx_ppo_head_forward.restype = C.c_int32
    L.lgx_ppo_head_backward.argtypes = [vp, vp]
    L.lgx_ppo_head_backward.restype = C.c_int32
    L.lgx_adam_step.argtypes = [vp, vp, vp, vp, C.c_int64, vp, f32, f32, f32, f32, vp, vp, vp]
    L.lgx_adam_step.restype = C.c_int32
    L.lgx_clip_adam.argtypes = [vp, vp, vp, vp, C.c_int64, vp, f32, f32, f32, f32, vp, f32, vp, vp]
    L.lgx_clip_adam.restype = C.c_int32
    L.lgx_copy_batch.argtypes = [vp, C.c_int32, vp]
    L.lgx_copy_batch.restype = C.c_int32
    L.lgx_act_head.argtypes = [vp, vp]
    L.lgx_act_head.restype = C.c_int32
    L.lgx_store_transition.argtypes = [vp, vp]
    L.lgx_store_transition.restype = C.c_int32
    L.lgx_track_episodes.argtypes = [vp, vp]
    L.lgx_track_episodes.restype = C.c_int32
    for fn in ("lgx_loss_heads_forward", "lgx_loss_heads_backward"):
        getattr(L, fn).argtypes = [vp, vp, vp]
        getattr(L, fn).restype = C.c_int32
    L.lgx_loss_heads_fused.argtypes = [vp, vp, vp, vp]
    L.lgx_loss_heads_fused.restype = C.c_int32
    L.lgx_loss_heads_tail.argtypes = [vp, vp, vp, vp, vp]
    L.lgx_loss_heads_tail.restype = C.c_int32
    L.lgx_adaptation_train.argtypes = [vp, vp]
    L.lgx_adaptation_train.restype = C.c_int32
    for fn in ("lgx_aux_loss_forward", "lgx_aux_loss_backward", "lgx_ppo_tail"):
        getattr(L, fn).argtypes = [vp, vp]
        getattr(L, fn).restype = C.c_int32
    L.lgx_gemm_group.argtypes = [vp, C.c_int32, vp]
    L.lgx_gemm_group.restype = C.c_int32
    L.lgx_mlp_pick_split_group.argtypes = [vp, vp, vp, C.c_int32, vp]
    L.lgx_mlp_pick_split_group.restype = C.c_int32
    L.lgx_transpose_batch.argtypes = [vp, C.c_int32, vp]
    L.lgx_transpose_batch.restype = C.c_int32
    L.lgx_gather_rows.argtypes = [vp, C.c_int32, vp, C.c_int64, vp]
    L.lgx_gather_rows.restype = C.c_int32
    L.lgx_gae.argtypes = [vp, vp]
    L.lgx_gae.restype = C.c_int32
    L.lgx_normalize_advantages.argtypes = [vp, C.c_int64, vp, C.c_double, vp]
    L.lgx_normalize_advantages.restype = C.c_int32
    L.lgx_splitk_reduce_batch.argtypes = [vp, C.c_int32, vp]
    L.lgx_splitk_reduce_batch.restype = C.c_int32
    L.lgx_chain.argtypes = [vp, C.c_int32, vp]
    L.lgx_chain.restype = C.c_int32
    L.lgx_adaptation_forward.argtypes = [vp, vp]
    L.lgx_adaptation_forward.restype = C.c_int32
    if L.lgx_mlp_abi_version() != ABI_VERSION:
        raise MlpLibError("liblgx_mlp ABI version mismatch; rebuild")
    L.lgx_mlp_sizeof_gemm_args.restype = C.c_int32
    if L.lgx_mlp_sizeof_gemm_args() != C.sizeof(GemmArgs):
        raise MlpLibError(f"lgx_gemm_args layout mismatch: C {L.lgx_mlp_sizeof_gemm_args()} vs ctypes "
                          f"{C.sizeof(GemmArgs)}")
    _lib = L
    return L


def _ptr(t):
    return None if t is None else t.data_ptr()


def _run(args):
    L = lib()
    rc = L.lgx_gemm(C.byref(args), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise MlpLibError("lgx_gemm: " + L.lgx_mlp_last_error().decode())


def _rowmajor(t):
    return t if t.stride(-1) == 1 else t.contiguous()


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise MlpLibError(f"{what}: " + lib().lgx_mlp_last_error().decode())


def copy_batch(dsts, srcs):
    """dst.copy_(src) for each pair (same dtype, contiguous, on the HIP device) in one launch."""
    descs = (CopyDesc * COPY_MAX)()
    n = 0
    for d, x in zip(dsts, srcs):
        if not (d.is_contiguous() and x.is_contiguous()) or d.dtype != x.dtype or d.numel() != x.numel():
            raise MlpLibError("copy_batch: contiguous tensors of equal dtype and size only")
        if n == COPY_MAX:
            _check(lib().lgx_copy_batch(descs, n, _stream()), "lgx_copy_batch")
            n = 0
        descs[n].src, descs[n].dst, descs[n].nbytes = x.data_ptr(), d.data_ptr(), x.numel() * x.element_size()
        n += 1
    _check(lib().lgx_copy_batch(descs, n, _stream()), "lgx_copy_batch")


def gather_rows(srcs, idx, dsts=None):
    """[t.index_select(0, idx) for t in srcs] (contiguous fp32/4-B tensors) in one launch.
    dsts (optional, per source): a preallocated [len(idx), width] destination with unit column
    stride and any row stride (e.g. a column span of a wider buffer), or None for a new
    contiguous tensor. Returns the destinations."""
    if idx.dtype != torch.int64:
        raise MlpLibError("gather_rows: int64 indices only")
    idx = idx.contiguous()
    dsts = list(dsts) if dsts is not None else [None] * len(srcs)
    outs = []
    for t, d in zip(srcs, dsts):
        if d is None:
            d = torch.empty((idx.numel(),) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
        elif (d.dim() != 2 or d.shape[0] != idx.numel() or d.shape[1] * 4 != (t.numel() // max(1, t.shape[0])) * 4
              or d.stride(1) != 1 or d.dtype != t.dtype):
            raise MlpLibError("gather_rows: a destination must be [rows, width] with unit column stride")
        outs.append(d)
    for i in range(0, len(srcs), COPY_MAX):
        chunk = list(zip(srcs[i:i + COPY_MAX], outs[i:i + COPY_MAX]))
        descs = (CopyDesc * COPY_MAX)()
        for k, (x, o) in enumerate(chunk):
            if not x.is_contiguous() or x.element_size() != 4:
                raise MlpLibError("gather_rows: contiguous 4-byte tensors only")
            descs[k].src, descs[k].dst = x.data_ptr(), o.data_ptr()
            descs[k].nbytes = (x.numel() // max(1, x.shape[0])) * 4
            descs[k].dst_stride = o.stride(0) * 4 if o.dim() == 2 else 0
        _check(lib().lgx_gather_rows(descs, len(chunk), idx.data_ptr(), idx.numel(), _stream()), "lgx_gather_rows")
    return outs


def act_head(mean, std, eps, actions, mu, sigma, logp, actions_copy=None, noise=None):
    """a = mean + std * eps and the Normal log-prob row sums, written into storage rows (and
    the actions also into `actions_copy`, e.g. the env's input buffer, when given).
    eps None: `noise` = (seed, step_dev, env_offset) and the kernel draws eps per global env
    and env step (Philox, lgx_mlp.h LGX_ACT_NOISE_STREAM)."""
    B, A = mean.shape
    if actions_copy is not None and (actions_copy.shape != mean.shape or not actions_copy.is_contiguous()):
        raise MlpLibError("act_head: actions_copy must be a contiguous [B, A] buffer")
    if eps is None:
        if noise is None:
            raise MlpLibError("act_head: eps=None needs noise=(seed, step_dev, env_offset)")
        seed, step_dev, off = noise
        if step_dev.dtype != torch.int64 or step_dev.device != mean.device:
            raise MlpLibError("act_head: step_dev must be an int64 tensor on the actions' device")
        extra = (step_dev.data_ptr(), int(seed) & 0xFFFFFFFFFFFFFFFF, int(off))
    else:
        extra = (None, 0, 0)
    args = ActHeadArgs(mean.data_ptr(), std.data_ptr(), None if eps is None else eps.data_ptr(), actions.data_ptr(),
                       mu.data_ptr(), sigma.data_ptr(), logp.data_ptr(), B, A,
                       None if actions_copy is None else actions_copy.data_ptr(), *extra)
    _check(lib().lgx_act_head(C.byref(args), _stream()), "lgx_act_head")


def store_transition(rewards, dones, time_outs, values, rewards_out, dones_out, values_out, gamma, track=None):
    """lgx_store_transition, or with `track` (track_episodes(..., launch=False)'s arguments) the
    step's transition and episode bookkeeping in one lgx_post_step launch."""
    args = TransitionArgs(rewards.data_ptr(), dones.data_ptr(), None if time_outs is None else time_outs.data_ptr(),
                          values.data_ptr(), rewards_out.data_ptr(), dones_out.data_ptr(), values_out.data_ptr(),
                          float(gamma), rewards.shape[0])
    if track is not None:
        _check(lib().lgx_post_step(C.byref(args), C.byref(track), _stream()), "lgx_post_step")
        return
    _check(lib().lgx_store_transition(C.byref(args), _stream()), "lgx_store_transition")


def track_episodes(rewards, dones, st, ep_a=None, ep_b=None, launch=True):
    """lgx_track_episodes on the runner's stats dict (on_policy_runner.py:160-170); with
    launch=False the arguments only (for store_transition's one-launch form)."""
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    args = TrackArgs(rewards.data_ptr(), dones.data_ptr(), st["cur_rew"].data_ptr(), st["cur_len"].data_ptr(),
                     st["rew_ring"].data_ptr(), st["len_ring"].data_ptr(), st["ptr"].data_ptr(), st["n"].data_ptr(),
                     p(ep_a), p(ep_b), p(st["ep_sum"] if ep_a is not None or ep_b is not None else None),
                     p(st["ep_cnt"] if ep_a is not None or ep_b is not None else None), rewards.shape[0],
                     0 if ep_a is None else ep_a.numel(), 0 if ep_b is None else ep_b.numel())
    if not launch:
        return args
    _check(lib().lgx_track_episodes(C.byref(args), _stream()), "lgx_track_episodes")


def gae(rewards, dones, values, last_values, returns, advantages, gamma, lam, moments, ws, counter):
    """lgx_gae over [T, N, 1] storage buffers: returns, raw advantages, fp64 moments[0:2]."""
    T, N = rewards.shape[0], rewards.shape[1]
    for t in (rewards, dones, values, last_values, returns, advantages):
        if not t.is_contiguous():
            raise MlpLibError("gae: contiguous buffers only")
    args = GaeArgs(rewards.data_ptr(), dones.data_ptr(), values.data_ptr(), last_values.data_ptr(), returns.data_ptr(),
                   advantages.data_ptr(), T, N, float(gamma), float(lam), moments.data_ptr(), ws.data_ptr(),
                   counter.data_ptr())
    _check(lib().lgx_gae(C.byref(args), _stream()), "lgx_gae")


def normalize_advantages(advantages, moments, count):
    _check(lib().lgx_normalize_advantages(advantages.data_ptr(), advantages.numel(), moments.data_ptr(), float(count),
                                          _stream()), "lgx_normalize_advantages")


def clip_adam(p, g, m, v, step, lr, beta1, beta2, eps, max_norm, coef_out=None):
    """lgx_clip_adam: clip_grad_norm_(g, max_norm) in place, step += 1 and one Adam step over one
    small flat segment (<= 65536 entries), in one launch; lr: float or 0-dim device tensor."""
    lr_dev = lr.data_ptr() if isinstance(lr, torch.Tensor) else None
    lr_f = 0.0 if isinstance(lr, torch.Tensor) else float(lr)
    _check(lib().lgx_clip_adam(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), g.numel(), lr_dev, lr_f,
                               float(beta1), float(beta2), float(eps), step.data_ptr(), float(max_norm),
                               None if coef_out is None else coef_out.data_ptr(), _stream()), "lgx_clip_adam")


def adam_step(p, g, m, v, step, lr, beta1, beta2, eps, grad_scale=None):
    """lgx_adam_step over flat fp32 segments (views); lr: float or 0-dim device tensor."""
    lr_dev = lr.data_ptr() if isinstance(lr, torch.Tensor) else None
    lr_f = 0.0 if isinstance(lr, torch.Tensor) else float(lr)
    L = lib()
    rc = L.lgx_adam_step(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), lr_dev, lr_f, beta1, beta2,
                         eps, step.data_ptr(), None if grad_scale is None else grad_scale.data_ptr(),
                         C.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise MlpLibError("lgx_adam_step: " + L.lgx_mlp_last_error().decode())


def gemm_raw(A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, M, N, K, epilogue=0, bias=None, act=None, ld_act=0):
    """One lgx_gemm on raw device addresses (ints) — for strided sub-views such as the
    conv1d windows of the adaptation encoder. k-contiguous operands only (split_k 1)."""
    _run(GemmArgs(A=A, lda=lda, a_kcontig=a_kcontig, B=B, ldb=ldb, b_kcontig=b_kcontig, C=C, ldc=ldc,
                  M=M, N=N, K=K, epilogue=epilogue, bias=bias, act=act, ld_act=ld_act, split_k=1))


def weight_grad_raw(G, ldg, X, ldx, rows, N, K, dW, db):
    """dW[N,K] += sum_r G[r*ldg + n] X[r*ldx + k]; db[N] += sum_r G[r*ldg + n] (raw addresses)."""
    split = max(2, int(lib().lgx_mlp_pick_split(N, K, rows)))
    ws = torch.empty(split * N * K + split * N, device=dW.device, dtype=torch.float32)
    _run(GemmArgs(A=G, lda=ldg, a_kcontig=0, B=X, ldb=ldx, b_kcontig=0, C=dW.data_ptr(), ldc=dW.stride(0),
                  M=N, N=K, K=rows, epilogue=EPI_ACCUM, split_k=split, workspace=ws.data_ptr(),
                  colsum=db.data_ptr(), colsum_ws=ws.data_ptr() + 4 * split * N * K))


# ---------------------------------------------------------------------------------------
# Deferred split-K reductions: inside `deferred_splitk()`, every weight-gradient GEMM
# leaves its split partials in its workspace, and the reductions of the whole backward
# pass run as ONE lgx_splitk_reduce_batch launch at exit (same fixed summation order as
# the immediate reduction, so the gradients are bit-identical).
# ---------------------------------------------------------------------------------------
_pending = None  # list of (SplitkDesc fields, workspace tensor, (lo, hi) byte ranges) while deferring


class deferred_splitk:
    def __enter__(self):
        global _pending
        if _pending is not None:
            raise RuntimeError("deferred_splitk does not nest")
        _pending = []
        return self

    def __exit__(self, *exc):
        global _pending
        try:
            if exc[0] is None:
                _flush()
        finally:
            _pending = None
        return False


def _flush():
    global _pending
    items, _pending[:] = list(_pending), []
    for i in range(0, len(items), SPLITK_MAX):
        chunk = items[i:i + SPLITK_MAX]
        descs = (SplitkDesc * SPLITK_MAX)()
        for k, (d, _ws, _rng) in enumerate(chunk):
            descs[k] = d
        _check(lib().lgx_splitk_reduce_batch(descs, len(chunk), _stream()), "lgx_splitk_reduce_batch")


class _immediate:
    """Settle pending reductions and reduce immediately inside (code that reads its
    weight gradients right away, e.g. the adaptation encoder's re-laid conv weights)."""

    def __enter__(self):
        global _pending, _pending_dw
        self._saved = _pending
        self._saved_dw = _pending_dw
        if _pending is not None:
            _flush()
        if _pending_dw is not None:
            _flush_dw()
        _pending = None
        _pending_dw = None

    def __exit__(self, *exc):
        global _pending, _pending_dw
        _pending = self._saved
        _pending_dw = self._saved_dw
        return False


def _overlaps(ranges):
    return any(lo < h and l2 < hi for (lo, hi) in ranges for (_, _, rs) in _pending for (l2, h) in rs)


def run_group(args):
    """lgx_gemm_group over a list of GemmArgs (one kind; chunks of GROUP_MAX)."""
    for i in range(0, len(args), GROUP_MAX):
        chunk = args[i:i + GROUP_MAX]
        arr = (GemmArgs * len(chunk))(*chunk)
        _check(lib().lgx_gemm_group(arr, len(chunk), _stream()), "lgx_gemm_group")


def run_chain(descs):
    """lgx_chain over a list of ChainDesc (chunks of CHAIN_MAX)."""
    for i in range(0, len(descs), CHAIN_MAX):
        chunk = descs[i:i + CHAIN_MAX]
        arr = (ChainDesc * len(chunk))(*chunk)
        _check(lib().lgx_chain(arr, len(chunk), _stream()), "lgx_chain")


def _chain_desc(x, layers):
    """ChainDesc for input x ([rows, K0], unit column stride) and layers
    [(B, C, epilogue, bias, act), ...] (B [N, K] k-contiguous, C [rows, N])."""
    d = ChainDesc(A=_ptr(x), lda=x.stride(0), rows=x.shape[0], nlayers=len(layers))
    for l, (B, Cm, epi, bias, act) in enumerate(layers):
        d.layers[l] = ChainLayer(B=_ptr(B), ldb=B.stride(0), C=_ptr(Cm), ldc=Cm.stride(0), K=B.shape[1],
                                 N=B.shape[0], epilogue=epi, bias=_ptr(bias), act=_ptr(act),
                                 ld_act=0 if act is None else act.stride(0))
    return d


def _narrow(W):
    return W.shape[0] <= CHAIN_MAXW and W.shape[1] <= CHAIN_MAXW


def _chain_start(chains, hs):
    """First depth d0 from which every chain's remaining layers (2..CHAIN_MAXL of them, all
    widths <= CHAIN_MAXW, non-empty input) run as one lgx_chain launch; None if none does."""
    if not USE_CHAIN or len(chains) > CHAIN_MAX or not hs[0].is_cuda or max(h.shape[0] for h in hs) > CHAIN_ROWS:
        return None
    d0 = 0
    for Ws, _b, _f in chains:
        t = len(Ws)
        while t > 0 and _narrow(Ws[t - 1]):
            t -= 1
        d0 = max(d0, t)
    lens = [len(Ws) for Ws, _b, _f in chains]
    if min(lens) - d0 < 1 or max(lens) - d0 < 2 or max(lens) - d0 > CHAIN_MAXL:
        return None
    if d0 == 0 and any(h.shape[1] == 0 for h in hs):
        return None
    return d0


def pick_split_group(shapes):
    """lgx_mlp_pick_split_group for [(M, N, K), ...] (weight-gradient GEMMs of one launch)."""
    n = len(shapes)
    I = C.c_int32 * n
    Ms, Ns, Ks, out = I(*[s[0] for s in shapes]), I(*[s[1] for s in shapes]), I(*[s[2] for s in shapes]), I()
    _check(lib().lgx_mlp_pick_split_group(Ms, Ns, Ks, n, out), "lgx_mlp_pick_split_group")
    return list(out)


# ---------------------------------------------------------------------------------------
# Deferred weight gradients: inside `deferred_weight_grads()` (a whole backward pass), every
# dW/db GEMM is recorded instead of launched; at exit they run as lgx_gemm_group launches
# (all layers of all networks share the grid, split-K chosen for the group: one K chunk,
# one residency wave) followed by one lgx_splitk_reduce_batch.
# ---------------------------------------------------------------------------------------
_pending_dw = None  # [(g, x, dW, db, epilogue, byte ranges)] while deferring


class deferred_weight_grads:
    def __enter__(self):
        global _pending_dw
        if _pending_dw is not None or _pending is not None:
            raise RuntimeError("deferred_weight_grads does not nest")
        _pending_dw = []
        return self

    def __exit__(self, *exc):
        global _pending_dw
        try:
            if exc[0] is None:
                _flush_dw()
        finally:
            _pending_dw = None
        return False


def _flush_dw():
    items, _pending_dw[:] = list(_pending_dw), []
    for i in range(0, len(items), GROUP_MAX):
        chunk = items[i:i + GROUP_MAX]
        shapes = [(g.shape[1], x.shape[1], g.shape[0]) for (g, x, *_r) in chunk]
        splits = pick_split_group(shapes)
        offs, tot = [], 0
        for (N, K, _rows), s in zip(shapes, splits):
            offs.append(tot)
            tot += (s * N * K + s * N + 3) // 4 * 4  # 16-B aligned partial blocks
        ws = torch.empty(tot, device=chunk[0][0].device, dtype=torch.float32)
        args, descs = [], (SplitkDesc * SPLITK_MAX)()
        for k, ((g, x, dW, db, epi, _rng), (N, K, rows), s, o) in enumerate(zip(chunk, shapes, splits, offs)):
            w = ws.data_ptr() + 4 * o
            cw = w + 4 * s * N * K
            args.append(GemmArgs(A=_ptr(g), lda=g.stride(0), a_kcontig=0, B=_ptr(x), ldb=x.stride(0), b_kcontig=0,
                                 C=_ptr(dW), ldc=dW.stride(0), M=N, N=K, K=rows, epilogue=epi, split_k=s,
                                 workspace=w, colsum=_ptr(db), colsum_ws=cw, defer_reduce=1))
            descs[k] = SplitkDesc(ws=w, colsum_ws=cw, C=dW.data_ptr(), ldc=dW.stride(0), colsum=db.data_ptr(), M=N,
                                  N=K, split=s, epilogue=epi)
        run_group(args)
        _check(lib().lgx_splitk_reduce_batch(descs, len(chunk), _stream()), "lgx_splitk_reduce_batch")


def linear_weight_grad(g, x, dW=None, db=None, accumulate=False):
    """dW[N,K] (+)= dY[M,N]^T X[M,K], db[N] (+)= sum_m dY[m,:] (split-K, deterministic order;
    the reduction is deferred inside `deferred_splitk()`, the whole GEMM inside
    `deferred_weight_grads()`)."""
    g = _rowmajor(g)
    x = _rowmajor(x)
    rows, N = g.shape
    K = x.shape[1]
    dev = g.device
    dW = torch.empty(N, K, device=dev, dtype=torch.float32) if dW is None else dW
    db = torch.empty(N, device=dev, dtype=torch.float32) if db is None else db
    if K == 0:
        # a layer on an empty input (ANYmal's scan encoder, num_scan_obs = 0): no weight entries,
        # the bias gradient is sum_rows dY — no GEMM, so no split-K workspace left unwritten
        s = g.sum(0)
        if accumulate:
            db.add_(s)
        else:
            db.copy_(s)
        return dW, db
    if _pending_dw is not None:
        rng = [(dW.data_ptr(), dW.data_ptr() + 4 * (dW.stride(0) * (N - 1) + K)), (db.data_ptr(), db.data_ptr() + 4 * N)]
        if any(lo < h and l2 < hi for (lo, hi) in rng for (*_r, rs) in _pending_dw for (l2, h) in rs):
            _flush_dw()  # an output a recorded GEMM still owes (accumulation): settle those first
        _pending_dw.append((g, x, dW, db, EPI_ACCUM if accumulate else 0, rng))
        return dW, db
    split = max(2, int(lib().lgx_mlp_pick_split(N, K, rows)))
    ws = torch.empty(split * N * K + split * N, device=dev, dtype=torch.float32)
    defer = _pending is not None
    if defer:  # an output an earlier deferred reduction still owes: settle those first
        rng = [(dW.data_ptr(), dW.data_ptr() + 4 * (dW.stride(0) * (N - 1) + K)), (db.data_ptr(), db.data_ptr() + 4 * N)]
        if _overlaps(rng):
            _flush()
    epi = EPI_ACCUM if accumulate else 0
    _run(GemmArgs(A=_ptr(g), lda=g.stride(0), a_kcontig=0, B=_ptr(x), ldb=x.stride(0), b_kcontig=0,
                  C=_ptr(dW), ldc=dW.stride(0), M=N, N=K, K=rows, epilogue=epi,
                  split_k=split, workspace=_ptr(ws), colsum=_ptr(db),
                  colsum_ws=ws.data_ptr() + 4 * split * N * K, defer_reduce=int(defer)))
    if defer:
        d = SplitkDesc(ws=ws.data_ptr(), colsum_ws=ws.data_ptr() + 4 * split * N * K, C=dW.data_ptr(),
                       ldc=dW.stride(0), colsum=db.data_ptr(), M=N, N=K, split=split, epilogue=epi)
        _pending.append((d, ws, rng))
    return dW, db


def linear_forward(x, W, b, elu, out=None):
    """Y[M,N] = act(X[M,K] W[N,K]^T + b)."""
    x = _rowmajor(x)
    M, K = x.shape
    N = W.shape[0]
    y = out if out is not None else torch.empty(M, N, device=x.device, dtype=torch.float32)
    if K == 0:  # nn.Linear on an empty input: the bias on every row
        bb = b.detach()
        return y.copy_((torch.nn.functional.elu(bb) if elu else bb).expand_as(y))
    _run(GemmArgs(A=_ptr(x), lda=x.stride(0), a_kcontig=1, B=_ptr(W), ldb=W.stride(0), b_kcontig=1,
                  C=_ptr(y), ldc=y.stride(0), M=M, N=N, K=K, epilogue=EPI_BIAS | (EPI_ELU if elu else 0),
                  bias=_ptr(b), split_k=1))
    return y


def linear_input_grad(g, W, y_prev=None, Wt=None):
    """dX[M,K] = (dY[M,N] W[N,K]) * ELU'(y_prev) (when the layer input is an ELU output).
    W is read in place: B(k=n_out, n=k_in) = W[n_out, k_in] is n-contiguous (float4 staging
    along n when aligned); pass Wt ([K,N] contiguous) to stream it k-contiguous instead."""
    g = _rowmajor(g)
    M, N = g.shape
    K = W.shape[1]
    dx = torch.empty(M, K, device=g.device, dtype=torch.float32)
    if Wt is None:
        _run(GemmArgs(A=_ptr(g), lda=g.stride(0), a_kcontig=1, B=_ptr(W), ldb=W.stride(0), b_kcontig=0,
                      C=_ptr(dx), ldc=dx.stride(0), M=M, N=K, K=N, epilogue=EPI_DELU if y_prev is not None else 0,
                      act=_ptr(y_prev), ld_act=0 if y_prev is None else y_prev.stride(0), split_k=1))
        return dx
    _run(GemmArgs(A=_ptr(g), lda=g.stride(0), a_kcontig=1, B=_ptr(Wt), ldb=Wt.stride(0), b_kcontig=1,
                  C=_ptr(dx), ldc=dx.stride(0), M=M, N=K, K=N, epilogue=EPI_DELU if y_prev is not None else 0,
                  act=_ptr(y_prev), ld_act=0 if y_prev is None else y_prev.stride(0), split_k=1))
    return dx


def _grad_of(p):
    """The parameter's .grad buffer (created zeroed if absent): the weight-gradient pass
    accumulates into it directly, so autograd has no AccumulateGrad add to run."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


class _MLPFunction(torch.autograd.Function):
    """The whole chain as one autograd node. The chain input is the concatenation of
    `nparts` tensors (the actor's [obs | latent | scan latent | est], actor_critic.py:79):
    the concatenation is built here, and the first layer's input gradient is computed only
    for the column span of the parts that need one (the actor's 55 latent columns, not
    its 627 — obs and est carry no gradient)."""

    @staticmethod
    def forward(ctx, nparts, elu_flags, *args):
        parts, wb = args[:nparts], args[nparts:]
        x = parts[0] if nparts == 1 else torch.cat(parts, dim=-1)
        n = len(elu_flags)
        outs = []
        h = x
        for i in range(n):
            h = linear_forward(h, wb[2 * i], wb[2 * i + 1], elu_flags[i])
            outs.append(h)
        ctx.elu_flags = elu_flags
        ctx.nparts = nparts
        ctx.widths = [t.shape[-1] for t in parts]
        ctx.params = wb  # the leaf Parameters (their .grad is written in backward)
        ctx.save_for_backward(x, *wb, *outs)
        return h

    @staticmethod
    def backward(ctx, grad_out):
        flags = ctx.elu_flags
        n = len(flags)
        np_ = ctx.nparts
        saved = ctx.saved_tensors
        x, wb, outs = saved[0], saved[1:1 + 2 * n], saved[1 + 2 * n:]
        g = grad_out
        if flags[-1]:  # a chain ending in an activation (not built by _mlp): its ELU' on the incoming grad
            y = outs[-1]
            g = g * torch.where(y > 0, torch.ones_like(y), y + 1.0)
        need = [ctx.needs_input_grad[2 + i] for i in range(np_)]
        part_grads = [None] * np_
        for i in reversed(range(n)):
            inp = x if i == 0 else outs[i - 1]
            if ctx.needs_input_grad[2 + np_ + 2 * i] or ctx.needs_input_grad[3 + np_ + 2 * i]:
                linear_weight_grad(g, inp, _grad_of(ctx.params[2 * i]), _grad_of(ctx.params[2 * i + 1]),
                                   accumulate=True)
            if i > 0:
                g = linear_input_grad(g, wb[2 * i], outs[i - 1] if flags[i - 1] else None)
            elif any(need):
                # dX for the columns [lo, hi) spanning the parts that need a gradient: W read in place
                offs = [0]
                for w in ctx.widths:
                    offs.append(offs[-1] + w)
                first = need.index(True)
                last = np_ - 1 - need[::-1].index(True)
                lo, hi = offs[first], offs[last + 1]
                dx = linear_input_grad(g, wb[0][:, lo:hi], None)
                for k in range(first, last + 1):
                    if need[k]:
                        part_grads[k] = dx[:, offs[k] - lo:offs[k + 1] - lo]
        return (None, None, *part_grads) + (None,) * (2 * n)


def mlp_forward(x, weights, biases, elu_flags):
    """Whole chain on the HIP device (autograd-aware). `x` is a tensor, or a tuple of
    tensors whose concatenation along the last dim is the chain input."""
    parts = tuple(x) if isinstance(x, (tuple, list)) else (x,)
    wb = [t for pair in zip(weights, biases) for t in pair]
    needs_graph = torch.is_grad_enabled() and (any(t.requires_grad for t in parts) or
                                               any(t.requires_grad for t in wb))
    if not needs_graph:
        h = parts[0] if len(parts) == 1 else torch.cat(parts, dim=-1)
        for W, b, e in zip(weights, biases, elu_flags):
            h = linear_forward(h, W, b, e)
        return h
    return _MLPFunction.apply(len(parts), tuple(elu_flags), *parts, *wb)


class HipMLP(nn.Sequential):
    """nn.Sequential of [Linear, ELU]* Linear that runs as fused HIP GEMMs on the GPU."""

    def _chain(self):
        layers, flags = [], []
        mods = list(self)
        i = 0
        while i < len(mods):
            m = mods[i]
            if not isinstance(m, nn.Linear) or m.bias is None:
                return None
            act = mods[i + 1] if i + 1 < len(mods) and not isinstance(mods[i + 1], nn.Linear) else None
            if act is not None and not (isinstance(act, nn.ELU) and act.alpha == 1.0):
                return None
            layers.append(m)
            flags.append(act is not None)
            i += 2 if act is not None else 1
        return layers, flags

    def forward(self, x):
        if x.device.type != "cuda":
            return super().forward(x)
        chain = self._chain()
        if chain is None:  # an activation the fused epilogues do not cover (only ELU is built)
            return super().forward(x)
        layers, flags = chain
        return mlp_forward(x, [m.weight for m in layers], [m.bias for m in layers], flags)

    def forward_parts(self, parts):
        """forward(torch.cat(parts, -1)); on the HIP device the concatenation happens inside
        the chain's autograd node, and the input gradient is only formed for the parts that
        require one."""
        chain = self._chain() if parts[0].device.type == "cuda" else None
        if chain is None:
            return self.forward(torch.cat(parts, dim=-1))
        layers, flags = chain
        return mlp_forward(tuple(parts), [m.weight for m in layers], [m.bias for m in layers], flags)


# ---------------------------------------------------------------------------------------
# Independent chains at equal depth in one launch per depth (lgx_gemm_group): the update's
# privileged/scan encoders, critic and estimator (ppo.py:186-206) and the rollout's
# (ppo.py:129-153) read only data, so layer d of every chain shares one grid. Backward
# aligns the chains at their outputs (step t = each chain's layer n - 1 - t): one grouped
# input-gradient launch per step; weight gradients as in _MLPFunction (deferred inside
# deferred_weight_grads()). Forward / input-gradient results equal the per-chain launches
# bit for bit.
# ---------------------------------------------------------------------------------------
def _fwd_args(h, W, b, elu, y):
    M, K = h.shape
    N = W.shape[0]
    return GemmArgs(A=_ptr(h), lda=h.stride(0), a_kcontig=1, B=_ptr(W), ldb=W.stride(0), b_kcontig=1, C=_ptr(y),
                    ldc=y.stride(0), M=M, N=N, K=K, epilogue=EPI_BIAS | (EPI_ELU if elu else 0), bias=_ptr(b),
                    split_k=1)


def _dx_args(g, W, y_prev, dx):
    M, N = g.shape
    K = W.shape[1]
    return GemmArgs(A=_ptr(g), lda=g.stride(0), a_kcontig=1, B=_ptr(W), ldb=W.stride(0), b_kcontig=0, C=_ptr(dx),
                    ldc=dx.stride(0), M=M, N=K, K=N, epilogue=EPI_DELU if y_prev is not None else 0,
                    act=_ptr(y_prev), ld_act=0 if y_prev is None else y_prev.stride(0), split_k=1)


def transpose_batch(mats):
    """[m.t().contiguous() for m in mats] (2-D fp32 views with unit column stride) in one launch."""
    outs = []
    for i in range(0, len(mats), TRANSPOSE_MAX):
        chunk = mats[i:i + TRANSPOSE_MAX]
        descs = (TransposeDesc * TRANSPOSE_MAX)()
        for k, m in enumerate(chunk):
            if m.dim() != 2 or m.stride(1) != 1 or m.dtype != torch.float32:
                raise MlpLibError("transpose_batch: 2-D fp32 with unit column stride only")
            o = torch.empty(m.shape[1], m.shape[0], device=m.device, dtype=torch.float32)
            descs[k] = TransposeDesc(m.data_ptr(), m.stride(0), m.shape[0], m.shape[1], o.data_ptr())
            outs.append(o)
        _check(lib().lgx_transpose_batch(descs, len(chunk), _stream()), "lgx_transpose_batch")
    return outs


def _dxt_args(g, Wt, y_prev, dx):
    """Input gradient dX = (dY W) * ELU'(y_prev) with W^T ([K_in, N_out] contiguous) streamed
    k-contiguous."""
    M, N = g.shape
    return GemmArgs(A=_ptr(g), lda=g.stride(0), a_kcontig=1, B=_ptr(Wt), ldb=Wt.stride(0), b_kcontig=1, C=_ptr(dx),
                    ldc=dx.stride(0), M=M, N=Wt.shape[0], K=N, epilogue=EPI_DELU if y_prev is not None else 0,
                    act=_ptr(y_prev), ld_act=0 if y_prev is None else y_prev.stride(0), split_k=1)


def _group_forward(xs, chains, finals=None):
    """Layer d of every chain in one launch; returns each chain's list of layer outputs.
    finals[c] (optional): where chain c's last layer writes (a [rows, out] span with unit
    column stride, e.g. the latent columns of the actor-input buffer)."""
    outs = [[] for _ in chains]
    hs = [_rowmajor(x) for x in xs]
    d0 = _chain_start(chains, hs)
    depth = max(len(c[2]) for c in chains) if d0 is None else d0
    for d in range(depth):
        args = []
        for c, (Ws, bs, flags) in enumerate(chains):
            if d < len(flags):
                y = finals[c] if finals is not None and finals[c] is not None and d == len(flags) - 1 else None
                if y is not None and (y.shape != (hs[c].shape[0], Ws[d].shape[0]) or y.stride(1) != 1):
                    raise MlpLibError("forward_group: output span shape does not match the chain")
                if y is None:
                    y = torch.empty(hs[c].shape[0], Ws[d].shape[0], device=hs[c].device, dtype=torch.float32)
                if hs[c].shape[1] == 0:
                    # a layer on an empty input (e.g. ANYmal's scan encoder, num_scan_obs = 0):
                    # nn.Linear gives its bias on every row
                    bb = bs[d].detach()
                    y.copy_((torch.nn.functional.elu(bb) if flags[d] else bb).expand_as(y))
                else:
                    args.append(_fwd_args(hs[c], Ws[d], bs[d], flags[d], y))
                outs[c].append(y)
                hs[c] = y
        run_group(args)
    if d0 is not None:  # the narrow tail of every chain: one launch, activations on chip
        descs = []
        for c, (Ws, bs, flags) in enumerate(chains):
            layers = []
            for d in range(d0, len(flags)):
                y = finals[c] if finals is not None and finals[c] is not None and d == len(flags) - 1 else None
                if y is not None and (y.shape != (hs[c].shape[0], Ws[d].shape[0]) or y.stride(1) != 1):
                    raise MlpLibError("forward_group: output span shape does not match the chain")
                if y is None:
                    y = torch.empty(hs[c].shape[0], Ws[d].shape[0], device=hs[c].device, dtype=torch.float32)
                layers.append((Ws[d], y, EPI_BIAS | (EPI_ELU if flags[d] else 0), bs[d], None))
                outs[c].append(y)
            descs.append(_chain_desc(hs[c], layers))
        run_chain(descs)
    return outs


def _concat(parts, buf=None):
    """torch.cat(parts, -1); with `buf` (a [rows, sum of widths] buffer), only the parts not
    already in place inside it are copied (the PPO update keeps the actor's obs and est
    columns in one buffer, so only the two latents move)."""
    if len(parts) == 1 and buf is None:
        return parts[0]
    if buf is None:
        return torch.cat(parts, dim=-1)
    off = 0
    for t in parts:
        w = t.shape[-1]
        dst = buf[:, off:off + w]
        if not (t.data_ptr() == dst.data_ptr() and t.stride() == dst.stride() and t.shape == dst.shape):
            dst.copy_(t)
        off += w
    if off != buf.shape[-1]:
        raise MlpLibError("concat buffer width does not match the parts")
    return buf


class _GroupFn(torch.autograd.Function):
    """Several independent chains as one autograd node. meta: per chain (nparts, flags,
    concat buffer or None, output span or None)."""

    @staticmethod
    def forward(ctx, meta, *flat):
        xs, chains, params, widths = [], [], [], []
        i = 0
        for nparts, flags, buf, _out in meta:
            parts = flat[i:i + nparts]
            i += nparts
            n = len(flags)
            wb = flat[i:i + 2 * n]
            i += 2 * n
            xs.append(_concat(parts, buf))
            chains.append((wb[0::2], wb[1::2], flags))
            params.append(wb)
            widths.append([t.shape[-1] for t in parts])
        outs = _group_forward(xs, chains, [m[3] for m in meta])
        ctx.meta, ctx.params, ctx.widths = tuple((m[0], m[1]) for m in meta), params, widths
        saved = []
        for x, wb, o in zip(xs, params, outs):
            saved += [x, *wb, *o]
        ctx.save_for_backward(*saved)
        return tuple(o[-1] for o in outs)

    @staticmethod
    def backward(ctx, *grad_outs):
        saved = ctx.saved_tensors
        meta = ctx.meta
        st, k, pos, gi = [], 0, 0, 0  # per chain: x, wb, outs, grad, first needs_input_grad index
        for (nparts, flags), g in zip(meta, grad_outs):
            n = len(flags)
            x, wb, outs = saved[k], saved[k + 1:k + 1 + 2 * n], saved[k + 1 + 2 * n:k + 1 + 3 * n]
            k += 1 + 3 * n
            if g is not None and flags[-1]:
                y = outs[-1]
                g = g * torch.where(y > 0, torch.ones_like(y), y + 1.0)
            st.append([x, wb, outs, g, pos])
            pos += nparts + 2 * n
        part_grads = [[None] * nparts for nparts, _f in meta]
        # the weights (or layer-0 column spans) whose input gradient this pass forms, transposed
        # in one launch so the input-gradient GEMMs stream W^T k-contiguous
        need_t, spans = [], {}
        for c, ((nparts, flags), item) in enumerate(zip(meta, st)):
            if item[3] is None:
                continue
            wb = item[1]
            for i in range(1, len(flags)):
                spans[(c, i)] = len(need_t)
                need_t.append(wb[2 * i])
            need = [ctx.needs_input_grad[1 + item[4] + j] for j in range(nparts)]
            if any(need):
                offs = [0]
                for w in ctx.widths[c]:
                    offs.append(offs[-1] + w)
                first, last = need.index(True), nparts - 1 - need[::-1].index(True)
                spans[(c, 0)] = len(need_t)
                need_t.append(wb[0][:, offs[first]:offs[last + 1]])
        wts = transpose_batch(need_t) if need_t else []
        # the input gradients through the chains' narrow tails (layers i >= max(d0, 1), as the
        # forward's lgx_chain) in one launch before the per-depth loop: chained[c] = (first
        # layer covered, {i - 1: dY_{i-1}})
        chained = [None] * len(meta)
        chains_w = [(item[1][0::2], None, flags) for (_n, flags), item in zip(meta, st)]
        d0 = _chain_start(chains_w, [item[0] for item in st]) if all(item[3] is not None for item in st) else None
        if d0 is not None:
            i_stop = max(d0, 1)
            descs = []
            for c, ((_n, flags), item) in enumerate(zip(meta, st)):
                x, wb, outs, g, _p0 = item
                n = len(flags)
                layers, got = [], {}
                for i in range(n - 1, i_stop - 1, -1):
                    dx = torch.empty(g.shape[0], wb[2 * i].shape[1], device=g.device, dtype=torch.float32)
                    yp = outs[i - 1] if flags[i - 1] else None
                    layers.append((wts[spans[(c, i)]], dx, EPI_DELU if yp is not None else 0, None, yp))
                    got[i - 1] = dx
                if layers:
                    descs.append(_chain_desc(_rowmajor(g), layers))
                    chained[c] = (i_stop, got)
            if descs:
                run_chain(descs)
        for t in range(max(len(f) for _n, f in meta)):
            args, news = [], []
            for c, ((nparts, flags), item) in enumerate(zip(meta, st)):
                x, wb, outs, g, p0 = item
                n = len(flags)
                i = n - 1 - t
                if g is None or i < 0:
                    continue
                inp = x if i == 0 else outs[i - 1]
                if ctx.needs_input_grad[1 + p0 + nparts + 2 * i] or ctx.needs_input_grad[2 + p0 + nparts + 2 * i]:
                    linear_weight_grad(g, inp, _grad_of(ctx.params[c][2 * i]), _grad_of(ctx.params[c][2 * i + 1]),
                                       accumulate=True)
                if i > 0 and chained[c] is not None and i >= chained[c][0]:
                    news.append((c, chained[c][1][i - 1]))  # formed by the chain launch
                    continue
                if i > 0:
                    dx = torch.empty(g.shape[0], wb[2 * i].shape[1], device=g.device, dtype=torch.float32)
                    args.append(_dxt_args(g, wts[spans[(c, i)]], outs[i - 1] if flags[i - 1] else None, dx))
                    news.append((c, dx))
                    continue
                need = [ctx.needs_input_grad[1 + p0 + j] for j in range(nparts)]
                if any(need):  # columns [lo, hi) spanning the parts that need a gradient
                    offs = [0]
                    for w in ctx.widths[c]:
                        offs.append(offs[-1] + w)
                    first = need.index(True)
                    last = nparts - 1 - need[::-1].index(True)
                    lo, hi = offs[first], offs[last + 1]
                    dx = torch.empty(g.shape[0], hi - lo, device=g.device, dtype=torch.float32)
                    args.append(_dxt_args(g, wts[spans[(c, 0)]], None, dx))
                    for j in range(first, last + 1):
                        if need[j]:
                            part_grads[c][j] = dx[:, offs[j] - lo:offs[j + 1] - lo]
                item[3] = None
            if args:
                run_group(args)
            for c, dx in news:
                st[c][3] = dx
        res = [None]
        for (nparts, flags), pg in zip(meta, part_grads):
            res += pg + [None] * (2 * len(flags))
        return tuple(res)


def forward_group(items):
    """Outputs of independent chains [(HipMLP, x or tuple of parts[, concat buffer[, output
    span]]), ...], one launch per depth on the HIP device (autograd-aware); elsewhere each
    module's own forward. An output span receives the chain's last layer in place (the update
    writes the encoders' latents straight into the actor-input buffer)."""
    resolved, bufs, finals = [], [], []
    for item in items:
        mod, x = item[0], item[1]
        parts = tuple(x) if isinstance(x, (tuple, list)) else (x,)
        chain = mod._chain() if isinstance(mod, HipMLP) and parts[0].device.type == "cuda" else None
        if chain is None:
            return [it[0].forward_parts(tuple(it[1])) if isinstance(it[1], (tuple, list)) else it[0](it[1])
                    for it in items]
        resolved.append((parts, chain))
        bufs.append(item[2] if len(item) > 2 else None)
        finals.append(item[3] if len(item) > 3 else None)
    wbs = [[t for pair in zip([m.weight for m in layers], [m.bias for m in layers]) for t in pair]
           for _p, (layers, _f) in resolved]
    needs_graph = torch.is_grad_enabled() and any(
        t.requires_grad for (parts, _c), wb in zip(resolved, wbs) for t in (*parts, *wb))
    if not needs_graph:
        xs = [_concat(p, b) for (p, _c), b in zip(resolved, bufs)]
        chains = [([m.weight for m in layers], [m.bias for m in layers], flags) for _p, (layers, flags) in resolved]
        return [o[-1] for o in _group_forward(xs, chains, finals)]
    meta = tuple((len(parts), tuple(flags), b, f) for (parts, (_l, flags)), b, f in zip(resolved, bufs, finals))
    flat = [t for (parts, _c), wb in zip(resolved, wbs) for t in (*parts, *wb)]
    return list(_GroupFn.apply(meta, *flat))


# ---------------------------------------------------------------------------------------
# Adaptation encoder (support_networks.py:116-175): Linear(P->30)+ELU per history step,
# Conv1d(30->20, k4, s2)+ELU, Conv1d(20->10, k2, s1)+ELU, Flatten, Linear(30->out)+ELU.
# Kept channels-last ([B, time, ch]) so every conv1d output position t reads ONE
# contiguous window (k x ch floats at row offset t*stride*ch): a conv is L_out GEMMs on
# strided row views. Weights are re-laid to the window order (tap-major) per call.
# ---------------------------------------------------------------------------------------
def _conv_w(w):
    """Conv1d weight [out, in, k] -> [out, k*in] (tap-major, matches the window layout)."""
    return w.permute(0, 2, 1).reshape(w.shape[0], -1).contiguous()


def _final_w(w, c3, l2):
    """fc_final weight indexed by torch's flatten (c*L + t) -> our (t*C + c) order."""
    return w.reshape(w.shape[0], c3, l2).permute(0, 2, 1).reshape(w.shape[0], -1).contiguous()


def _conv_dims(mod, H):
    c1 = mod.fc_encoder[0].out_features
    conv1, conv2 = mod.conv_layers[0], mod.conv_layers[2]
    k1, s1 = conv1.kernel_size[0], conv1.stride[0]
    k2, s2 = conv2.kernel_size[0], conv2.stride[0]
    L1 = (H - k1) // s1 + 1
    L2 = (L1 - k2) // s2 + 1
    return c1, conv1.out_channels, conv2.out_channels, k1, s1, k2, s2, L1, L2


class _AdaptationFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, dims, want_grad, fc_w, fc_b, c1_w, c1_b, c2_w, c2_b, f_w, f_b):
        global ADAPT_INPLACE_CALLS
        C1, C2, C3, k1, s1, k2, s2, L1, L2 = dims
        Bn, H, P = h.shape
        dev = h.device
        # no gradient wanted and h the first H of Hs > H blocks of a contiguous [B, Hs * P]
        # buffer (the history inside the obs rows): the per-step layer runs on all Hs blocks
        # of every row, read in place, instead of on a packed copy of the H history blocks
        # (the conv windows below only read blocks < H); one copy of B x H x P floats less
        Hs = h.stride(0) // P if h.stride(2) == 1 and h.stride(1) == P and h.stride(0) % P == 0 else 0
        # (ctx.needs_input_grad reports requires_grad whatever the grad mode, so the caller
        # decides: want_grad = grad mode on and some input requires grad)
        inplace = (not want_grad and Hs > H and
                   h.storage_offset() + Bn * Hs * P <= h.untyped_storage().nbytes() // h.element_size())
        # the fused kernel's limits (lgx_adaptation_forward): its intermediates fit 64 KB of LDS
        # for 16 rows, row pitch >= H * P, 32-bit row offsets; beyond them, the per-layer launches
        fits = (16 * (H * C1 + L1 * C2 + L2 * C3) * 4 <= 64 * 1024 and h.stride(0) >= H * P and
                Bn * h.stride(0) <= 2 ** 31 - 1)
        if not want_grad and USE_ADAPT_FUSED and fits and h.stride(2) == 1 and h.stride(1) == P and Bn > 0:
            # no gradient: the whole encoder in one launch (lgx_adaptation_forward), reading the
            # history rows in place; bit-identical to the per-layer launches below
            if inplace:
                ADAPT_INPLACE_CALLS += 1
            W1, W2, Wf = _conv_w(c1_w), _conv_w(c2_w), _final_w(f_w, C3, L2)
            out = torch.empty(Bn, f_w.shape[0], device=dev)
            args = AdaptArgs(x=h.data_ptr(), ldx=h.stride(0), B=Bn, H=H, P=P, w0=_ptr(fc_w), b0=_ptr(fc_b), C1=C1,
                             w1=_ptr(W1), b1=_ptr(c1_b), C2=C2, k1=k1, s1=s1, w2=_ptr(W2), b2=_ptr(c2_b), C3=C3,
                             k2=k2, s2=s2, wf=_ptr(Wf), bf=_ptr(f_b), NO=f_w.shape[0], out=_ptr(out),
                             ldo=out.stride(0))
            _check(lib().lgx_adaptation_forward(C.byref(args), _stream()), "lgx_adaptation_forward")
            ctx.dims = dims
            return out
        if inplace:
            ADAPT_INPLACE_CALLS += 1
            x = h.as_strided((Bn * Hs, P), (P, 1))
        else:
            Hs = H
            x = _rowmajor(h.reshape(Bn * H, P))
        y0 = linear_forward(x, fc_w, fc_b, True)                         # [B, Hs, C1]
        # each conv's output positions are independent GEMMs: one grouped launch per conv
        # (bit-identical to launching them one by one)
        W1 = _conv_w(c1_w)
        y1 = torch.empty(Bn, L1, C2, device=dev)
        run_group([GemmArgs(A=y0.data_ptr() + 4 * t * s1 * C1, lda=Hs * C1, a_kcontig=1, B=W1.data_ptr(),
                            ldb=W1.stride(0), b_kcontig=1, C=y1.data_ptr() + 4 * t * C2, ldc=L1 * C2, M=Bn, N=C2,
                            K=k1 * C1, epilogue=EPI_BIAS | EPI_ELU, bias=c1_b.data_ptr(), split_k=1)
                   for t in range(L1)])
        W2 = _conv_w(c2_w)
        y2 = torch.empty(Bn, L2, C3, device=dev)
        run_group([GemmArgs(A=y1.data_ptr() + 4 * t * s2 * C2, lda=L1 * C2, a_kcontig=1, B=W2.data_ptr(),
                            ldb=W2.stride(0), b_kcontig=1, C=y2.data_ptr() + 4 * t * C3, ldc=L2 * C3, M=Bn, N=C3,
                            K=k2 * C2, epilogue=EPI_BIAS | EPI_ELU, bias=c2_b.data_ptr(), split_k=1)
                   for t in range(L2)])
        Wf = _final_w(f_w, C3, L2)
        out = linear_forward(y2.reshape(Bn, L2 * C3), Wf, f_b, True)
        ctx.dims = dims
        ctx.params = (fc_w, fc_b, c1_w, c1_b, c2_w, c2_b, f_w, f_b)
        if not inplace:  # (the in-place path wants no gradient)
            ctx.save_for_backward(x, y0, y1, y2, out, W1, W2, Wf)
        return out

    @staticmethod
    def backward(ctx, g_out):
        with _immediate():
            return _AdaptationFn._backward(ctx, g_out)

    @staticmethod
    def _backward(ctx, g_out):
        C1, C2, C3, k1, s1, k2, s2, L1, L2 = ctx.dims
        x, y0, y1, y2, out, W1, W2, Wf = ctx.saved_tensors
        fc_w, fc_b, c1_w, c1_b, c2_w, c2_b, f_w, f_b = ctx.params
        Bn = out.shape[0]
        H = y0.shape[0] // Bn
        dev = out.device
        # fc_final (its output ELU first)
        gz = g_out * torch.where(out > 0, torch.ones_like(out), out + 1.0)
        dWf = torch.zeros_like(Wf)
        linear_weight_grad(gz, y2.reshape(Bn, L2 * C3), dWf, _grad_of(f_b), accumulate=True)
        _grad_of(f_w).add_(dWf.reshape(-1, L2, C3).permute(0, 2, 1).reshape(f_w.shape[0], -1))
        g2 = linear_input_grad(gz, Wf, y2.reshape(Bn, L2 * C3))          # [B, L2, C3], pre-activation
        # conv2: per output position t, window t*s2 .. t*s2+k2-1 of y1
        dW2 = torch.zeros_like(W2)
        g1 = torch.zeros(Bn, L1, C2, device=dev)
        W2t = W2.t().contiguous()
        for t in range(L2):
            gp = g2.data_ptr() + 4 * t * C3
            weight_grad_raw(gp, L2 * C3, y1.data_ptr() + 4 * t * s2 * C2, L1 * C2, Bn, C3, k2 * C2, dW2,
                            _grad_of(c2_b))
            gemm_raw(gp, L2 * C3, 1, W2t.data_ptr(), W2t.stride(0), 1, g1.data_ptr() + 4 * t * s2 * C2, L1 * C2,
                     Bn, k2 * C2, C3, EPI_DELU | EPI_ACCUM, act=y1.data_ptr() + 4 * t * s2 * C2, ld_act=L1 * C2)
        _grad_of(c2_w).add_(dW2.reshape(C3, k2, C2).permute(0, 2, 1))
        # conv1
        dW1 = torch.zeros_like(W1)
        g0 = torch.zeros(Bn, H, C1, device=dev)
        W1t = W1.t().contiguous()
        for t in range(L1):
            gp = g1.data_ptr() + 4 * t * C2
            weight_grad_raw(gp, L1 * C2, y0.data_ptr() + 4 * t * s1 * C1, H * C1, Bn, C2, k1 * C1, dW1,
                            _grad_of(c1_b))
            gemm_raw(gp, L1 * C2, 1, W1t.data_ptr(), W1t.stride(0), 1, g0.data_ptr() + 4 * t * s1 * C1, H * C1,
                     Bn, k1 * C1, C2, EPI_DELU | EPI_ACCUM, act=y0.data_ptr() + 4 * t * s1 * C1, ld_act=H * C1)
        _grad_of(c1_w).add_(dW1.reshape(C2, k1, C1).permute(0, 2, 1))
        # fc_encoder over all B*H steps
        g0 = g0.reshape(Bn * H, C1)
        linear_weight_grad(g0, x, _grad_of(fc_w), _grad_of(fc_b), accumulate=True)
        dh = None
        if ctx.needs_input_grad[0]:
            dh = linear_input_grad(g0, fc_w, None).reshape(Bn, H, -1)
        return (dh, None, None) + (None,) * 8


ADAPT_INPLACE_CALLS = 0  # forwards that took the in-place history read (tests check it ran)


def adaptation_forward(mod, hist):
    """AdaptationEncoder.forward on the HIP GEMMs; hist [B, H, P]."""
    H = hist.shape[1]
    dims = _conv_dims(mod, H)
    if dims[8] * dims[2] != mod.fc_final[0].in_features:
        raise ValueError(f"adaptation encoder: flatten size {dims[8] * dims[2]} != fc_final input "
                         f"{mod.fc_final[0].in_features} (the reference assumes history 10, Q17)")
    ps = (mod.fc_encoder[0].weight, mod.fc_encoder[0].bias, mod.conv_layers[0].weight, mod.conv_layers[0].bias,
          mod.conv_layers[2].weight, mod.conv_layers[2].bias, mod.fc_final[0].weight, mod.fc_final[0].bias)
    want_grad = torch.is_grad_enabled() and (hist.requires_grad or any(p.requires_grad for p in ps))
    return _AdaptationFn.apply(hist, dims, want_grad, *ps)


def adaptation_forward_into(mod, hist, out):
    """AdaptationEncoder.forward without gradient in ONE launch (lgx_adaptation_forward), writing
    into `out` ([B, output_dim] fp32, unit column stride, any row stride: e.g. the latent span of
    the fused act kernel's encoder-output buffer). hist [B, H, P] with unit column stride and row
    pitch P (the history inside the obs rows, read in place). Same numbers as adaptation_forward."""
    Bn, H, P = hist.shape
    C1, C2, C3, k1, s1, k2, s2, L1, L2 = dims = _conv_dims(mod, H)
    f_w = mod.fc_final[0].weight
    if dims[8] * dims[2] != f_w.shape[1]:
        raise ValueError("adaptation encoder: flatten size does not match fc_final (history 10, Q17)")
    if (hist.stride(2) != 1 or hist.stride(1) != P or hist.stride(0) < H * P or Bn * hist.stride(0) > 2 ** 31 - 1
            or 16 * (H * C1 + L1 * C2 + L2 * C3) * 4 > 64 * 1024):
        raise MlpLibError("adaptation_forward_into: history layout / sizes outside the fused kernel's limits")
    if out.shape != (Bn, f_w.shape[0]) or out.stride(1) != 1 or out.dtype != torch.float32:
        raise MlpLibError("adaptation_forward_into: out must be fp32 [B, output_dim] with unit column stride")
    fc_w, fc_b = mod.fc_encoder[0].weight, mod.fc_encoder[0].bias
    W1, W2, Wf = _conv_w(mod.conv_layers[0].weight), _conv_w(mod.conv_layers[2].weight), _final_w(f_w, C3, L2)
    args = AdaptArgs(x=hist.data_ptr(), ldx=hist.stride(0), B=Bn, H=H, P=P, w0=_ptr(fc_w), b0=_ptr(fc_b), C1=C1,
                     w1=_ptr(W1), b1=_ptr(mod.conv_layers[0].bias), C2=C2, k1=k1, s1=s1, w2=_ptr(W2),
                     b2=_ptr(mod.conv_layers[2].bias), C3=C3, k2=k2, s2=s2, wf=_ptr(Wf), bf=_ptr(mod.fc_final[0].bias),
                     NO=f_w.shape[0], out=_ptr(out), ldo=out.stride(0))
    _check(lib().lgx_adaptation_forward(C.byref(args), _stream()), "lgx_adaptation_forward")
    return out


# ---------------------------------------------------------------------------------------
# PPO loss head (ppo.py:196-262 over actor_critic.py's Normal(mu, std)): surrogate, clipped
# value loss, entropy and KL as one forward and one backward kernel (lgx_ppo_head_*).
# ---------------------------------------------------------------------------------------
_head_counter = {}


def _counter(dev, kind="head"):
    c = _head_counter.get((dev, kind))
    if c is None:
        c = _head_counter[(dev, kind)] = torch.zeros(1, dtype=torch.int32, device=dev)
    return c


def _seed_vector(gs, dev):
    """The incoming output gradients as one contiguous fp32 vector: read in place when they
    already sit back to back in one buffer (the PPO update's seeds), else stacked."""
    if all(t is not None and t.dtype == torch.float32 and t.numel() == 1 for t in gs):
        p0 = gs[0].data_ptr()
        if all(t.data_ptr() == p0 + 4 * k for k, t in enumerate(gs)):
            return gs[0].as_strided((len(gs),), (1,))
    z = torch.zeros((), device=dev)
    return torch.stack([t if t is not None else z for t in gs]).float().contiguous()


class _PPOHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, value, std, actions, old_logp, adv, target_values, returns, old_mu, old_sigma, clip,
                clipped_value, kl_dst, out):
        B, A = mu.shape
        dev = mu.device
        ts = [_rowmajor(t.reshape(B, -1)) for t in (mu, value, actions, old_logp, adv, target_values, returns, old_mu,
                                                     old_sigma)]
        mu_, value_, actions_, old_logp_, adv_, tv_, ret_, old_mu_, old_sigma_ = ts
        std_ = std.contiguous()
        out = torch.empty(4, device=dev) if out is None else out
        ws = torch.empty(16 * ((B + 63) // 64), device=dev)  # per-block partials, blocks of >= 64 rows
        a = HeadArgs(mu=mu_.data_ptr(), value=value_.data_ptr(), std=std_.data_ptr(), actions=actions_.data_ptr(),
                     old_logp=old_logp_.data_ptr(), adv=adv_.data_ptr(), target_values=tv_.data_ptr(),
                     returns=ret_.data_ptr(), old_mu=old_mu_.data_ptr(), old_sigma=old_sigma_.data_ptr(), B=B, A=A,
                     clip=float(clip), clipped_value=int(bool(clipped_value)), out=out.data_ptr(), ws=ws.data_ptr(),
                     counter=_counter(dev).data_ptr(), kl_dst=None if kl_dst is None else kl_dst.data_ptr())
        L = lib()
        if L.lgx_ppo_head_forward(C.byref(a), C.c_void_p(torch.cuda.current_stream().cuda_stream)) != 0:
            raise MlpLibError("lgx_ppo_head_forward: " + L.lgx_mlp_last_error().decode())
        ctx.save_for_backward(mu_, value_, std_, actions_, old_logp_, adv_, tv_, ret_)
        ctx.std_param = std  # its .grad (a view into the flat gradients) takes dstd in place
        ctx.set_materialize_grads(False)  # the KL output carries no gradient: no zero fill
        ctx.clip, ctx.clipped = float(clip), int(bool(clipped_value))
        ctx.value_shape = value.shape
        ctx.mark_non_differentiable(out)
        return out[0], out[1], out[2], out[3]

    @staticmethod
    def backward(ctx, g_surr, g_value, g_ent, g_kl):
        mu, value, std, actions, old_logp, adv, tv, ret = ctx.saved_tensors
        B, A = mu.shape
        dev = mu.device
        g = _seed_vector((g_surr, g_value, g_ent), dev)
        dmu = torch.empty_like(mu)
        dvalue = torch.empty(B, device=dev)
        sp = ctx.std_param
        direct = sp.requires_grad and sp.is_leaf and sp.grad is not None and sp.grad.is_contiguous() and \
            not sp._backward_hooks
        dstd = sp.grad if direct else torch.empty_like(std)
        ws = torch.empty(16 * ((B + 63) // 64), device=dev)  # per-block partials, blocks of >= 64 rows
        a = HeadArgs(mu=mu.data_ptr(), value=value.data_ptr(), std=std.data_ptr(), actions=actions.data_ptr(),
                     old_logp=old_logp.data_ptr(), adv=adv.data_ptr(), target_values=tv.data_ptr(),
                     returns=ret.data_ptr(), B=B, A=A, clip=ctx.clip, clipped_value=ctx.clipped, g=g.data_ptr(),
                     dmu=dmu.data_ptr(), dvalue=dvalue.data_ptr(), dstd=dstd.data_ptr(), ws=ws.data_ptr(),
                     counter=_counter(dev).data_ptr(), accumulate_dstd=int(direct))
        L = lib()
        if L.lgx_ppo_head_backward(C.byref(a), C.c_void_p(torch.cuda.current_stream().cuda_stream)) != 0:
            raise MlpLibError("lgx_ppo_head_backward: " + L.lgx_mlp_last_error().decode())
        return (dmu, dvalue.view(ctx.value_shape), None if direct else dstd) + (None,) * 11


def ppo_head(mu, value, std, actions, old_logp, adv, target_values, returns, old_mu, old_sigma, clip, clipped_value,
             kl_dst=None, out=None):
    """(surrogate_loss, value_loss, entropy_mean, kl_mean) on the HIP device; kl carries no grad
    (and is also written to `kl_dst`, a 1-element device tensor, when given). `out`: an
    optional persistent [4] buffer the four values are written to (fixed addresses)."""
    return _PPOHeadFn.apply(mu, value, std, actions, old_logp, adv, target_values, returns, old_mu, old_sigma, clip,
                            clipped_value, kl_dst, out)


# ---------------------------------------------------------------------------------------
# ROA regulariser ||z_priv - sg(z_adapt)|| and estimator loss ||e - t||^2 (ppo.py:190-206)
# as one forward and one backward kernel (lgx_aux_loss_*).
# ---------------------------------------------------------------------------------------
class _AuxLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, a, e, t, out):
        p, a, e, t = (_rowmajor(x) for x in (p, a, e, t))
        B, L = p.shape
        E = e.shape[1]
        dev = p.device
        out = torch.empty(2, device=dev) if out is None else out
        ws = torch.empty(2 * ((B + 63) // 64), device=dev)  # per-block partials, blocks of >= 64 rows
        args = AuxArgs(p=p.data_ptr(), a=a.data_ptr(), L=L, e=e.data_ptr(), t=t.data_ptr(), E=E, B=B,
                       out=out.data_ptr(), ws=ws.data_ptr(), counter=_counter(dev, "aux").data_ptr())
        _check(lib().lgx_aux_loss_forward(C.byref(args), _stream()), "lgx_aux_loss_forward")
        ctx.save_for_backward(p, a, e, t)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_reg, g_est):
        p, a, e, t = ctx.saved_tensors
        B, L = p.shape
        dev = p.device
        g = _seed_vector((g_reg, g_est), dev)
        dp = torch.empty_like(p)
        de = torch.empty_like(e)
        args = AuxArgs(p=p.data_ptr(), a=a.data_ptr(), L=L, e=e.data_ptr(), t=t.data_ptr(), E=e.shape[1], B=B,
                       g=g.data_ptr(), dp=dp.data_ptr(), de=de.data_ptr())
        _check(lib().lgx_aux_loss_backward(C.byref(args), _stream()), "lgx_aux_loss_backward")
        return dp, None, de, None, None


def aux_losses(priv_latent, adapt_latent, pred, true_est, out=None):
    """(mean ||priv_latent - adapt_latent||_2, mean ||pred - true_est||_2^2); gradients flow
    to priv_latent and pred only (adapt_latent and true_est are constants). `out`: optional
    persistent [2] buffer for the two values."""
    return _AuxLossFn.apply(priv_latent, adapt_latent.detach(), pred, true_est.detach(), out)


class _LossHeadsFn(torch.autograd.Function):
    """_PPOHeadFn and _AuxLossFn as one autograd node: one launch each way
    (lgx_loss_heads_forward / _backward), the same arguments and results."""

    @staticmethod
    def forward(ctx, mu, value, std, actions, old_logp, adv, target_values, returns, old_mu, old_sigma, p, a, e, t,
                clip, clipped_value, kl_dst, out, out_aux):
        B, A = mu.shape
        dev = mu.device
        ts = [_rowmajor(x.reshape(B, -1)) for x in (mu, value, actions, old_logp, adv, target_values, returns, old_mu,
                                                     old_sigma)]
        mu_, value_, actions_, old_logp_, adv_, tv_, ret_, old_mu_, old_sigma_ = ts
        std_ = std.contiguous()
        p_ = _rowmajor(p)  # row stride passed (ld_p): p may be a column span of the actor-input buffer
        a_, e_, t_ = (x.contiguous() for x in (a, e, t))
        out = torch.empty(4, device=dev) if out is None else out
        out_aux = torch.empty(2, device=dev) if out_aux is None else out_aux
        ws = torch.empty(16 * ((B + 63) // 64), device=dev)  # per-block partials, blocks of >= 64 rows
        ws_aux = torch.empty(2 * ((B + 63) // 64), device=dev)  # per-block partials, blocks of >= 64 rows
        h = HeadArgs(mu=mu_.data_ptr(), value=value_.data_ptr(), std=std_.data_ptr(), actions=actions_.data_ptr(),
                     old_logp=old_logp_.data_ptr(), adv=adv_.data_ptr(), target_values=tv_.data_ptr(),
                     returns=ret_.data_ptr(), old_mu=old_mu_.data_ptr(), old_sigma=old_sigma_.data_ptr(), B=B, A=A,
                     clip=float(clip), clipped_value=int(bool(clipped_value)), out=out.data_ptr(), ws=ws.data_ptr(),
                     counter=_counter(dev).data_ptr(), kl_dst=None if kl_dst is None else kl_dst.data_ptr())
        x = AuxArgs(p=p_.data_ptr(), a=a_.data_ptr(), L=p_.shape[1], e=e_.data_ptr(), t=t_.data_ptr(), E=e_.shape[1],
                    B=B, out=out_aux.data_ptr(), ws=ws_aux.data_ptr(), counter=_counter(dev, "aux").data_ptr(),
                    ld_p=p_.stride(0))
        _check(lib().lgx_loss_heads_forward(C.byref(h), C.byref(x), _stream()), "lgx_loss_heads_forward")
        ctx.save_for_backward(mu_, value_, std_, actions_, old_logp_, adv_, tv_, ret_, p_, a_, e_, t_)
        ctx.std_param = std
        ctx.set_materialize_grads(False)
        ctx.clip, ctx.clipped = float(clip), int(bool(clipped_value))
        ctx.value_shape = value.shape
        ctx.mark_non_differentiable(out, out_aux)
        return out[0], out[1], out[2], out[3], out_aux[0], out_aux[1]

    @staticmethod
    def backward(ctx, g_surr, g_value, g_ent, g_kl, g_reg, g_est):
        mu, value, std, actions, old_logp, adv, tv, ret, p, a, e, t = ctx.saved_tensors
        B, A = mu.shape
        dev = mu.device
        g = _seed_vector((g_surr, g_value, g_ent), dev)
        g_aux = _seed_vector((g_reg, g_est), dev)
        dmu = torch.empty_like(mu)
        dvalue = torch.empty(B, device=dev)
        sp = ctx.std_param
        direct = sp.requires_grad and sp.is_leaf and sp.grad is not None and sp.grad.is_contiguous() and \
            not sp._backward_hooks
        dstd = sp.grad if direct else torch.empty_like(std)
        dp = torch.empty(p.shape, device=dev, dtype=torch.float32)  # contiguous even when p is a span
        de = torch.empty_like(e)
        ws = torch.empty(16 * ((B + 63) // 64), device=dev)  # per-block partials, blocks of >= 64 rows
        h = HeadArgs(mu=mu.data_ptr(), value=value.data_ptr(), std=std.data_ptr(), actions=actions.data_ptr(),
                     old_logp=old_logp.data_ptr(), adv=adv.data_ptr(), target_values=tv.data_ptr(),
                     returns=ret.data_ptr(), B=B, A=A, clip=ctx.clip, clipped_value=ctx.clipped, g=g.data_ptr(),
                     dmu=dmu.data_ptr(), dvalue=dvalue.data_ptr(), dstd=dstd.data_ptr(), ws=ws.data_ptr(),
                     counter=_counter(dev).data_ptr(), accumulate_dstd=int(direct))
        x = AuxArgs(p=p.data_ptr(), a=a.data_ptr(), L=p.shape[1], e=e.data_ptr(), t=t.data_ptr(), E=e.shape[1], B=B,
                    g=g_aux.data_ptr(), dp=dp.data_ptr(), de=de.data_ptr(), ld_p=p.stride(0))
        _check(lib().lgx_loss_heads_backward(C.byref(h), C.byref(x), _stream()), "lgx_loss_heads_backward")
        return (dmu, dvalue.view(ctx.value_shape), None if direct else dstd) + (None,) * 7 + \
            (dp, None, de, None) + (None,) * 5


def loss_heads(mu, value, std, actions, old_logp, adv, target_values, returns, old_mu, old_sigma, clip, clipped_value,
               priv_latent, adapt_latent, pred, true_est, kl_dst=None, out=None, out_aux=None):
    """ppo_head(...) + aux_losses(...) in one launch each way: (surrogate_loss, value_loss,
    entropy_mean, kl_mean, regularisation, estimator_loss)."""
    return _LossHeadsFn.apply(mu, value, std, actions, old_logp, adv, target_values, returns, old_mu, old_sigma,
                              priv_latent, adapt_latent.detach(), pred, true_est.detach(), clip, clipped_value, kl_dst,
                              out, out_aux)


def ppo_tail(grads, params, exp_avg, exp_avg_sq, main, est, adapt, kl_index, max_norm, betas_main, eps_main,
             betas_est, eps_est, est_lr, desired_kl, lr64, lr32, step_main, step_est, loss_ptrs, sums, ws, counter,
             s8=None):
    """lgx_ppo_tail: clip + Adam of both optimizers, the KL schedule and the loss sums
    (one minibatch's optimizer tail, two launches). main/est/adapt: (lo, hi) element ranges.
    s8: optional (table from tail_s8_table, count): the updated weights' S8 copies."""
    a = TailArgs(grads=grads.data_ptr(), params=params.data_ptr(), exp_avg=exp_avg.data_ptr(),
                 exp_avg_sq=exp_avg_sq.data_ptr(), main_lo=main[0], main_hi=main[1], est_lo=est[0], est_hi=est[1],
                 adapt_lo=adapt[0], adapt_hi=adapt[1], kl_index=kl_index, max_norm=max_norm,
                 b1_main=betas_main[0], b2_main=betas_main[1], eps_main=eps_main, b1_est=betas_est[0],
                 b2_est=betas_est[1], eps_est=eps_est, est_lr=est_lr, desired_kl=desired_kl,
                 lr64=lr64.data_ptr(), lr32=lr32.data_ptr(), step_main=step_main.data_ptr(),
                 step_est=step_est.data_ptr(), sums=sums.data_ptr(), nloss=len(loss_ptrs), ws=ws.data_ptr(),
                 counter=counter.data_ptr())
    for k, t in enumerate(loss_ptrs):
        a.loss_ptrs[k] = t.data_ptr()
    if s8 is not None:
        a.s8, a.n_s8 = C.addressof(s8[0]), s8[1]
    _check(lib().lgx_ppo_tail(C.byref(a), _stream()), "lgx_ppo_tail")
