/* lgx_mlp.h — C ABI of liblgx_mlp.so: the learner's fused MLP layer GEMMs on MI355X.
 *
 * Replaces the nn.Linear + nn.ELU chains of the rsl_rl networks
 * (reference rsl_rl/rsl_rl/modules/actor_critic.py:64-87 actor/critic MLPs,
 * support_networks.py:22-33 scan encoder, :60-70 MlpEstimator, :100-112 privileged
 * encoder) in forward (rollout ppo.py:129-153 and update ppo.py:186-201) and backward
 * (loss.backward(), ppo.py:262 / :207).
 *
 * One entry point computes, for row-major fp32 operands,
 *     C[m, n] = epilogue( sum_k A(m, k) * B(k, n) )
 * with A(m,k) = A[m*lda + k] (a_kcontig = 1) or A[k*lda + m] (a_kcontig = 0), and the
 * same for B(k,n) = B[n*ldb + k] (b_kcontig = 1) or B[k*ldb + n] (b_kcontig = 0). So
 *     forward   Y  = X W^T + b       a_kcontig = 1, b_kcontig = 1 (+ bias, ELU)
 *     input grad dX = dY W (* ELU'(Y_prev))   a_kcontig = 1, b_kcontig = 0
 *     weight grad dW = dY^T X, db = sum_rows dY    a_kcontig = 0, b_kcontig = 0, split-K
 * Arithmetic: products in 3 x bf16 MFMA (a = a_hi + a_lo, a_hi*b_hi + a_hi*b_lo +
 * a_lo*b_hi, fp32 accumulation): ~2^-16 relative per product, tighter than the TF32
 * the reference trains with (legged_gym/scripts/train.py:39 set_float32_matmul_precision('high')).
 * All work is stream-ordered on `stream` (hipStream_t); no host synchronisation.
 * Return 0 on success, negative on invalid arguments / launch failure (lgx_mlp_last_error).
 */
#ifndef LGX_MLP_H
#define LGX_MLP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define LGX_MLP_ABI_VERSION 11

enum {
  LGX_EPI_BIAS = 1,  /* + bias[n] */
  LGX_EPI_ELU = 2,   /* then ELU(alpha = 1): v > 0 ? v : expm1(v) */
  LGX_EPI_DELU = 4,  /* * ELU'(z) from the ELU output y = act[m*ld_act + n]: y > 0 ? 1 : y + 1 */
  LGX_EPI_ACCUM = 8  /* C += result (else C = result) */
};

typedef struct lgx_gemm_args {
  const float* A; int64_t lda; int32_t a_kcontig;
  const float* B; int64_t ldb; int32_t b_kcontig;
  float* C; int64_t ldc;
  int32_t M, N, K;
  int32_t epilogue;          /* LGX_EPI_* bits */
  const float* bias;         /* [N] for LGX_EPI_BIAS */
  const float* act; int64_t ld_act;  /* ELU outputs for LGX_EPI_DELU */
  int32_t split_k;           /* >= 1; > 1 needs workspace (split_k * M * N floats) */
  float* workspace;
  float* colsum;             /* optional [M]: sum_k A(m,k) (the bias gradient); needs a_kcontig = 0 */
  float* colsum_ws;          /* split_k * M floats when colsum != NULL */
  int32_t defer_reduce;      /* split_k > 1: leave the partials in workspace/colsum_ws; the
                                caller reduces them later with lgx_splitk_reduce_batch */
} lgx_gemm_args;

int32_t lgx_mlp_abi_version(void);
/* sizeof(lgx_gemm_args) as compiled (binding layout check; no device needed). */
int32_t lgx_mlp_sizeof_gemm_args(void);
/* Suggested split-K factor for an M x N x K weight-gradient GEMM. */
int32_t lgx_mlp_pick_split(int32_t M, int32_t N, int32_t K);
int32_t lgx_gemm(const lgx_gemm_args* args, void* stream);

/* Several independent GEMMs (lgx_gemm semantics each) in ONE launch: the logical output
 * tiles of all entries share the grid, so the small layers of one network depth (or the
 * whole backward pass's weight gradients) fill the chip together instead of one launch
 * each (rsl_rl actor_critic.py:64-87 / support_networks.py: the actor, critic, encoder and
 * estimator chains are independent at equal depth). All entries are of one kind:
 *   forward       a_kcontig = 1, b_kcontig = 1 (split_k 1)
 *   input grad    a_kcontig = 1, b_kcontig = 0 (split_k 1)
 *   weight grad   a_kcontig = 0, b_kcontig = 0, colsum set, split_k >= 2, defer_reduce = 1
 *                 (reduce with lgx_splitk_reduce_batch)
 * Each entry's arithmetic and summation order are those of lgx_gemm with the same split_k
 * (bit-identical results). Entries must not write overlapping outputs. */
#define LGX_GEMM_GROUP_MAX 20
int32_t lgx_gemm_group(const lgx_gemm_args* args, int32_t n, void* stream);
/* The narrow consecutive layers of up to LGX_CHAIN_MAX independent chains in ONE launch
 * (the encoders' and estimator's layers after the first, the actor/critic 256->128->out
 * tails, and the input-gradient passes back through them: rsl_rl actor_critic.py:64-87,
 * support_networks.py:22-112). Layer l of a chain computes, for its `rows` rows,
 *     C_l[m*ldc + n] = epilogue_l( sum_k A_l(m, k) * B_l[n*ldb + k] )
 * with A_0(m, k) = A[m*lda + k] and A_l = C_{l-1} for l > 0 (the previous layer's output,
 * kept on chip between layers and also written to C_{l-1}); K_0 = the chain's input width,
 * K_l = N_{l-1}; every K_l, N_l <= LGX_CHAIN_MAXW. Epilogues: LGX_EPI_BIAS (+ LGX_EPI_ELU)
 * for a forward pass, LGX_EPI_DELU (act = the ELU output at the same rows) for an input-
 * gradient pass over transposed weights. Each layer's arithmetic and summation order are
 * those of lgx_gemm with a_kcontig = b_kcontig = 1, split_k 1: bit-identical results. */
#define LGX_CHAIN_MAX 4
#define LGX_CHAIN_MAXL 3
#define LGX_CHAIN_MAXW 256
typedef struct lgx_chain_layer {
  const float* B; int64_t ldb;       /* [N][K] k-contiguous (W for forward, W^T for input grad) */
  float* C; int64_t ldc;
  int32_t K, N, epilogue;
  const float* bias;
  const float* act; int64_t ld_act;
} lgx_chain_layer;
typedef struct lgx_chain_desc {
  const float* A; int64_t lda;
  int32_t rows, nlayers;             /* 1 <= nlayers <= LGX_CHAIN_MAXL */
  lgx_chain_layer layers[LGX_CHAIN_MAXL];
} lgx_chain_desc;
int32_t lgx_chain(const lgx_chain_desc* chains, int32_t n, void* stream);
/* The adaptation encoder's forward for a pass that needs no gradient (the PPO update's
 * adaptation latents, rsl_rl ppo.py's ROA regulariser; support_networks.py:116-175) in ONE
 * launch: per history position t < H, y0 = ELU(w0 x_t + b0) (Linear P -> C1, x_t = x[r*ldx +
 * t*P ..]); y1 = ELU(Conv1d(C1 -> C2, k1, s1)); y2 = ELU(Conv1d(C2 -> C3, k2, s2)); out =
 * ELU(wf flatten(y2) + bf). Conv weights tap-major [C_out][k*C_in], wf position-major
 * [NO][L2*C3] (hip_mlp._conv_w / _final_w). Only `out` [B][NO] is written; each layer's
 * arithmetic and summation order are those of lgx_gemm (bit-identical to the per-layer
 * launches). Requires 16 * (H*C1 + L1*C2 + L2*C3) floats <= 64 KB. */
typedef struct lgx_adapt_args {
  const float* x; int64_t ldx;
  int32_t B, H, P;
  const float* w0; const float* b0; int32_t C1;
  const float* w1; const float* b1; int32_t C2, k1, s1;
  const float* w2; const float* b2; int32_t C3, k2, s2;
  const float* wf; const float* bf; int32_t NO;
  float* out; int64_t ldo;
} lgx_adapt_args;
int32_t lgx_adaptation_forward(const lgx_adapt_args* a, void* stream);
/* ABI 9 (f32-MFMA form: ABI 10). One DAgger minibatch of the adaptation encoder (rsl_rl
 * ppo.py:309-349: adaptation forward, loss = mean_i ||target_i - latent_i||_2, backward) in ONE
 * launch. A block walks 16-row chunks with everything in LDS; every stage (the four forward
 * layers, each input gradient, each weight gradient) is a GEMM on v_mfma_f32_16x16x4_f32 (exact
 * f32 products, fp32 sums; f.out, the latent, optional). The weight / bias gradients of the
 * block's rows are summed in a fixed order into one partial row per block: gws[block][NP] in the
 * flat parameter layout (fc_encoder w, b, conv1 w [out][in][k], b, conv2 w, b, fc_final w
 * [out][c * L2 + t], b; NP their total), and loss_ws[block] = sum of the block's ||.|| / B. The
 * grid is min(blocks, ceil(B/16)) blocks; the caller sums the partial rows (the gradient and the
 * loss). Shapes outside the kernel's tiling return an error (hip_mlp.adaptation_train_supported
 * states them: <= 4 positions after each convolution, P <= 64, C1 <= 32 or 64, the per-wave
 * weight-gradient tiles, <= 80 KB of LDS). f.w1 / f.w2 / f.wf in lgx_adaptation_forward's
 * layouts (tap-major, (t, c) flatten). */
typedef struct lgx_adapt_train_args {
  lgx_adapt_args f;
  const float* target; int64_t ldt;
  float* gws; float* loss_ws;
  int32_t blocks;
} lgx_adapt_train_args;
int32_t lgx_adaptation_train(const lgx_adapt_train_args* t, void* stream);
/* Split-K factors for n weight-gradient GEMMs launched as one group: one K chunk for all
 * (a multiple of 32 rows, >= 256), the smallest whose block count fits one residency wave
 * of the chip; every split >= 2. */
int32_t lgx_mlp_pick_split_group(const int32_t* M, const int32_t* N, const int32_t* K, int32_t n, int32_t* split);
/* Deferred split-K reductions of several weight-gradient GEMMs in ONE launch (a whole
 * backward pass's dW/db, rsl_rl ppo.py:262 loss.backward()): for each entry
 *   C[m*ldc + n] (+)= sum_{z in order} ws[(z*M + m)*N + n]
 *   colsum[m]    (+)= sum_{z in order} colsum_ws[z*M + m]          (colsum != NULL)
 * (+= when epilogue has LGX_EPI_ACCUM). Fixed summation order: the result equals the
 * immediate reduction of lgx_gemm bit for bit. Entries must not overlap in C / colsum. */
#define LGX_SPLITK_MAX 24
typedef struct lgx_splitk_desc {
  const float* ws; const float* colsum_ws;
  float* C; int64_t ldc; float* colsum;
  int32_t M, N, split, epilogue;
} lgx_splitk_desc;
int32_t lgx_splitk_reduce_batch(const lgx_splitk_desc* descs, int32_t n, void* stream);
/* Up to LGX_TRANSPOSE_MAX matrix transposes in one launch: dst[c * rows + r] = src[r * ld + c]
 * (r < rows, c < cols; dst contiguous [cols, rows]). The backward pass transposes the layer
 * weights it needs once, so input-gradient GEMMs read W^T k-contiguous (lgx_gemm with
 * b_kcontig = 1) instead of W n-contiguous. */
#define LGX_TRANSPOSE_MAX 24
typedef struct lgx_transpose_desc {
  const float* src; int64_t ld; int32_t rows, cols; float* dst;
} lgx_transpose_desc;
int32_t lgx_transpose_batch(const lgx_transpose_desc* descs, int32_t n, void* stream);
const char* lgx_mlp_last_error(void);

/* One Adam step over a contiguous parameter segment (fp32), replacing torch.optim.Adam's
 * step (rsl_rl ppo.py:58-66 optimizers; the arithmetic of torch's fused Adam):
 *   t = *step (already incremented by the caller), g' = g * (grad_scale ? *grad_scale : 1)
 *   m = b1 m + (1-b1) g';  v = b2 v + (1-b2) g'^2
 *   p -= (lr / (1-b1^t)) * m / (sqrt(v) / sqrt(1-b2^t) + eps)
 * lr is read from lr_dev when non-NULL (device-side KL schedule), else lr. grad_scale is
 * the clip_grad_norm_ coefficient (device scalar). Stream-ordered; graph-capturable. */
int32_t lgx_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                      const float* lr_dev, float lr, float beta1, float beta2, float eps, const float* step,
                      const float* grad_scale, void* stream);
/* ABI 10. clip_grad_norm_ + one Adam step over a small segment in ONE launch (one block; the
 * DAgger step, rsl_rl ppo.py:336-345 — clip_grad_norm_(adaptation_encoder.parameters()), then
 * adaptation_optimizer.step()):
 *   coef = min(max_norm / (||grad||_2 + 1e-6), 1);  grad *= coef (in place, as torch leaves it)
 *   *step += 1;  Adam as lgx_adam_step with the clipped gradient;  *coef_out = coef (optional)
 * ||grad|| is summed in a fixed order (deterministic). n <= LGX_CLIP_ADAM_MAX. */
#define LGX_CLIP_ADAM_MAX 65536
int32_t lgx_clip_adam(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, const float* lr_dev,
                      float lr, float beta1, float beta2, float eps, float* step, float max_norm, float* coef_out,
                      void* stream);

/* PPO loss head (rsl_rl ppo.py:196-262 with the Gaussian policy of actor_critic.py:
 * Normal(mu, std) log_prob / entropy), forward and backward in one kernel each.
 * Row i of B (A actions):
 *   logp_i  = sum_j -(a-mu)^2/(2 std_j^2) - log std_j - log sqrt(2 pi)
 *   r_i     = exp(logp_i - old_logp_i)
 *   surr    = mean_i max(-adv_i r_i, -adv_i clamp(r_i, 1-clip, 1+clip))
 *   vloss   = mean_i max((v-R)^2, (tv + clamp(v-tv, -clip, clip) - R)^2)   (clipped_value)
 *             mean_i (R - v)^2                                              (otherwise)
 *   entropy = sum_j 0.5 + 0.5 log(2 pi) + log std_j      (= mean_i of the row entropy)
 *   kl      = mean_i sum_j log(std_j/old_sigma + 1e-5) + (old_sigma^2 + (old_mu-mu)^2)/(2 std_j^2) - 0.5
 * out[4] = {surr, vloss, entropy, kl}. Backward takes g[3] = d(loss)/d{surr, vloss,
 * entropy} and writes dmu [B,A], dvalue [B], dstd [A] with torch's gradient rules (max
 * splits ties evenly, clamp passes on [lo, hi]). Row sums are reduced deterministically
 * (per-block partials, fixed-order sum by the last block). ws: >= 16 * ceil(B/256) floats;
 * counter: one zero-initialised uint32 (left at zero). */
typedef struct lgx_ppo_head_args {
  const float* mu; const float* value; const float* std; const float* actions;
  const float* old_logp; const float* adv; const float* target_values; const float* returns;
  const float* old_mu; const float* old_sigma;
  int32_t B, A; float clip; int32_t clipped_value;
  float* out;
  const float* g;
  float* dmu; float* dvalue; float* dstd;
  float* ws; uint32_t* counter;
  float* kl_dst;             /* optional: forward also writes the KL mean here (the KL slot
                                of the flat gradient buffer that rides the all-reduce) */
  int32_t accumulate_dstd;   /* backward: dstd += (the parameter's .grad) instead of = */
} lgx_ppo_head_args;

int32_t lgx_ppo_head_forward(const lgx_ppo_head_args* args, void* stream);
int32_t lgx_ppo_head_backward(const lgx_ppo_head_args* args, void* stream);

/* ROA regulariser and estimator loss (rsl_rl ppo.py:204-206 and :190-192):
 *   reg = mean_i || p_i - a_i ||_2          (p = privileged latent, a = sg(adaptation latent), [B, L])
 *   est = mean_i || e_i - t_i ||_2^2        (e = estimator output, t = true estimated obs, [B, E])
 * Forward writes out[0] = reg, out[1] = est (deterministic: per-block partials summed in
 * block order by the last block). Backward takes g[0], g[1] (device scalars: d loss/d reg,
 * d loss/d est) and writes dp = g0 (p - a) / (B ||p - a||) (0 where the norm is 0, as
 * torch's norm backward) and de = g1 * 2 (e - t) / B. ws >= 2 * ceil(B/256) floats; counter
 * one zero-initialised uint32. */
typedef struct lgx_aux_loss_args {
  const float* p; const float* a; int32_t L;
  const float* e; const float* t; int32_t E;
  int32_t B;
  float* out; const float* g; float* dp; float* de;
  float* ws; uint32_t* counter;
  int64_t ld_p;              /* row stride of p (0: L); p may be a column span of a wider buffer */
} lgx_aux_loss_args;
int32_t lgx_aux_loss_forward(const lgx_aux_loss_args* args, void* stream);
int32_t lgx_aux_loss_backward(const lgx_aux_loss_args* args, void* stream);
/* Both loss heads of one minibatch in one launch each way (blockIdx.y selects the head):
 * the same results as lgx_ppo_head_* and lgx_aux_loss_* on the same arguments. head->B must
 * equal aux->B. */
int32_t lgx_loss_heads_forward(const lgx_ppo_head_args* head, const lgx_aux_loss_args* aux, void* stream);
int32_t lgx_loss_heads_backward(const lgx_ppo_head_args* head, const lgx_aux_loss_args* aux, void* stream);
/* ABI 7. Both heads' forward sums AND input gradients in ONE launch (the gradients need none
 * of the forward's sums): the outputs of lgx_loss_heads_forward + lgx_loss_heads_backward on
 * the same arguments (head->ws >= (3 + 16) * ceil(B/256) floats), where the narrow output
 * gradients may ALSO (or instead: a NULL fp32 pointer) be written in S8 (include/lgx_s8.h:
 * bf16 hi / lo per 8 columns, pitch in elements, a multiple of 8) with one column-sum partial
 * per 256-row block ([ceil(B/256)][A], [..][1], [..][E]; E <= 8) — the S8 update's GEMM
 * operands and last-layer bias-gradient partials (rsl_rl ppo.py:196-262 then the backward). */
typedef struct lgx_heads_s8_args {
  void* dmu_s8; int64_t ld_dmu; float* dmu_cs;
  void* dvalue_s8; int64_t ld_dvalue; float* dvalue_cs;
  void* de_s8; int64_t ld_de; float* de_cs;
  /* ABI 8, optional (NULL: unused). The per-sample discrete decisions of the PPO head, one byte
   * per row: bits 0-1 the surrogate max (ppo.py:254) weight of the unclipped term times 2 (0, 1:
   * a tie, 2), bit 2 the ratio inside [1-clip, 1+clip] (the clamp's gradient, :252), bits 3-4 the
   * value-loss max (:261) weight of the unclipped term times 2, bit 5 v - target inside
   * [-clip, clip] (:258). decisions_out: this launch writes its own decisions. decisions_in: the
   * launch takes its decisions from here instead (forward maxima and gradients; the continuous
   * quantities stay its own), so a test can replay a reference run's decisions and its
   * trajectory cannot leave the reference's at a sample sitting within rounding of a clip
   * boundary (tests/test_gpu_learner_golden.py). ABI 9: a decisions_in byte with bit 6 (0x40)
   * set leaves that row its own decisions (replaying only the near-tie samples). */
  const uint8_t* decisions_in; uint8_t* decisions_out;
} lgx_heads_s8_args;
int32_t lgx_loss_heads_fused(const lgx_ppo_head_args* head, const lgx_aux_loss_args* aux,
                             const lgx_heads_s8_args* s8, void* stream);

/* ABI 9. lgx_loss_heads_fused with the actor's and the critic's LAST layers fused around the
 * PPO head (the S8 update; rsl_rl actor_critic.py:82-107, ppo.py:196-262 and the backward of
 * those two layers), per block of LGX_HEADS_TAIL_ROWS rows:
 *   mu = y W^T + b, value = y_c W_c^T + b_c   fp32 FMAs over k in order; y, y_c: the last hidden
 *                                             layers' S8 outputs [B][H] read as hi + lo; W [A][H],
 *                                             W_c [1][H_c] fp32 (nn.Linear layout)
 *   the PPO head of lgx_loss_heads_fused on them (head->mu / head->value are IGNORED as inputs);
 *   the aux head as there (blockIdx.y = 1)
 *   dy = (dmu W) * ELU'(y), dy_c = (dvalue W_c) * ELU'(y_c) -> S8 [B][H] with one column-sum
 *                                             partial per block ([ceil(B/32)][H]: the hidden
 *                                             layers' bias-gradient partials)
 * It replaces the last layers' forward launch, lgx_loss_heads_fused and the last layers' input-
 * gradient launch. Here s8->dmu_cs / dvalue_cs are per 32-row block ([ceil(B/32)][A], [..][1]),
 * head->ws >= (3 + 16) * ceil(B/32) floats; mu_out / value_out (optional): fp32 copies of mu
 * [B][A] and value [B]. H, H_c multiples of 8 in [8, 256]; A <= 16.
 * The PPO head's totals are NOT formed in this launch (no last-block pass; head->counter is not
 * used): head->ws holds one row of 3 + 16 floats per block, {surrogate / B, value loss / B,
 * KL / B, dstd partial [A]} (block 0's dstd partial includes the entropy term), and the caller
 * sums the rows (out[0..1], out[3] / kl_dst, dstd: lgx_s8_reduce jobs); out[2] (the entropy) is
 * written here. The aux head forms its totals as in lgx_loss_heads_fused. */
#define LGX_HEADS_TAIL_ROWS 32
typedef struct lgx_heads_tail_args {
  const void* y; int64_t ld_y; const float* W; const float* b;
  void* dy; int64_t ld_dy; float* dy_cs;
  const void* yc; int64_t ld_yc; const float* Wc; const float* bc;
  void* dyc; int64_t ld_dyc; float* dyc_cs;
  float* mu_out; float* value_out;
  int32_t H, Hc;
} lgx_heads_tail_args;
int32_t lgx_loss_heads_tail(const lgx_ppo_head_args* head, const lgx_aux_loss_args* aux,
                            const lgx_heads_s8_args* s8, const lgx_heads_tail_args* tail, void* stream);

/* The optimizer tail of one PPO minibatch (rsl_rl ppo.py:264-291) in two launches, over
 * the flat gradient/parameter/moment buffers (one layout):
 *   coef_e = min(max_norm / (||g[est]|| + 1e-6), 1)            clip_grad_norm_(estimator)
 *   Adam(est segment, est_lr, coef_e)                           estimator_optimizer.step()
 *   adaptive KL schedule in fp64 on lr64 (kl = g[kl_index]; skipped when kl_index < 0):
 *     kl > 2 d: lr = max(lr / 1.5, 1e-5);  d/2 > kl > 0: lr = min(lr * 1.5, 1e-2)
 *   coef_m = min(max_norm / (||g[main] ++ g[adapt]|| + 1e-6), 1)  clip_grad_norm_(actor_critic)
 *   g[adapt] *= coef_m (the stale DAgger gradients, a reference quirk)
 *   Adam(main segment, (float) lr, coef_m)                      optimizer.step()
 *   sums[i] += *loss_ptrs[i] (i < nloss)                        loss bookkeeping
 * Adam arithmetic as lgx_adam_step; step_main / step_est are incremented here. Norms are
 * block partials summed in block order (deterministic): the first launch writes them, every
 * block of the second sums them (no last-block pass). ws >= 2 * 512 floats + 8; counter:
 * unused (kept for the layout).
 * ABI 11, optional (n_s8 = 0: none): the updated weights also written in S8 (the update's GEMM
 * operands, include/lgx_s8.h) by the Adam launch itself, so the next minibatch needs no weight
 * split launch. Each lgx_tail_s8_seg maps the logical columns [c0, c0 + w) of one weight W [N][K]
 * (row-major in params from index p0) to S8 destination columns 0.. of dst: S8 rows of pitch ld
 * elements (32 B per 8-column group: 8 hi then 8 lo bf16), or, packed != 0, the fragment-packed
 * copy (lgx_s8_split packed_steps = ld: per 16-row tile and 32-deep K step 64 lanes x 16 B of hi,
 * then of lo). The conversion is lgx_s8_split's (hi = RN bf16(x), lo = RN bf16(x - hi)), so the
 * copies equal a split of the updated weights bit for bit; pad columns are not written (a split
 * zeroed them). The table (host memory, n_s8 <= LGX_TAIL_S8_MAX entries sorted by p0, a weight's
 * entries consecutive, at most 4 per weight; every weight inside the main or the estimator
 * segment) is read at the
 * call: a captured graph keeps the table of its capture. */
#define LGX_TAIL_MAX_LOSSES 8
#define LGX_TAIL_S8_MAX 32
typedef struct lgx_tail_s8_seg {
  int64_t p0;         /* params index of W[0][0] */
  int32_t N, K;       /* W rows, columns */
  int32_t c0, w;      /* the logical columns this entry covers */
  char* dst;          /* S8 column 0 of this entry (row 0) */
  int32_t ld;         /* S8 row pitch in elements; packed: K steps per 16-row tile */
  int32_t packed;
} lgx_tail_s8_seg;
typedef struct lgx_ppo_tail_args {
  float* grads; float* params; float* exp_avg; float* exp_avg_sq;
  int64_t main_lo, main_hi, est_lo, est_hi, adapt_lo, adapt_hi, kl_index;
  float max_norm;
  float b1_main, b2_main, eps_main, b1_est, b2_est, eps_est, est_lr;
  double desired_kl;
  double* lr64; float* lr32;
  float* step_main; float* step_est;
  const float* loss_ptrs[LGX_TAIL_MAX_LOSSES]; float* sums; int32_t nloss;
  float* ws; uint32_t* counter;
  const lgx_tail_s8_seg* s8; int32_t n_s8;  /* ABI 11 */
} lgx_ppo_tail_args;
int32_t lgx_ppo_tail(const lgx_ppo_tail_args* args, void* stream);

/* ---- rollout bookkeeping (ppo.py:129-171, rollout_storage.py:87-105), one launch each */

/* Up to LGX_COPY_MAX device-to-device copies in one launch (the storage writes of one
 * rollout step). Each entry: nbytes from src to dst; 16-byte aligned entries whose size
 * is a multiple of 16 take the vector path. dst_stride is read by lgx_gather_rows only
 * (added in ABI v5: the descriptor is 32 bytes; v4 callers used 24). */
#define LGX_COPY_MAX 16
typedef struct lgx_copy_desc {
  const void* src; void* dst; int64_t nbytes;
  int64_t dst_stride;  /* lgx_gather_rows: bytes between destination rows (0: nbytes, packed) */
} lgx_copy_desc;
int32_t lgx_copy_batch(const lgx_copy_desc* descs, int32_t n, void* stream);
/* Row gather of up to LGX_COPY_MAX row-major buffers in one launch (the storage permuted once
 * per update, rollout_storage.py:134-181): dst row r (at dst + r * dst_stride) = src row
 * idx[r] (r < rows), nbytes each; a strided destination places rows inside a wider buffer
 * (the update's actor-input rows). 16-B vector path when nbytes, dst_stride and both bases
 * are 16-B aligned; rows * (nbytes / 4) < 2^31. */
int32_t lgx_gather_rows(const lgx_copy_desc* descs, int32_t n, const int64_t* idx, int64_t rows, void* stream);

/* PPO.act action head (actor_critic.py:205-226 + ppo.py:141-146) for a diagonal Gaussian:
 *   a = mean + std * eps,  logp_i = sum_j -(a-mean)^2/(2 std_j^2) - log std_j - log sqrt(2 pi)
 * (torch.distributions.Normal.log_prob op order), written straight into the storage rows:
 * actions [B,A], mu [B,A] (= mean), sigma [B,A] (= std broadcast), logp [B].
 * eps: a given [B,A] standard-normal sample, or NULL: drawn in the kernel per (global env
 * env_offset + row, env step *step_dev, action) from the env's Philox4x32-10 counter layout on
 * stream LGX_ACT_NOISE_STREAM (Box-Muller) — the noise of an env does not depend on which
 * rank or shard steps it, so sharded rollouts equal one GPU's. step_dev: the env's device step
 * counter (lgx_step_dev; the number of the step these actions drive). Fields after
 * actions_copy: ABI v5. */
#define LGX_ACT_NOISE_STREAM 2
typedef struct lgx_act_head_args {
  const float* mean; const float* std; const float* eps;
  float* actions; float* mu; float* sigma; float* logp;
  int32_t B, A;
  float* actions_copy;       /* optional second destination of the actions (the env's input buffer) */
  const int64_t* step_dev;   /* eps == NULL: device step counter */
  uint64_t seed;             /* eps == NULL: the env's seed (Philox key) */
  int64_t env_offset;        /* eps == NULL: global id of row 0 */
} lgx_act_head_args;
int32_t lgx_act_head(const lgx_act_head_args* args, void* stream);

/* PPO.process_env_step (ppo.py:156-171) into the storage rows of this step:
 *   rewards_out[i] = rewards[i] + gamma * (values[i] * time_outs[i])   (time_outs may be NULL)
 *   dones_out[i] = dones[i] (uint8), values_out[i] = values[i]. */
typedef struct lgx_transition_args {
  const float* rewards; const uint8_t* dones; const uint8_t* time_outs; const float* values;
  float* rewards_out; uint8_t* dones_out; float* values_out;
  float gamma; int32_t B;
} lgx_transition_args;
int32_t lgx_store_transition(const lgx_transition_args* args, void* stream);

/* OnPolicyRunner.learn's per-step episode bookkeeping (on_policy_runner.py:160-170) in one
 * launch, device-side form of its deques (rewbuffer/lenbuffer keep the last 100 completed
 * episodes; ep_infos accumulate infos['episode']):
 *   cur_rew += rewards;  cur_len += 1
 *   for the done envs in env order (rank r of k): if r >= k - 100:
 *       rew_ring[(ptr + r) % 100] = cur_rew;  len_ring[(ptr + r) % 100] = cur_len
 *   ptr = (ptr + k) % 100;  n = min(n + k, 100);  cur_rew, cur_len = 0 where done
 *   ep_sum[0:na] += ep_a[0:na];  ep_sum[na:na+nb] += ep_b[0:nb];  ep_cnt += 1  (ep_* optional)
 * One workgroup; the done ranks come from a block-wide scan. Replaces the cumsum / where /
 * scatter / masked_fill / stack sequence of the runner's torch form, bit for bit. */
typedef struct lgx_track_args {
  const float* rewards; const uint8_t* dones;
  float* cur_rew; float* cur_len; float* rew_ring; float* len_ring;  /* rings: >= 100 floats */
  int64_t* ptr; int64_t* n;
  const float* ep_a; const float* ep_b; float* ep_sum; float* ep_cnt;
  int32_t N, na, nb;
} lgx_track_args;
int32_t lgx_track_episodes(const lgx_track_args* args, void* stream);
/* ABI 11. lgx_store_transition and lgx_track_episodes of one rollout step in ONE launch (both
 * read the env's rewards / dones and write disjoint buffers; the same arithmetic as the two
 * launches, bit for bit). track NULL: lgx_store_transition alone. */
int32_t lgx_post_step(const lgx_transition_args* transition, const lgx_track_args* track, void* stream);

/* RolloutStorage.compute_returns (rollout_storage.py:110-124) over [T, N] rows, one thread
 * per env walking the steps backwards in torch's operation order:
 *   nt = 1 - dones[t];  delta = (rewards[t] + (nt*gamma) * V[t+1]) - V[t]   (V[T] = last_values)
 *   A = delta + ((nt*gamma)*lam) * A;  returns[t] = A + V[t];  advantages[t] = returns[t] - V[t]
 * and moments[0..1] = (sum, sum of squares) of the advantages in fp64 (per-block partials
 * summed in block order by the last block: deterministic). ws >= 2 * ceil(N / 256) doubles;
 * counter: one zero-initialised uint32 (left at zero). */
typedef struct lgx_gae_args {
  const float* rewards; const uint8_t* dones; const float* values; const float* last_values;
  float* returns; float* advantages;
  int32_t T, N; float gamma, lam;
  double* moments; double* ws; uint32_t* counter;
} lgx_gae_args;
int32_t lgx_gae(const lgx_gae_args* args, void* stream);
/* advantages = (advantages - mean) / (std + 1e-8) with mean = moments[0] / count and the
 * unbiased std sqrt((moments[1] - count mean^2) / (count - 1)) (fp64, then fp32 like torch's
 * mean()/std() scalars); count = the number of advantages over all ranks. */
int32_t lgx_normalize_advantages(float* advantages, int64_t n, const double* moments, double count, void* stream);

#ifdef __cplusplus
}
#endif
#endif
