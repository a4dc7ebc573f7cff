/* lgx_s8.h — C ABI of liblgx_s8.so: the learner's GEMM core on pre-split operands (MI355X).
 *
 * Replaces the same nn.Linear + nn.ELU chains as lgx_mlp.h (reference rsl_rl
 * modules/actor_critic.py:64-87, support_networks.py:22-112; forward ppo.py:186-206, backward
 * ppo.py:262 / :207) inside the PPO update, with every GEMM operand stored PRE-SPLIT by the
 * kernel that produced it instead of split in each GEMM's K loop.
 *
 * S8 layout ("split rows"). A logical fp32 matrix X[rows][cols] is stored as 4-byte words,
 * row pitch `ld` elements (a multiple of 8; 16-B aligned rows). Columns are grouped by 8: group
 * g of row r occupies bytes [32 g, 32 g + 32) of the row: 8 x bf16 hi, then 8 x bf16 lo, where
 *     hi = bf16_rne(x),  lo = bf16_rne(x - hi)        (x ~ hi + lo to ~2^-17 relative)
 * — the split the fp32 GEMMs of lgx_mlp.h perform on the fly, so the products are the same
 * (3 x bf16 MFMA: lo*hi + hi*lo + hi*hi per 32-deep K step, fp32 accumulation).
 * Pad columns [cols, ld) hold zeros. The producers write them in the last group of a row (the
 * rest is never written), so an S8 buffer is allocated zeroed once and reused.
 *
 * One GEMM:  C[m][n] = epilogue( sum_k A(m, k) B(k, n) ), with each operand in one of two modes:
 *     ROW  A(m, k) = S8 element (m, k) — k along the source row (forward X, W; input-grad dY)
 *     TR   A(m, k) = S8 element (k, m) — k = source row (input-grad W; weight-grad dY and X)
 * so  forward     Y  = X W^T + b     A = X ROW,  B = W ROW, then bias, ELU
 *     input grad  dX = dY W          A = dY ROW, B = W TR,  then * ELU'(Y_prev) (Y_prev in S8)
 *     weight grad dW = dY^T X        A = dY TR,  B = X TR,  split-K fp32 partials
 * Operand contract: a ROW operand's pitch covers round_up(K, 32) columns (zeros past K in at
 * least one of the two operands; the producers' zero pads give that); a TR operand's rows
 * [K, round_up(K, 32)) exist (zero in at least one operand). Rows/columns past M or N are read
 * clamped and never stored.
 * All work is stream-ordered on `stream` (hipStream_t). Return 0 on success, negative on invalid
 * arguments or launch failure (lgx_s8_last_error).
 */
#ifndef LGX_S8_H
#define LGX_S8_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define LGX_S8_ABI_VERSION 4

enum { LGX_S8_FWD = 0, LGX_S8_DX = 1, LGX_S8_DW = 2 };  /* GEMM kinds (operand modes above) */

enum {
  LGX_S8_EPI_BIAS = 1,   /* FWD: + bias[n] */
  LGX_S8_EPI_ELU = 2,    /* FWD: then ELU(alpha = 1) */
  LGX_S8_EPI_DELU = 4,   /* DX: * ELU'(z) from the ELU output y = act (S8): y > 0 ? 1 : y + 1 */
  LGX_S8_EPI_ACCUM = 8   /* DW with split 1: C += result */
};

typedef struct lgx_s8_gemm_args {
  const void* A; int64_t lda;   /* S8 operands, pitch in elements */
  const void* B; int64_t ldb;
  int32_t M, N, K;
  int32_t epilogue;             /* LGX_S8_EPI_* */
  void* C; int64_t ldc;         /* FWD / DX: S8 output (optional if C32 is set) */
  float* C32; int64_t ldc32;    /* FWD / DX: fp32 copy of the output (optional); DW: fp32 output
                                   (split 1) or the partial workspace [split][M][N] (split > 1) */
  const float* bias;            /* FWD, LGX_S8_EPI_BIAS: [N] */
  const void* act; int64_t ld_act;      /* DX, LGX_S8_EPI_DELU: Y_prev (S8) */
  const float* addend; int64_t ld_add;  /* DX (optional): + addend[m][n] for n < add_cols, after ELU' */
  int32_t add_cols;
  float* colsum_ws;             /* FWD / DX (optional): [ceil(M / LGX_S8_TILE_M)][N] fp32 column
                                   sums of the output over each 64-row half tile (the next weight
                                   gradient's bias gradient, reduced with lgx_s8_reduce) */
  int32_t split;                /* DW: K split (>= 1); kchunk = round_up(ceil(K / split), 32) */
  int32_t pad0;
} lgx_s8_gemm_args;

/* fp32 -> S8 (weights after each optimizer step; the update's network inputs, gathered in the
 * minibatch permutation; the loss heads' narrow gradients). Row r of dst = split of src row
 * (idx ? idx[r] : r), zeros in columns [cols, round_up(cols, 8)). With colsum_ws set (cols <= 64)
 * also the column sums of each 256-row block: colsum_ws[blk * cols + c] (blk = r / 256). */
typedef struct lgx_s8_split_args {
  const float* src; int64_t ld_src;
  void* dst; int64_t ld_dst;    /* dst points at the S8 group of column 0 (a multiple of 8) */
  int32_t rows, cols;
  float* colsum_ws;
  const int64_t* idx;           /* optional row gather (rollout_storage.py:141-147's permutation) */
  int32_t packed_steps;         /* > 0: dst is fragment-packed (a chain's weights, below) with this
                                   many 32-deep K steps per 16-row tile; ld_dst unused */
  int32_t transpose;            /* packed only: dst = src^T (src [cols][rows]: an input-gradient
                                   chain's W^T) */
} lgx_s8_split_args;

/* out[r * ld_out + c] (+)= sum_{s < nsplit} ws[s * stride + r * ld_ws + c], r < rows, c < cols
 * (fixed order: deterministic) — split-K partials into weight gradients (also column spans:
 * a weight whose input columns sit at other positions in S8 space), bias-gradient partials. */
typedef struct lgx_s8_reduce_args {
  const float* ws; int64_t stride, ld_ws;
  float* out; int64_t ld_out;
  int32_t rows, cols, nsplit, accumulate;
} lgx_s8_reduce_args;

#define LGX_S8_GROUP_MAX 20
#define LGX_S8_BATCH_MAX 48
#define LGX_S8_TILE_M 64         /* rows of one colsum_ws partial (FWD / DX; ABI 4: was 128) */
#define LGX_S8_SPLIT_ROWS 256    /* rows of one lgx_s8_split colsum partial */

int32_t lgx_s8_abi_version(void);
int32_t lgx_s8_sizeof_gemm_args(void);
const char* lgx_s8_last_error(void);
/* n independent GEMMs of one kind in one launch (each problem's tiles dealt over the 8 XCDs). */
int32_t lgx_s8_gemm_group(const lgx_s8_gemm_args* args, int32_t n, int32_t kind, void* stream);
/* Split factors for n weight-gradient GEMMs sharing one launch (out[i] >= 1). */
int32_t lgx_s8_pick_split(const int32_t* M, const int32_t* N, const int32_t* K, int32_t n, int32_t* out);
int32_t lgx_s8_split(const lgx_s8_split_args* args, int32_t n, void* stream);
int32_t lgx_s8_reduce(const lgx_s8_reduce_args* args, int32_t n, void* stream);

/* ---- ABI v2: the rollout's act networks in ONE launch (PPO.act, ppo.py:129-153): the
 * estimator, scan encoder and privileged encoder, the actor on [obs | priv latent | scan latent
 * | est] (actor_critic.py:79-107) and the critic (:110-115), [Linear, ELU]* Linear chains whose
 * weights are in the act-packed S8 format written by lgx_s8_act_pack and biases fp32. The actor
 * input is the S8 update's segmented layout: part p starts at column seg[p] (seg[0] = 0, a
 * multiple of 4 each, zero gaps), width = its K (a multiple of 32); the actor's first-layer
 * weights use the same layout. Writes mu [B, A] (row stride ld_mu) and value [B]. 32 rows per
 * block, one block per CU; widths: actor input <= LGX_S8_ACT_MAXIN, hidden layers <=
 * LGX_S8_ACT_MAXH (actor, critic) / LGX_S8_ACT_MAXENC (encoders), <= LGX_S8_ACT_MAXL layers. */
#define LGX_S8_ACT_ROWS 32
#define LGX_S8_ACT_MAXIN 640
#define LGX_S8_ACT_MAXH 512
#define LGX_S8_ACT_MAXENC 256
#define LGX_S8_ACT_MAXL 6
typedef struct lgx_s8_act_layer {
  const void* W; int64_t ldw;   /* act-packed weights; ldw = K steps per tile (ceil(K / 32)) */
  const float* b;
  int32_t K, N, elu, pad0;
} lgx_s8_act_layer;
typedef struct lgx_s8_act_args {
  int32_t B, width;
  const float* obs; int64_t ld_obs; int32_t n_obs;                 /* actor / estimator input */
  const float* priv_obs; int64_t ld_priv; int32_t n_priv_in;
  const float* scan_obs; int64_t ld_scan; int32_t n_scan_in;
  const float* critic_obs; int64_t ld_critic; int32_t n_critic_in;
  int32_t est_c0;                                                   /* estimator input: obs columns [est_c0, est_c0 + K) */
  int32_t seg[4];
  lgx_s8_act_layer est[LGX_S8_ACT_MAXL], scan[LGX_S8_ACT_MAXL], priv[LGX_S8_ACT_MAXL];
  lgx_s8_act_layer actor[LGX_S8_ACT_MAXL], critic[LGX_S8_ACT_MAXL];
  int32_t n_est, n_scan, n_priv, n_actor, n_critic;
  float* mu; int64_t ld_mu;
  float* value;
  /* optional (NULL: skipped): this step's storage rows (rollout_storage.py:87-105, written at
   * act time), contiguous [B, width of the input]: the kernel copies obs, priv_obs, scan_obs,
   * critic_obs and est_obs ([B, n_est_obs], read for this copy only) into them */
  float* obs_st; float* priv_st; float* scan_st; float* critic_st; float* est_st;
  const float* est_obs; int64_t ld_est; int32_t n_est_obs, pad1;
  /* n_est = n_scan = n_priv = 0: the encoders ran elsewhere; their outputs [B, w] (row stride
   * ld) are copied into the actor-input parts 1..3 (priv latent, scan latent, est) instead */
  const float* part_src[3]; int64_t part_ld[3]; int32_t part_w[3];
  int32_t nets;  // 0: actor and critic blocks; 1: the actor blocks only; 2: the critic blocks only
  /* optional act head (actions != NULL; lgx_act_head's semantics, lgx_mlp.h): from the actor's
   * output mu, a = mu + std * eps and the Normal log-prob, into this step's storage rows
   * actions / mu_st / sigma_st [B, A] and logp_st [B] (+ actions_copy); eps [B, A] given, or
   * drawn from (seed, *step_dev, env_offset) as lgx_act_head does; mu is then not written */
  const float* std; const float* eps;
  float* actions; float* mu_st; float* sigma_st; float* logp_st; float* actions_copy;
  const int64_t* step_dev; uint64_t seed; int64_t env_offset;
} lgx_s8_act_args;
int32_t lgx_s8_act(const lgx_s8_act_args* args, void* stream);
/* The act-packed format: for each 16-row output tile t and 32-deep K step s, one 2 KB block
 * [hi: 64 lanes x 16 B][lo: 64 lanes x 16 B] where lane (c, g) = (lane & 15, lane >> 4) holds
 * the bf16 hi (lo = bf16(x - hi)) of W[16 t + c][32 s + 8 g .. + 7] — exactly the MFMA B
 * fragment, so a wave loads it as 1 KB contiguous (whole cache lines); block (t, s) at byte
 * ((t * steps + s) * 2048). Rows >= N and columns outside the spans are zero. Spans place
 * logical input columns at packed columns (the actor's first layer: [obs | priv latent | scan
 * latent | est] at seg[]); one span (0, 0, K) otherwise. One launch packs up to
 * LGX_S8_BATCH_MAX layers (the rollout's first step: the update changed the weights). */
typedef struct lgx_s8_act_pack_args {
  const float* W; int64_t ld;   /* fp32 [N][ld] (nn.Linear.weight) */
  void* dst;                    /* >= ceil(N / 16) * steps * 2048 bytes */
  int32_t N, steps;             /* steps = ceil(packed K / 32) */
  int32_t nspans;               /* 1..4 */
  int32_t span_c0[4], span_p0[4], span_w[4];  /* logical column, packed column, width */
} lgx_s8_act_pack_args;
int32_t lgx_s8_act_pack(const lgx_s8_act_pack_args* args, int32_t n, void* stream);
const char* lgx_s8_act_last_error(void);
int32_t lgx_s8_sizeof_act_args(void);
int32_t lgx_s8_sizeof_act_pack_args(void);

/* Chains (lgx_s8chain.hip): the narrow encoders of the update (the privileged and scan
 * encoders, support_networks.py:25-80, as PPO.update runs them in ppo.py:201-233) as ONE launch
 * instead of one grouped launch per depth — their forward, and their input gradients. Per
 * chain: A = the S8 input rows [rows][>= K_0] (pitch lda elements; columns past K_0 are read as
 * zero), then up to LGX_S8_CHAIN_MAXL layers y_l = epi(y_{l-1} W_l^T + b_l) with W_l S8
 * [N_l][ldw_l] (or fragment-packed), K_l = N_{l-1}. epi (`elu`): 0 none, 1 ELU (forward), 2
 * times ELU'(act) with act the S8 ELU output at the same rows (input gradient: W_l = the
 * forward weight transposed, bias null). Each layer's output goes to C_l (S8, pitch ldc_l,
 * pads zero; may be null) and / or C32_l (fp32; may be null); colsum_ws (exactly on the elu = 2
 * layers): the column sums of each 32-row block, colsum_ws[block * N + n] (a bias gradient is
 * their lgx_s8_reduce). Same operand contract, products and epilogues as lgx_s8_gemm_group;
 * widths <= LGX_S8_CHAIN_MAXW. */
#define LGX_S8_CHAIN_MAX 4
#define LGX_S8_CHAIN_MAXL 3
#define LGX_S8_CHAIN_MAXW 256
typedef struct lgx_s8_chain_layer {
  const void* W; int64_t ldw;   /* S8 [N][ldw] */
  const float* bias;
  void* C; int64_t ldc;         /* S8 output (or null) */
  float* C32; int64_t ldc32;    /* fp32 output (or null) */
  const void* act; int64_t ld_act;  /* S8 ELU output for elu = 2 */
  float* colsum_ws;
  int32_t K, N, elu;
  int32_t packed;               /* W fragment-packed (lgx_s8_split packed_steps = ceil(K / 32)):
                                   per (16-row tile, K step) 2 KB = 64 lanes x 16 B hi, then lo */
} lgx_s8_chain_layer;
typedef struct lgx_s8_chain_args {
  const void* A; int64_t lda;   /* S8 input rows */
  int32_t rows, nlayers;
  lgx_s8_chain_layer layers[LGX_S8_CHAIN_MAXL];
} lgx_s8_chain_args;
int32_t lgx_s8_chain(const lgx_s8_chain_args* chains, int32_t n, void* stream);
int32_t lgx_s8_sizeof_chain_args(void);

#ifdef __cplusplus
}
#endif
#endif
