/* hvit.h -- C ABI of the MI355X (gfx950) HybridViT hot-path library (libhvit.so).
 *
 * The reference exposes this path only as the PyTorch nn.Module API of
 * models/hybrid_vit.py (HybridViT.__init__ :36-170, forward :396-469) with no
 * native operator or FFI of its own.  This header is the C ABI
 * that module binds (via ctypes).  Each entry point replaces
 * the aten op sequence of one reference module, cited per function.
 *
 * Conventions
 *  - Plain pointers to device memory + sizes; no torch types.  The library never
 *    allocates or frees device memory and keeps no pointer past a call; the
 *    caller provides every output, saved activation and workspace.
 *  - Activations are NHWC (channels innermost).  A token tensor [B, N, D] is the
 *    NHWC image [B, H', W', D] of the patch grid, N = H' * W'.
 *  - dtype codes: HVIT_F32 (exact-f32 MFMA path, used for 1e-3 parity) or
 *    HVIT_BF16 (bf16 MFMA, f32 accumulate).  Statistics, the ViT residual
 *    stream, LayerNorm inputs and all weight gradients are f32.
 *  - Work is enqueued on `stream` (a hipStream_t); no host synchronisation, no
 *    allocation: every call is hipGraph-capturable.
 *  - Return 0 on success; otherwise an HVIT_ERR_* code, with a message from
 *    hvit_last_error().  There is no fallback path.
 */
#ifndef HVIT_H_
#define HVIT_H_

#ifdef __cplusplus
extern "C" {
#endif

enum { HVIT_F32 = 0, HVIT_BF16 = 1 };
enum { HVIT_OK = 0, HVIT_ERR_ARG = 1, HVIT_ERR_LAUNCH = 2 };
enum {
  HVIT_ACT_NONE = 0,
  HVIT_ACT_GELU_DUAL = 1,
  HVIT_ACT_TANH = 2,
  HVIT_ACT_GELU_BWD = 3,
  HVIT_ACT_GELU_DUAL_D = 4, /* GELU_DUAL that stores gelu'(v) instead of v (for MUL_AUX) */
  HVIT_ACT_MUL_AUX = 5,     /* GELU_BWD whose aux already holds gelu'(h): v *= aux */
  HVIT_ACT_RELU = 6,        /* conv forward only: v = max(v + bias, 0) (eval-mode BatchNorm folded) */
  HVIT_ACT_GELU = 7,        /* linear forward: y = dropout(gelu(v)) only (fc1 when no backward runs) */
  HVIT_ACT_RELU_POOL2 = 8,  /* conv forward only (bf16, even Ho / Wo, 64-channel-multiple sources): relu(v + bias)
                               then 2x2 max-pool, y = [N, Ho/2, Wo/2, Cout] (eval BatchNorm folded, pooled block) */
  HVIT_ACT_GELU_DUAL_DK = 9 /* GELU_DUAL_D storing dropout-mask * gelu'(v): the backward's MUL_AUX then needs no
                               mask (pass no dropout there) */
};
/* flags of the backward calls that accumulate into caller memory:
 * HVIT_ACC_ZEROED says the caller already zeroed the accumulator outputs (one
 * fill for a whole backward pass), so the call skips its own clear.
 * Determinism: every reduction of the train step is a fixed-order sum of
 * per-workgroup partial rows (plain stores), so results are bit-identical from
 * run to run and between eager launches and hipGraph replays.  The one
 * exception is hvit_layernorm_bwd called WITHOUT a workspace (float atomics). */
enum { HVIT_ACC_ZEROED = 1,
       /* hvit_layernorm_bwd_drop only: leave the per-workgroup partial rows in
        * ws ([ws_elems / (3*D)][3*D] f32, row order = summation order) for the
        * caller to sum -- e.g. as the side job {ws, acc3, 3*D, 3*D, rows} of its
        * next GEMM launch; acc3 is not touched */
       HVIT_ACC_DEFER = 2 };

/* Counter-based dropout: element i is kept iff a 16-bit hash of (seed, site, i)
 * is >= round(p * 65536); kept values are scaled by 1/(1-p).  Forward and
 * backward regenerate identical masks.  p = 0 disables.  seed_ptr (nullable,
 * device memory): the effective seed is seed ^ *seed_ptr, read by the kernel
 * at run time, so a captured hipGraph draws new masks each replay once the
 * word is advanced on the stream (hvit_rng_advance). */
typedef struct {
  float p;
  unsigned long long seed;
  unsigned int site;
  const unsigned long long* seed_ptr;
} hvit_dropout_t;

/* Split-K partial slabs handed from one launch to a later one: dst[i] =
 * sum over z < splits of src[z * stride + i], i < n (f32). */
typedef struct {
  const float* src;
  float* dst;
  long long n;
  long long stride;
  int splits;
} hvit_slab_sum_t;

/* Fused GEMM epilogue (applied in this order):
 *   v  = acc (+ bias[n]) (+ rowadd[(m % rowadd_rows) * N + n])
 *   GELU_DUAL: y = v (pre-activation); out2 = dropout(gelu(v))      -> stop
 *     (GELU_DUAL_D: y = gelu'(v) instead, the MUL_AUX operand of the backward;
 *      GELU_DUAL_DK: y = keep * scale * gelu'(v), the dropout mask folded in)
 *   TANH: v = tanh(v) ; v = dropout(v) ; GELU_BWD: v *= gelu'(aux[m, n])
 *     (MUL_AUX: v *= aux[m, n])
 *   resid: v = resid[m, n] + rowscale[m / rows_per_sample] * v     (f32)
 *   y[m, n] = v ; colsum (f32 [ceil(M/64)][N], overwritten): row r = sum of v
 *     over rows 64r .. 64r+63 where the GEMM tile starting there is <= 64 rows
 *     tall, else the tile's whole column sum in its first 64-row row and zeros
 *     in the others (deterministic partial rows: the column sum is their
 *     row-order sum, e.g. an hvit_slab_sum_t {colsum, out, N, N, ceil(M/64)}
 *     side job of the next launch)                                             */
typedef struct {
  int act;
  void* out2;
  int out2_dt;
  const void* aux;
  int aux_dt;
  hvit_dropout_t dropout;
  const float* resid;
  const float* rowscale;
  int rows_per_sample;
  const float* rowadd;
  int rowadd_rows;
  float* colsum; /* partial rows, see above */
  /* side job (n = 0: none; hvit_linear_fwd / hvit_linear_dgrad only): the
   * slabs of a deferred weight gradient (hvit_linear_wgrad_defer) summed by
   * this launch's workgroups before their own tiles -- no reduction launch of
   * its own.  Complete when this call's launch is. */
  hvit_slab_sum_t side;
} hvit_epilogue_t;

/* Convolution geometry.  Input image = concat(src1[C1], src2[C2]) (channels)
 * of an Hs x Ws NHWC source, nearest-upsampled by U; kernel KS x KS, stride,
 * zero pad.  Output Ho = (Hs*U + 2*pad - KS)/stride + 1 (same for W). */
typedef struct {
  const void* src1;
  int C1;
  const void* src2;
  int C2;
  int N, Hs, Ws, U;
  int KS, stride, pad;
  int Cout;
} hvit_conv_geom_t;

const char* hvit_last_error(void);
const char* hvit_version(void);

/* ---- Linear (nn.Linear: attention.py:55,58 qkv/proj; components.py:224,227
 * MLP; hybrid_vit.py:153 to_feature_map; 1x1 skip convs hybrid_vit.py:158-165
 * as a Linear over NHWC pixels).  w is [N][K] (torch layout). */
int hvit_linear_fwd(int dt, const void* x, const void* w, const float* bias, int M, int N, int K, void* y,
                    int y_dt, const hvit_epilogue_t* epi, void* stream);          /* y[M,N] = x[M,K] w^T */
int hvit_linear_dgrad(int dt, const void* dy, const void* w, int M, int N, int K, void* dx, int dx_dt,
                      const hvit_epilogue_t* epi, void* stream);                 /* dx[M,K] = dy[M,N] w */
long long hvit_wgrad_workspace(int M, int N, int K);                              /* f32 elements */
/* The same with the split-K partial sums reduced inside the GEMM launch (the
 * last K slice of each output tile sums the slabs; no separate reduction
 * launch): tickets = hvit_wgrad_tickets(M, N, K) uint32 arrival counters, zeroed
 * by the caller when flags has HVIT_ACC_ZEROED (else the call clears them);
 * they are left zeroed.  Falls back to the two-launch form where the ring
 * kernels do not apply. */
long long hvit_wgrad_tickets(int M, int N, int K);
int hvit_linear_wgrad_tk(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* db, float* ws,
                         long long ws_elems, unsigned* tickets, long long tickets_elems, int flags, void* stream);
/* Tuning knobs (A/B measurements, tests): what 0 = GEMM pipeline of the bf16
 * linears (-1 automatic, 0: two-stage kernels; 1-5: LDS-ring configurations,
 * gemm_ring.h); what 1 = the fused first block's matrix-core kernels (1 on, 0:
 * the VALU kernels); what 2 = workgroup target of the linear weight gradients'
 * split-K choice for the calls that follow (0: default 256; also sizes
 * hvit_wgrad_workspace); what 4 = the attention backward for bf16 / head_dim 64 /
 * N <= 256 (1: the single-pass kernel, 0: the dQ and dK/dV kernel pair); what 5
 * = the fp8 attention forward form (1: v2, 0: round 4's kernel, 2: v2 as two
 * 8-wave workgroups per (b, h)).
 * Returns the previous value (-1 for an unknown knob). */
int hvit_gemm_tune(int what, int value);
/* Diagnostics only (tools/wgrad_layout_probe.py): C[M,N] = sum_k A[m,k] B[n,k]
 * as f32 split-K slabs ws[splits][M*N + M]; kca / kcb: 1 = operand stored with
 * K contiguous ([M][K] / [N][K]), 0 = [K][M] / [K][N]; cfg 0 = gemm.h's kernels,
 * 1-5 = a ring configuration (error if it does not apply). */
int hvit_probe_gemm_splitk(int kca, int kcb, const void* a, const void* b, int M, int N, int K, int splits,
                           float* ws, int cfg, void* stream);
/* dw[N,K] = dy^T x; db[N] = colsum(dy) (nullable; fused when db == dw + N*K) */
int hvit_linear_wgrad(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* db,
                      float* ws, long long ws_elems, void* stream);
/* The weight gradient with its split-K reduction deferred: when the GEMM
 * splits K, it leaves the partial slabs in ws and fills *job (job->n > 0) for
 * the caller to pass as the `side` job of the next hvit_linear_fwd / _dgrad
 * epilogue on the same stream (or to hvit_sum_slabs_strided); dw is final only
 * after that.  Otherwise dw is written and job->n = 0.  No bias gradient.
 * side (nullable): an earlier launch's slabs, summed by this launch. */
int hvit_linear_wgrad_defer(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* ws,
                            long long ws_elems, const hvit_slab_sum_t* side, hvit_slab_sum_t* job, void* stream);
/* The same with the bias gradient db = colsum(dy) (db == dw + N*K, or NULL) of
 * a biased Linear (the head, hybrid_vit.py:153, and the skip projections,
 * :158-165): the tall-skinny kernel defers its [dw | db] slabs as one job;
 * the other paths defer dw's (when split) and write db now.  dw and db are
 * final once job (if job->n > 0) has been carried. */
int hvit_linear_wgrad_bias_defer(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* db,
                                 float* ws, long long ws_elems, const hvit_slab_sum_t* side, hvit_slab_sum_t* job,
                                 void* stream);
int hvit_sum_slabs_strided(const float* ws, int splits, long long stride, long long n, float* out, void* stream);

/* ---- Grouped weight gradients (the ViT Linears' dW of several blocks in one
 * launch; attention.py:55,58 qkv / proj, components.py:224,227 fc1 / fc2 --
 * the reference's autograd computes each as its own addmm).  Problem p:
 * dw[n_out][k_in] = dy[M][0:n_out]^T x[M][0:k_in] (bf16 operands with row
 * pitches ldy / ldx, f32 result, overwritten).  Every 256x256 output tile runs
 * over the whole token range M; when the tiles do not divide evenly over the
 * CUs, the remainder tiles are split into K pieces summed in piece order by
 * the last piece to arrive (deterministic).  ws: hvit_linear_wgrad_group_ws()
 * f32 elements; tickets: hvit_linear_wgrad_group_tickets() uint32 counters,
 * zeroed by the caller once, left zeroed by every call. */
typedef struct {
  const void* dy;
  int ldy;
  const void* x;
  int ldx;
  float* dw;
  int n_out, k_in;
  /* patch > 0: x is not a token-major matrix but the NHWC image [*, img_h,
   * img_w, img_c] of a patch embedding (Conv2d k = stride = patch,
   * components.py:275-280, hybrid_vit.py:127): token t = (image, py, px) of the
   * (img_h/patch) x (img_w/patch) grid, row t of x = the patch's (ky, kx, c)
   * values, k_in = patch^2 * img_c; dw is then [n_out][ky][kx][c] (the packed
   * conv layout, hvit_conv_weight_unpack gives torch's).  Needs a grid width
   * dividing 32, tokens per image a multiple of 32, patch * img_c a multiple
   * of 256.  ldx is ignored. */
  int patch, img_h, img_w, img_c;
} hvit_wgrad_prob_t;
int hvit_linear_wgrad_group_ok(int dt, int M, int n_out, int k_in); /* 1: the shape can join a group */
int hvit_linear_wgrad_group_patch_ok(int dt, int M, int n_out, int patch, int img_h, int img_w, int img_c);
long long hvit_linear_wgrad_group_ws(void);
long long hvit_linear_wgrad_group_tickets(void);
int hvit_linear_wgrad_group(int dt, int M, const hvit_wgrad_prob_t* probs, int nprobs, float* ws, long long ws_elems,
                            unsigned* tickets, long long n_tickets, void* stream);

/* ---- Convolution as implicit GEMM (ConvBlock conv components.py:55-62,
 * TransposeConvBlock upsample+conv components.py:146-158, PatchEmbedding
 * conv components.py:275-280, decoder concat hybrid_vit.py:389).
 * Weights are pre-packed with hvit_conv_weight_pack: mode 0 [Cout][KS][KS][Cin]
 * for fwd / wgrad / patch dgrad; mode 1 (flipped) [Cin][KS][KS][Cout] for the
 * 3x3 dgrad.  conv_fwd optionally writes BatchNorm partials
 * [ceil(P/R)][Cout][2] (mean, M2 per R-row tile, R = hvit_conv_bn_tile_rows)
 * for hvit_bn_finalize; its
 * epilogue (nullable) may apply tanh (final decoder conv, components.py:166-167),
 * a row-periodic add (pos_embed, components.py:384) and dropout.
 * conv_dgrad: same-conv -> gradient of the (upsampled, concatenated) conv input
 * [N, Hs*U, Ws*U, C1+C2] (finish with hvit_upsample_split_bwd); patch conv
 * (KS == stride, pad 0) -> gradient of src1 [N, Hs, Ws, C1] directly. */
int hvit_conv_bn_tile_rows(const hvit_conv_geom_t* g);
int hvit_conv_fwd(int dt, const hvit_conv_geom_t* g, const void* w_packed, const float* bias, void* y, int y_dt,
                  float* bn_partials, const hvit_epilogue_t* epi, void* stream);
int hvit_conv_dgrad(int dt, const hvit_conv_geom_t* g, const void* dy, const void* w_packed, void* dx, int dx_dt,
                    void* stream);
long long hvit_conv_wgrad_workspace(const hvit_conv_geom_t* g);
int hvit_conv_wgrad(int dt, const hvit_conv_geom_t* g, const void* dy, float* dw_packed, float* ws,
                    long long ws_elems, void* stream);
/* The same with dw written in the conv Parameter's layout [Cout][Cin][KS][KS]
 * (Cin = C1 + C2): the split-K slab reduction stores that order directly, so
 * no hvit_conv_weight_unpack pass runs; dw_packed (Cout*Cin*KS*KS f32) is
 * scratch for the unsplit case. */
int hvit_conv_wgrad_torch(int dt, const hvit_conv_geom_t* g, const void* dy, float* dw, float* dw_packed, float* ws,
                          long long ws_elems, void* stream);                           /* dw_packed mode-0 layout */
int hvit_conv_weight_pack(const float* w, int Cout, int Cin, int KS, int mode, void* out, int out_dt,
                          void* stream);
int hvit_conv_weight_unpack(const float* dw_packed, int Cout, int Cin, int KS, float* dw, void* stream);
/* Eval-mode BatchNorm folded into the conv (components.py:55-85 in eval):
 * w_packed (mode 0, w_dt) = w * gamma * invstd per output channel, bias =
 * beta - mean * gamma * invstd, so relu(bn(conv(x, w))) = conv(x, w_packed) +
 * bias through hvit_conv_fwd with act HVIT_ACT_RELU (mean / invstd from
 * hvit_bn_eval_prep). */
int hvit_bn_fold(const float* w, int Cout, int Cin, int KS, const float* mean, const float* invstd,
                 const float* gamma, const float* beta, void* w_packed, int w_dt, float* bias, void* stream);

/* ---- Multi-head self-attention core (attention.py:82-107): softmax(q k^T *
 * scale) -> dropout -> @ v with qkv [B, N, 3, H, hd] (the qkv Linear output)
 * and o [B, N, H*hd]; lse [B, H, N] f32.  probs (optional, [B, H, N, N] f32)
 * receives the post-dropout attention map for return_attentions
 * (hybrid_vit.py:422-453).  Backward writes dq, dk, dv into dqkv (qkv layout);
 * delta_ws is [B, H, N] f32 scratch.  head_dim in {16, 32, 64}. */
int hvit_mhsa_fwd(int dt, const void* qkv, int B, int N, int H, int hd, float scale,
                  const hvit_dropout_t* dropout, void* o, float* lse, float* probs, void* stream);
int hvit_mhsa_bwd(int dt, const void* qkv, const void* o, const void* dout, const float* lse, int B, int N, int H,
                  int hd, float scale, const hvit_dropout_t* dropout, void* dqkv, float* delta_ws, void* stream);
/* The same with the attention-dropout decisions kept: the forward writes one
 * bit per (query, key) to keep_bits (hvit_mhsa_keep_bits_elems(B, N, H) 32-bit
 * words, 16-byte aligned) and the backward reads them instead of regenerating
 * the mask (bf16, head_dim 64, N <= 512, N % 4 == 0; other shapes and p = 0
 * ignore keep_bits).  Results equal hvit_mhsa_fwd / hvit_mhsa_bwd.
 * hvit_mhsa_keep_bits_used: 1 when the (dt, N, hd) kernels use keep bits (the
 * caller allocates none otherwise). */
long long hvit_mhsa_keep_bits_elems(int B, int N, int H);
int hvit_mhsa_keep_bits_used(int dt, int N, int hd);
int hvit_mhsa_fwd_kb(int dt, const void* qkv, int B, int N, int H, int hd, float scale, const hvit_dropout_t* dropout,
                     void* o, float* lse, unsigned* keep_bits, void* stream);
int hvit_mhsa_bwd_kb(int dt, const void* qkv, const void* o, const void* dout, const float* lse, int B, int N, int H,
                     int hd, float scale, const hvit_dropout_t* dropout, const unsigned* keep_bits, void* dqkv,
                     float* delta_ws, void* stream);
/* The backward with keep_bits optional (NULL: regenerate the mask) and the qkv
 * Linear's bias gradient (attention.py:55, Linear(dim, 3*dim) bias) formed on
 * the way: dbias_rows (f32 [hvit_mhsa_bias_rows(...)][3 * H * hd], NULL for
 * none) receives partial column sums of dqkv (overwritten) whose sum over the
 * rows is the bias gradient -- one row per attention workgroup, written by
 * the backward kernels themselves (other shapes: column reductions of dqkv).
 * Sum them with an hvit_slab_sum_t {dbias_rows, db, 3*H*hd, 3*H*hd, rows}. */
long long hvit_mhsa_bias_rows(int dt, int B, int N, int H, int hd);
int hvit_mhsa_bwd_db(int dt, const void* qkv, const void* o, const void* dout, const float* lse, int B, int N, int H,
                     int hd, float scale, const hvit_dropout_t* dropout, const unsigned* keep_bits, void* dqkv,
                     float* delta_ws, float* dbias_rows, void* stream);
/* fp8 (OCP e4m3) forward of the same core for BASELINE config 5: bf16 qkv / o,
 * per-(b, h) power-of-two scales for K and V and per-query scales for Q
 * (e4m3 range from the absolute maxima), QK^T on v_mfma_f32_16x16x32_fp8_fp8,
 * PV on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4.  hd = 64, N <= 256.
 * The dropout mask and lse match hvit_mhsa_fwd's, so hvit_mhsa_bwd (bf16) is
 * its backward. */
int hvit_mhsa_fwd_fp8(const void* qkv, int B, int N, int H, int hd, float scale, const hvit_dropout_t* dropout,
                      void* o, float* lse, void* stream);
/* The same storing its dropout decisions in hvit_mhsa_fwd_kb's keep-bit layout
 * (keep_bits nullable; N % 4 == 0), for hvit_mhsa_bwd_kb / _bwd_db. */
int hvit_mhsa_fwd_fp8_kb(const void* qkv, int B, int N, int H, int hd, float scale, const hvit_dropout_t* dropout,
                         void* o, float* lse, unsigned* keep_bits, void* stream);

/* ---- LayerNorm eps (attention.py:152-153, :271): x f32 [M, D] -> y; saves
 * mean / rstd [M].  Backward: dx = resid + dLN (resid may be NULL or alias dx),
 * dgamma / dbeta [D] overwritten. */
int hvit_layernorm_fwd(const float* x, const float* gamma, const float* beta, int M, int D, float eps, void* y,
                       int y_dt, float* mean, float* rstd, void* stream);
long long hvit_layernorm_bwd_ws_elems(int M, int D);   /* f32 slab for dgamma/dbeta partials */
/* The backward with the dropout + DropPath scaling of its output fused
 * (TransformerEncoderBlock, attention.py:206-211: the residual branch's
 * Dropout and DropPath before the proj / fc2 Linear): besides dx, writes
 * g_out = dx * keep / (1 - p) * rowscale[m / rows_per_sample] (g_dt) and
 * accumulates into acc3 = [dgamma | dbeta | colsum(g_out)] (3*D f32; caller-
 * zeroed with HVIT_ACC_ZEROED, else overwritten); ws =
 * hvit_layernorm_bwd_drop_ws_elems floats.  Same results as hvit_layernorm_bwd
 * followed by hvit_dropout_scale with a column sum. */
long long hvit_layernorm_bwd_drop_ws_elems(int M, int D);
int hvit_layernorm_bwd_drop(const void* dy, int dy_dt, const float* x, const float* mean, const float* rstd,
                            const float* gamma, int M, int D, const float* resid, float* dx, float* acc3,
                            const hvit_dropout_t* dropout, const float* rowscale, int rows_per_sample, void* g_out,
                            int g_dt, float* ws, long long ws_elems, int flags, void* stream);
int hvit_layernorm_bwd(const void* dy, int dy_dt, const float* x, const float* mean, const float* rstd,
                       const float* gamma, int M, int D, const float* resid, float* dx, float* dgamma,
                       float* dbeta, float* ws, long long ws_elems, int flags, void* stream);  /* ws may be
                       NULL; without ws, dgamma/dbeta are atomic targets (flags: HVIT_ACC_ZEROED) */

/* ---- BatchNorm2d -> ReLU -> Dropout2d -> MaxPool2d(pool) tail of ConvBlock /
 * TransposeConvBlock (components.py:67-85, :161-178).  z is the pre-BN conv
 * output NHWC [N, H, W, C] (C a power of two <= 256).  Train mode: mean /
 * invstd from hvit_bn_finalize (which also updates running stats with
 * momentum and the unbiased variance, and increments num_batches_tracked);
 * eval: hvit_bn_eval_prep (hvit_bn_finalize uses its partials buffer as scratch: overwritten).
 * Backward: dz from dy = grad of the pooled output;
 * sums (hvit_bn_act_bwd_sums_elems(C) floats: [2][C] result followed by
 * per-workgroup partial rows, all overwritten -- no zeroing needed, flags is
 * ignored) receives (dbeta, dgamma) in its first 2*C entries. */
long long hvit_bn_act_bwd_sums_elems(int C);
int hvit_bn_finalize(float* partials, int ntiles, int tile_rows, long long M, int C, float* mean,
                     float* invstd, float* running_mean, float* running_var, long long* num_batches_tracked,
                     float momentum, float eps, void* stream);
int hvit_bn_eval_prep(const float* running_mean, const float* running_var, int C, float eps, float* mean,
                      float* invstd, void* stream);
int hvit_bn_act_fwd(int dt, const void* z, int N, int H, int W, int C, const float* mean, const float* invstd,
                    const float* gamma, const float* beta, const hvit_dropout_t* dropout2d, int pool, void* y,
                    int y_dt, void* stream);
int hvit_bn_act_bwd(int dt, const void* z, int N, int H, int W, int C, const float* mean, const float* invstd,
                    const float* gamma, const float* beta, const hvit_dropout_t* dropout2d, int pool,
                    const void* dy, int dy_dt, int training, void* dz, int dz_dt, float* sums, int flags,
                    void* stream);

/* ---- The first encoder ConvBlock fused (hybrid_vit.py:196-208 -> components.py:
 * 55-85 with Cin = 1: Conv3x3 no bias -> BatchNorm2d -> ReLU -> Dropout2d ->
 * MaxPool2d(pool)), the conv output z never stored: hvit_c1block_stats writes
 * the BatchNorm partials of z (hvit_conv_fwd's layout, tile rows =
 * hvit_conv_bn_tile_rows) for hvit_bn_finalize; hvit_c1block_fwd recomputes z
 * and writes the pooled output y [N, H/pool, W/pool, Cout]; hvit_c1block_bwd
 * recomputes z, forms dz (hvit_bn_act_bwd's arithmetic) and reduces it straight
 * into the weight gradient dw_packed [Cout][9] f32 (sums: [dbeta | dgamma], 2*Cout
 * floats, overwritten; ws = hvit_c1block_bwd_ws floats, which also holds the
 * sums' per-workgroup partial rows).  g: C1 = 1, C2 = 0, U = 1, KS = 3, stride 1,
 * pad 1, Cout a power of two <= 256.  There is no input gradient (the model
 * input). */
int hvit_c1block_stats(int dt, const hvit_conv_geom_t* g, const void* w_packed, float* bn_partials, void* stream);
int hvit_c1block_fwd(int dt, const hvit_conv_geom_t* g, const void* w_packed, const float* mean,
                     const float* invstd, const float* gamma, const float* beta, const hvit_dropout_t* dropout2d,
                     int pool, void* y, int y_dt, void* stream);
long long hvit_c1block_bwd_ws(const hvit_conv_geom_t* g, int pool);
int hvit_c1block_bwd(int dt, const hvit_conv_geom_t* g, const void* w_packed, const float* mean, const float* invstd,
                     const float* gamma, const float* beta, const hvit_dropout_t* dropout2d, int pool, const void* dy,
                     int dy_dt, int training, float* sums, int flags, float* dw_packed, float* ws,
                     long long ws_elems, void* stream);

/* ---- Resampling (F.interpolate bilinear align_corners=False, hybrid_vit.py:
 * 381-386 and :459-465; nearest x2 backward + concat split, components.py:146,
 * hybrid_vit.py:389).  NHWC. */
int hvit_bilinear_fwd(const void* x, int x_dt, int N, int Hi, int Wi, int C, int Ho, int Wo, void* y, int y_dt,
                      void* stream);
int hvit_bilinear_bwd(const void* dy, int dy_dt, int N, int Ho, int Wo, int C, int Hi, int Wi, void* dx,
                      int dx_dt, int accumulate, void* stream);
int hvit_upsample_split_bwd(const void* du, int du_dt, int N, int H, int W, int U, int C1, int C2, void* dx1,
                            int dx1_dt, void* dx2, int dx2_dt, void* stream);

/* ---- Elementwise / reductions */
int hvit_cast(const void* src, int src_dt, void* dst, int dst_dt, long long n, void* stream);
/* Multi-tensor weight preparation, one launch for many parameters (replaces
 * per-weight hvit_cast / hvit_conv_weight_pack in the module forward):
 * kind 0 = cast f32 -> dt (numel elements), kind 1 / 2 = conv packing mode 0 / 1
 * of a [cout][cin][ks][ks] f32 weight, kind 3 = eval BatchNorm folded into a
 * mode-0 packing (hvit_bn_fold's result with mean = rmean, invstd =
 * rsqrt(rvar + eps): dst = w * gamma * invstd per output channel, bias[cout] =
 * beta - rmean * gamma * invstd; the bn fields are read for kind 3 only).
 * numel % 4 == 0, 16-byte aligned src. */
typedef struct {
  const float* src;
  void* dst;
  long long numel;
  int kind, dt;
  int cout, cin, ks;
  const float *gamma, *beta, *rmean, *rvar;
  float* bias;
  float eps;
} hvit_wprep_item_t;
int hvit_weight_prep(int count, const hvit_wprep_item_t* items, void* stream);
long long hvit_dropout_colsum_ws_elems(int N);
int hvit_dropout_scale(const void* g, int g_dt, long long M, int N, const hvit_dropout_t* dropout,
                       const float* rowscale, int rows_per_sample, void* out, int out_dt, float* colsum, float* ws,
                       long long ws_elems, void* stream);  /* colsum (nullable, f32 [N]) += column sums of out
                       (the bias gradient of the GEMM that consumes out); ws: hvit_dropout_colsum_ws_elems(N)
                       floats of per-workgroup partials (NULL: a slower two-pass fallback) */
int hvit_tanh_bwd(const void* dy, int dy_dt, const float* y, long long n, void* dz, int dz_dt, void* stream);
int hvit_reduce_rows(const void* x, int dt, long long M, long long N, long long ld, int accumulate, float* out,
                     void* stream);       /* out[n] (+)= sum_m x[m*ld+n], fixed summation order (no atomics) */
int hvit_sum_slabs(const float* ws, int splits, long long n, float* out, void* stream);
int hvit_droppath_scale(int B, const hvit_dropout_t* dropout, float* out, void* stream);  /* DropPath
                                                                     components.py:407-427 */
int hvit_droppath_scales(int B, int n, const hvit_dropout_t* dropouts, float* out, void* stream);
                     /* n <= 32 sites in one launch: out[j*B + b] = hvit_droppath_scale(B, &dropouts[j])[b]
                        (every transformer block's two branch multipliers, components.py:407-427) */

/* ---- Train-step neighbours.
 * CombinedLoss (training/losses.py:286-387; STOILoss :109-141, PerceptualLoss
 * :270-283): pred/target are [B][P] f32 (P = C*F*T per sample, contiguous).
 * hvit_loss_fwd writes stats [B][6] (per-sample sums the backward reads) and
 * out[5] = {total, l1, mse, stoi, perceptual}; terms with weight 0 are left
 * out of the total, as in the reference.  hvit_loss_bwd writes
 * dpred = gout[0] * d total / d pred (gout may be NULL: 1). */
typedef struct {
  float w_l1, w_mse, w_stoi, w_perc;
  int log_compression; /* log(x + 1e-8) on the L1 / MSE inputs (losses.py:319-321) */
} hvit_loss_cfg_t;
long long hvit_loss_ws_elems(int B, long long P);
int hvit_loss_fwd(const float* pred, const float* tgt, int B, long long P, const hvit_loss_cfg_t* cfg, float* ws,
                  long long ws_elems, float* stats, float* out, void* stream);
int hvit_loss_bwd(const float* pred, const float* tgt, int B, long long P, const hvit_loss_cfg_t* cfg,
                  const float* stats, const float* gout, float* dpred, void* stream);

/* clip_grad_norm_ (training/trainer.py:170-174 -> torch.nn.utils, norm 2) and
 * AdamW (training/optimizer.py:53-61 -> torch.optim.AdamW).  Tensor lists are
 * passed by value to the kernels (40 per launch), so nothing is copied to the
 * device.  hvit_clip_coef writes out[0] = total 2-norm of all tensors,
 * out[1] = min(max_norm / (norm + 1e-6), 1); hvit_scale_tensors multiplies
 * each tensor in place by coef[1] (torch's in-place clip).  hvit_adamw applies
 * one AdamW step per item, multiplying each gradient by coef[1] when coef is
 * non-NULL (clip fused into the update, gradients left untouched), and writes
 * the updated weight as bf16 to shadow_bf16 when non-NULL. */
typedef struct {
  void* ptr;
  long long numel;
} hvit_tensor_t;
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  void* shadow_bf16;
  long long numel;
  const float* step; /* nullable device step counter: when set, this tensor's bias corrections come from
                        *step on the device (torch.optim.AdamW capturable=True semantics; advance it with
                        hvit_step_bump); NULL: hyper bc1 / bc2 */
} hvit_adamw_item_t;
typedef struct {
  float lr, beta1, beta2, eps, weight_decay;
  float bc1, bc2; /* 1 - beta1^step, 1 - beta2^step (items without a device step) */
} hvit_adamw_hyper_t;
long long hvit_clip_ws_elems(int count);
int hvit_clip_coef(int count, const hvit_tensor_t* grads, float max_norm, float* ws, long long ws_elems, float* out,
                   void* stream);
int hvit_scale_tensors(int count, const hvit_tensor_t* tensors, const float* coef, void* stream);
int hvit_adamw(int count, const hvit_adamw_item_t* items, const hvit_adamw_hyper_t* hp, const float* coef,
               void* stream);
/* hvit_adamw with the hyper-parameters read on the device when hyper_dev (f32[5]
 * = lr, beta1, beta2, eps, weight_decay) is non-NULL: a captured optimizer step
 * (hipGraph) then replays the values the caller last wrote there (an LR
 * scheduler's), not the ones of capture time; hp's bc1 / bc2 still serve items
 * without a device step counter. */
int hvit_adamw_dev(int count, const hvit_adamw_item_t* items, const hvit_adamw_hyper_t* hp, const float* coef,
                   const float* hyper_dev, void* stream);
/* Device-resident training counters, advanced on the stream (so a captured train
 * step, hipGraph, replays with fresh values): hvit_rng_advance steps the dropout
 * state {base, counter} and writes the next forward's seed to *seed_out (what
 * that forward's hvit_dropout_t.seed_ptr points at; the model calls it once per
 * training forward); hvit_step_bump adds inc to n f32 step counters. */
int hvit_rng_advance(unsigned long long* state, unsigned long long* seed_out, void* stream);
int hvit_step_bump(float* steps, int n, float inc, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HVIT_H_ */
