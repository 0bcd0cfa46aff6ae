#pragma once
// Host-side helpers shared by the C-ABI entry points built on the MFMA GEMM template (gemm.h):
//   Linear fwd / dgrad / wgrad  (nn.Linear in attention.py:55,58 and
//     components.py:224,227; to_feature_map hybrid_vit.py:153; the 1x1 skip
//     projections hybrid_vit.py:158-165 on NHWC pixels)
//   Conv fwd / dgrad / wgrad     (3x3 ConvBlock / TransposeConvBlock convs,
//     components.py:55-62, :149-158, with nearest-x2 upsample and the decoder's
//     channel concat folded into the operand gather; the k=s=4 patch embedding,
//     components.py:275-280, with the [B,N,D] token layout written directly).
#include <algorithm>

#include <cstdlib>

#include "gemm.h"

using namespace hvit;

extern "C" int hvit_sum_slabs_strided(const float* ws, int splits, long long stride, long long n, float* out,
                                      void* stream);

namespace {

Epi to_epi(const hvit_epilogue_t* e, void* out, int out_dt, long ldo) {
  Epi ep;
  ep.out = out;
  ep.out_dt = out_dt;
  ep.ldo = ldo;
  if (!e) return ep;
  // GELU_DUAL_D / MUL_AUX: GELU_DUAL / GELU_BWD with gelu'(h) in place of h
  // (GELU_DUAL_DK: gd = 2, the stored gelu'(h) carries the dropout multiplier)
  ep.act = (e->act == HVIT_ACT_GELU_DUAL_D || e->act == HVIT_ACT_GELU_DUAL_DK) ? HVIT_ACT_GELU_DUAL
           : e->act == HVIT_ACT_MUL_AUX                                      ? HVIT_ACT_GELU_BWD
                                                                              : e->act;
  ep.gd = e->act == HVIT_ACT_GELU_DUAL_DK ? 2 : (e->act == HVIT_ACT_GELU_DUAL_D || e->act == HVIT_ACT_MUL_AUX);
  if (e->act == HVIT_ACT_RELU || e->act == HVIT_ACT_RELU_POOL2) {  // flags of the plain-store epilogue
    ep.act = HVIT_ACT_NONE;
    ep.relu = 1;
    ep.pool2 = e->act == HVIT_ACT_RELU_POOL2;
  }
  ep.out2 = e->out2;
  ep.out2_dt = e->out2_dt;
  ep.ldo2 = ldo;
  if (e->act == HVIT_ACT_GELU) {  // GELU_DUAL storing only dropout(gelu(v)), into y
    ep.act = HVIT_ACT_GELU_DUAL;
    ep.out2 = out;
    ep.out2_dt = out_dt;
    ep.out = nullptr;
  }
  ep.aux = e->aux;
  ep.aux_dt = e->aux_dt;
  ep.ldaux = ldo;
  if (e->dropout.p > 0.f) {
    ep.drop_thr = drop_threshold(e->dropout.p);
    ep.drop_scale = 1.f / (1.f - e->dropout.p);
    ep.drop_key = rng_key(e->dropout.seed, e->dropout.site);
    ep.drop_seedp = e->dropout.seed_ptr;
    ep.drop_seed = e->dropout.seed;
    ep.drop_site = e->dropout.site;
  }
  ep.resid = e->resid;
  ep.ldr = ldo;
  ep.rowscale = e->rowscale;
  ep.rows_per_sample = e->rows_per_sample > 0 ? e->rows_per_sample : 1;
  ep.rowadd = e->rowadd;
  ep.rowadd_ld = ldo;
  ep.rowadd_mod = e->rowadd_rows > 0 ? e->rowadd_rows : 1;
  ep.colsum = e->colsum;
  return ep;
}

// the side job of a linear fwd / dgrad epilogue: handed to the GEMM kernels
// (Epi::sj_*, float4 granules) when vector-aligned and the launch has rows,
// else run here as its own reduction launch
int take_side(const hvit_slab_sum_t* jp, Epi& ep, int M, hipStream_t st) {
  if (!jp || jp->n <= 0) return HVIT_OK;
  const hvit_slab_sum_t& j = *jp;
  HVIT_CHECK(j.src && j.dst && j.splits > 0 && j.stride >= j.n, "epilogue side job: bad slabs");
  if (M > 0 && j.n % 4 == 0 && j.stride % 4 == 0 && aligned16(j.src) && aligned16(j.dst)) {
    ep.sj_src = j.src;
    ep.sj_dst = j.dst;
    ep.sj_n4 = (long)(j.n / 4);
    ep.sj_stride4 = (long)(j.stride / 4);
    ep.sj_splits = j.splits;
    return HVIT_OK;
  }
  return hvit_sum_slabs_strided(j.src, j.splits, j.stride, j.n, j.dst, st);
}

int check_epi(const hvit_epilogue_t* e) {
  if (!e) return HVIT_OK;
  HVIT_CHECK(e->act >= HVIT_ACT_NONE && e->act <= HVIT_ACT_GELU_DUAL_DK, "epilogue: bad act %d", e->act);
  HVIT_CHECK((e->act != HVIT_ACT_GELU_DUAL && e->act != HVIT_ACT_GELU_DUAL_D && e->act != HVIT_ACT_GELU_DUAL_DK) || e->out2,
             "epilogue: GELU_DUAL needs out2");
  HVIT_CHECK((e->act != HVIT_ACT_GELU_BWD && e->act != HVIT_ACT_MUL_AUX) || e->aux, "epilogue: GELU_BWD needs aux");
  HVIT_CHECK(!(e->dropout.p < 0.f || e->dropout.p >= 1.f), "epilogue: dropout p out of range");
  return HVIT_OK;
}

// choose split-K so that a wgrad launch has enough workgroups: about 256
// workgroups of the given tile (one per CU, two for 64x64 tiles; each keeps
// >= 4 K-stages)
// (conv: the implicit-im2col weight gradient, whose 128x64 tiles fit more
// workgroups per CU; HVIT_WG_TARGET / HVIT_CONV_WG_TARGET override the targets
// for A/B measurements only)
// wg_target: the caller's workgroup target for the linear weight gradients
// that follow (hvit_set_wgrad_target; 0 = the default above) -- the side-stream
// weight gradients, which share the chip with the data-gradient chain
long wg_target = 0;
int wgrad_splits(long M, long N, long K, int bm, int bn, int bk = 64, bool conv = false) {
  long tiles = (long)cdiv(M, bm) * cdiv(N, bn);
  const long target = bm * bn <= 64 * 64 ? 512 : conv ? 256 : wg_target > 0 ? wg_target : 256;
  long want = (target + tiles - 1) / tiles;
  long maxs = K / (4 * bk);
  // a multiple of 8 slices: with the XCD-aware tile order (gemm.h tile_of)
  // each XCD then reduces whole K slices, whose operand rows stay in its L2
  if (want > 4 && maxs >= 8) want = std::min((want + 7) / 8 * 8, maxs / 8 * 8);
  if (want > maxs) want = maxs;
  if (want > 256) want = 256;
  if (want < 1) want = 1;
  return (int)want;
}
// Split-K of the conv weight gradient (implicit-im2col tiles, up to 3
// workgroups resident per CU).  tiles * splits workgroups are dealt evenly
// over the 256 CUs, so the busiest CU runs ceil(nwg / 256) of them: pick the
// split count that keeps the CUs evenly loaded (nwg / (256 ceil(nwg / 256))
// near 1) with >= 1.5 workgroups per CU on average for latency hiding, and
// prefer fewer splits (less slab traffic).  Measured on enc1 (9 tiles,
// tools/wgrad_sweep.py, B=32): 288 WGs 226 us, 432 -> 169, 576 -> 203,
// 792 -> 185.  HVIT_CONV_WG_TARGET selects the older fixed-target rule (A/B).
int conv_wgrad_splits(int M, long N, long K, int bm, int bn, int bk = 64) {
  const long tiles = (long)cdiv(M, bm) * cdiv(N, bn);
  const long maxs = std::max(1L, std::min(256L, K / (4 * bk)));
  int best = 1;
  double bs = -1e30;
  for (long s = 1; s <= maxs; ++s) {
    const long nwg = tiles * s;
    if (nwg > 768 && s > 1) break;
    const long per = (nwg + 255) / 256;
    double score = (double)nwg / (256.0 * per) - 0.02 * (double)nwg / 256.0;
    if (nwg < 384) score -= 0.5 * (384.0 - (double)nwg) / 384.0;
    if (score > bs + 1e-9) {
      bs = score;
      best = (int)s;
    }
  }
  return best;
}
// wgrad tiles: dense x dense -> 128x128; dense x im2col -> 128x64 (fits the
// register budget of the gathered operand's cursors)
constexpr int LIN_WG_BM = 128, LIN_WG_BN = 128, LIN_WG_TILE = 128;
// (64x64 when Cout <= 64 so no half-empty tiles)
struct ConvWgTile {
  int bm, bn, tile;
  explicit ConvWgTile(int cout) : bm(cout <= 64 ? 64 : 128), bn(64), tile(cout <= 64 ? 64 : 12864) {}
};

template <typename T>
LdConv<T, true> conv_a(const hvit_conv_geom_t* g, const void* s1, int C1, const void* s2, int C2, int Hs, int Ws,
                       int U, int KS, int S, int Pd) {
  LdConv<T, true> l;
  l.src1 = (const T*)s1;
  l.src2 = (const T*)s2;
  l.C1 = C1;
  l.C2 = C2;
  l.Ctot = C1 + C2;
  l.Hs = Hs;
  l.Ws = Ws;
  l.U = U;
  l.Hi = Hs * U;
  l.Wi = Ws * U;
  l.KS = KS;
  l.S = S;
  l.Pd = Pd;
  l.Ho = (l.Hi + 2 * Pd - KS) / S + 1;
  l.Wo = (l.Wi + 2 * Pd - KS) / S + 1;
  l.P = g->N * l.Ho * l.Wo;
  l.Kt = KS * KS * l.Ctot;
  constexpr int E = Elem<T>::PER16;
  l.vec_ok = (C1 % E == 0) && (C2 % E == 0) && aligned16(s1) && (!s2 || aligned16(s2));
  return l;
}

// the fast loader applies when every 64-channel stage stays inside one tap
// and one source, U is 1 or 2, and byte offsets fit 31 bits
template <typename T>
bool conv_fast_ok(const LdConv<T, true>& l, int N) {
  if (sizeof(T) != 2 || !l.vec_ok) return false;
  if (l.C1 % 64 || l.C2 % 64 || (l.U != 1 && l.U != 2)) return false;
  const long b1 = (long)N * l.Hs * l.Ws * l.C1 * sizeof(T), b2 = (long)N * l.Hs * l.Ws * l.C2 * sizeof(T);
  return b1 < (1L << 31) && b2 < (1L << 31);
}
template <typename T>
LdConvF<T> conv_fast(const LdConv<T, true>& l, int N) {
  LdConvF<T> f;
  f.src1 = l.src1;
  f.src2 = l.src2 ? l.src2 : l.src1;
  f.C1 = l.C1;
  f.C2 = l.C2;
  f.Ctot = l.Ctot;
  f.Hs = l.Hs;
  f.Ws = l.Ws;
  f.Hi = l.Hi;
  f.Wi = l.Wi;
  f.ushift = l.U == 2 ? 1 : 0;
  f.KS = l.KS;
  f.S = l.S;
  f.Pd = l.Pd;
  f.Ho = l.Ho;
  f.Wo = l.Wo;
  f.P = l.P;
  f.Kt = l.Kt;
  f.bytes1 = (unsigned)((long)N * l.Hs * l.Ws * l.C1 * sizeof(T));
  f.bytes2 = (unsigned)((long)N * l.Hs * l.Ws * l.C2 * sizeof(T));
  return f;
}

template <typename T, bool KC>
LdDense<T, KC> dense(const void* p, long ld, int rows, int K) {
  LdDense<T, KC> l;
  l.p = (const T*)p;
  l.ld = ld;
  l.rows = rows;
  l.K = K;
  l.vok = aligned16(p) && (ld % Elem<T>::PER16 == 0);
  return l;
}

int check_geom(const hvit_conv_geom_t* g) {
  HVIT_CHECK(g && g->src1, "conv: null geometry/source");
  HVIT_CHECK(g->C1 > 0 && g->C2 >= 0 && (g->C2 == 0 || g->src2), "conv: bad channels");
  HVIT_CHECK(g->N > 0 && g->Hs > 0 && g->Ws > 0 && g->U >= 1 && g->KS > 0 && g->stride > 0 && g->pad >= 0,
             "conv: bad geometry");
  HVIT_CHECK(g->Cout > 0, "conv: bad Cout");
  return HVIT_OK;
}

// thin-channel stencil kernels (thinconv.hip)
bool thin_c1(const hvit_conv_geom_t* g) {
  return g->C1 == 1 && g->C2 == 0 && g->U == 1 && g->KS == 3 && g->stride == 1 && g->pad == 1 &&
         g->Cout % 8 == 0 && g->Cout <= 256 && 256 % g->Cout == 0;
}
bool thin_o1(const hvit_conv_geom_t* g) {
  return g->Cout == 1 && g->C2 == 0 && g->KS == 3 && g->stride == 1 && g->pad == 1 && g->C1 % 8 == 0 &&
         g->C1 / 8 <= 64 && 64 % (g->C1 / 8) == 0 && aligned16(g->src1);
}

}  // namespace

int hvit_thin_c1_fwd(int dt, const hvit_conv_geom_t* g, const void* w, void* y, int y_dt, float* stats, hipStream_t st);
// split-K slabs a conv weight gradient left for its caller to reduce
// (hvit_conv_wgrad_torch): splits > 1 when there are any
struct ConvSlabs {
  int splits = 1;
  long long slab = 0;
};
int hvit_sum_slabs_unpack(const float* ws, int splits, long long slab, int Cout, int Cin, int KS, float* dw,
                          float* tmp, hipStream_t st);
int hvit_thin_c1_bn_tile_rows();
long long hvit_thin_c1_wgrad_ws(const hvit_conv_geom_t* g);
int hvit_thin_c1_wgrad(int dt, const hvit_conv_geom_t* g, const void* dz, float* dw, float* ws, long long ws_elems,
                       hipStream_t st);
int hvit_thin_o1_fwd(int dt, const hvit_conv_geom_t* g, const void* w, void* y, int y_dt, int act_tanh, hipStream_t st);
int hvit_thin_o1_dgrad(int dt, const hvit_conv_geom_t* g, const void* dz, const void* w, void* du, hipStream_t st);
long long hvit_thin_o1_wgrad_ws(const hvit_conv_geom_t* g);
int hvit_thin_o1_wgrad(int dt, const hvit_conv_geom_t* g, const void* dz, float* dw, float* ws, long long ws_elems,
                       hipStream_t st);

#define DT_DISPATCH(dt, ...)                   \
  if ((dt) == HVIT_BF16) {                     \
    using T = bf16_t;                          \
    __VA_ARGS__;                               \
  } else if ((dt) == HVIT_F32) {               \
    using T = float;                           \
    __VA_ARGS__;                               \
  } else {                                     \
    hvit_set_error("bad dtype %d", (int)(dt)); \
    return HVIT_ERR_ARG;                       \
  }

