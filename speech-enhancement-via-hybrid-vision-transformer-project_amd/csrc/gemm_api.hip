// C-ABI entry points built on the MFMA GEMM template (gemm.h):
//   Linear fwd / dgrad / wgrad  (nn.Linear in attention.py:55,58 and
//     components.py:224,227; to_feature_map hybrid_vit.py:153; the 1x1 skip
//     projections hybrid_vit.py:158-165 on NHWC pixels)
//   Conv fwd / dgrad / wgrad     (3x3 ConvBlock / TransposeConvBlock convs,
//     components.py:55-62, :149-158, with nearest-x2 upsample and the decoder's
//     channel concat folded into the operand gather; the k=s=4 patch embedding,
//     components.py:275-280, with the [B,N,D] token layout written directly).
#include <algorithm>

#include "gemm.h"

using namespace hvit;

namespace {

Epi to_epi(const hvit_epilogue_t* e, void* out, int out_dt, long ldo) {
  Epi ep;
  ep.out = out;
  ep.out_dt = out_dt;
  ep.ldo = ldo;
  if (!e) return ep;
  ep.act = e->act;
  ep.out2 = e->out2;
  ep.out2_dt = e->out2_dt;
  ep.ldo2 = ldo;
  ep.aux = e->aux;
  ep.aux_dt = e->aux_dt;
  ep.ldaux = ldo;
  if (e->dropout.p > 0.f) {
    ep.drop_thr = drop_threshold(e->dropout.p);
    ep.drop_scale = 1.f / (1.f - e->dropout.p);
    ep.seed = e->dropout.seed;
    ep.site = e->dropout.site;
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

int check_epi(const hvit_epilogue_t* e) {
  if (!e) return HVIT_OK;
  HVIT_CHECK(e->act >= HVIT_ACT_NONE && e->act <= HVIT_ACT_GELU_BWD, "epilogue: bad act %d", e->act);
  HVIT_CHECK(e->act != HVIT_ACT_GELU_DUAL || e->out2, "epilogue: GELU_DUAL needs out2");
  HVIT_CHECK(e->act != HVIT_ACT_GELU_BWD || e->aux, "epilogue: GELU_BWD needs aux");
  HVIT_CHECK(!(e->dropout.p < 0.f || e->dropout.p >= 1.f), "epilogue: dropout p out of range");
  return HVIT_OK;
}

// choose split-K so that a wgrad launch has enough workgroups: about 256
// workgroups of the given tile (one per CU, two for 64x64 tiles; each keeps
// >= 4 K-stages)
int wgrad_splits(long M, long N, long K, int bm, int bn, int bk = 64) {
  long tiles = (long)cdiv(M, bm) * cdiv(N, bn);
  const long target = bm * bn <= 64 * 64 ? 512 : 256;  // small tiles: two per CU
  long want = (target + tiles - 1) / tiles;
  long maxs = K / (4 * bk);
  if (want > maxs) want = maxs;
  if (want > 256) want = 256;
  if (want < 1) want = 1;
  return (int)want;
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
int hvit_sum_slabs_strided(const float* ws, int splits, long long stride, long long n, float* out, void* stream);
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

extern "C" int hvit_linear_fwd(int dt, const void* x, const void* w, const float* bias, int M, int N, int K,
                               void* y, int y_dt, const hvit_epilogue_t* epi, void* stream) {
  HVIT_CHECK(x && w && y, "hvit_linear_fwd: null pointer");
  HVIT_CHECK(M >= 0 && N > 0 && K > 0, "hvit_linear_fwd: bad shape M=%d N=%d K=%d", M, N, K);
  HVIT_CHECK(aligned16(x) && aligned16(w), "hvit_linear_fwd: x/w must be 16-byte aligned");
  if (int rc = check_epi(epi)) return rc;
  Epi ep = to_epi(epi, y, y_dt, N);
  ep.bias = bias;
  DT_DISPATCH(dt, {
    HVIT_CHECK(K % Elem<T>::PER16 == 0, "hvit_linear_fwd: K=%d must be a multiple of %d", K, Elem<T>::PER16);
    return launch_gemm<T>(dense<T, true>(x, K, M, K), dense<T, true>(w, K, N, K), M, N, K, 1, ep,
                          (hipStream_t)stream);
  });
}

extern "C" int hvit_linear_dgrad(int dt, const void* dy, const void* w, int M, int N, int K, void* dx, int dx_dt,
                                 const hvit_epilogue_t* epi, void* stream) {
  HVIT_CHECK(dy && w && dx, "hvit_linear_dgrad: null pointer");
  HVIT_CHECK(M >= 0 && N > 0 && K > 0, "hvit_linear_dgrad: bad shape");
  HVIT_CHECK(aligned16(dy) && aligned16(w), "hvit_linear_dgrad: alignment");
  if (int rc = check_epi(epi)) return rc;
  Epi ep = to_epi(epi, dx, dx_dt, K);
  DT_DISPATCH(dt, {
    HVIT_CHECK(N % Elem<T>::PER16 == 0 && K % Elem<T>::PER16 == 0, "hvit_linear_dgrad: N, K alignment");
    return launch_gemm<T>(dense<T, true>(dy, N, M, N), dense<T, false>(w, K, K, N), M, K, N, 1, ep,
                          (hipStream_t)stream);
  });
}

extern "C" long long hvit_wgrad_workspace(int M, int N, int K) {
  // dw is [N_out x K_in] reduced over M rows; slabs only when splitting, each
  // slab followed by N_out bias partials
  int s = wgrad_splits(N, K, M, LIN_WG_BM, LIN_WG_BN);
  return s > 1 ? (long long)s * ((long long)N * K + N) : 0;
}

// db (nullable): bias gradient sum_m dy[m][n].  The fused path (bf16, db ==
// dw + N*K) takes it from the A tiles the wgrad GEMM already stages (row sums
// over the token reduction); otherwise a column reduction of dy.
extern "C" int hvit_linear_wgrad(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* db,
                                 float* ws, long long ws_elems, void* stream) {
  HVIT_CHECK(dy && x && dw, "hvit_linear_wgrad: null pointer");
  HVIT_CHECK(M >= 0 && N > 0 && K > 0, "hvit_linear_wgrad: bad shape");
  HVIT_CHECK(aligned16(dy) && aligned16(x), "hvit_linear_wgrad: alignment");
  hipStream_t st = (hipStream_t)stream;
  const long long NK = (long long)N * K;
  int splits = wgrad_splits(N, K, M, LIN_WG_BM, LIN_WG_BN);
  if ((long long)splits * (NK + N) > ws_elems || !ws) splits = 1;
  if (M == 0) {
    (void)hipMemsetAsync(dw, 0, sizeof(float) * NK, st);
    if (db) (void)hipMemsetAsync(db, 0, sizeof(float) * N, st);
    return HVIT_OK;
  }
  const bool fused_db = db && dt == HVIT_BF16 && db == dw + NK;
  Epi ep;
  ep.out_dt = HVIT_F32;
  ep.ldo = K;
  DT_DISPATCH(dt, {
    HVIT_CHECK(N % Elem<T>::PER16 == 0 && K % Elem<T>::PER16 == 0, "hvit_linear_wgrad: N, K alignment");
    splits = plan_splits<T>(M, splits);
    ep.mode = splits > 1 ? EPI_SLAB : EPI_STORE;
    ep.out = splits > 1 ? (void*)ws : (void*)dw;
    ep.slab_stride = NK + N;
    if (fused_db) {
      ep.rs_ptr = splits > 1 ? ws + NK : db;
      ep.rs_stride = splits > 1 ? NK + N : 0;
    }
    int rc = launch_gemm<T>(dense<T, false>(dy, N, N, M), dense<T, false>(x, K, K, M), N, K, M, splits, ep, st,
                            LIN_WG_TILE);
    if (rc) return rc;
  });
  if (splits > 1) {
    // sums [dw | db] when fused (db follows dw), else dw alone
    if (int rc = hvit_sum_slabs_strided(ws, splits, NK + N, fused_db ? NK + N : NK, dw, stream)) return rc;
  }
  if (db && !fused_db) return hvit_reduce_rows(dy, dt, M, N, N, 0, db, stream);
  return HVIT_OK;
}

// rows per BatchNorm partial tile written by hvit_conv_fwd for geometry g
extern "C" int hvit_conv_bn_tile_rows(const hvit_conv_geom_t* g) {
  return g && thin_c1(g) ? hvit_thin_c1_bn_tile_rows() : 64;
}

extern "C" int hvit_conv_fwd(int dt, const hvit_conv_geom_t* g, const void* w_packed, const float* bias,
                             void* y, int y_dt, float* bn_partials, const hvit_epilogue_t* epi, void* stream) {
  if (int rc = check_geom(g)) return rc;
  HVIT_CHECK(w_packed && y, "hvit_conv_fwd: null pointer");
  if (int rc = check_epi(epi)) return rc;
  HVIT_CHECK(!epi || epi->act == HVIT_ACT_NONE || epi->act == HVIT_ACT_TANH,
             "hvit_conv_fwd: act must be NONE or TANH");
  HVIT_CHECK(!epi || !epi->resid, "hvit_conv_fwd: residual epilogue unsupported");
  HVIT_CHECK(aligned16(w_packed), "hvit_conv_fwd: weight alignment");
  const bool plain_epi = !epi || (epi->dropout.p == 0.f && !epi->rowadd && !epi->colsum);
  if (thin_c1(g) && plain_epi && !bias && (!epi || epi->act == HVIT_ACT_NONE) && aligned16(y))
    return hvit_thin_c1_fwd(dt, g, w_packed, y, y_dt, bn_partials, (hipStream_t)stream);
  // BN partial tiles follow hvit_conv_bn_tile_rows(g): the thin path must have been taken
  HVIT_CHECK(!bn_partials || !thin_c1(g), "hvit_conv_fwd: Cin=1 BatchNorm partials need the thin path "
                                           "(no bias / epilogue, 16-byte aligned output)");
  if (thin_o1(g) && plain_epi && !bias && !bn_partials)
    return hvit_thin_o1_fwd(dt, g, w_packed, y, y_dt, epi && epi->act == HVIT_ACT_TANH, (hipStream_t)stream);
  Epi ep = to_epi(epi, y, y_dt, g->Cout);
  ep.bias = bias;
  ep.stats = bn_partials;
  DT_DISPATCH(dt, {
    auto la = conv_a<T>(g, g->src1, g->C1, g->src2, g->C2, g->Hs, g->Ws, g->U, g->KS, g->stride, g->pad);
    HVIT_CHECK(la.Ho > 0 && la.Wo > 0, "hvit_conv_fwd: empty output");
    int Kt = la.Kt;
    if constexpr (sizeof(T) == 2) {
      if (conv_fast_ok(la, g->N))
        return launch_gemm<T>(conv_fast(la, g->N), dense<T, true>(w_packed, Kt, g->Cout, Kt), la.P, g->Cout, Kt, 1,
                              ep, (hipStream_t)stream);
    }
    // odd reduction length (Cin=1 first conv): weights take the scalar load path
    return launch_gemm<T>(la, dense<T, true>(w_packed, Kt, g->Cout, Kt), la.P, g->Cout, Kt, 1, ep,
                          (hipStream_t)stream);
  });
}

extern "C" int hvit_conv_dgrad(int dt, const hvit_conv_geom_t* g, const void* dy, const void* w, void* dx,
                               int dx_dt, void* stream) {
  if (int rc = check_geom(g)) return rc;
  HVIT_CHECK(dy && w && dx, "hvit_conv_dgrad: null pointer");
  HVIT_CHECK(aligned16(dy) && aligned16(w), "hvit_conv_dgrad: alignment");
  hipStream_t st = (hipStream_t)stream;
  const int Ctot = g->C1 + g->C2;
  const int Hi = g->Hs * g->U, Wi = g->Ws * g->U;
  const int Ho = (Hi + 2 * g->pad - g->KS) / g->stride + 1;
  const int Wo = (Wi + 2 * g->pad - g->KS) / g->stride + 1;
  if (g->KS == g->stride && g->pad == 0) {
    // non-overlapping patches: dX[patch pixel] = dT[token] . W  scattered back (col2im)
    HVIT_CHECK(g->U == 1 && g->C2 == 0, "hvit_conv_dgrad: patch path needs U=1, one source");
    if (Ho * g->KS != Hi || Wo * g->KS != Wi)
      (void)hipMemsetAsync(dx, 0, (size_t)g->N * Hi * Wi * Ctot * (dx_dt == HVIT_F32 ? 4 : 2), st);
    Epi ep;
    ep.mode = EPI_PATCH;
    ep.out = dx;
    ep.out_dt = dx_dt;
    ep.pP = g->KS;
    ep.pC = Ctot;
    ep.pHp = Ho;
    ep.pWp = Wo;
    ep.pH = Hi;
    ep.pW = Wi;
    const int Kt = g->KS * g->KS * Ctot;
    const int M = g->N * Ho * Wo;
    DT_DISPATCH(dt, {
      HVIT_CHECK(g->Cout % Elem<T>::PER16 == 0 && Kt % Elem<T>::PER16 == 0, "hvit_conv_dgrad: patch alignment");
      return launch_gemm<T>(dense<T, true>(dy, g->Cout, M, g->Cout), dense<T, false>(w, Kt, Kt, g->Cout), M, Kt,
                            g->Cout, 1, ep, st);
    });
  }
  HVIT_CHECK(g->stride == 1 && g->pad == g->KS / 2 && (g->KS & 1), "hvit_conv_dgrad: only odd same-convs");
  if (thin_o1(g) && dx_dt == dt && aligned16(dx)) return hvit_thin_o1_dgrad(dt, g, dy, w, dx, st);
  Epi ep;
  ep.out = dx;
  ep.out_dt = dx_dt;
  ep.ldo = Ctot;
  DT_DISPATCH(dt, {
    // dU = conv(dy, flipped/transposed W): im2col over dy (Cout channels, stride 1)
    auto la = conv_a<T>(g, dy, g->Cout, nullptr, 0, Ho, Wo, 1, g->KS, 1, g->pad);
    int Kt = la.Kt;
    if constexpr (sizeof(T) == 2) {
      if (conv_fast_ok(la, g->N))
        return launch_gemm<T>(conv_fast(la, g->N), dense<T, true>(w, Kt, Ctot, Kt), la.P, Ctot, Kt, 1, ep, st);
    }
    return launch_gemm<T>(la, dense<T, true>(w, Kt, Ctot, Kt), la.P, Ctot, Kt, 1, ep, st);
  });
}

extern "C" long long hvit_conv_wgrad_workspace(const hvit_conv_geom_t* g) {
  if (!g) return 0;
  if (thin_c1(g)) return hvit_thin_c1_wgrad_ws(g);
  if (thin_o1(g)) return hvit_thin_o1_wgrad_ws(g);
  const int Hi = g->Hs * g->U, Wi = g->Ws * g->U;
  const long Ho = (Hi + 2 * g->pad - g->KS) / g->stride + 1;
  const long Wo = (Wi + 2 * g->pad - g->KS) / g->stride + 1;
  const long Kt = (long)g->KS * g->KS * (g->C1 + g->C2);
  const ConvWgTile t(g->Cout);
  int s = wgrad_splits(g->Cout, Kt, g->N * Ho * Wo, t.bm, t.bn);
  return s > 1 ? (long long)s * g->Cout * Kt : 0;
}

extern "C" int hvit_conv_wgrad(int dt, const hvit_conv_geom_t* g, const void* dy, float* dw_packed, float* ws,
                               long long ws_elems, void* stream) {
  if (int rc = check_geom(g)) return rc;
  HVIT_CHECK(dy && dw_packed, "hvit_conv_wgrad: null pointer");
  HVIT_CHECK(aligned16(dy), "hvit_conv_wgrad: alignment");
  hipStream_t st = (hipStream_t)stream;
  if (thin_c1(g)) return hvit_thin_c1_wgrad(dt, g, dy, dw_packed, ws, ws_elems, st);
  if (thin_o1(g)) return hvit_thin_o1_wgrad(dt, g, dy, dw_packed, ws, ws_elems, st);
  DT_DISPATCH(dt, {
    auto la = conv_a<T>(g, g->src1, g->C1, g->src2, g->C2, g->Hs, g->Ws, g->U, g->KS, g->stride, g->pad);
    LdConv<T, false> lb;
    static_assert(sizeof(lb) == sizeof(la), "layout");
    __builtin_memcpy(&lb, &la, sizeof(la));
    LdConvWF<T> lf;
    const bool wfast = sizeof(T) == 2 && la.vec_ok && (la.U == 1 || la.U == 2) &&
                       (long)g->N * la.Hs * la.Ws * std::max(la.C1, la.C2) < (1L << 31);
    if (wfast) {
      lf.src1 = la.src1;
      lf.src2 = la.src2 ? la.src2 : la.src1;
      lf.C1 = la.C1;
      lf.C2 = la.C2;
      lf.Ctot = la.Ctot;
      lf.Hs = la.Hs;
      lf.Ws = la.Ws;
      lf.Hi = la.Hi;
      lf.Wi = la.Wi;
      lf.ushift = la.U == 2 ? 1 : 0;
      lf.KS = la.KS;
      lf.S = la.S;
      lf.Pd = la.Pd;
      lf.Ho = la.Ho;
      lf.Wo = la.Wo;
      lf.P = la.P;
      lf.Kt = la.Kt;
    }
    const int M = g->Cout, N = la.Kt, K = la.P;
    const ConvWgTile t(M);
    int splits = wgrad_splits(M, N, K, t.bm, t.bn);
    if ((long long)splits * M * N > ws_elems || !ws) splits = 1;
    splits = plan_splits<T>(K, splits);
    Epi ep;
    ep.mode = splits > 1 ? EPI_SLAB : EPI_STORE;
    ep.out = splits > 1 ? (void*)ws : (void*)dw_packed;
    ep.out_dt = HVIT_F32;
    ep.ldo = N;
    int rc = wfast ? launch_gemm<T>(dense<T, false>(dy, M, M, K), lf, M, N, K, splits, ep, st, t.tile)
                   : launch_gemm<T>(dense<T, false>(dy, M, M, K), lb, M, N, K, splits, ep, st, t.tile);
    if (rc) return rc;
    if (splits > 1) return hvit_sum_slabs(ws, splits, (long long)M * N, dw_packed, stream);
    return HVIT_OK;
  });
}

#ifdef HVIT_GEMM_STAMPS
__device__ unsigned long long hvit::g_gemm_stamps[65536 * 4];
extern "C" int hvit_debug_gemm_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hvit::g_gemm_stamps), sizeof(unsigned long long) * n) == hipSuccess
             ? 0
             : 1;
}
#endif
