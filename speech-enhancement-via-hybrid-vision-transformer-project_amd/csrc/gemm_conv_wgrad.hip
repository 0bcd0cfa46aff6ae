// C-ABI conv weight gradient (im2col operand, split-K slabs) on the MFMA GEMM.
#include "gemm_host.h"

// shifted-row-window path for the 3x3 convs (conv_wgrad_rows.hip)
bool conv_wgrad_rows_geom_ok(const hvit_conv_geom_t* g);
bool conv_wgrad_rows_ok(int dt, const hvit_conv_geom_t* g);
long long conv_wgrad_rows_ws(const hvit_conv_geom_t* g);
int conv_wgrad_rows(const hvit_conv_geom_t* g, const void* dy, float* dw_packed, float* ws, long long ws_elems,
                    hipStream_t st, ConvSlabs* slabs = nullptr);

extern "C" long long hvit_conv_wgrad_workspace(const hvit_conv_geom_t* g) {
  if (!g) return 0;
  if (thin_c1(g)) return hvit_thin_c1_wgrad_ws(g);
  if (thin_o1(g)) return hvit_thin_o1_wgrad_ws(g);
  const int Hi = g->Hs * g->U, Wi = g->Ws * g->U;
  const long Ho = (Hi + 2 * g->pad - g->KS) / g->stride + 1;
  const long Wo = (Wi + 2 * g->pad - g->KS) / g->stride + 1;
  const long Kt = (long)g->KS * g->KS * (g->C1 + g->C2);
  const ConvWgTile t(g->Cout);
  int s = conv_wgrad_splits(g->Cout, Kt, g->N * Ho * Wo, t.bm, t.bn);
  const long long gen = s > 1 ? (long long)s * g->Cout * Kt : 0;
  // the dtype is not known here: room for either path
  return conv_wgrad_rows_geom_ok(g) ? std::max(gen, conv_wgrad_rows_ws(g)) : gen;
}

static int conv_wgrad_impl(int dt, const hvit_conv_geom_t* g, const void* dy, float* dw_packed, float* ws,
                           long long ws_elems, void* stream, ConvSlabs* slabs);

extern "C" int hvit_conv_wgrad(int dt, const hvit_conv_geom_t* g, const void* dy, float* dw_packed, float* ws,
                               long long ws_elems, void* stream) {
  return conv_wgrad_impl(dt, g, dy, dw_packed, ws, ws_elems, stream, nullptr);
}

extern "C" int hvit_conv_wgrad_torch(int dt, const hvit_conv_geom_t* g, const void* dy, float* dw, float* dw_packed,
                                     float* ws, long long ws_elems, void* stream) {
  if (int rc = check_geom(g)) return rc;
  HVIT_CHECK(dw && dw_packed, "hvit_conv_wgrad_torch: null pointer");
  const int Cin = g->C1 + g->C2, KS = g->KS, Cout = g->Cout;
  hipStream_t st = (hipStream_t)stream;
  // Cin = 1 (the first encoder conv): the packed order is already [Cout][1][KS][KS]
  if (Cin == 1) return conv_wgrad_impl(dt, g, dy, dw, ws, ws_elems, stream, nullptr);
  ConvSlabs sl;
  if (int rc = conv_wgrad_impl(dt, g, dy, dw_packed, ws, ws_elems, stream, &sl)) return rc;
  if (sl.splits > 1) return hvit_sum_slabs_unpack(ws, sl.splits, sl.slab, Cout, Cin, KS, dw, dw_packed, st);
  return hvit_conv_weight_unpack(dw_packed, Cout, Cin, KS, dw, stream);
}

static int conv_wgrad_impl(int dt, const hvit_conv_geom_t* g, const void* dy, float* dw_packed, float* ws,
                           long long ws_elems, void* stream, ConvSlabs* slabs) {
  if (int rc = check_geom(g)) return rc;
  HVIT_CHECK(dy && dw_packed, "hvit_conv_wgrad: null pointer");
  HVIT_CHECK(aligned16(dy), "hvit_conv_wgrad: alignment");
  hipStream_t st = (hipStream_t)stream;
  if (thin_c1(g)) return hvit_thin_c1_wgrad(dt, g, dy, dw_packed, ws, ws_elems, st);
  if (thin_o1(g)) return hvit_thin_o1_wgrad(dt, g, dy, dw_packed, ws, ws_elems, st);
  if (conv_wgrad_rows_ok(dt, g)) return conv_wgrad_rows(g, dy, dw_packed, ws, ws_elems, st, slabs);
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
    int splits = conv_wgrad_splits(M, N, K, t.bm, t.bn);
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
    if (splits > 1) {
      if (slabs) {  // the caller reduces them (hvit_conv_wgrad_torch)
        slabs->splits = splits;
        slabs->slab = (long long)M * N;
        return HVIT_OK;
      }
      return hvit_sum_slabs(ws, splits, (long long)M * N, dw_packed, stream);
    }
    return HVIT_OK;
  });
}
