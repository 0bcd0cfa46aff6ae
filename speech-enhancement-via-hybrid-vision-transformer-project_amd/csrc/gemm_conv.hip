// C-ABI conv forward (3x3 implicit GEMM, patch embedding) on the MFMA GEMM.
#include "gemm_host.h"

// rows per BatchNorm partial tile written by hvit_conv_fwd for geometry g
extern "C" int hvit_conv_bn_tile_rows(const hvit_conv_geom_t* g) {
  return g && thin_c1(g) ? hvit_thin_c1_bn_tile_rows() : 64;
}

extern "C" int hvit_conv_fwd(int dt, const hvit_conv_geom_t* g, const void* w_packed, const float* bias,
                             void* y, int y_dt, float* bn_partials, const hvit_epilogue_t* epi, void* stream) {
  if (int rc = check_geom(g)) return rc;
  HVIT_CHECK(w_packed && y, "hvit_conv_fwd: null pointer");
  if (int rc = check_epi(epi)) return rc;
  HVIT_CHECK(!epi || epi->act == HVIT_ACT_NONE || epi->act == HVIT_ACT_TANH || epi->act == HVIT_ACT_RELU ||
                 epi->act == HVIT_ACT_RELU_POOL2,
             "hvit_conv_fwd: act must be NONE, TANH, RELU or RELU_POOL2");
  HVIT_CHECK(!epi || (epi->act != HVIT_ACT_RELU && epi->act != HVIT_ACT_RELU_POOL2) || !bn_partials,
             "hvit_conv_fwd: RELU with BatchNorm partials");
  const bool pool2 = epi && epi->act == HVIT_ACT_RELU_POOL2;
  HVIT_CHECK(!epi || !epi->resid, "hvit_conv_fwd: residual epilogue unsupported");
  HVIT_CHECK(aligned16(w_packed), "hvit_conv_fwd: weight alignment");
  const bool plain_epi = !epi || (epi->dropout.p == 0.f && !epi->rowadd && !epi->colsum);
  if (pool2) {
    // the eval-mode encoder block with its max-pool (components.py:55-85 with pool 2, BatchNorm folded):
    // the implicit-im2col loader walks output pixels window by window, the epilogue keeps each
    // window's maximum; y is [N, Ho/2, Wo/2, Cout]
    HVIT_CHECK(dt == HVIT_BF16 && y_dt == HVIT_BF16 && plain_epi && !epi->resid && aligned16(y) && g->Cout % 4 == 0,
               "hvit_conv_fwd: RELU_POOL2 needs bf16 in / out, no dropout / rowadd / colsum, aligned output");
    auto la = conv_a<bf16_t>(g, g->src1, g->C1, g->src2, g->C2, g->Hs, g->Ws, g->U, g->KS, g->stride, g->pad);
    HVIT_CHECK(la.Ho > 0 && la.Wo > 0 && la.Ho % 2 == 0 && la.Wo % 2 == 0, "hvit_conv_fwd: RELU_POOL2 needs even Ho, Wo");
    HVIT_CHECK(conv_fast_ok(la, g->N), "hvit_conv_fwd: RELU_POOL2 needs 64-channel-multiple sources (fast loader)");
    Epi ep = to_epi(epi, y, y_dt, g->Cout);
    ep.bias = bias;
    LdConvF<bf16_t> f = conv_fast(la, g->N);
    f.pool2 = 1;
    return launch_gemm<bf16_t>(f, dense<bf16_t, true>(w_packed, la.Kt, g->Cout, la.Kt), la.P, g->Cout, la.Kt, 1, ep,
                               (hipStream_t)stream);
  }
  if (thin_c1(g) && plain_epi && !bias && (!epi || epi->act == HVIT_ACT_NONE) && aligned16(y))
    return hvit_thin_c1_fwd(dt, g, w_packed, y, y_dt, bn_partials, (hipStream_t)stream);
  // BN partial tiles follow hvit_conv_bn_tile_rows(g): the thin path must have been taken
  HVIT_CHECK(!bn_partials || !thin_c1(g), "hvit_conv_fwd: Cin=1 BatchNorm partials need the thin path "
                                           "(no bias / epilogue, 16-byte aligned output)");
  if (thin_o1(g) && plain_epi && !bias && !bn_partials && (!epi || epi->act != HVIT_ACT_RELU))
    return hvit_thin_o1_fwd(dt, g, w_packed, y, y_dt, epi && epi->act == HVIT_ACT_TANH, (hipStream_t)stream);
  HVIT_CHECK(!epi || epi->side.n <= 0, "hvit_conv_fwd: epilogue side jobs are for the linear entry points");
  Epi ep = to_epi(epi, y, y_dt, g->Cout);
  ep.bias = bias;
  ep.stats = bn_partials;
  DT_DISPATCH(dt, {
    auto la = conv_a<T>(g, g->src1, g->C1, g->src2, g->C2, g->Hs, g->Ws, g->U, g->KS, g->stride, g->pad);
    HVIT_CHECK(la.Ho > 0 && la.Wo > 0, "hvit_conv_fwd: empty output");
    int Kt = la.Kt;
    if constexpr (sizeof(T) == 2) {
      constexpr int ft = 0;  // automatic tile (forced 128x128 / 128x64 measured slower)
      if (conv_fast_ok(la, g->N))
        return launch_gemm<T>(conv_fast(la, g->N), dense<T, true>(w_packed, Kt, g->Cout, Kt), la.P, g->Cout, Kt, 1,
                              ep, (hipStream_t)stream, ft);
    }
    // odd reduction length (Cin=1 first conv): weights take the scalar load path
    return launch_gemm<T>(la, dense<T, true>(w_packed, Kt, g->Cout, Kt), la.P, g->Cout, Kt, 1, ep,
                          (hipStream_t)stream);
  });
}

