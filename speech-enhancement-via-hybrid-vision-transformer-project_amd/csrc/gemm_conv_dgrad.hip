// C-ABI conv data gradient (3x3 implicit GEMM, patch col2im) on the MFMA GEMM.
#include "gemm_host.h"

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

