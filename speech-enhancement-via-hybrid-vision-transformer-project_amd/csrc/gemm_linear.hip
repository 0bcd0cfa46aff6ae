// C-ABI Linear fwd / dgrad / wgrad on the MFMA GEMM (see gemm_host.h).
#include "gemm_host.h"
#include "gemm_ring.h"

int hvit_attn_tune(int value);
int hvit_fp8_tune(int value);  // attention_fp8.hip

extern "C" int hvit_linear_fwd(int dt, const void* x, const void* w, const float* bias, int M, int N, int K,
                               void* y, int y_dt, const hvit_epilogue_t* epi, void* stream) {
  HVIT_CHECK(x && w && y, "hvit_linear_fwd: null pointer");
  HVIT_CHECK(M >= 0 && N > 0 && K > 0, "hvit_linear_fwd: bad shape M=%d N=%d K=%d", M, N, K);
  HVIT_CHECK(aligned16(x) && aligned16(w), "hvit_linear_fwd: x/w must be 16-byte aligned");
  if (int rc = check_epi(epi)) return rc;
  HVIT_CHECK(!epi || epi->act != HVIT_ACT_RELU, "hvit_linear_fwd: RELU is a conv-forward epilogue");
  Epi ep = to_epi(epi, y, y_dt, N);
  ep.bias = bias;
  if (int rc = take_side(epi ? &epi->side : nullptr, ep, M, (hipStream_t)stream)) return rc;
  if (M == 0) return HVIT_OK;
  if (dt == HVIT_BF16) {
    int rc = 0;
    if (try_ring(dense<bf16_t, true>(x, K, M, K), dense<bf16_t, true>(w, K, N, K), M, N, K, 1, ep,
                 (hipStream_t)stream, &rc))
      return rc;
  }
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
  HVIT_CHECK(!epi || epi->act != HVIT_ACT_RELU, "hvit_linear_dgrad: RELU is a conv-forward epilogue");
  Epi ep = to_epi(epi, dx, dx_dt, K);
  if (int rc = take_side(epi ? &epi->side : nullptr, ep, M, (hipStream_t)stream)) return rc;
  if (M == 0) return HVIT_OK;
  if (dt == HVIT_BF16 && N % 8 == 0) {
    int rc = 0;
    if (try_ring(dense<bf16_t, true>(dy, N, M, N), dense<bf16_t, false>(w, K, K, N), M, K, N, 1, ep,
                 (hipStream_t)stream, &rc))
      return rc;
  }
  DT_DISPATCH(dt, {
    HVIT_CHECK(N % Elem<T>::PER16 == 0 && K % Elem<T>::PER16 == 0, "hvit_linear_dgrad: N, K alignment");
    return launch_gemm<T>(dense<T, true>(dy, N, M, N), dense<T, false>(w, K, K, N), M, K, N, 1, ep,
                          (hipStream_t)stream);
  });
}

bool hvit_wgrad_small_ok(int dt, int M, int N, int K);  // wgrad_small.hip
long long hvit_wgrad_small_ws(int M, int N, int K);
int hvit_wgrad_small(const void* dy, const void* x, int M, int N, int K, float* dw, float* db, float* ws,
                     long long ws_elems, void* stream,
                     hvit_slab_sum_t* job = nullptr);

// Weight-gradient plan (hvit_gemm_tune(6, v)): 0 = round 5's (ring_pick /
// gemm.h per shape, split-K to ~256 workgroups), 1 = eight K slices for the
// token-major ViT shapes (1,024 tokens each at B = 32) on the 128x128 ring, or
// gemm.h's 128x128 kernels for N * K <= 512 * 512 (tools/wgrad_layout_probe.py,
// profiles/r6_wgrad_layout_probe.txt)
static int& wgrad_plan_ref() {
  static int v = 0;
  return v;
}
static int wgrad_plan_splits(int M) { return std::max(1, std::min(8, M / 1024)); }

extern "C" long long hvit_wgrad_workspace(int M, int N, int K) {
  // dw is [N_out x K_in] reduced over M rows; slabs only when splitting, each
  // slab followed by N_out bias partials (enough for every tile configuration
  // the entry point may pick: gemm.h's 128x128, the ring's 128x128 / 128x64,
  // the tall-skinny kernel of wgrad_small.hip)
  int s = std::max(wgrad_splits(N, K, M, LIN_WG_BM, LIN_WG_BN), wgrad_splits(N, K, M, 128, 64));
  s = std::max(s, wgrad_plan_splits(M));
  const long long g = s > 1 ? (long long)s * ((long long)N * K + N) : 0;
  // + room for the two-level bias column sums of a tall dy (hvit_reduce_rows_ws)
  return std::max(std::max(g, 64LL * N),
                  hvit_wgrad_small_ok(HVIT_BF16, M, N, K) ? hvit_wgrad_small_ws(M, N, K) : 0LL);
}

// per-tile arrival counters of the in-kernel split-K reduction (ring kernels;
// the smallest tile any configuration uses, 128x64)
extern "C" long long hvit_wgrad_tickets(int M, int N, int K) {
  (void)M;
  return (long long)cdiv(N, 128) * cdiv(K, 64);
}

// db (nullable): bias gradient sum_m dy[m][n].  The fused path (bf16, db ==
// dw + N*K) takes it from the A tiles the wgrad GEMM already stages (row sums
// over the token reduction); otherwise a column reduction of dy.
static int linear_wgrad_impl(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* db,
                             float* ws, long long ws_elems, unsigned* tickets, long long tickets_elems, int flags,
                             void* stream, hvit_slab_sum_t* job = nullptr,
                             const hvit_slab_sum_t* side = nullptr);

extern "C" int hvit_linear_wgrad(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* db,
                                 float* ws, long long ws_elems, void* stream) {
  return linear_wgrad_impl(dt, dy, x, M, N, K, dw, db, ws, ws_elems, nullptr, 0, 0, stream);
}

extern "C" int hvit_linear_wgrad_tk(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* db,
                                    float* ws, long long ws_elems, unsigned* tickets, long long tickets_elems, int flags,
                                    void* stream) {
  return linear_wgrad_impl(dt, dy, x, M, N, K, dw, db, ws, ws_elems, tickets, tickets_elems, flags, stream);
}

extern "C" int hvit_linear_wgrad_defer(int dt, const void* dy, const void* x, int M, int N, int K, float* dw,
                                       float* ws, long long ws_elems, const hvit_slab_sum_t* side,
                                       hvit_slab_sum_t* job, void* stream) {
  HVIT_CHECK(job, "hvit_linear_wgrad_defer: null job");
  *job = hvit_slab_sum_t{nullptr, nullptr, 0, 0, 0};
  return linear_wgrad_impl(dt, dy, x, M, N, K, dw, nullptr, ws, ws_elems, nullptr, 0, 0, stream, job, side);
}

// hvit_linear_wgrad_defer with the bias gradient: db == dw + N*K (or NULL);
// the tall-skinny path defers [dw | db] as one job, the others defer dw (when
// split) and finish db now
extern "C" int hvit_linear_wgrad_bias_defer(int dt, const void* dy, const void* x, int M, int N, int K, float* dw,
                                            float* db, float* ws, long long ws_elems, const hvit_slab_sum_t* side,
                                            hvit_slab_sum_t* job, void* stream) {
  HVIT_CHECK(job, "hvit_linear_wgrad_bias_defer: null job");
  *job = hvit_slab_sum_t{nullptr, nullptr, 0, 0, 0};
  return linear_wgrad_impl(dt, dy, x, M, N, K, dw, db, ws, ws_elems, nullptr, 0, 0, stream, job, side);
}

// the split-K slab sum: deferred into *job when the caller asked, else launched
static int slab_reduce(const float* ws, int splits, long long stride, long long n, float* out, void* stream,
                       hvit_slab_sum_t* job) {
  if (job) {
    *job = hvit_slab_sum_t{ws, out, n, stride, splits};
    return HVIT_OK;
  }
  return hvit_sum_slabs_strided(ws, splits, stride, n, out, stream);
}

static int linear_wgrad_impl(int dt, const void* dy, const void* x, int M, int N, int K, float* dw, float* db,
                             float* ws, long long ws_elems, unsigned* tickets, long long tickets_elems, int flags,
                             void* stream, hvit_slab_sum_t* job, const hvit_slab_sum_t* side) {
  HVIT_CHECK(dy && x && dw, "hvit_linear_wgrad: null pointer");
  HVIT_CHECK(M >= 0 && N > 0 && K > 0, "hvit_linear_wgrad: bad shape");
  HVIT_CHECK(aligned16(dy) && aligned16(x), "hvit_linear_wgrad: alignment");
  hipStream_t st = (hipStream_t)stream;
  // a side job carried by this launch's GEMM kernels (epi_side); paths that
  // launch none of them run it first as its own reduction
  Epi sj;
  if (int rc = take_side(side, sj, M, st)) return rc;
  const long long NK = (long long)N * K;
  int splits = wgrad_splits(N, K, M, LIN_WG_BM, LIN_WG_BN);
  if ((long long)splits * (NK + N) > ws_elems || !ws) splits = 1;
  auto side_alone = [&]() -> int {
    if (!sj.sj_n4) return HVIT_OK;
    const int r = hvit_sum_slabs_strided(sj.sj_src, sj.sj_splits, sj.sj_stride4 * 4, sj.sj_n4 * 4, sj.sj_dst, stream);
    sj.sj_n4 = 0;
    return r;
  };
  auto carry = [&](Epi& e) {
    e.sj_src = sj.sj_src;
    e.sj_dst = sj.sj_dst;
    e.sj_n4 = sj.sj_n4;
    e.sj_stride4 = sj.sj_stride4;
    e.sj_splits = sj.sj_splits;
  };
  if (M == 0) {
    if (int rc = side_alone()) return rc;
    (void)hipMemsetAsync(dw, 0, sizeof(float) * NK, st);
    if (db) (void)hipMemsetAsync(db, 0, sizeof(float) * N, st);
    return HVIT_OK;
  }
  // tall-skinny shapes (head, skip projections): one 64x64 tile per workgroup
  // over a chunk of rows
  if (!tickets && hvit_wgrad_small_ok(dt, M, N, K) && (!db || db == dw + NK) &&
      ws_elems >= hvit_wgrad_small_ws(M, N, K)) {
    if (int rc = side_alone()) return rc;
    return hvit_wgrad_small(dy, x, M, N, K, dw, db, ws, ws_elems, stream, job);
  }
  const bool fused_db = db && dt == HVIT_BF16 && db == dw + NK;
  // ring-pipelined kernels (gemm_ring.h) for bf16 without fused bias row sums
  const bool plan1 = wgrad_plan_ref() == 1 && dt == HVIT_BF16 && !fused_db && ring_default_cfg() < 0;
  const int rcfg = ring_default_cfg() >= 0 ? ring_default_cfg()
                   : plan1                 ? ((long)N * K <= 512L * 512 ? 0 : 2)
                                           : ring_pick(false, false, N, K, M);
  if (plan1) splits = wgrad_plan_splits(M);
  if ((long long)splits * (NK + N) > ws_elems || !ws) splits = 1;
  if (dt == HVIT_BF16 && !fused_db && N % 8 == 0 && K % 8 == 0 && rcfg > 0) {
    const RingCfg r = ring_cfg(rcfg);
    int s = plan1 ? wgrad_plan_splits(M) : wgrad_splits(N, K, M, r.bm, r.bn);
    if ((long long)s * (NK + N) > ws_elems || !ws) s = 1;
    s = plan_splits<bf16_t>(M, s);
    Epi e;
    e.out_dt = HVIT_F32;
    e.ldo = K;
    e.mode = s > 1 ? EPI_SLAB : EPI_STORE;
    e.out = s > 1 ? (void*)ws : (void*)dw;
    e.slab_stride = NK + N;
    carry(e);
    // in-kernel reduction when the caller provides the ticket counters
    const bool tk = s > 1 && tickets && tickets_elems >= (long long)(N / r.bm) * (K / r.bn);
    if (tk) {
      e.tickets = tickets;
      e.red_out = dw;
      if (!(flags & HVIT_ACC_ZEROED)) (void)hipMemsetAsync(tickets, 0, sizeof(unsigned) * (N / r.bm) * (K / r.bn), st);
    }
    int rc = 0;
    if (try_ring(dense<bf16_t, false>(dy, N, N, M), dense<bf16_t, false>(x, K, K, M), N, K, M, s, e, st, &rc, rcfg)) {
      if (rc) return rc;
      if (s > 1 && !tk)
        if (int rc2 = slab_reduce(ws, s, NK + N, NK, dw, stream, job)) return rc2;
      // (the slabs are consumed on the stream before this reuses ws; a deferred job
      // has no bias gradient)
      if (db) return hvit_reduce_rows_ws(dy, dt, M, N, N, 0, db, job ? nullptr : ws, ws_elems, stream);
      return HVIT_OK;
    }
  }
  Epi ep;
  ep.out_dt = HVIT_F32;
  ep.ldo = K;
  carry(ep);
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
    if (int rc = slab_reduce(ws, splits, NK + N, fused_db ? NK + N : NK, dw, stream, fused_db ? nullptr : job))
      return rc;
  }
  if (db && !fused_db) return hvit_reduce_rows_ws(dy, dt, M, N, N, 0, db, job ? nullptr : ws, ws_elems, stream);
  return HVIT_OK;
}

#ifdef HVIT_GEMM_STAMPS
__device__ unsigned long long hvit::g_gemm_stamps[65536 * 4];
extern "C" int hvit_debug_gemm_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hvit::g_gemm_stamps), sizeof(unsigned long long) * n) == hipSuccess
             ? 0
             : 1;
}
#endif

// Tuning knob for A/B measurements (tools/ring_bench.py): what 0 = the ring
// GEMM configuration of the bf16 linears (-1 = automatic per shape, 0 =
// gemm.h's kernels only, 1-5 = one ring configuration; see gemm_ring.h).
// Returns the previous value.
int hvit_c1_tune(int value);  // c1block.hip
int hvit_wgrad_group_tune(int value);  // wgrad_group.hip

extern "C" int hvit_gemm_tune(int what, int value) {
  if (what == 1) return hvit_c1_tune(value);
  // (3: the round-5 persistent epilogue-overlapped kernels, measured slower and
  // removed in round 6 -- git history before that round has gemm_pp.hip)
  if (what == 6) {  // weight-gradient plan (wgrad_plan_ref)
    const int old = wgrad_plan_ref();
    wgrad_plan_ref() = value;
    return old;
  }
  if (what == 8) {  // LDS-DMA stage buffers of the long-K 128x64 / 64x64 kernels (dma_depth_ref)
    const int old = dma_depth_ref();
    if (value >= 2 && value <= 4) dma_depth_ref() = value;
    return old;
  }
  if (what == 7) return hvit_wgrad_group_tune(value);  // grouped weight gradients: 0 256x256 tiles, 1 256x128
  if (what == 4) return hvit_attn_tune(value);  // attention backward for N <= 256: 1 single pass, 0 two kernels
  if (what == 5) return hvit_fp8_tune(value);  // fp8 attention forward: 0 round-4 kernel, 1 v2 16 waves, 2 v2 8 waves
  if (what == 2) {  // workgroup target of the linear weight gradients' split-K (0: default)
    const int old = (int)wg_target;
    wg_target = value > 0 ? value : 0;
    return old;
  }
  if (what != 0) return -1;
  const int old = ring_cfg_ref();
  ring_cfg_ref() = value;
  return old;
}

// Diagnostics (tools/wgrad_layout_probe.py): a weight-gradient-shaped split-K
// GEMM C[M, N] = sum_k A[m, k] B[n, k] into f32 slabs ws[splits][M * N + M]
// with each operand K-contiguous (kc = 1: rows of K, the forward layout) or
// M / N-contiguous (kc = 0: [K][M] / [K][N], the layout a weight gradient
// reads its token-major operands in), on pipeline cfg (0: gemm.h's kernels,
// 1-5: a gemm_ring.h configuration).  Used to price the operand layout and the
// tile / split choice of the weight gradients; not on the model's path.
extern "C" int hvit_probe_gemm_splitk(int kca, int kcb, const void* a, const void* b, int M, int N, int K, int splits,
                                      float* ws, int cfg, void* stream) {
  HVIT_CHECK(a && b && ws && M > 0 && N > 0 && K > 0 && splits >= 1, "hvit_probe_gemm_splitk: bad args");
  HVIT_CHECK(aligned16(a) && aligned16(b) && M % 8 == 0 && N % 8 == 0 && K % 64 == 0, "hvit_probe_gemm_splitk: align");
  Epi e;
  e.out_dt = HVIT_F32;
  e.ldo = N;
  e.mode = splits > 1 ? EPI_SLAB : EPI_STORE;
  e.out = ws;
  e.slab_stride = (long)M * N + M;
  hipStream_t st = (hipStream_t)stream;
  auto go = [&](auto la, auto lb) -> int {
    int rc = 0;
    if (cfg > 0) {
      if (try_ring(la, lb, M, N, K, splits, e, st, &rc, cfg)) return rc;
      hvit_set_error("hvit_probe_gemm_splitk: ring configuration %d does not apply", cfg);
      return HVIT_ERR_ARG;
    }
    return launch_gemm<bf16_t>(la, lb, M, N, K, splits, e, st);
  };
  if (kca && kcb) return go(dense<bf16_t, true>(a, K, M, K), dense<bf16_t, true>(b, K, N, K));
  if (kca) return go(dense<bf16_t, true>(a, K, M, K), dense<bf16_t, false>(b, N, N, K));
  if (kcb) return go(dense<bf16_t, false>(a, M, M, K), dense<bf16_t, true>(b, K, N, K));
  return go(dense<bf16_t, false>(a, M, M, K), dense<bf16_t, false>(b, N, N, K));
}
