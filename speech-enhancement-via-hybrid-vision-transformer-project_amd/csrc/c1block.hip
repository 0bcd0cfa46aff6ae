// The first encoder ConvBlock (components.py:15-99 via hybrid_vit.py:196-208:
// Conv3x3 Cin=1 no-bias -> BatchNorm2d -> ReLU -> Dropout2d -> MaxPool2d) as
// one fused block that never stores the conv output z (gfx950).
//
// At B=32 z is [32, 256, 256, 64] = 268 MB in bf16; the unfused path wrote it
// once and read it three times (BN apply, the backward's two passes), then
// wrote and re-read the same volume again as dz for the weight gradient.  A
// Cin = 1 3x3 conv is 9 MACs per output, so recomputing z from the 4 MB input
// inside each pass costs far less than moving it:
//   stats : z on the fly -> BatchNorm (mean, M2) tile partials   (thinconv.hip c1_fwd, no z store)
//   apply : z on the fly -> BN, ReLU, Dropout2d, max-pool -> y    (reads x, writes y)
//   sums  : z on the fly + dy -> per-channel (sum g, sum g xhat)  (training backward)
//   bwd   : z on the fly + dy -> dz in registers -> dW += dz * x  (no dz in HBM)
// A workgroup owns RB pooled rows of one sample: it stages the RB*P + 2 input
// rows they need (zero padded) in LDS; a thread owns CV channels with their
// 9*CV weights in registers and walks pooling windows, reading each window's
// (P+2)^2 input patch from LDS once.  Dropout2d multipliers are bnact.hip's
// counter hash of (sample, channel) and the max-pool routing is its
// first-maximum rule, so the fused and unfused paths implement the same
// function (z is kept in f32 here instead of being rounded to bf16 in HBM).
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace hvit_c1 {

// the backward sums' partial rows: one [2C] row per sums workgroup, written
// into the weight-gradient workspace (which the backward kernel overwrites only
// after the rows are reduced) and summed in row order: no atomics
constexpr int THREADS = 256;

struct Args {
  const void* x;  // [N, H, W] (Cin = 1), dtype dt
  const void* w;  // packed [Cout][9], dtype dt
  int N, H, W, C;
  int RB;  // pooled rows per workgroup
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  uint32_t thr;
  float dscale;
  uint32_t key;
  const unsigned long long* seedp;
  unsigned long long seed;
  uint32_t site;
  __device__ __forceinline__ void resolve() {
    if (seedp && thr) key = rng_key(seed ^ *seedp, site);
  }
};

template <typename T>
__device__ __forceinline__ float ldv(const void* p, long i) {
  return Elem<T>::to_f(((const T*)p)[i]);
}

// row and column of window `it` among rows of `w` windows, for it < 4 * w (a
// workgroup owns RB <= 4 rows): compares instead of an integer division (a
// ~25-instruction VALU sequence per use in these VALU-bound loops)
__device__ __forceinline__ void win_rc(int it, int w, int& r, int& ox) {
  r = (it >= w ? 1 : 0) + (it >= 2 * w ? 1 : 0) + (it >= 3 * w ? 1 : 0);
  ox = it - r * w;
}

// rows [y_lo, y_lo + nrows) of sample n, `pitch` floats each: column c holds
// x = c - 1 (zero outside [0, W)); rows outside the image are zeros.  Loads go
// out in batches of UB per thread (one load -> store chain per element would
// serialise the staging on memory latency).
template <typename T>
__device__ __forceinline__ void stage_rows(const Args& a, int n, int y_lo, int nrows, int pitch, float* xs) {
  const int tot = nrows * pitch;
  constexpr int UB = 8;
  for (int i0 = threadIdx.x; i0 < tot; i0 += THREADS * UB) {
    float v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = i0 + u * THREADS;
      const int r = i / pitch, c = i - r * pitch;
      const int y = y_lo + r, x = c - 1;
      const bool ok = i < tot && y >= 0 && y < a.H && x >= 0 && x < a.W;
      const float e = ldv<T>(a.x, ok ? ((long)n * a.H + y) * a.W + x : 0);
      v[u] = ok ? e : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UB; ++u)
      if (i0 + u * THREADS < tot) xs[i0 + u * THREADS] = v[u];
  }
  __syncthreads();
}

// the (P+2)^2 input patch of the window whose top-left pixel is staged row r*P,
// column ox*P (staged row 0 = image row oy0*P - 1, column 0 = x = -1)
template <int P>
__device__ __forceinline__ void load_patch(const float* xs, int pitch, int r, int ox, float (&pt)[P + 2][P + 2]) {
  const float* b = xs + r * P * pitch + ox * P;
#pragma unroll
  for (int i = 0; i < P + 2; ++i)
#pragma unroll
    for (int j = 0; j < P + 2; ++j) pt[i][j] = b[i * pitch + j];
}

template <int P, int CV>
__device__ __forceinline__ void conv_at(const float (&pt)[P + 2][P + 2], int qy, int qx, const float (&wr)[9][CV],
                                        float* z) {
#pragma unroll
  for (int e = 0; e < CV; ++e) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) s += pt[qy + k / 3][qx + k % 3] * wr[k][e];
    z[e] = s;
  }
}

template <typename T, int CV>
__device__ __forceinline__ void load_w(const Args& a, int c, float (&wr)[9][CV]) {
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < CV; ++e) wr[t][e] = ldv<T>(a.w, (c + e) * 9 + t);
}

template <int CV>
__device__ __forceinline__ void loadc(const float* p, int c, float* o) {
#pragma unroll
  for (int e = 0; e < CV; ++e) o[e] = p[c + e];
}

// relu(bn(z)) = max(z*sc + sh, 0); xhat = (z - mu)*is
template <int CV>
__device__ __forceinline__ void bn_consts(const Args& a, int c, float* sc, float* sh, float* mu, float* is) {
  float ga[CV], be[CV];
  loadc<CV>(a.mean, c, mu);
  loadc<CV>(a.invstd, c, is);
  loadc<CV>(a.gamma, c, ga);
  loadc<CV>(a.beta, c, be);
#pragma unroll
  for (int e = 0; e < CV; ++e) {
    sc[e] = is[e] * ga[e];
    sh[e] = be[e] - mu[e] * sc[e];
  }
}

// Dropout2d multipliers of channels c .. c+CV-1 of sample n (bnact.hip drop_mask)
template <int CV>
__device__ __forceinline__ void drop_cv(const Args& a, int n, int c, float* m) {
#pragma unroll
  for (int e = 0; e < CV; ++e) m[e] = 1.f;
  if (!a.thr) return;
  const uint64_t i0 = (uint64_t)n * a.C + c;
#pragma unroll
  for (int e4 = 0; e4 < CV; e4 += 4) {
    const f32x4 k = keep4_at(a.key, i0 + e4, a.thr, a.dscale);
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e4 + e] = k[e];
  }
}

template <typename TO, int CV>
__device__ __forceinline__ void store_cv(TO* p, const float* v) {
  if constexpr (sizeof(TO) == 2) {
    uint32_t u[CV / 2];
#pragma unroll
    for (int i = 0; i < CV / 2; ++i) u[i] = f2bf2(v[2 * i], v[2 * i + 1]);
    if constexpr (CV == 8) *(u32x4*)p = (u32x4){u[0], u[1], u[2], u[3]};
    else *(uint2*)p = make_uint2(u[0], u[1]);
  } else {
#pragma unroll
    for (int i = 0; i < CV; i += 4) *(f32x4*)(p + i) = (f32x4){v[i], v[i + 1], v[i + 2], v[i + 3]};
  }
}
template <typename TD, int CV>
__device__ __forceinline__ void load_cv(const TD* p, float* v) {
  if constexpr (sizeof(TD) == 2) {
    uint32_t u[CV / 2];
    if constexpr (CV == 8) {
      const u32x4 q = *(const u32x4*)p;
#pragma unroll
      for (int i = 0; i < 4; ++i) u[i] = q[i];
    } else {
      const uint2 q = *(const uint2*)p;
      u[0] = q.x;
      u[1] = q.y;
    }
#pragma unroll
    for (int i = 0; i < CV / 2; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < CV; i += 4) {
      const f32x4 q = *(const f32x4*)(p + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[i + j] = q[j];
    }
  }
}

// forward apply: y[n, oy, ox, c..] = Dropout2d(max over the window of relu(bn(z)))
template <typename T, typename TO, int P, int CV>
__global__ __launch_bounds__(THREADS) void c1_apply_kernel(Args a_, TO* __restrict__ y) {
  Args a = a_;
  a.resolve();
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int Ho = a.H / P, Wo = a.W / P;
  const int chunks = (Ho + a.RB - 1) / a.RB;
  const int n = blockIdx.x / chunks, oy0 = (blockIdx.x - n * chunks) * a.RB;
  const int pitch = a.W + 2;
  stage_rows<T>(a, n, oy0 * P - 1, a.RB * P + 2, pitch, xs);
  const int CC = a.C / CV, c = (threadIdx.x % CC) * CV, lanes = THREADS / CC;
  float wr[9][CV], sc[CV], sh[CV], mu[CV], is[CV], m[CV];
  load_w<T, CV>(a, c, wr);
  bn_consts<CV>(a, c, sc, sh, mu, is);
  drop_cv<CV>(a, n, c, m);
  const int rows = min(a.RB, Ho - oy0);
  for (int it = threadIdx.x / CC; it < rows * Wo; it += lanes) {
    int r, ox;
    win_rc(it, Wo, r, ox);
    float pt[P + 2][P + 2];
    load_patch<P>(xs, pitch, r, ox, pt);
    float best[CV];
#pragma unroll
    for (int e = 0; e < CV; ++e) best[e] = 0.f;  // the relu floor
#pragma unroll
    for (int q = 0; q < P * P; ++q) {
      float z[CV];
      conv_at<P, CV>(pt, q / P, q % P, wr, z);
#pragma unroll
      for (int e = 0; e < CV; ++e) best[e] = fmaxf(best[e], __builtin_fmaf(z[e], sc[e], sh[e]));
    }
#pragma unroll
    for (int e = 0; e < CV; ++e) best[e] *= m[e];
    store_cv<TO, CV>(y + (((long)n * Ho + oy0 + r) * Wo + ox) * a.C + c, best);
  }
}

// routed gradient of one full window: the first maximum of relu(bn(z)) over the
// window (torch's max-pool rule) gets g = dy * mask where the relu is open;
// arg = its position, zs = its z
template <int P, int CV>
__device__ __forceinline__ void route(const float (&zq)[P * P][CV], const float* sc, const float* sh, const float* d,
                                      const float* m, int* arg, float* g, float* zs) {
#pragma unroll
  for (int e = 0; e < CV; ++e) {
    float best = fmaxf(__builtin_fmaf(zq[0][e], sc[e], sh[e]), 0.f);
    float z = zq[0][e];
    int ai = 0;
#pragma unroll
    for (int q = 1; q < P * P; ++q) {
      const float v = fmaxf(__builtin_fmaf(zq[q][e], sc[e], sh[e]), 0.f);
      const bool gt = v > best;
      best = gt ? v : best;
      z = gt ? zq[q][e] : z;
      ai = gt ? q : ai;
    }
    arg[e] = ai;
    g[e] = best > 0.f ? d[e] * m[e] : 0.f;
    zs[e] = z;
  }
}

// backward reduce pass: per-channel sum g (dbeta), sum g * xhat (dgamma) over the
// full windows; one partial row [2C] per workgroup in part (no atomics)
template <typename T, typename TD, int P, int CV>
__global__ __launch_bounds__(THREADS) void c1_sums_kernel(Args a_, const TD* __restrict__ dy, float* __restrict__ part) {
  Args a = a_;
  a.resolve();
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int Ho = a.H / P, Wo = a.W / P;
  const int chunks = (Ho + a.RB - 1) / a.RB;
  const int n = blockIdx.x / chunks, oy0 = (blockIdx.x - n * chunks) * a.RB;
  const int pitch = a.W + 2;
  const int nrows = a.RB * P + 2;
  stage_rows<T>(a, n, oy0 * P - 1, nrows, pitch, xs);
  float* red = xs + nrows * pitch;  // [4 waves][2][C]
  const int CC = a.C / CV, c = (threadIdx.x % CC) * CV, lanes = THREADS / CC;
  float wr[9][CV], sc[CV], sh[CV], mu[CV], is[CV], m[CV], acc1[CV], acc2[CV];
  load_w<T, CV>(a, c, wr);
  bn_consts<CV>(a, c, sc, sh, mu, is);
  drop_cv<CV>(a, n, c, m);
#pragma unroll
  for (int e = 0; e < CV; ++e) acc1[e] = acc2[e] = 0.f;
  const int rows = min(a.RB, Ho - oy0);
  for (int it = threadIdx.x / CC; it < rows * Wo; it += lanes) {
    int r, ox;
    win_rc(it, Wo, r, ox);
    float d[CV];
    load_cv<TD, CV>(dy + (((long)n * Ho + oy0 + r) * Wo + ox) * a.C + c, d);
    float pt[P + 2][P + 2];
    load_patch<P>(xs, pitch, r, ox, pt);
    float zq[P * P][CV];
#pragma unroll
    for (int q = 0; q < P * P; ++q) conv_at<P, CV>(pt, q / P, q % P, wr, zq[q]);
    int arg[CV];
    float g[CV], zs[CV];
    route<P, CV>(zq, sc, sh, d, m, arg, g, zs);
#pragma unroll
    for (int e = 0; e < CV; ++e) {
      acc1[e] += g[e];
      acc2[e] += g[e] * ((zs[e] - mu[e]) * is[e]);
    }
  }
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
  for (int e = 0; e < CV; ++e) {
    float v1 = acc1[e], v2 = acc2[e];
    for (int o = CC; o < 64; o <<= 1) {
      v1 += __shfl_xor(v1, o, 64);
      v2 += __shfl_xor(v2, o, 64);
    }
    if (ln < CC) {
      red[(wv * 2) * a.C + c + e] = v1;
      red[(wv * 2 + 1) * a.C + c + e] = v2;
    }
  }
  __syncthreads();
  float* row = part + (size_t)2 * a.C * blockIdx.x;
  for (int i = threadIdx.x; i < 2 * a.C; i += THREADS)
    row[i] = red[i] + red[2 * a.C + i] + red[4 * a.C + i] + red[6 * a.C + i];
}

// backward apply + weight gradient: dz of every pixel (all windows, the
// partial ones at odd edges included: training-mode BN gives them ca + cb z),
// accumulated straight into dW[c][tap] += dz * x_tap; partials part[blk][C*9]
template <typename T, typename TD, int P, int CV, int CC>
__global__ __launch_bounds__(THREADS) void c1_bwd_kernel(Args a_, const TD* __restrict__ dy,
                                                         const float* __restrict__ sums, int training,
                                                         float* __restrict__ part) {
  Args a = a_;
  a.resolve();
  extern __shared__ __attribute__((aligned(16))) float xs[];
  constexpr int lanes = THREADS / CC;
  const int Ho = a.H / P, Wo = a.W / P;
  const int Hw = (a.H + P - 1) / P, Ww = (a.W + P - 1) / P;
  const int chunks = (Hw + a.RB - 1) / a.RB;
  const int n = blockIdx.x / chunks, oy0 = (blockIdx.x - n * chunks) * a.RB;
  const int pitch = a.W + 2;
  const int nrows = a.RB * P + 2;
  stage_rows<T>(a, n, oy0 * P - 1, nrows, pitch, xs);
  float* red = xs + nrows * pitch;  // [4 waves][C * 9]
  const int c = (threadIdx.x % CC) * CV;
  const float invM = 1.f / (float)((long)a.N * a.H * a.W);
  float wr[9][CV], sc[CV], sh[CV], m[CV], ca[CV], cb[CV];
  load_w<T, CV>(a, c, wr);
  {
    float mu[CV], is[CV], s1v[CV], s2v[CV];
    bn_consts<CV>(a, c, sc, sh, mu, is);
    loadc<CV>(sums, c, s1v);
    loadc<CV>(sums + a.C, c, s2v);
    // dz = sc*(g - s1 - xhat*s2) = sc*g + ca + cb*z  (bnact.hip's apply pass)
#pragma unroll
    for (int e = 0; e < CV; ++e) {
      const float s1 = training ? s1v[e] * invM : 0.f, s2 = training ? s2v[e] * invM : 0.f;
      cb[e] = -sc[e] * s2 * is[e];
      ca[e] = -sc[e] * s1 - cb[e] * mu[e];
    }
  }
  drop_cv<CV>(a, n, c, m);
  float acc[9][CV];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < CV; ++e) acc[t][e] = 0.f;
  const int rows = min(a.RB, Hw - oy0);
  for (int it = threadIdx.x / CC; it < rows * Ww; it += lanes) {
    int r, ox;
    win_rc(it, Ww, r, ox);
    const int oy = oy0 + r;
    const bool full = oy < Ho && ox < Wo;
    float d[CV];
#pragma unroll
    for (int e = 0; e < CV; ++e) d[e] = 0.f;
    if (full) load_cv<TD, CV>(dy + (((long)n * Ho + oy) * Wo + ox) * a.C + c, d);
    float pt[P + 2][P + 2];
    load_patch<P>(xs, pitch, r, ox, pt);
    float zq[P * P][CV];
#pragma unroll
    for (int q = 0; q < P * P; ++q) conv_at<P, CV>(pt, q / P, q % P, wr, zq[q]);
    int arg[CV];
    float g[CV], zs[CV];
    route<P, CV>(zq, sc, sh, d, m, arg, g, zs);  // d = 0 outside full windows -> g = 0
#pragma unroll
    for (int q = 0; q < P * P; ++q) {
      const int qy = q / P, qx = q % P;
      // pixels past an odd edge belong to no window but still have a dz
      const float inb = (oy * P + qy < a.H && ox * P + qx < a.W) ? 1.f : 0.f;
#pragma unroll
      for (int e = 0; e < CV; ++e) {
        const float gq = arg[e] == q ? g[e] : 0.f;
        const float dz = inb * (training ? sc[e] * gq + ca[e] + cb[e] * zq[q][e] : sc[e] * gq);
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t][e] += dz * pt[qy + t / 3][qx + t % 3];
      }
    }
  }
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < CV; ++e) {
      float v = acc[t][e];
#pragma unroll
      for (int o = CC; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      if (ln < CC) red[wv * a.C * 9 + (c + e) * 9 + t] = v;
    }
  __syncthreads();
  const int R = a.C * 9;
  for (int i = threadIdx.x; i < R; i += THREADS)
    part[(size_t)blockIdx.x * R + i] = red[i] + red[R + i] + red[2 * R + i] + red[3 * R + i];
}

// ============================================================================
// bf16 throughput path on the matrix cores (pool 2, Cout in {16, 32, 64}).
//
// The VALU kernels above spend 9 FMAs per output recomputing z and are
// VALU-bound (60-105 us per pass at B=32).  Here z comes from one
// v_mfma_f32_16x16x32_bf16 per 16 pixels x 16 channels: A = the 16 pixels' 9
// taps (k 0..8, the other 23 k zero), B = the weights [tap][channel].  Rows are
// ordered window-major -- row 4*wi + q is position q = 2*qy + qx of window wi
// -- so the accumulator layout (lane l: rows 4*(l>>4) + j, column l & 15) puts
// one whole pooling window of one channel in each lane's 4 registers: max-pool
// routing, BatchNorm and ReLU need no lane exchange.  Column n of channel block
// cb is channel NCB*n + cb, so a lane's NCB channels are contiguous in NHWC
// (one 8-byte store of 4 bf16 for Cout = 64).
//
// The weight gradient dW[tap][c] = sum_px x_tap[px] dz[px][c] is a second
// MFMA with K = pixels: a lane's dz registers of two 16-pixel groups ARE its
// B fragment (k = 8*(l>>4) + j <-> group j>>2, row 4*(l>>4) + (j&3): any k
// order works for a sum, as long as A uses the same), and A = the taps of those
// pixels read from LDS.  dz enters as bf16 hi + lo (two MFMAs), so the product
// keeps ~16 mantissa bits of dz; x is exact in bf16.
// BatchNorm statistics: from the 10x10 Gram matrix of (taps, 1) over a
// 1024-pixel tile (c1m_stats_kernel), in the tile layout of
// hvit_conv_bn_tile_rows (thinconv.hip c1_fwd).
constexpr int STATS_TILE = 1024;  // == hvit_thin_c1_bn_tile_rows()

__device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, a), __builtin_bit_cast(s16x8, b), c, 0,
                                                 0, 0);
}

// A fragment of a 16 x 32 tap matrix: lane l holds row l & 15, k = 8*(l>>4)+j;
// taps 0..7 on lanes 0-15, tap 8 on lanes 16-31 (j = 0), zeros elsewhere
__device__ __forceinline__ u32x4 tap_frag(const float* t, int l) {
  const u32x4 lo = {f2bf2(t[0], t[1]), f2bf2(t[2], t[3]), f2bf2(t[4], t[5]), f2bf2(t[6], t[7])};
  const u32x4 hi = {f2bf2(t[8], 0.f), 0u, 0u, 0u};
  const u32x4 zero = {0u, 0u, 0u, 0u};
  return l < 16 ? lo : (l < 32 ? hi : zero);
}

// B fragments of the weights: channel block cb, column n = l & 15 -> channel NCB*n + cb
template <int NCB>
__device__ __forceinline__ void weight_frags(const bf16_t* w, int l, u32x4 (&bw)[NCB]) {
  const int n = l & 15;
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const bf16_t* wc = w + (NCB * n + cb) * 9;
    float t[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) t[k] = bf2f(wc[k]);
    bw[cb] = tap_frag(t, l);
  }
}

// per-lane channel constants of channels c0 .. c0+NCB-1
template <int NCB>
struct ChanConsts {
  float sc[NCB], sh[NCB], mu[NCB], is[NCB], m[NCB];
  __device__ __forceinline__ void load(const Args& a, int n, int c0) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      const int c = c0 + cb;
      mu[cb] = a.mean[c];
      is[cb] = a.invstd[c];
      sc[cb] = is[cb] * a.gamma[c];
      sh[cb] = a.beta[c] - mu[cb] * sc[cb];
      m[cb] = a.thr ? (rng_u16k(a.key, (uint64_t)n * a.C + c) >= a.thr ? a.dscale : 0.f) : 1.f;
    }
  }
};

template <typename TD, int NCB>
__device__ __forceinline__ void load_ncb(const TD* p, float* v) {
  if constexpr (sizeof(TD) == 2) {
    if constexpr (NCB == 4) {
      const uint2 q = *(const uint2*)p;
      v[0] = __uint_as_float(q.x << 16);
      v[1] = __uint_as_float(q.x & 0xffff0000u);
      v[2] = __uint_as_float(q.y << 16);
      v[3] = __uint_as_float(q.y & 0xffff0000u);
    } else if constexpr (NCB == 2) {
      const uint32_t q = *(const uint32_t*)p;
      v[0] = __uint_as_float(q << 16);
      v[1] = __uint_as_float(q & 0xffff0000u);
    } else {
      v[0] = bf2f(p[0]);
    }
  } else {
#pragma unroll
    for (int e = 0; e < NCB; ++e) v[e] = p[e];
  }
}
// the same NCB channels as raw bits, converted at their use: the load of the
// next window group is issued before the current one's arithmetic (the dy
// stream was latency-bound: one dependent HBM round trip per group)
template <typename TD, int NCB>
struct RawNcb {
  float v[NCB];
  __device__ __forceinline__ void load(const TD* p) {
#pragma unroll
    for (int e = 0; e < NCB; ++e) v[e] = p[e];
  }
  __device__ __forceinline__ void get(float* o) const {
#pragma unroll
    for (int e = 0; e < NCB; ++e) o[e] = v[e];
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int e = 0; e < NCB; ++e) v[e] = 0.f;
  }
};
template <>
struct RawNcb<bf16_t, 4> {
  uint2 q;
  __device__ __forceinline__ void load(const bf16_t* p) { q = *(const uint2*)p; }
  __device__ __forceinline__ void get(float* o) const {
    o[0] = __uint_as_float(q.x << 16);
    o[1] = __uint_as_float(q.x & 0xffff0000u);
    o[2] = __uint_as_float(q.y << 16);
    o[3] = __uint_as_float(q.y & 0xffff0000u);
  }
  __device__ __forceinline__ void zero() { q = make_uint2(0u, 0u); }
};
template <>
struct RawNcb<bf16_t, 2> {
  uint32_t q;
  __device__ __forceinline__ void load(const bf16_t* p) { q = *(const uint32_t*)p; }
  __device__ __forceinline__ void get(float* o) const {
    o[0] = __uint_as_float(q << 16);
    o[1] = __uint_as_float(q & 0xffff0000u);
  }
  __device__ __forceinline__ void zero() { q = 0u; }
};
template <>
struct RawNcb<bf16_t, 1> {
  bf16_t q;
  __device__ __forceinline__ void load(const bf16_t* p) { q = *p; }
  __device__ __forceinline__ void get(float* o) const { o[0] = bf2f(q); }
  __device__ __forceinline__ void zero() { q = 0; }
};

template <typename TO, int NCB>
__device__ __forceinline__ void store_ncb(TO* p, const float* v) {
  if constexpr (sizeof(TO) == 2) {
    if constexpr (NCB == 4) *(uint2*)p = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
    else if constexpr (NCB == 2) *(uint32_t*)p = f2bf2(v[0], v[1]);
    else p[0] = f2bf(v[0]);
  } else {
#pragma unroll
    for (int e = 0; e < NCB; ++e) p[e] = v[e];
  }
}

// z of the 16 rows of window group g (windows 4g .. 4g+3 of the block, row-major
// over rows x ww windows per row), one accumulator per channel block.  Windows
// past nwin are clamped (their results are discarded by the caller).
template <int NCB>
__device__ __forceinline__ void group_z(const float* xs, int pitch, int g, int nwin, int ww, int l,
                                        const u32x4 (&bw)[NCB], f32x4 (&z)[NCB]) {
  const int row = l & 15;
  const int it = min(4 * g + (row >> 2), nwin - 1);
  int r, ox;
  win_rc(it, ww, r, ox);
  const float* b = xs + (r * 2 + ((row & 3) >> 1)) * pitch + ox * 2 + (row & 1);
  float t[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) t[k] = b[(k / 3) * pitch + k % 3];
  const u32x4 af = tap_frag(t, l);
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) z[cb] = mfma16(af, bw[cb], (f32x4){0.f, 0.f, 0.f, 0.f});
}

// first-maximum routing of one window (4 positions in registers): arg, relu'd
// maximum, z at the maximum
__device__ __forceinline__ void route4(const f32x4& z, float sc, float sh, int& arg, float& best, float& zs) {
  best = fmaxf(__builtin_fmaf(z[0], sc, sh), 0.f);
  zs = z[0];
  arg = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q) {
    const float v = fmaxf(__builtin_fmaf(z[q], sc, sh), 0.f);
    const bool gt = v > best;
    best = gt ? v : best;
    zs = gt ? z[q] : zs;
    arg = gt ? q : arg;
  }
}

template <typename TO, int NCB>
__global__ __launch_bounds__(THREADS) void c1m_apply_kernel(Args a_, TO* __restrict__ y) {
  Args a = a_;
  a.resolve();
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int Ho = a.H / 2, Wo = a.W / 2;
  const int chunks = (Ho + a.RB - 1) / a.RB;
  const int n = blockIdx.x / chunks, oy0 = (blockIdx.x - n * chunks) * a.RB;
  const int pitch = a.W + 4;
  stage_rows<bf16_t>(a, n, oy0 * 2 - 1, a.RB * 2 + 2, pitch, xs);
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = NCB * (l & 15);
  u32x4 bw[NCB];
  weight_frags<NCB>((const bf16_t*)a.w, l, bw);
  ChanConsts<NCB> k;
  k.load(a, n, c0);
  const int nwin = min(a.RB, Ho - oy0) * Wo;
  for (int g = wv; 4 * g < nwin; g += THREADS / 64) {
    f32x4 z[NCB];
    group_z<NCB>(xs, pitch, g, nwin, Wo, l, bw, z);
    const int it = 4 * g + (l >> 4);
    if (it < nwin) {
      int r, ox;
    win_rc(it, Wo, r, ox);
      float o[NCB];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        float best = 0.f;  // the relu floor
#pragma unroll
        for (int q = 0; q < 4; ++q) best = fmaxf(best, __builtin_fmaf(z[cb][q], k.sc[cb], k.sh[cb]));
        o[cb] = best * k.m[cb];
      }
      store_ncb<TO, NCB>(y + (((long)n * Ho + oy0 + r) * Wo + ox) * a.C + c0, o);
    }
  }
}

template <typename TD, int NCB>
__global__ __launch_bounds__(THREADS) void c1m_sums_kernel(Args a_, const TD* __restrict__ dy,
                                                           float* __restrict__ part) {
  Args a = a_;
  a.resolve();
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int Ho = a.H / 2, Wo = a.W / 2;
  const int chunks = (Ho + a.RB - 1) / a.RB;
  const int n = blockIdx.x / chunks, oy0 = (blockIdx.x - n * chunks) * a.RB;
  const int pitch = a.W + 4;
  const int nrows = a.RB * 2 + 2;
  stage_rows<bf16_t>(a, n, oy0 * 2 - 1, nrows, pitch, xs);
  float* red = xs + nrows * pitch;  // [4 waves][2][C]
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = NCB * (l & 15);
  u32x4 bw[NCB];
  weight_frags<NCB>((const bf16_t*)a.w, l, bw);
  ChanConsts<NCB> k;
  k.load(a, n, c0);
  float s1[NCB], s2[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) s1[cb] = s2[cb] = 0.f;
  const int nwin = min(a.RB, Ho - oy0) * Wo;
  // dy of group g for this lane (window 4g + (l >> 4)), one group ahead
  auto issue = [&](int g, RawNcb<TD, NCB>& raw) {
    const int it = 4 * g + (l >> 4);
    if (4 * g < nwin && it < nwin) {
      int r, ox;
    win_rc(it, Wo, r, ox);
      raw.load(dy + (((long)n * Ho + oy0 + r) * Wo + ox) * a.C + c0);
    } else {
      raw.zero();
    }
  };
  RawNcb<TD, NCB> nxt;
  issue(wv, nxt);
  for (int g = wv; 4 * g < nwin; g += THREADS / 64) {
    const RawNcb<TD, NCB> cur = nxt;
    issue(g + THREADS / 64, nxt);
    f32x4 z[NCB];
    group_z<NCB>(xs, pitch, g, nwin, Wo, l, bw, z);
    const int it = 4 * g + (l >> 4);
    if (it < nwin) {
      float d[NCB];
      cur.get(d);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        int arg;
        float best, zs;
        route4(z[cb], k.sc[cb], k.sh[cb], arg, best, zs);
        const float gv = best > 0.f ? d[cb] * k.m[cb] : 0.f;
        s1[cb] += gv;
        s2[cb] += gv * ((zs - k.mu[cb]) * k.is[cb]);
      }
    }
  }
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      s1[cb] += __shfl_xor(s1[cb], o, 64);
      s2[cb] += __shfl_xor(s2[cb], o, 64);
    }
    if (l < 16) {
      red[(wv * 2) * a.C + c0 + cb] = s1[cb];
      red[(wv * 2 + 1) * a.C + c0 + cb] = s2[cb];
    }
  }
  __syncthreads();
  float* row = part + (size_t)2 * a.C * blockIdx.x;
  for (int i = threadIdx.x; i < 2 * a.C; i += THREADS)
    row[i] = red[i] + red[2 * a.C + i] + red[4 * a.C + i] + red[6 * a.C + i];
}

// FULL: even H and W, whole row chunks and whole group pairs (the model's
// 256 x 256 input): no window / pixel range tests.
template <typename TD, int NCB, bool FULL = false>
__global__ __launch_bounds__(THREADS) void c1m_bwd_kernel(Args a_, const TD* __restrict__ dy,
                                                          const float* __restrict__ sums, int training,
                                                          float* __restrict__ part) {
  Args a = a_;
  a.resolve();
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int Ho = a.H / 2, Wo = a.W / 2;
  const int Hw = (a.H + 1) / 2, Ww = (a.W + 1) / 2;
  const int chunks = (Hw + a.RB - 1) / a.RB;
  const int n = blockIdx.x / chunks, oy0 = (blockIdx.x - n * chunks) * a.RB;
  const int pitch = a.W + 4;
  const int nrows = a.RB * 2 + 2;
  stage_rows<bf16_t>(a, n, oy0 * 2 - 1, nrows, pitch, xs);
  float* red = xs + nrows * pitch;  // [4 waves][C * 9]
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = NCB * (l & 15);
  u32x4 bw[NCB];
  weight_frags<NCB>((const bf16_t*)a.w, l, bw);
  ChanConsts<NCB> k;
  k.load(a, n, c0);
  // dz = sc*g + ca + cb*z  (training), sc*g (eval): bnact.hip's apply pass
  float ca[NCB], cbz[NCB];
  const float invM = 1.f / (float)((long)a.N * a.H * a.W);
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const float s1 = training ? sums[c0 + cb] * invM : 0.f, s2 = training ? sums[a.C + c0 + cb] * invM : 0.f;
    cbz[cb] = -k.sc[cb] * s2 * k.is[cb];
    ca[cb] = -k.sc[cb] * s1 - cbz[cb] * k.mu[cb];
  }
  f32x4 acc[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc[cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // wgrad A fragment: lane l holds tap m = l & 15 (0 past tap 8) of the pixels
  // k = 8*(l>>4) + j -> group j>>2, window l>>4, position j&3
  const int m = l & 15;
  const int mo = m < 9 ? (m / 3) * pitch + m % 3 : 0;
  const int nwin = min(a.RB, Hw - oy0) * Ww;
  // dy of group g for this lane (zero outside the full windows), issued one
  // iteration (two groups) ahead
  auto issue = [&](int g, RawNcb<TD, NCB>& raw) {
    const int it = 4 * g + (l >> 4);
    // (prefetches run past the block's last group: the window range test stays)
    const int itc = min(it, nwin - 1);
    int r, ox;
    win_rc(itc, Ww, r, ox);
    const int oy = oy0 + r;
    if (it < nwin && (FULL || (oy < Ho && ox < Wo))) raw.load(dy + (((long)n * Ho + oy) * Wo + ox) * a.C + c0);
    else raw.zero();
  };
  RawNcb<TD, NCB> nxt[2];
  issue(2 * wv, nxt[0]);
  issue(2 * wv + 1, nxt[1]);
  for (int g0 = 2 * wv; 4 * g0 < nwin; g0 += 2 * (THREADS / 64)) {
    u32x4 bhi[NCB], blo[NCB];
    float xa[8];
    const RawNcb<TD, NCB> cur[2] = {nxt[0], nxt[1]};
    issue(g0 + 2 * (THREADS / 64), nxt[0]);
    issue(g0 + 2 * (THREADS / 64) + 1, nxt[1]);
#pragma unroll
    for (int gs = 0; gs < 2; ++gs) {
      const int g = g0 + gs;
      f32x4 z[NCB];
      group_z<NCB>(xs, pitch, g, nwin, Ww, l, bw, z);
      const int it = 4 * g + (l >> 4);
      const bool valid = FULL || it < nwin;
      const int itc = FULL ? it : min(it, nwin - 1);
      int r, ox;
    win_rc(itc, Ww, r, ox);
      const int oy = oy0 + r;
      float d[NCB];
      cur[gs].get(d);
      // the lane's 4 pixels: inside the image and inside the block's windows?
      float inb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        inb[q] = (FULL || (valid && oy * 2 + (q >> 1) < a.H && ox * 2 + (q & 1) < a.W)) ? 1.f : 0.f;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        int arg;
        float best, zs;
        route4(z[cb], k.sc[cb], k.sh[cb], arg, best, zs);
        const float gv = best > 0.f ? d[cb] * k.m[cb] : 0.f;
        float dz[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float gq = arg == q ? gv : 0.f;
          const float v = fmaf(cbz[cb], z[cb][q], fmaf(k.sc[cb], gq, ca[cb]));  // ca = cbz = 0 in eval
          dz[q] = FULL ? v : inb[q] * v;
        }
        float lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) lo[q] = dz[q] - bf2f(f2bf(dz[q]));
        bhi[cb][2 * gs] = f2bf2(dz[0], dz[1]);
        bhi[cb][2 * gs + 1] = f2bf2(dz[2], dz[3]);
        blo[cb][2 * gs] = f2bf2(lo[0], lo[1]);
        blo[cb][2 * gs + 1] = f2bf2(lo[2], lo[3]);
      }
      // taps of this lane's wgrad pixels in group gs: window (l >> 4) of the
      // group as above, positions q = 0..3 (k = 8*(l>>4) + 4*gs + q)
      const float* b = xs + (r * 2) * pitch + ox * 2 + mo;
#pragma unroll
      for (int q = 0; q < 4; ++q) xa[4 * gs + q] = m < 9 ? b[(q >> 1) * pitch + (q & 1)] : 0.f;
    }
    // dz of invalid / outside pixels is 0, so their (clamped) taps add nothing
    const u32x4 aw = {f2bf2(xa[0], xa[1]), f2bf2(xa[2], xa[3]), f2bf2(xa[4], xa[5]), f2bf2(xa[6], xa[7])};
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      acc[cb] = mfma16(aw, bhi[cb], acc[cb]);
      acc[cb] = mfma16(aw, blo[cb], acc[cb]);
    }
  }
  // acc[cb]: lane l holds taps 4*(l>>4) + j of channel NCB*(l&15) + cb
  const int R = a.C * 9;
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tap = 4 * (l >> 4) + j;
      if (tap < 9) red[wv * R + (c0 + cb) * 9 + tap] = acc[cb][j];
    }
  __syncthreads();
  for (int i = threadIdx.x; i < R; i += THREADS)
    part[(size_t)blockIdx.x * R + i] = red[i] + red[R + i] + red[2 * R + i] + red[3 * R + i];
}

// BatchNorm (mean, M2) partials of z over 1024-pixel raster tiles (the layout
// hvit_bn_finalize reads with tile_rows = STATS_TILE), without forming z:
// z_c = w_c . t over the 9 taps t of a pixel, so a tile's
//   sum z_c = w_c . S,  sum z_c^2 = w_c^T G w_c,  S = sum_px t,  G = sum_px t t^T.
// G (with a constant-1 tap 9, so G[9][.] = S and G[9][9] = the pixel count)
// is one 16x16x32 MFMA per 32 pixels: A = B = the taps, lane l holding tap l&15
// of pixels k = 8*(l>>4) + j.  Taps are exact bf16 values, the products exact
// in f32.  Per channel the tile then needs 100 FMAs instead of 2 per pixel.
__global__ __launch_bounds__(THREADS) void c1m_stats_kernel(const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ w, float* __restrict__ stats,
                                                            int N, int H, int W, int C) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  __shared__ float gr[4][16][17];
  const int P = N * H * W;
  const int p0 = blockIdx.x * STATS_TILE, pend = min(P, p0 + STATS_TILE);
  const long base = (long)p0 - W - 1;
  const int ns = (pend - p0) + 2 * W + 2;
  {
    constexpr int UB = 8;
    for (int i0 = threadIdx.x; i0 < ns; i0 += THREADS * UB) {
      float v[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int i = i0 + u * THREADS;
        const long q = base + i;
        const bool ok = i < ns && q >= 0 && q < P;
        const float e = bf2f(x[ok ? q : 0]);
        v[u] = ok ? e : 0.f;
      }
#pragma unroll
      for (int u = 0; u < UB; ++u)
        if (i0 + u * THREADS < ns) xs[i0 + u * THREADS] = v[u];
    }
    __syncthreads();
  }
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int m = l & 15;  // this lane's tap: (dy, dx) = (m / 3, m % 3) for m < 9, 1 for m == 9, 0 above
  const int dy = m < 9 ? m / 3 - 1 : 0, dx = m < 9 ? m % 3 - 1 : 0;
  const int toff = dy * W + dx;
  const int HW = H * W;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int g = wv; 32 * g < pend - p0; g += THREADS / 64) {
    // pixels p0 + 32g + 8*(l>>4) + j, j = 0..7: (y, x) of the first, then stepped
    int p = p0 + 32 * g + 8 * (l >> 4);
    const int rem = p % HW;
    int yy = rem / W, xx = rem - yy * W;
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool in = p < pend;
      const bool ok = in && (unsigned)(yy + dy) < (unsigned)H && (unsigned)(xx + dx) < (unsigned)W;
      const float v = xs[min(p, pend - 1) - base + toff];
      t[j] = m < 9 ? (ok ? v : 0.f) : (m == 9 && in ? 1.f : 0.f);
      ++p;
      if (++xx == W) {
        xx = 0;
        if (++yy == H) yy = 0;
      }
    }
    const u32x4 f = {f2bf2(t[0], t[1]), f2bf2(t[2], t[3]), f2bf2(t[4], t[5]), f2bf2(t[6], t[7])};
    acc = mfma16(f, f, acc);
  }
  // acc: lane l holds G[4*(l>>4) + j][l & 15]; sum the four waves
#pragma unroll
  for (int j = 0; j < 4; ++j) gr[wv][4 * (l >> 4) + j][m] = acc[j];
  __syncthreads();
  if (threadIdx.x < 100) {
    const int r = threadIdx.x / 10, c = threadIdx.x % 10;
    gr[0][r][c] = gr[0][r][c] + gr[1][r][c] + gr[2][r][c] + gr[3][r][c];
  }
  __syncthreads();
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    float wc[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wc[k] = bf2f(w[c * 9 + k]);
    const float n = gr[0][9][9];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int a = 0; a < 9; ++a) {
      s1 += wc[a] * gr[0][9][a];
      float ga = 0.f;
#pragma unroll
      for (int b = 0; b < 9; ++b) ga += gr[0][a][b] * wc[b];
      s2 += wc[a] * ga;
    }
    const float mean = n > 0.f ? s1 / n : 0.f;
    stats[((size_t)blockIdx.x * C + c) * 2] = mean;
    stats[((size_t)blockIdx.x * C + c) * 2 + 1] = fmaxf(s2 - s1 * mean, 0.f);
  }
}

// pooled rows per workgroup: the staged rows (pitch W + 4) stay within 32 KiB of LDS
inline int rows_per_block(int W, int P) {
  const int maxrows = (32768 / 4) / (W + 4);
  int rb = (maxrows - 2) / P;
  return rb > 4 ? 4 : rb;
}

// the matrix-core kernels apply (bf16 operands, pool 2, 16 <= Cout <= 64);
// hvit_gemm_tune(1, 0) forces the VALU kernels (tests)
inline int& mfma_knob() {
  static int knob = 1;
  return knob;
}
inline bool use_mfma(int dt, int pool, int C) {
  return mfma_knob() != 0 && dt == HVIT_BF16 && pool == 2 && (C == 16 || C == 32 || C == 64);
}

int make_args(Args& a, int dt, const hvit_conv_geom_t* g, const void* w, const float* mean, const float* invstd,
              const float* gamma, const float* beta, const hvit_dropout_t* dr, int pool) {
  HVIT_CHECK(g && g->src1 && w && mean && invstd && gamma && beta, "c1block: null pointer");
  HVIT_CHECK(g->C1 == 1 && g->C2 == 0 && g->U == 1 && g->KS == 3 && g->stride == 1 && g->pad == 1,
             "c1block: Cin = 1 3x3 same conv only");
  HVIT_CHECK(g->Cout >= 8 && g->Cout <= 256 && (g->Cout & (g->Cout - 1)) == 0,
             "c1block: Cout=%d must be a power of two in [8, 256]", g->Cout);
  HVIT_CHECK(pool == 1 || pool == 2, "c1block: pool must be 1 or 2");
  HVIT_CHECK(dt == HVIT_BF16 || dt == HVIT_F32, "c1block: bad dtype");
  a.x = g->src1;
  a.w = w;
  a.N = g->N;
  a.H = g->Hs;
  a.W = g->Ws;
  a.C = g->Cout;
  a.RB = rows_per_block(g->Ws, pool);
  HVIT_CHECK(a.RB >= 1 && a.RB <= 4, "c1block: W=%d too wide for the staged rows", g->Ws);  // win_rc: RB <= 4
  a.mean = mean;
  a.invstd = invstd;
  a.gamma = gamma;
  a.beta = beta;
  a.thr = dr ? drop_threshold(dr->p) : 0;
  a.dscale = (dr && dr->p > 0.f) ? 1.f / (1.f - dr->p) : 1.f;
  a.key = dr ? rng_key(dr->seed, dr->site) : 0u;
  a.seedp = dr ? dr->seed_ptr : nullptr;
  a.seed = dr ? dr->seed : 0ull;
  a.site = dr ? dr->site : 0u;
  return HVIT_OK;
}

// fn(std::integral_constant<int, P>) for the runtime pool size
template <typename F>
void with_pool(int pool, F&& fn) {
  if (pool == 2) fn(std::integral_constant<int, 2>());
  else fn(std::integral_constant<int, 1>());
}

// fn(std::integral_constant<int, NCB>) for Cout = 16 * NCB
template <typename F>
void with_ncb(int C, F&& fn) {
  if (C == 64) fn(std::integral_constant<int, 4>());
  else if (C == 32) fn(std::integral_constant<int, 2>());
  else fn(std::integral_constant<int, 1>());
}

}  // namespace hvit_c1

using namespace hvit_c1;

int hvit_c1_tune(int value) {
  const int old = mfma_knob();
  mfma_knob() = value;
  return old;
}

int hvit_thin_c1_fwd(int dt, const hvit_conv_geom_t* g, const void* w, void* y, int y_dt, float* stats,
                     hipStream_t st);
int hvit_thin_c1_bn_tile_rows();

extern "C" int hvit_c1block_stats(int dt, const hvit_conv_geom_t* g, const void* w_packed, float* bn_partials,
                                  void* stream) {
  HVIT_CHECK(g && g->src1 && w_packed && bn_partials, "hvit_c1block_stats: null pointer");
  HVIT_CHECK(g->C1 == 1 && g->C2 == 0 && g->U == 1 && g->KS == 3 && g->stride == 1 && g->pad == 1,
             "hvit_c1block_stats: Cin = 1 3x3 same conv only");
  const int C = g->Cout;
  const size_t lds = sizeof(float) * (STATS_TILE + 2 * (size_t)g->Ws + 2);
  if (use_mfma(dt, 2, C) && lds <= 48 * 1024) {
    HVIT_CHECK(hvit_thin_c1_bn_tile_rows() == STATS_TILE, "hvit_c1block_stats: tile size mismatch");
    const long P = (long)g->N * g->Hs * g->Ws;
    HVIT_CHECK(P < (1L << 31), "hvit_c1block_stats: too many pixels");
    if (P <= 0) return HVIT_OK;
    hipLaunchKernelGGL(c1m_stats_kernel, dim3(cdiv(P, STATS_TILE)), dim3(THREADS), lds, (hipStream_t)stream,
                       (const bf16_t*)g->src1, (const bf16_t*)w_packed, bn_partials, g->N, g->Hs, g->Ws, C);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  return hvit_thin_c1_fwd(dt, g, w_packed, nullptr, dt, bn_partials, (hipStream_t)stream);
}

extern "C" int hvit_c1block_fwd(int dt, const hvit_conv_geom_t* g, const void* w_packed, const float* mean,
                                const float* invstd, const float* gamma, const float* beta,
                                const hvit_dropout_t* dropout2d, int pool, void* y, int y_dt, void* stream) {
  Args a;
  if (int rc = make_args(a, dt, g, w_packed, mean, invstd, gamma, beta, dropout2d, pool)) return rc;
  HVIT_CHECK(y && aligned16(y), "hvit_c1block_fwd: y null or misaligned");
  HVIT_CHECK(y_dt == HVIT_BF16 || y_dt == HVIT_F32, "hvit_c1block_fwd: bad y dtype");
  const int Ho = a.H / pool;
  if (Ho <= 0 || a.W / pool <= 0 || a.N <= 0) return HVIT_OK;
  const int blocks = a.N * ((Ho + a.RB - 1) / a.RB);
  hipStream_t st = (hipStream_t)stream;
  if (use_mfma(dt, pool, a.C)) {
    const size_t lds = sizeof(float) * (a.RB * 2 + 2) * (a.W + 4);
    with_ncb(a.C, [&](auto nc) {
      constexpr int NCB = decltype(nc)::value;
      if (y_dt == HVIT_BF16)
        hipLaunchKernelGGL((c1m_apply_kernel<bf16_t, NCB>), dim3(blocks), dim3(THREADS), lds, st, a, (bf16_t*)y);
      else
        hipLaunchKernelGGL((c1m_apply_kernel<float, NCB>), dim3(blocks), dim3(THREADS), lds, st, a, (float*)y);
    });
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  const size_t lds = sizeof(float) * (a.RB * pool + 2) * (a.W + 2);
  with_pool(pool, [&](auto pc) {
    constexpr int P = decltype(pc)::value;
    if (dt == HVIT_BF16 && y_dt == HVIT_BF16)
      hipLaunchKernelGGL((c1_apply_kernel<bf16_t, bf16_t, P, 8>), dim3(blocks), dim3(THREADS), lds, st, a,
                         (bf16_t*)y);
    else if (dt == HVIT_BF16)
      hipLaunchKernelGGL((c1_apply_kernel<bf16_t, float, P, 8>), dim3(blocks), dim3(THREADS), lds, st, a, (float*)y);
    else if (y_dt == HVIT_F32)
      hipLaunchKernelGGL((c1_apply_kernel<float, float, P, 8>), dim3(blocks), dim3(THREADS), lds, st, a, (float*)y);
    else
      hipLaunchKernelGGL((c1_apply_kernel<float, bf16_t, P, 8>), dim3(blocks), dim3(THREADS), lds, st, a,
                         (bf16_t*)y);
  });
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" long long hvit_c1block_bwd_ws(const hvit_conv_geom_t* g, int pool) {
  if (!g || (pool != 1 && pool != 2) || g->Ws <= 0 || g->N <= 0) return 0;
  const int rb = rows_per_block(g->Ws, pool);
  if (rb < 1) return 0;
  const int Hw = (g->Hs + pool - 1) / pool;
  return (long long)g->N * ((Hw + rb - 1) / rb) * g->Cout * 9;
}

int hvit_sum_slabs(const float* ws, int splits, long long n, float* out, void* stream);

extern "C" int hvit_c1block_bwd(int dt, const hvit_conv_geom_t* g, const void* w_packed, const float* mean,
                                const float* invstd, const float* gamma, const float* beta,
                                const hvit_dropout_t* dropout2d, int pool, const void* dy, int dy_dt, int training,
                                float* sums, int flags, float* dw_packed, float* ws, long long ws_elems,
                                void* stream) {
  Args a;
  if (int rc = make_args(a, dt, g, w_packed, mean, invstd, gamma, beta, dropout2d, pool)) return rc;
  HVIT_CHECK(dy && sums && dw_packed && ws, "hvit_c1block_bwd: null pointer");
  HVIT_CHECK(dy_dt == HVIT_BF16 || dy_dt == HVIT_F32, "hvit_c1block_bwd: bad dy dtype");
  HVIT_CHECK(aligned16(dy), "hvit_c1block_bwd: dy alignment");
  HVIT_CHECK(ws_elems >= hvit_c1block_bwd_ws(g, pool), "hvit_c1block_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int C = a.C;
  (void)flags;  // (partial rows, plain stores: no zeroed accumulator needed)
  if (a.N <= 0 || a.H <= 0 || a.W <= 0) {
    (void)hipMemsetAsync(sums, 0, sizeof(float) * 2 * C, st);
    (void)hipMemsetAsync(dw_packed, 0, sizeof(float) * C * 9, st);
    return HVIT_OK;
  }
  const bool mf = use_mfma(dt, pool, C);
  const int Ho = a.H / pool;
  const size_t lds_rows = sizeof(float) * (a.RB * pool + 2) * (a.W + (mf ? 4 : 2));
  constexpr int CV = 4;
  if (Ho > 0 && a.W / pool > 0) {  // dbeta / dgamma in both modes; training-mode dz also uses them
    const int blocks = a.N * ((Ho + a.RB - 1) / a.RB);
    const size_t lds = lds_rows + sizeof(float) * 8 * C;
    if (mf) {
      with_ncb(C, [&](auto nc) {
        constexpr int NCB = decltype(nc)::value;
        if (dy_dt == HVIT_BF16)
          hipLaunchKernelGGL((c1m_sums_kernel<bf16_t, NCB>), dim3(blocks), dim3(THREADS), lds, st, a,
                             (const bf16_t*)dy, ws);
        else
          hipLaunchKernelGGL((c1m_sums_kernel<float, NCB>), dim3(blocks), dim3(THREADS), lds, st, a,
                             (const float*)dy, ws);
      });
    } else {
      with_pool(pool, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        if (dt == HVIT_BF16 && dy_dt == HVIT_BF16)
          hipLaunchKernelGGL((c1_sums_kernel<bf16_t, bf16_t, P, CV>), dim3(blocks), dim3(THREADS), lds, st, a,
                             (const bf16_t*)dy, ws);
        else if (dt == HVIT_BF16)
          hipLaunchKernelGGL((c1_sums_kernel<bf16_t, float, P, CV>), dim3(blocks), dim3(THREADS), lds, st, a,
                             (const float*)dy, ws);
        else if (dy_dt == HVIT_BF16)
          hipLaunchKernelGGL((c1_sums_kernel<float, bf16_t, P, CV>), dim3(blocks), dim3(THREADS), lds, st, a,
                             (const bf16_t*)dy, ws);
        else
          hipLaunchKernelGGL((c1_sums_kernel<float, float, P, CV>), dim3(blocks), dim3(THREADS), lds, st, a,
                             (const float*)dy, ws);
      });
    }
    HVIT_LAUNCH_CHECK();
    HVIT_CHECK((long long)blocks * 2 * C <= ws_elems, "hvit_c1block_bwd: workspace too small for the sums rows");
    if (int rc = hvit_reduce_rows(ws, HVIT_F32, blocks, 2 * C, 2 * C, 0, sums, st)) return rc;
  } else {
    (void)hipMemsetAsync(sums, 0, sizeof(float) * 2 * C, st);
  }
  const int Hw = (a.H + pool - 1) / pool;
  const int blocks = a.N * ((Hw + a.RB - 1) / a.RB);
  const size_t lds = lds_rows + sizeof(float) * 4 * C * 9;
  HVIT_CHECK(lds <= 64 * 1024, "hvit_c1block_bwd: LDS %zu too large", lds);
  if (mf) {
    with_ncb(C, [&](auto nc) {
      constexpr int NCB = decltype(nc)::value;
      const int Ww = (a.W + pool - 1) / pool;
      const bool full = pool == 2 && a.H % 2 == 0 && a.W % 2 == 0 && Hw % a.RB == 0 && (a.RB * Ww) % 8 == 0;
      if (dy_dt == HVIT_BF16 && full)
        hipLaunchKernelGGL((c1m_bwd_kernel<bf16_t, NCB, true>), dim3(blocks), dim3(THREADS), lds, st, a,
                           (const bf16_t*)dy, sums, training, ws);
      else if (dy_dt == HVIT_BF16)
        hipLaunchKernelGGL((c1m_bwd_kernel<bf16_t, NCB>), dim3(blocks), dim3(THREADS), lds, st, a, (const bf16_t*)dy,
                           sums, training, ws);
      else
        hipLaunchKernelGGL((c1m_bwd_kernel<float, NCB>), dim3(blocks), dim3(THREADS), lds, st, a, (const float*)dy,
                           sums, training, ws);
    });
    HVIT_LAUNCH_CHECK();
    return hvit_sum_slabs(ws, blocks, (long long)C * 9, dw_packed, stream);
  }
  auto go = [&](auto ccc) {
    constexpr int CC = decltype(ccc)::value;
    with_pool(pool, [&](auto pc) {
      constexpr int P = decltype(pc)::value;
      if (dt == HVIT_BF16 && dy_dt == HVIT_BF16)
        hipLaunchKernelGGL((c1_bwd_kernel<bf16_t, bf16_t, P, CV, CC>), dim3(blocks), dim3(THREADS), lds, st, a,
                           (const bf16_t*)dy, sums, training, ws);
      else if (dt == HVIT_BF16)
        hipLaunchKernelGGL((c1_bwd_kernel<bf16_t, float, P, CV, CC>), dim3(blocks), dim3(THREADS), lds, st, a,
                           (const float*)dy, sums, training, ws);
      else if (dy_dt == HVIT_BF16)
        hipLaunchKernelGGL((c1_bwd_kernel<float, bf16_t, P, CV, CC>), dim3(blocks), dim3(THREADS), lds, st, a,
                           (const bf16_t*)dy, sums, training, ws);
      else
        hipLaunchKernelGGL((c1_bwd_kernel<float, float, P, CV, CC>), dim3(blocks), dim3(THREADS), lds, st, a,
                           (const float*)dy, sums, training, ws);
    });
  };
  switch (C / CV) {
    case 2: go(std::integral_constant<int, 2>()); break;
    case 4: go(std::integral_constant<int, 4>()); break;
    case 8: go(std::integral_constant<int, 8>()); break;
    case 16: go(std::integral_constant<int, 16>()); break;
    case 32: go(std::integral_constant<int, 32>()); break;
    case 64: go(std::integral_constant<int, 64>()); break;
    default: hvit_set_error("hvit_c1block_bwd: Cout=%d unsupported", C); return HVIT_ERR_ARG;
  }
  HVIT_LAUNCH_CHECK();
  return hvit_sum_slabs(ws, blocks, (long long)C * 9, dw_packed, stream);
}
