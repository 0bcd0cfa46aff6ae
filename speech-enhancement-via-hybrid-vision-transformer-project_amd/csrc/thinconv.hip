// Thin-channel 3x3 convolutions (gfx950) where an MFMA tile would be mostly
// padding:
//   * Cin = 1  : the first encoder conv (ConvBlock 0, components.py:55-62) on
//                the magnitude spectrogram -- fwd with fused BatchNorm partials,
//                and wgrad (a 2M-pixel reduction into 9*Cout weights);
//   * Cout = 1 : the final decoder conv + tanh (TransposeConvBlock final,
//                components.py:149-167) -- fwd, dgrad and wgrad.
// All are HBM-bound stencils on NHWC data: 16-byte channel vectors, one pass
// over the large tensor, weights in LDS.  Called from the hvit_conv_* entry
// points when the geometry matches (3x3, stride 1, pad 1).
#include <algorithm>

#include "common.h"

namespace hvit {

template <typename T>
struct Vec8 {  // 8 consecutive elements as floats (16 B for bf16, 32 B for f32)
  __device__ __forceinline__ static void load(const T* p, float* f) {
    if constexpr (sizeof(T) == 2) {
      u32x4 u = *(const u32x4*)p;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(u[i] << 16);
        f[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
      }
    } else {
      f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[i] = a[i];
        f[4 + i] = b[i];
      }
    }
  }
  __device__ __forceinline__ static void store(T* p, const float* f) {
    if constexpr (sizeof(T) == 2) {
      u32x4 u;
#pragma unroll
      for (int i = 0; i < 4; ++i) u[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
      *(u32x4*)p = u;
    } else {
      *(f32x4*)p = (f32x4){f[0], f[1], f[2], f[3]};
      *(f32x4*)(p + 4) = (f32x4){f[4], f[5], f[6], f[7]};
    }
  }
};

constexpr int TC_PIX = 64;   // pixels per stats tile (= BN partial tile rows)
constexpr int TC_TILES = 16;  // tiles per block

// ---------------------------------------------------------------- Cin = 1 ---
// A block owns a contiguous range [p0, pend) of flattened pixels p = (n, y, x)
// of the single-channel input.  Every 3x3 tap of those pixels that lies inside
// its image sits at flattened offset p + dy*W + dx, so the block stages the
// range widened by W + 1 on each side into LDS once (f32) and reads taps from
// there: no per-tap global loads, no per-pixel integer division (PixCursor
// walks (y, x) incrementally).  Dynamic LDS: strip_floats(pixels, W) floats.
__host__ __device__ inline int strip_floats(int pix, int W) { return pix + 2 * W + 2; }

template <typename T>
__device__ __forceinline__ long stage_strip(const T* __restrict__ x, int P, int p0, int pend, int W, float* xs) {
  const long base = (long)p0 - W - 1;
  const int n = (pend - p0) + 2 * W + 2;
  // batches of loads in flight per thread (a load -> store chain per element
  // serialised the staging on memory latency)
  constexpr int UB = 8;
  for (int i0 = threadIdx.x; i0 < n; i0 += 256 * UB) {
    float v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = i0 + u * 256;
      const long q = base + i;
      const bool ok = i < n && q >= 0 && q < P;
      const float e = Elem<T>::to_f(x[ok ? q : 0]);  // unconditional load (clamped): no branch per element
      v[u] = ok ? e : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UB; ++u)
      if (i0 + u * 256 < n) xs[i0 + u * 256] = v[u];
  }
  __syncthreads();
  return base;
}

struct PixCursor {
  int y, x;
  __device__ __forceinline__ PixCursor(int p, int H, int W) {
    const int rem = p % (H * W);
    y = rem / W;
    x = rem - y * W;
  }
  __device__ __forceinline__ void advance(int d, int H, int W) {
    x += d;
    while (x >= W) {
      x -= W;
      if (++y == H) y = 0;
    }
  }
};

// xv[t] = input at tap t = (dy+1)*3 + (dx+1) of the pixel whose staged centre is c
__device__ __forceinline__ void taps9(const float* c, int y, int x, int H, int W, float* xv) {
  const bool up = y > 0, dn = y + 1 < H, lf = x > 0, rt = x + 1 < W;
  xv[0] = (up && lf) ? c[-W - 1] : 0.f;
  xv[1] = up ? c[-W] : 0.f;
  xv[2] = (up && rt) ? c[-W + 1] : 0.f;
  xv[3] = lf ? c[-1] : 0.f;
  xv[4] = c[0];
  xv[5] = rt ? c[1] : 0.f;
  xv[6] = (dn && lf) ? c[W - 1] : 0.f;
  xv[7] = dn ? c[W] : 0.f;
  xv[8] = (dn && rt) ? c[W + 1] : 0.f;
}

// z[p][co] = sum_tap x[p + tap] * w[co][tap]; BN partials per 64-pixel tile.
// BN partial tile of the Cin = 1 path: one (mean, M2) per channel and block
constexpr int C1_BLOCK_PIX = TC_PIX * TC_TILES;

template <typename T, typename TO>
__global__ __launch_bounds__(256) void c1_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w, TO* __restrict__ z,
                                                     float* __restrict__ stats, int N, int H, int W, int Cout) {
  // Each thread owns one 8-channel group cc (fixed: 256 % CC == 0) with its 72
  // weights in registers and walks the block's C1_BLOCK_PIX pixels with a
  // stride of 256 / CC, keeping a Welford (mean, M2) per channel in registers;
  // lanes of the same group merge (Chan) through shuffles, the four waves
  // through LDS, once per block: BN partial tile = the block's pixels.
  __shared__ float red[4][256][3];  // [wave][channel][count, mean, M2]
  extern __shared__ float xs[];     // the block's input strip (stage_strip)
  const int CC = Cout / 8;
  const int cc = threadIdx.x % CC, pl = threadIdx.x / CC, lanes = 256 / CC;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  float wr[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) wr[t][e] = Elem<T>::to_f(w[(cc * 8 + e) * 9 + t]);
  const int P = N * H * W;
  const int p0 = blockIdx.x * C1_BLOCK_PIX, pend = min(P, p0 + C1_BLOCK_PIX);
  const long base = stage_strip(x, P, p0, pend, W, xs);
  float mu[8], m2[8], cnt = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) mu[e] = m2[e] = 0.f;
  PixCursor pc(p0 + pl, H, W);
  for (int p = p0 + pl; p < pend; p += lanes, pc.advance(lanes, H, W)) {
    float xv[9];
    taps9(xs + (p - base), pc.y, pc.x, H, W, xv);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t) acc += xv[t] * wr[t][e];
      o[e] = acc;
    }
    if (z) Vec8<TO>::store(z + (size_t)p * Cout + cc * 8, o);  // null: statistics only (c1block.hip)
    cnt += 1.f;
    const float inv = __builtin_amdgcn_rcpf(cnt);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = o[e] - mu[e];
      mu[e] += d * inv;
      m2[e] += d * (o[e] - mu[e]);
    }
  }
  if (!stats) return;
  for (int off = CC; off < 64; off <<= 1) {
    const float cb = __shfl_xor(cnt, off, 64);
    const float ct = cnt + cb;
    const float fb = ct > 0.f ? cb / ct : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float mb = __shfl_xor(mu[e], off, 64), qb = __shfl_xor(m2[e], off, 64);
      const float d = mb - mu[e];
      m2[e] += qb + d * d * cnt * fb;
      mu[e] += d * fb;
    }
    cnt = ct;
  }
  if (ln < CC) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[wv][cc * 8 + e][0] = cnt;
      red[wv][cc * 8 + e][1] = mu[e];
      red[wv][cc * 8 + e][2] = m2[e];
    }
  }
  __syncthreads();
  if (threadIdx.x < Cout) {
    const int c = threadIdx.x;
    float na = 0.f, ma = 0.f, qa = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float nb = red[v][c][0];
      if (nb <= 0.f) continue;
      const float nt = na + nb, d = red[v][c][1] - ma;
      qa += red[v][c][2] + d * d * na * nb / nt;
      ma += d * nb / nt;
      na = nt;
    }
    stats[((size_t)blockIdx.x * Cout + c) * 2] = ma;
    stats[((size_t)blockIdx.x * Cout + c) * 2 + 1] = qa;
  }
}

// partial[blk][co][tap] = sum over the block's pixels of dz[p][co] * x[p + tap]
// (pixel chunks sized for >= 4 workgroups per CU at the model's shapes)
// Cin = 1 wgrad: pixels per workgroup sized so the grid is one round of
// three resident workgroups per CU (2M pixels at B=32 -> 2752 per workgroup)
constexpr int C1W_MIN_PIX = 512, C1W_GRID = 768;
__host__ __device__ inline int c1w_pix(long P) {
  const long per = (P + C1W_GRID - 1) / C1W_GRID;
  return (int)std::max<long>(C1W_MIN_PIX, (per + 63) / 64 * 64);
}
constexpr int C1_WG_PF = 8;    // dz prefetch depth (pixels per thread)

// 8 consecutive elements kept raw in registers until used
template <typename T>
struct Raw8 {
  u32x4 u;
  __device__ __forceinline__ void load(const T* p) { u = *(const u32x4*)p; }
  __device__ __forceinline__ void to_f(float* f) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(u[i] << 16);
      f[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  }
};
template <>
struct Raw8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *(const f32x4*)p;
    b = *(const f32x4*)(p + 4);
  }
  __device__ __forceinline__ void to_f(float* f) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[i] = a[i];
      f[4 + i] = b[i];
    }
  }
};
constexpr int WG_PIX_O1 = 256; // Cout = 1 wgrad (131k pixels at B=32)
// CC = Cout / 8 is a template parameter so the lane reductions below unroll
// (a runtime-bounded shuffle loop serialised 72 x 3 ds_bpermute round trips)
template <typename T, int CC>
__global__ __launch_bounds__(256) void c1_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dz,
                                                       float* __restrict__ part, int N, int H, int W, int Cout) {
  // thread = (8-channel group cc, pixel lane); 72 accumulators in registers;
  // wave-level shuffles then LDS across the 4 waves.  Dynamic LDS: the input
  // strip (stage_strip), then the [4 waves][Cout * 9] reduction buffer (sized
  // by Cout so more workgroups fit per CU: more dz bytes in flight)
  extern __shared__ float xs[];
  constexpr int lanes = 256 / CC;
  const int cc = threadIdx.x % CC, pl = threadIdx.x / CC;
  const int P = N * H * W;
  const int wg_pix = c1w_pix(P);
  const int pbeg = blockIdx.x * wg_pix, pend = min(P, pbeg + wg_pix);
  float* red = xs + strip_floats(wg_pix, W);
  const long base = stage_strip(x, P, pbeg, pend, W, xs);
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[t][e] = 0.f;
  // dz loads run C1_WG_PF pixels ahead of the accumulation (a ring of raw
  // 16/32-byte registers): one load in flight per thread left the loop
  // latency-bound at this occupancy
  PixCursor pc(pbeg + pl, H, W);
  int p = pbeg + pl;
  Raw8<T> q[C1_WG_PF];
#pragma unroll
  for (int k = 0; k < C1_WG_PF; ++k)
    if (p + k * lanes < pend) q[k].load(dz + (size_t)(p + k * lanes) * Cout + cc * 8);
  while (p < pend) {
#pragma unroll
    for (int k = 0; k < C1_WG_PF; ++k) {
      if (p >= pend) break;
      float d[8];
      q[k].to_f(d);
      const int pn = p + C1_WG_PF * lanes;
      if (pn < pend) q[k].load(dz + (size_t)pn * Cout + cc * 8);
      float xv[9];
      taps9(xs + (p - base), pc.y, pc.x, H, W, xv);
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[t][e] += d[e] * xv[t];
      p += lanes;
      pc.advance(lanes, H, W);
    }
  }
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = acc[t][e];
      for (int o = CC; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      if (ln < CC) red[wv * Cout * 9 + (cc * 8 + e) * 9 + t] = v;
    }
  __syncthreads();
  const int R = Cout * 9;
  for (int i = threadIdx.x; i < R; i += 256)
    part[(size_t)blockIdx.x * R + i] = red[i] + red[R + i] + red[2 * R + i] + red[3 * R + i];
}

// --------------------------------------------------------------- Cout = 1 ---
// the staged input strip of `pix` output pixels (taps reach W + 1 either way), whole KiB
__host__ __device__ inline size_t o1_strip_bytes(int pix, int W, int C, size_t esz) {
  return ((size_t)(pix + 2 * W + 2) * C * esz + 1023) / 1024 * 1024;
}

// y[p] = act(sum_{tap, ci} in[p + tap][ci] * w[tap][ci]); in = src upsampled by U
template <typename T, typename TO>
__global__ __launch_bounds__(256) void o1_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w, TO* __restrict__ y,
                                                     int N, int Hs, int Ws, int U, int C, int act_tanh) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  for (int i = threadIdx.x; i < 9 * C; i += 256) sm[i] = Elem<T>::to_f(w[i]);  // packed [tap][ci]
  __syncthreads();
  const int H = Hs * U, W = Ws * U;
  const int P = N * H * W;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < P; p += gridDim.x * 256) {
    const int n = p / (H * W), rem = p - n * H * W, yy = rem / W, xx = rem - yy * W;
    float s = 0.f;
    for (int t = 0; t < 9; ++t) {
      const int iy = yy + t / 3 - 1, ix = xx + t % 3 - 1;
      if (iy < 0 || ix < 0 || iy >= H || ix >= W) continue;
      const T* src = x + ((size_t)(n * Hs + iy / U) * Ws + ix / U) * C;
      const float* wt = sm + t * C;
      for (int c = 0; c < C; c += 8) {
        float v[8];
        Vec8<T>::load(src + c, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[e] * wt[c + e];
      }
    }
    if (act_tanh) s = tanhf(s);
    y[p] = Elem<TO>::from_f(s);
  }
}

// The same for U == 1, bf16, CC = C / 8 <= 8 (the decoder's final 3x3 conv,
// 64 -> 1): a workgroup's 256 output pixels, their input strip [p0 - W - 1,
// pend + W + 1) staged once by LDS-DMA (as o1_wgrad_strip_kernel); thread
// (pixel, channel chunk) sums its 9 taps x 8 channels with the weights in
// registers, the CC chunks of a pixel (adjacent lanes) are added by shuffles.
// The element-wise form above re-read every input vector once per tap from
// L2 and spent three integer divisions per pixel (~24 us for 131k pixels).
template <int CC>
__global__ __launch_bounds__(256) void o1_fwd_strip_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                           void* __restrict__ y, int y_f32, int N, int H, int W,
                                                           int act_tanh, int pix) {
  extern __shared__ __attribute__((aligned(16))) char o1s[];
  constexpr int C = CC * 8;
  const int P = N * H * W;
  const int p0 = blockIdx.x * pix, pend = min(P, p0 + pix);
  const long base = (long)p0 - W - 1;
  const int ns = (pend - p0) + 2 * W + 2;
  {
    constexpr int upp = C * 2 / 16;
    const int nu = ns * upp;
    const long u0 = base * upp, ulim = (long)P * upp;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)(ulim * 16), 0x00020000);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i0 = wid * 64; i0 < nu; i0 += 256) {
      const long q = u0 + i0 + lane;
      const unsigned voff = (i0 + lane < nu && q >= 0 && q < ulim) ? (unsigned)(q * 16) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(o1s + (size_t)i0 * 16), 16,
                                               voff, 0, 0, 0);
    }
  }
  const int cc = threadIdx.x % CC, lg = threadIdx.x / CC;
  constexpr int G = 256 / CC;
  float wr[9][8];  // w packed [tap][ci]: this thread's chunk
#pragma unroll
  for (int t = 0; t < 9; ++t) Vec8<bf16_t>::load(w + t * C + cc * 8, wr[t]);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the strip
  __syncthreads();
  const bf16_t* xs = (const bf16_t*)o1s;
  PixCursor pc(p0 + lg, H, W);
  // (the CC lanes of a pixel share p: they leave the loop together, so the
  // chunk shuffles below only meet active lanes)
  for (int p = p0 + lg; p < pend; p += G, pc.advance(G, H, W)) {
    float s = 0.f;
    const bf16_t* c = xs + (size_t)(p - base) * C + cc * 8;
    const bool up = pc.y > 0, dn = pc.y + 1 < H, lf = pc.x > 0, rt = pc.x + 1 < W;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3 - 1, dx = t % 3 - 1;
      const bool ok = (dy < 0 ? up : dy > 0 ? dn : true) && (dx < 0 ? lf : dx > 0 ? rt : true);
      if (!ok) continue;
      float v[8];
      Vec8<bf16_t>::load(c + (dy * W + dx) * C, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[e] * wr[t][e];
    }
#pragma unroll
    for (int o = 1; o < CC; o <<= 1) s += __shfl_xor(s, o, 64);
    if (cc == 0) {
      if (act_tanh) s = tanhf(s);
      if (y_f32) ((float*)y)[p] = s;
      else ((bf16_t*)y)[p] = f2bf(s);
    }
  }
}

// du[q][ci] = sum_tap dz[q - (tap - 1)] * w[tap][ci]   (q over the conv-input grid)
template <typename T, typename TD>
__global__ __launch_bounds__(256) void o1_dgrad_kernel(const TD* __restrict__ dz, const T* __restrict__ w,
                                                       T* __restrict__ du, int N, int H, int W, int C) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  // w is the dgrad (mode-1, flipped) packing [ci][ky'][kx'][co=1]:
  // sm[tap][ci] = w_fwd[0][ci][tap] = w[ci*9 + 8 - tap]
  for (int i = threadIdx.x; i < 9 * C; i += 256) sm[i] = Elem<T>::to_f(w[(i % C) * 9 + 8 - i / C]);
  __syncthreads();
  const int CC = C / 8;
  const long total = (long)N * H * W * CC;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int cc = i % CC;
    const int q = i / CC;
    const int n = q / (H * W), rem = q - n * H * W, yy = rem / W, xx = rem - yy * W;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int py = yy - (t / 3 - 1), px = xx - (t % 3 - 1);
      if (py < 0 || px < 0 || py >= H || px >= W) continue;
      const float d = Elem<TD>::to_f(dz[(n * H + py) * W + px]);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += d * sm[t * C + cc * 8 + e];
    }
    Vec8<T>::store(du + (size_t)q * C + cc * 8, o);
  }
}

// The same for U == 1, bf16, CC <= 8: a workgroup's 256 input pixels, the dz
// values their taps reach ([q0 - W - 1, qend + W + 1), f32) staged in LDS once;
// thread (pixel, chunk) with its 9 x 8 weights in registers, one 16-byte store.
template <int CC>
__global__ __launch_bounds__(256) void o1_dgrad_strip_kernel(const bf16_t* __restrict__ dz, const bf16_t* __restrict__ w,
                                                             bf16_t* __restrict__ du, int N, int H, int W) {
  extern __shared__ __attribute__((aligned(16))) float dzs[];
  constexpr int C = CC * 8;
  const int P = N * H * W;
  const int q0 = blockIdx.x * WG_PIX_O1, qend = min(P, q0 + WG_PIX_O1);
  const long base = (long)q0 - W - 1;
  const int ns = (qend - q0) + 2 * W + 2;
  for (int i = threadIdx.x; i < ns; i += 256) {
    const long q = base + i;
    dzs[i] = (q >= 0 && q < P) ? bf2f(dz[q]) : 0.f;
  }
  const int cc = threadIdx.x % CC, lg = threadIdx.x / CC;
  constexpr int G = 256 / CC;
  // w: the dgrad (mode-1, flipped) packing [ci][ky'][kx'][co = 1]: tap t's weight of
  // channel ci is w[ci * 9 + 8 - t] (o1_dgrad_kernel's table)
  float wr[9][8];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int t = 0; t < 9; ++t) wr[t][e] = bf2f(w[(cc * 8 + e) * 9 + 8 - t]);
  __syncthreads();
  PixCursor pc(q0 + lg, H, W);
  for (int q = q0 + lg; q < qend; q += G, pc.advance(G, H, W)) {
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float* c = dzs + (q - base);
    // tap t reads dz at (y - dy, x - dx): inside the image?
    const bool up = pc.y + 1 < H, dn = pc.y > 0, lf = pc.x + 1 < W, rt = pc.x > 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3 - 1, dx = t % 3 - 1;
      const bool ok = (dy < 0 ? up : dy > 0 ? dn : true) && (dx < 0 ? lf : dx > 0 ? rt : true);
      if (!ok) continue;
      const float d = c[-dy * W - dx];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += d * wr[t][e];
    }
    Vec8<bf16_t>::store(du + (size_t)q * C + cc * 8, o);
  }
}

// part[blk][tap][ci] = sum_p dz[p] * in[p + tap][ci]
template <typename T, typename TD>
__global__ __launch_bounds__(256) void o1_wgrad_kernel(const T* __restrict__ x, const TD* __restrict__ dz,
                                                       float* __restrict__ part, int N, int Hs, int Ws, int U, int C) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4 waves][9*C]
  const int CC = C / 8;  // power of two dividing 64
  const int G = 256 / CC;
  const int cc = threadIdx.x % CC, lg = threadIdx.x / CC;
  const int H = Hs * U, W = Ws * U;
  const int P = N * H * W;
  const int pbeg = blockIdx.x * WG_PIX_O1, pend = min(P, pbeg + WG_PIX_O1);
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[t][e] = 0.f;
#pragma unroll 2
  for (int p = pbeg + lg; p < pend; p += G) {
    const float d = Elem<TD>::to_f(dz[p]);
    const int n = p / (H * W), rem = p - n * H * W, yy = rem / W, xx = rem - yy * W;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = yy + t / 3 - 1, ix = xx + t % 3 - 1;
      if (iy < 0 || ix < 0 || iy >= H || ix >= W) continue;
      float v[8];
      Vec8<T>::load(x + ((size_t)(n * Hs + iy / U) * Ws + ix / U) * C + cc * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[t][e] += d * v[e];
    }
  }
  // lanes of a wave with the same cc differ by multiples of CC
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = acc[t][e];
      for (int o = CC; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      if (ln < CC) red[wv * 9 * C + t * C + cc * 8 + e] = v;
    }
  __syncthreads();
  for (int i = threadIdx.x; i < 9 * C; i += 256)
    part[(size_t)blockIdx.x * 9 * C + i] = red[i] + red[9 * C + i] + red[18 * C + i] + red[27 * C + i];
}

// The same for U == 1 with the input staged once: NHWC pixels are contiguous
// in the flattened index p = (n, y, x), so every tap of the block's pixels lies
// in [p0 - W - 1, pend + W + 1), staged into LDS (native dtype, 16-B vectors);
// each input vector then leaves HBM once instead of once per tap, and the
// per-pixel index math is the incremental PixCursor.
template <typename T, typename TD, int CC>
__global__ __launch_bounds__(256) void o1_wgrad_strip_kernel(const T* __restrict__ x, const TD* __restrict__ dz,
                                                             float* __restrict__ part, int N, int H, int W) {
  extern __shared__ __attribute__((aligned(16))) char o1s[];
  T* xs = (T*)o1s;
  constexpr int C = CC * 8;
  constexpr int G = 256 / CC;
  const int cc = threadIdx.x % CC, lg = threadIdx.x / CC;
  const int P = N * H * W;
  const int p0 = blockIdx.x * WG_PIX_O1, pend = min(P, p0 + WG_PIX_O1);
  const long base = (long)p0 - W - 1;
  const int ns = (pend - p0) + 2 * W + 2;
  const int upp = C * (int)sizeof(T) / 16;  // 16-B units per pixel
  float* red = (float*)(o1s + o1_strip_bytes(WG_PIX_O1, W, C, sizeof(T)));
  // LDS-DMA staging: 16-B units, lane-linear destinations (a wave-instruction
  // fills 1 KiB; o1_strip_bytes rounds the strip up to whole KiB), units outside
  // the tensor read as zeros through the buffer range check
  {
    const int nu = ns * upp;
    const long u0 = base * upp, ulim = (long)P * upp;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)(ulim * 16), 0x00020000);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i0 = wid * 64; i0 < nu; i0 += 256) {
      const long q = u0 + i0 + lane;
      const unsigned voff = (i0 + lane < nu && q >= 0 && q < ulim) ? (unsigned)(q * 16) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(o1s + (size_t)i0 * 16), 16,
                                               voff, 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  }
  float* dzs = red + 4 * 9 * C;  // the block's dz values (one per pixel)
  if (p0 + (int)threadIdx.x < pend) dzs[threadIdx.x] = Elem<TD>::to_f(dz[p0 + threadIdx.x]);
  __syncthreads();
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[t][e] = 0.f;
  PixCursor pc(p0 + lg, H, W);
  for (int p = p0 + lg; p < pend; p += G, pc.advance(G, H, W)) {
    const float d = dzs[p - p0];
    const T* c = xs + (size_t)(p - base) * C + cc * 8;
    const bool up = pc.y > 0, dn = pc.y + 1 < H, lf = pc.x > 0, rt = pc.x + 1 < W;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3 - 1, dx = t % 3 - 1;
      const bool ok = (dy < 0 ? up : dy > 0 ? dn : true) && (dx < 0 ? lf : dx > 0 ? rt : true);
      if (!ok) continue;
      float v[8];
      Vec8<T>::load(c + (dy * W + dx) * C, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[t][e] += d * v[e];
    }
  }
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = acc[t][e];
      for (int o = CC; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      if (ln < CC) red[wv * 9 * C + t * C + cc * 8 + e] = v;
    }
  __syncthreads();
  for (int i = threadIdx.x; i < 9 * C; i += 256)
    part[(size_t)blockIdx.x * 9 * C + i] = red[i] + red[9 * C + i] + red[18 * C + i] + red[27 * C + i];
}

}  // namespace hvit

using namespace hvit;

// dynamic LDS above the 64 KiB default needs an opt-in per kernel
template <typename K>
static void allow_lds(K kern, size_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// host dispatchers (called from gemm_api.hip) -----------------------------------
int hvit_thin_c1_fwd(int dt, const hvit_conv_geom_t* g, const void* w, void* y, int y_dt, float* stats,
                     hipStream_t st) {
  HVIT_CHECK(g->Cout % 8 == 0 && g->Cout <= 256, "thin conv: Cout=%d must be a multiple of 8 <= 256", g->Cout);
  const int P = g->N * g->Hs * g->Ws;
  const size_t smem = sizeof(float) * strip_floats(C1_BLOCK_PIX, g->Ws);
  HVIT_CHECK(smem + sizeof(float) * 4 * 256 * 3 <= 160 * 1024, "thin conv: W=%d too wide for the LDS strip", g->Ws);
  dim3 grid(cdiv(P, C1_BLOCK_PIX));
  auto go = [&](auto kern, auto xp, auto yp) {
    allow_lds(kern, smem);
    hipLaunchKernelGGL(kern, grid, dim3(256), smem, st, xp, (decltype(xp))w, yp, stats, g->N, g->Hs, g->Ws, g->Cout);
  };
  if (dt == HVIT_BF16 && y_dt == HVIT_BF16)
    go(c1_fwd_kernel<bf16_t, bf16_t>, (const bf16_t*)g->src1, (bf16_t*)y);
  else if (dt == HVIT_BF16)
    go(c1_fwd_kernel<bf16_t, float>, (const bf16_t*)g->src1, (float*)y);
  else if (y_dt == HVIT_F32)
    go(c1_fwd_kernel<float, float>, (const float*)g->src1, (float*)y);
  else
    go(c1_fwd_kernel<float, bf16_t>, (const float*)g->src1, (bf16_t*)y);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

int hvit_thin_c1_bn_tile_rows() { return C1_BLOCK_PIX; }

long long hvit_thin_c1_wgrad_ws(const hvit_conv_geom_t* g) {
  const long P = (long)g->N * g->Hs * g->Ws;
  const int wp = c1w_pix(P);
  return (long long)((P + wp - 1) / wp) * g->Cout * 9;
}

int hvit_thin_c1_wgrad(int dt, const hvit_conv_geom_t* g, const void* dz, float* dw, float* ws, long long ws_elems,
                       hipStream_t st) {
  HVIT_CHECK(g->Cout <= 256 && 256 % g->Cout == 0, "thin conv wgrad: Cout=%d must divide 256", g->Cout);
  const long P = (long)g->N * g->Hs * g->Ws;
  const int wp = c1w_pix(P);
  const int nb = (int)((P + wp - 1) / wp);
  HVIT_CHECK(ws && ws_elems >= (long long)nb * g->Cout * 9, "thin conv wgrad: workspace too small");
  const size_t smem = sizeof(float) * (strip_floats(wp, g->Ws) + 4 * 9 * g->Cout);
  HVIT_CHECK(smem <= 160 * 1024, "thin conv wgrad: W=%d too wide for the LDS strip", g->Ws);
  auto go = [&](auto kern, auto xp) {
    allow_lds(kern, smem);
    hipLaunchKernelGGL(kern, dim3(nb), dim3(256), smem, st, xp, (decltype(xp))dz, ws, g->N, g->Hs, g->Ws, g->Cout);
  };
#define C1W_CASE(cc)                                                  \
  case cc:                                                            \
    if (dt == HVIT_BF16)                                              \
      go(c1_wgrad_kernel<bf16_t, cc>, (const bf16_t*)g->src1);        \
    else                                                              \
      go(c1_wgrad_kernel<float, cc>, (const float*)g->src1);          \
    break;
  switch (g->Cout / 8) {
    C1W_CASE(1) C1W_CASE(2) C1W_CASE(4) C1W_CASE(8) C1W_CASE(16) C1W_CASE(32)
    default: HVIT_CHECK(false, "thin conv wgrad: Cout=%d unsupported", g->Cout);
  }
#undef C1W_CASE
  HVIT_LAUNCH_CHECK();
  return hvit_sum_slabs(ws, nb, (long long)g->Cout * 9, dw, st);
}

int hvit_thin_o1_fwd(int dt, const hvit_conv_geom_t* g, const void* w, void* y, int y_dt, int act_tanh,
                     hipStream_t st) {
  const int C = g->C1;
  HVIT_CHECK(C % 8 == 0, "thin conv: Cin=%d must be a multiple of 8", C);
  const long P = (long)g->N * g->Hs * g->U * g->Ws * g->U;
  // 128 output pixels per workgroup (1,024 workgroups at B = 32: four per CU overlap
  // their strip loads with each other's sums): 14.7 us vs 15.8 at 256, 24.9 at 512;
  // a thread-per-pixel form (no lane shuffles, weights from LDS) ran 15.7-17.1
  constexpr int fpix = 128;
  const size_t sstrip = o1_strip_bytes(fpix, g->Ws, C, 2);
  if (g->U == 1 && dt == HVIT_BF16 && C / 8 <= 8 && sstrip <= 150 * 1024 && P * C * 2L < (1L << 31)) {
    const int nb = (int)((P + fpix - 1) / fpix);
    auto go = [&](auto kern) {
      allow_lds(kern, sstrip);
      hipLaunchKernelGGL(kern, dim3(nb), dim3(256), sstrip, st, (const bf16_t*)g->src1, (const bf16_t*)w, y,
                         y_dt == HVIT_F32 ? 1 : 0, g->N, g->Hs, g->Ws, act_tanh, fpix);
    };
    switch (C / 8) {
      case 1: go(o1_fwd_strip_kernel<1>); break;
      case 2: go(o1_fwd_strip_kernel<2>); break;
      case 4: go(o1_fwd_strip_kernel<4>); break;
      case 8: go(o1_fwd_strip_kernel<8>); break;
      default: goto flat;
    }
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
flat:
  const size_t smem = 9 * C * sizeof(float);
  dim3 grid((unsigned)std::min<long>((P + 255) / 256, 8192));
  if (dt == HVIT_BF16 && y_dt == HVIT_F32)
    hipLaunchKernelGGL((o1_fwd_kernel<bf16_t, float>), grid, dim3(256), smem, st, (const bf16_t*)g->src1,
                       (const bf16_t*)w, (float*)y, g->N, g->Hs, g->Ws, g->U, C, act_tanh);
  else if (dt == HVIT_BF16)
    hipLaunchKernelGGL((o1_fwd_kernel<bf16_t, bf16_t>), grid, dim3(256), smem, st, (const bf16_t*)g->src1,
                       (const bf16_t*)w, (bf16_t*)y, g->N, g->Hs, g->Ws, g->U, C, act_tanh);
  else if (y_dt == HVIT_F32)
    hipLaunchKernelGGL((o1_fwd_kernel<float, float>), grid, dim3(256), smem, st, (const float*)g->src1,
                       (const float*)w, (float*)y, g->N, g->Hs, g->Ws, g->U, C, act_tanh);
  else
    hipLaunchKernelGGL((o1_fwd_kernel<float, bf16_t>), grid, dim3(256), smem, st, (const float*)g->src1,
                       (const float*)w, (bf16_t*)y, g->N, g->Hs, g->Ws, g->U, C, act_tanh);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

// dz dtype = dt (the compute dtype); du at conv-input resolution [N, H, W, C]
int hvit_thin_o1_dgrad(int dt, const hvit_conv_geom_t* g, const void* dz, const void* w, void* du, hipStream_t st) {
  const int C = g->C1;
  HVIT_CHECK(C % 8 == 0, "thin conv: Cin=%d must be a multiple of 8", C);
  const int H = g->Hs * g->U, W = g->Ws * g->U;
  const long total = (long)g->N * H * W * (C / 8);
  const size_t smem = 9 * C * sizeof(float);
  if (g->U == 1 && dt == HVIT_BF16 && C / 8 <= 8 && (64 % (C / 8)) == 0) {
    const long P = (long)g->N * H * W;
    const int nb = (int)((P + WG_PIX_O1 - 1) / WG_PIX_O1);
    const size_t sd = sizeof(float) * (WG_PIX_O1 + 2 * W + 2);
    HVIT_CHECK(sd <= 64 * 1024, "thin conv dgrad: W=%d too wide", W);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(nb), dim3(256), sd, st, (const bf16_t*)dz, (const bf16_t*)w, (bf16_t*)du, g->N, H,
                         W);
    };
    switch (C / 8) {
      case 1: go(o1_dgrad_strip_kernel<1>); break;
      case 2: go(o1_dgrad_strip_kernel<2>); break;
      case 4: go(o1_dgrad_strip_kernel<4>); break;
      default: go(o1_dgrad_strip_kernel<8>); break;
    }
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  dim3 grid((unsigned)std::min<long>((total + 255) / 256, 16384));
  if (dt == HVIT_BF16)
    hipLaunchKernelGGL((o1_dgrad_kernel<bf16_t, bf16_t>), grid, dim3(256), smem, st, (const bf16_t*)dz,
                       (const bf16_t*)w, (bf16_t*)du, g->N, H, W, C);
  else
    hipLaunchKernelGGL((o1_dgrad_kernel<float, float>), grid, dim3(256), smem, st, (const float*)dz,
                       (const float*)w, (float*)du, g->N, H, W, C);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

long long hvit_thin_o1_wgrad_ws(const hvit_conv_geom_t* g) {
  const long P = (long)g->N * g->Hs * g->U * g->Ws * g->U;
  return (long long)((P + WG_PIX_O1 - 1) / WG_PIX_O1) * 9 * g->C1;
}

int hvit_thin_o1_wgrad(int dt, const hvit_conv_geom_t* g, const void* dz, float* dw, float* ws, long long ws_elems,
                       hipStream_t st) {
  const int C = g->C1;
  HVIT_CHECK(C % 8 == 0 && C / 8 <= 64 && 64 % (C / 8) == 0, "thin conv wgrad: Cin=%d unsupported", C);
  const long P = (long)g->N * g->Hs * g->U * g->Ws * g->U;
  const int nb = (int)((P + WG_PIX_O1 - 1) / WG_PIX_O1);
  HVIT_CHECK(ws && ws_elems >= (long long)nb * 9 * C, "thin conv wgrad: workspace too small");
  const size_t esz = dt == HVIT_BF16 ? 2 : 4;
  const size_t sstrip = o1_strip_bytes(WG_PIX_O1, g->Ws, C, esz) + (4 * 9 * C + WG_PIX_O1) * sizeof(float);
  if (g->U == 1 && sstrip <= 150 * 1024 && P * C * (long)esz < (1L << 31)) {  // staged strip (every final conv of the model)
    auto go = [&](auto kern, auto xp) {
      allow_lds(kern, sstrip);
      hipLaunchKernelGGL(kern, dim3(nb), dim3(256), sstrip, st, xp, (decltype(xp))dz, ws, g->N, g->Hs, g->Ws);
    };
#define O1W_CASE(cc)                                                              \
  case cc:                                                                        \
    if (dt == HVIT_BF16)                                                          \
      go(o1_wgrad_strip_kernel<bf16_t, bf16_t, cc>, (const bf16_t*)g->src1);      \
    else                                                                          \
      go(o1_wgrad_strip_kernel<float, float, cc>, (const float*)g->src1);         \
    break;
    switch (C / 8) {
      O1W_CASE(1) O1W_CASE(2) O1W_CASE(4) O1W_CASE(8) O1W_CASE(16) O1W_CASE(32) O1W_CASE(64)
      default: HVIT_CHECK(false, "thin conv wgrad: Cin=%d unsupported", C);
    }
#undef O1W_CASE
  } else {
    const size_t smem = 4 * 9 * C * sizeof(float);
    if (dt == HVIT_BF16)
      hipLaunchKernelGGL((o1_wgrad_kernel<bf16_t, bf16_t>), dim3(nb), dim3(256), smem, st, (const bf16_t*)g->src1,
                         (const bf16_t*)dz, ws, g->N, g->Hs, g->Ws, g->U, C);
    else
      hipLaunchKernelGGL((o1_wgrad_kernel<float, float>), dim3(nb), dim3(256), smem, st, (const float*)g->src1,
                         (const float*)dz, ws, g->N, g->Hs, g->Ws, g->U, C);
  }
  HVIT_LAUNCH_CHECK();
  return hvit_sum_slabs(ws, nb, 9LL * C, dw, st);
}
