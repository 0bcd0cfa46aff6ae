// Spatial resampling on NHWC activations for gfx950:
//  * bilinear resize, align_corners=False (F.interpolate as used by the skip
//    connections, models/hybrid_vit.py:381-386, and the final resize, :459-465)
//    with torch's source-index rule (area_pixel_compute_source_index: src =
//    scale*(dst+0.5)-0.5 clamped at 0, scale = in/out in f32);
//  * its backward as a GATHER (each input pixel sums the output pixels that
//    sample it) -- deterministic, no atomics;
//  * the backward of nearest x2 upsample fused with the split of the
//    concatenated decoder input (components.py:146 + hybrid_vit.py:389).
#include "common.h"

namespace hvit {

struct LinIdx {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ LinIdx lin_idx(int o, int in, float scale) {
  float src = scale * ((float)o + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  int i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  int p = i0 < in - 1 ? 1 : 0;
  LinIdx r;
  r.i0 = i0;
  r.i1 = i0 + p;
  r.l1 = src - (float)i0;
  r.l0 = 1.f - r.l1;
  return r;
}

__global__ __launch_bounds__(256) void bilinear_fwd_kernel(const void* x, int x_dt, void* y, int y_dt, int N,
                                                          int Hi, int Wi, int C, int Ho, int Wo, float sh,
                                                          float sw) {
  const int total = N * Ho * Wo * C;  // < 2^31 (checked on the host)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % C;
    const int p = i / C;
    const int ox = p % Wo;
    const int t = p / Wo;
    const int oy = t % Ho;
    const int n = t / Ho;
    LinIdx ly = lin_idx(oy, Hi, sh), lx = lin_idx(ox, Wi, sw);
    const int b = n * Hi;
    float v00 = ld_dt(x, ((b + ly.i0) * Wi + lx.i0) * C + c, x_dt);
    float v01 = ld_dt(x, ((b + ly.i0) * Wi + lx.i1) * C + c, x_dt);
    float v10 = ld_dt(x, ((b + ly.i1) * Wi + lx.i0) * C + c, x_dt);
    float v11 = ld_dt(x, ((b + ly.i1) * Wi + lx.i1) * C + c, x_dt);
    float v = ly.l0 * (lx.l0 * v00 + lx.l1 * v01) + ly.l1 * (lx.l0 * v10 + lx.l1 * v11);
    st_dt(y, i, v, y_dt);
  }
}

// The same with one output row per blockIdx.y and CV channels per thread
// (bf16 CV = 8: four 16-byte loads, one 16-byte store; f32 CV = 1: the C = 1
// final resize): the row / column index math once per CV channels and no
// per-element division (the element-wise form above spent most of its time in
// three integer divisions per element).  Same arithmetic per element.
template <typename T, int CV>
__global__ __launch_bounds__(256) void bilinear_fwd_rows_kernel(const T* __restrict__ x, T* __restrict__ y, int Hi,
                                                               int Wi, int C, int Ho, int Wo, float sh, float sw) {
  const int r = blockIdx.y;  // n * Ho + oy
  const int n = r / Ho, oy = r - n * Ho;
  const int G = C / CV;
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= Wo * G) return;
  const int ox = item / G, cg = item - ox * G;
  const LinIdx ly = lin_idx(oy, Hi, sh), lx = lin_idx(ox, Wi, sw);
  const T* r0 = x + ((long)(n * Hi + ly.i0) * Wi) * C + cg * CV;
  const T* r1 = x + ((long)(n * Hi + ly.i1) * Wi) * C + cg * CV;
  T* out = y + ((long)r * Wo + ox) * C + cg * CV;
  if constexpr (CV == 8) {
    const u32x4 a = *(const u32x4*)(r0 + (long)lx.i0 * C), b = *(const u32x4*)(r0 + (long)lx.i1 * C);
    const u32x4 c = *(const u32x4*)(r1 + (long)lx.i0 * C), d = *(const u32x4*)(r1 + (long)lx.i1 * C);
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        auto f = [&](uint32_t u) { return h ? __uint_as_float(u & 0xffff0000u) : __uint_as_float(u << 16); };
        const float v00 = f(a[e]), v01 = f(b[e]), v10 = f(c[e]), v11 = f(d[e]);
        v[h] = ly.l0 * (lx.l0 * v00 + lx.l1 * v01) + ly.l1 * (lx.l0 * v10 + lx.l1 * v11);
      }
      o[e] = f2bf2(v[0], v[1]);
    }
    *(u32x4*)out = o;
  } else {
#pragma unroll
    for (int e = 0; e < CV; ++e) {
      const float v00 = Elem<T>::to_f(r0[(long)lx.i0 * C + e]), v01 = Elem<T>::to_f(r0[(long)lx.i1 * C + e]);
      const float v10 = Elem<T>::to_f(r1[(long)lx.i0 * C + e]), v11 = Elem<T>::to_f(r1[(long)lx.i1 * C + e]);
      out[e] = Elem<T>::from_f(ly.l0 * (lx.l0 * v00 + lx.l1 * v01) + ly.l1 * (lx.l0 * v10 + lx.l1 * v11));
    }
  }
}

// weight with which output index o samples input index i along one dim
__device__ __forceinline__ float lin_w(int o, int i, int in, float scale) {
  LinIdx l = lin_idx(o, in, scale);
  float w = 0.f;
  if (l.i0 == i) w += l.l0;
  if (l.i1 == i) w += l.l1;
  return w;
}
__device__ __forceinline__ void out_range(int i, int in, int out, float scale, int& lo, int& hi) {
  // outputs whose source lies in [i-1, i+1]
  float inv = 1.f / scale;
  lo = (int)floorf(((float)i - 1.f + 0.5f) * inv - 0.5f) - 1;
  hi = (int)ceilf(((float)i + 1.f + 0.5f) * inv - 0.5f) + 1;
  if (lo < 0) lo = 0;
  if (hi > out - 1) hi = out - 1;
}

constexpr int TAPS = 16;
__device__ __forceinline__ int taps_of(int i, int in, int out, float scale, int* o_idx, float* w) {
  int lo, hi;
  out_range(i, in, out, scale, lo, hi);
  int nt = 0;
  for (int o = lo; o <= hi && nt < TAPS; ++o) {
    const float wt = lin_w(o, i, in, scale);
    if (wt != 0.f) {
      o_idx[nt] = o;
      w[nt] = wt;
      ++nt;
    }
  }
  return nt;
}

// generic (any C / dtype pair): one thread per input element
__global__ __launch_bounds__(256) void bilinear_bwd_kernel(const void* dy, int dy_dt, void* dx, int dx_dt, int N,
                                                          int Hi, int Wi, int C, int Ho, int Wo, float sh,
                                                          float sw, int accumulate) {
  const int total = N * Hi * Wi * C;  // < 2^31 (checked on the host)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % C;
    const int p = i / C;
    const int ix = p % Wi;
    const int t = p / Wi;
    const int iy = t % Hi;
    const int n = t / Hi;
    int oy[TAPS], ox[TAPS];
    float wy[TAPS], wx[TAPS];
    const int ny = taps_of(iy, Hi, Ho, sh, oy, wy);
    const int nx = taps_of(ix, Wi, Wo, sw, ox, wx);
    float acc = 0.f;
    for (int a = 0; a < ny; ++a) {
      const int base = (n * Ho + oy[a]) * Wo;
      float row = 0.f;
      for (int b = 0; b < nx; ++b) row += wx[b] * ld_dt(dy, (base + ox[b]) * C + c, dy_dt);
      acc += wy[a] * row;
    }
    if (accumulate) acc += ld_dt(dx, i, dx_dt);
    st_dt(dx, i, acc, dx_dt);
  }
}

// Vectorised gather backward: one thread per (input pixel, 16-byte channel
// group); the output taps that sample the pixel (<= TAPS per dimension) and
// their weights are computed once per thread and reused for all CV channels.
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void bilinear_bwd_vec_kernel(const TI* __restrict__ dy, TO* __restrict__ dx,
                                                              int N, int Hi, int Wi, int C, int Ho, int Wo,
                                                              float sh, float sw, int accumulate) {
  constexpr int CV = 8;  // channels per thread (one or two 16-byte vectors)
  const int G = C / CV;
  const int total = N * Hi * Wi * G;  // < 2^31 (checked on the host)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cg = i % G;
    const int p = i / G;
    const int ix = p % Wi;
    const int t = p / Wi;
    const int iy = t % Hi;
    const int n = t / Hi;
    int oy[TAPS], ox[TAPS];
    float wy[TAPS], wx[TAPS];
    const int ny = taps_of(iy, Hi, Ho, sh, oy, wy);
    const int nx = taps_of(ix, Wi, Wo, sw, ox, wx);
    float acc[CV];
#pragma unroll
    for (int e = 0; e < CV; ++e) acc[e] = 0.f;
    for (int a = 0; a < ny; ++a) {
      const TI* row = dy + ((size_t)(n * Ho + oy[a]) * Wo) * C + cg * CV;
      for (int b = 0; b < nx; ++b) {
        const float w = wy[a] * wx[b];
        const TI* q = row + (size_t)ox[b] * C;
        float v[CV];
        if constexpr (sizeof(TI) == 2) {
          const u32x4 u = *(const u32x4*)q;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] = __uint_as_float(u[e] << 16);
            v[2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
          }
        } else {
          const f32x4 lo = *(const f32x4*)q, hi = *(const f32x4*)(q + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = lo[e];
            v[4 + e] = hi[e];
          }
        }
#pragma unroll
        for (int e = 0; e < CV; ++e) acc[e] += w * v[e];
      }
    }
    TO* d = dx + (size_t)p * C + cg * CV;
    if constexpr (sizeof(TO) == 2) {
      if (accumulate) {
        const u32x4 u = *(const u32x4*)d;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] += __uint_as_float(u[e] << 16);
          acc[2 * e + 1] += __uint_as_float(u[e] & 0xffff0000u);
        }
      }
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf2(acc[2 * e], acc[2 * e + 1]);
      *(u32x4*)d = o;
    } else {
      f32x4 lo = {acc[0], acc[1], acc[2], acc[3]}, hi = {acc[4], acc[5], acc[6], acc[7]};
      if (accumulate) {
        lo += *(const f32x4*)d;
        hi += *(const f32x4*)(d + 4);
      }
      *(f32x4*)d = lo;
      *(f32x4*)(d + 4) = hi;
    }
  }
}

// Row-blocked gather backward: one workgroup per RB input rows (n, iy .. iy +
// RB - 1; RB > 1 only when one row has fewer (column, channel group) items
// than threads -- the C = 1 final-output resize: 64 items per row left three
// quarters of every workgroup idle, 0.3 TB/s).  The output taps of every input
// column of the row (and of the rows themselves) are computed once into LDS,
// then threads walk (row, column, channel group) items.
constexpr int RB_MAXW = 256, RB_TAPS = 12, RB_MAXR = 8;
template <typename TI, typename TO, int CV>
__global__ __launch_bounds__(256) void bilinear_bwd_rows_kernel(const TI* __restrict__ dy, TO* __restrict__ dx,
                                                               int Hi, int Wi, int C, int Ho, int Wo, float sh,
                                                               float sw, int accumulate, int RB) {
  __shared__ int xo[RB_MAXW][RB_TAPS];
  __shared__ float xw[RB_MAXW][RB_TAPS];
  __shared__ int xn[RB_MAXW];
  __shared__ int yo[RB_MAXR][RB_TAPS];
  __shared__ float yw[RB_MAXR][RB_TAPS];
  __shared__ int yn[RB_MAXR];
  const int rpn = (Hi + RB - 1) / RB;  // row blocks per sample
  const int n = blockIdx.x / rpn, iy0 = (blockIdx.x - n * rpn) * RB;
  for (int ix = threadIdx.x; ix < Wi; ix += blockDim.x) {
    int lo, hi;
    out_range(ix, Wi, Wo, sw, lo, hi);
    int nt = 0;
    for (int o = lo; o <= hi && nt < RB_TAPS; ++o) {
      const float wt = lin_w(o, ix, Wi, sw);
      if (wt != 0.f) {
        xo[ix][nt] = o;
        xw[ix][nt] = wt;
        ++nt;
      }
    }
    xn[ix] = nt;
  }
  if (threadIdx.x < RB) {
    const int r = threadIdx.x, iy = iy0 + r;
    int nt = 0;
    if (iy < Hi) {
      int lo, hi;
      out_range(iy, Hi, Ho, sh, lo, hi);
      for (int o = lo; o <= hi && nt < RB_TAPS; ++o) {
        const float wt = lin_w(o, iy, Hi, sh);
        if (wt != 0.f) {
          yo[r][nt] = o;
          yw[r][nt] = wt;
          ++nt;
        }
      }
    }
    yn[r] = nt;
  }
  __syncthreads();
  const int G = C / CV;
  const int per_row = Wi * G;
  for (int item = threadIdx.x; item < RB * per_row; item += blockDim.x) {
    const int r = item / per_row, rem = item - r * per_row;
    const int iy = iy0 + r;
    if (iy >= Hi) break;  // (items are row-major: every later item is past the last row too)
    const int ix = rem / G, cg = rem - ix * G;
    float acc[CV];
    TO* d = dx + ((size_t)(n * Hi + iy) * Wi + ix) * C + cg * CV;
    // the accumulated-into gradient first: its load is independent of the taps
    // (issued after the tap loop it waited behind the previous item's store)
    if constexpr (CV == 8 && sizeof(TO) == 2) {
      if (accumulate) {
        const u32x4 u = *(const u32x4*)d;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] = __uint_as_float(u[e] << 16);
          acc[2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
        }
      } else {
#pragma unroll
        for (int e = 0; e < CV; ++e) acc[e] = 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < CV; ++e) acc[e] = accumulate ? Elem<TO>::to_f(d[e]) : 0.f;
    }
    const int nx = xn[ix], ny = yn[r];
    for (int a = 0; a < ny; ++a) {
      const TI* row = dy + ((size_t)(n * Ho + yo[r][a]) * Wo) * C + cg * CV;
      const float wa = yw[r][a];
      for (int b = 0; b < nx; ++b) {
        const float w = wa * xw[ix][b];
        const TI* q = row + (size_t)xo[ix][b] * C;
        if constexpr (CV == 8 && sizeof(TI) == 2) {
          const u32x4 u = *(const u32x4*)q;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[2 * e] += w * __uint_as_float(u[e] << 16);
            acc[2 * e + 1] += w * __uint_as_float(u[e] & 0xffff0000u);
          }
        } else {
#pragma unroll
          for (int e = 0; e < CV; ++e) acc[e] += w * Elem<TI>::to_f(q[e]);
        }
      }
    }
    if constexpr (CV == 8 && sizeof(TO) == 2) {
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf2(acc[2 * e], acc[2 * e + 1]);
      *(u32x4*)d = o;
    } else {
#pragma unroll
      for (int e = 0; e < CV; ++e) d[e] = Elem<TO>::from_f(acc[e]);
    }
  }
}

// The backward of an exact even-factor downsample (Hi = k Ho, Wi = k Wo, k even:
// the skip resizes of the encoder outputs onto the decoder grid, k = 2 and 4).
// With align_corners=False output pixel o samples src = k o + (k - 1) / 2, i.e.
// input pixels k o + k/2 - 1 and k o + k/2 at weight 0.5 each: every input
// pixel is sampled by at most one output pixel, at weight 0.5 * 0.5 or not at
// all.  bf16, 8-channel groups: one thread per (output pixel, channel group)
// adds 0.25 dy to its 2x2 sampled input pixels (acc = dx; acc += 0.25 * dy in
// f32, one bf16 rounding: the gather form's arithmetic) and, when not
// accumulating, zeroes the rest of its k x k block (accumulating, those keep
// their value, as the gather form rewrites them unchanged) -- no tap tables,
// no per-item divisions, and at k = 4 a quarter of the input gradient's bytes.
// blockIdx.y = n * Ho + oy; G = C / 8 a power of two.
__global__ __launch_bounds__(256) void bilinear_bwd_down_kernel(const bf16_t* __restrict__ dy,
                                                               bf16_t* __restrict__ dx, int Wo, int C, int gshift,
                                                               int k, int accumulate) {
  const int r = blockIdx.y;
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= (Wo << gshift)) return;
  const int ox = item >> gshift, cg = item & ((1 << gshift) - 1);
  const u32x4 g = *(const u32x4*)(dy + ((long)r * Wo + ox) * C + cg * 8);
  const long Wi = (long)k * Wo;
  const int h = k / 2 - 1;  // first sampled row / column of the block
  bf16_t* blk = dx + ((long)k * r * Wi + (long)k * ox) * C + cg * 8;
  bf16_t* d[4];
  u32x4 old[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    d[q] = blk + ((h + (q >> 1)) * Wi + h + (q & 1)) * C;
    old[q] = accumulate ? *(const u32x4*)d[q] : (u32x4){0u, 0u, 0u, 0u};
  }
  const float w = 0.25f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float lo = __uint_as_float(old[q][e] << 16), hi = __uint_as_float(old[q][e] & 0xffff0000u);
      lo += w * __uint_as_float(g[e] << 16);
      hi += w * __uint_as_float(g[e] & 0xffff0000u);
      o[e] = f2bf2(lo, hi);
    }
    *(u32x4*)d[q] = o;
  }
  if (!accumulate && k > 2)
    for (int yy = 0; yy < k; ++yy)
      for (int xx = 0; xx < k; ++xx)
        if (yy - h < 0 || yy - h > 1 || xx - h < 0 || xx - h > 1)
          *(u32x4*)(blk + (yy * Wi + xx) * C) = (u32x4){0u, 0u, 0u, 0u};
}

// dU [N, H*U, W*U, C1+C2] -> dx1 [N, H, W, C1], dx2 [N, H, W, C2] (sum over U x U)
__global__ __launch_bounds__(256) void up_split_bwd_kernel(const void* du, int du_dt, int N, int H, int W, int U,
                                                          int C1, int C2, void* dx1, int dx1_dt, void* dx2,
                                                          int dx2_dt) {
  const int Ct = C1 + C2;
  const int total = N * H * W * Ct;  // < 2^31 (checked on the host)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % Ct;
    const int p = i / Ct;
    const int x = p % W;
    const int t = p / W;
    const int y = t % H;
    const int n = t / H;
    float s = 0.f;
    for (int a = 0; a < U; ++a)
      for (int b = 0; b < U; ++b)
        s += ld_dt(du, ((long)((n * H + y) * U + a) * (W * U) + x * U + b) * Ct + c, du_dt);
    if (c < C1) st_dt(dx1, p * C1 + c, s, dx1_dt);
    else st_dt(dx2, p * C2 + (c - C1), s, dx2_dt);
  }
}

// The same for bf16 with C1 % 8 == C2 % 8 == 0: a thread sums the U x U
// 16-byte channel groups of one output pixel (f32 accumulation in the same
// a-major, b-minor order) and stores one 16-byte group; two integer divisions
// per 8 channels instead of four per channel.
__global__ __launch_bounds__(256) void up_split_bwd_vec_kernel(const bf16_t* __restrict__ du, int N, int H, int W,
                                                              int U, int C1, int C2, bf16_t* __restrict__ dx1,
                                                              bf16_t* __restrict__ dx2) {
  const int Ct = C1 + C2, G8 = Ct >> 3;
  const int total = N * H * W * G8;  // < 2^31 (checked on the host)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int p = i / G8;
    const int c0 = (i - p * G8) << 3;
    const int t = p / W;  // n * H + y
    const int x = p - t * W;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int a = 0; a < U; ++a)
      for (int b = 0; b < U; ++b) {
        const u32x4 u = *(const u32x4*)(du + ((long)(t * U + a) * (W * U) + x * U + b) * Ct + c0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[2 * e] += __uint_as_float(u[e] << 16);
          s[2 * e + 1] += __uint_as_float(u[e] & 0xffff0000u);
        }
      }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf2(s[2 * e], s[2 * e + 1]);
    if (c0 < C1) *(u32x4*)(dx1 + (long)p * C1 + c0) = o;
    else *(u32x4*)(dx2 + (long)p * C2 + (c0 - C1)) = o;
  }
}

static int grid_for(long n) {
  long g = (n + 255) / 256;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace hvit

using namespace hvit;

extern "C" int hvit_bilinear_fwd(const void* x, int x_dt, int N, int Hi, int Wi, int C, int Ho, int Wo,
                                 void* y, int y_dt, void* stream) {
  HVIT_CHECK(x && y, "hvit_bilinear_fwd: null pointer");
  HVIT_CHECK(Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && C > 0, "hvit_bilinear_fwd: bad sizes");
  long total = (long)N * Ho * Wo * C;
  if (total <= 0) return HVIT_OK;
  HVIT_CHECK(total < (1L << 31) && (long)N * Hi * Wi * C < (1L << 31), "resample: tensor too large");
  float sh = (float)Hi / (float)Ho, sw = (float)Wi / (float)Wo;
  if (x_dt == y_dt && (long)N * Ho < 65536) {
    if (x_dt == HVIT_BF16 && C % 8 == 0 && aligned16(x) && aligned16(y)) {
      hipLaunchKernelGGL((bilinear_fwd_rows_kernel<bf16_t, 8>), dim3(cdiv((long)Wo * (C / 8), 256), N * Ho), dim3(256),
                         0, (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y, Hi, Wi, C, Ho, Wo, sh, sw);
      HVIT_LAUNCH_CHECK();
      return HVIT_OK;
    }
    if (x_dt == HVIT_F32 && C == 1) {
      hipLaunchKernelGGL((bilinear_fwd_rows_kernel<float, 1>), dim3(cdiv(Wo, 256), N * Ho), dim3(256), 0,
                         (hipStream_t)stream, (const float*)x, (float*)y, Hi, Wi, C, Ho, Wo, sh, sw);
      HVIT_LAUNCH_CHECK();
      return HVIT_OK;
    }
  }
  hipLaunchKernelGGL(bilinear_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, x_dt,
                     y, y_dt, N, Hi, Wi, C, Ho, Wo, sh, sw);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_bilinear_bwd(const void* dy, int dy_dt, int N, int Ho, int Wo, int C, int Hi, int Wi,
                                 void* dx, int dx_dt, int accumulate, void* stream) {
  HVIT_CHECK(dy && dx, "hvit_bilinear_bwd: null pointer");
  HVIT_CHECK(Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && C > 0, "hvit_bilinear_bwd: bad sizes");
  long total = (long)N * Hi * Wi * C;
  if (total <= 0) return HVIT_OK;
  HVIT_CHECK(total < (1L << 31) && (long)N * Ho * Wo * C < (1L << 31), "resample: tensor too large");
  float sh = (float)Hi / (float)Ho, sw = (float)Wi / (float)Wo;
  // vector path: 8-channel groups, at most TAPS output taps per dimension
  const bool taps_ok = (float)Ho / (float)Hi <= 6.f && (float)Wo / (float)Wi <= 6.f;
  const bool rows_ok = (float)Ho / (float)Hi <= 4.f && (float)Wo / (float)Wi <= 4.f && Wi <= RB_MAXW &&
                       (long)N * Hi < (1L << 31) && dy_dt == dx_dt;
  // input rows per workgroup: enough (column, channel group) items for the 256 threads
  auto rows_per_wg = [&](int cv) {
    const long items = (long)Wi * (C / cv);
    int rb = 1;
    while (rb < RB_MAXR && items * rb * 2 <= 256) rb *= 2;
    return rb;
  };
  const int G8 = C / 8, kd = Hi / Ho;
  if ((kd == 2 || kd == 4) && Hi == kd * Ho && Wi == kd * Wo && C % 8 == 0 && (G8 & (G8 - 1)) == 0 &&
      dy_dt == HVIT_BF16 && dx_dt == HVIT_BF16 && aligned16(dy) && aligned16(dx) && (long)N * Ho < 65536) {
    int gshift = 0;
    while ((1 << gshift) < G8) ++gshift;
    hipLaunchKernelGGL(bilinear_bwd_down_kernel, dim3(cdiv((long)Wo * G8, 256), N * Ho), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)dy, (bf16_t*)dx, Wo, C, gshift, kd, accumulate);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  if (rows_ok && C % 8 == 0 && dy_dt == HVIT_BF16 && aligned16(dy) && aligned16(dx)) {
    const int rb = rows_per_wg(8);
    hipLaunchKernelGGL((bilinear_bwd_rows_kernel<bf16_t, bf16_t, 8>), dim3(N * cdiv(Hi, rb)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)dy, (bf16_t*)dx, Hi, Wi, C, Ho, Wo, sh, sw, accumulate, rb);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  if (rows_ok && C == 1 && dy_dt == HVIT_F32) {
    const int rb = rows_per_wg(1);
    hipLaunchKernelGGL((bilinear_bwd_rows_kernel<float, float, 1>), dim3(N * cdiv(Hi, rb)), dim3(256), 0,
                       (hipStream_t)stream, (const float*)dy, (float*)dx, Hi, Wi, C, Ho, Wo, sh, sw, accumulate, rb);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  if (C % 8 == 0 && taps_ok && dy_dt == dx_dt && aligned16(dy) && aligned16(dx)) {
    const long groups = (long)N * Hi * Wi * (C / 8);
    if (dy_dt == HVIT_BF16)
      hipLaunchKernelGGL((bilinear_bwd_vec_kernel<bf16_t, bf16_t>), dim3(grid_for(groups)), dim3(256), 0,
                         (hipStream_t)stream, (const bf16_t*)dy, (bf16_t*)dx, N, Hi, Wi, C, Ho, Wo, sh, sw,
                         accumulate);
    else
      hipLaunchKernelGGL((bilinear_bwd_vec_kernel<float, float>), dim3(grid_for(groups)), dim3(256), 0,
                         (hipStream_t)stream, (const float*)dy, (float*)dx, N, Hi, Wi, C, Ho, Wo, sh, sw,
                         accumulate);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  HVIT_CHECK(taps_ok, "hvit_bilinear_bwd: upsampling factor above 6 not supported");
  hipLaunchKernelGGL(bilinear_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, dy, dy_dt,
                     dx, dx_dt, N, Hi, Wi, C, Ho, Wo, sh, sw, accumulate);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_upsample_split_bwd(const void* du, int du_dt, int N, int H, int W, int U, int C1, int C2,
                                       void* dx1, int dx1_dt, void* dx2, int dx2_dt, void* stream) {
  HVIT_CHECK(du && dx1 && (C2 == 0 || dx2), "hvit_upsample_split_bwd: null pointer");
  HVIT_CHECK(U >= 1 && C1 > 0 && C2 >= 0, "hvit_upsample_split_bwd: bad sizes");
  long total = (long)N * H * W * (C1 + C2);
  if (total <= 0) return HVIT_OK;
  HVIT_CHECK(total * U * U < (1L << 31), "resample: tensor too large");
  if (du_dt == HVIT_BF16 && dx1_dt == HVIT_BF16 && (C2 == 0 || dx2_dt == HVIT_BF16) && C1 % 8 == 0 && C2 % 8 == 0 &&
      aligned16(du) && aligned16(dx1) && (C2 == 0 || aligned16(dx2))) {
    hipLaunchKernelGGL(up_split_bwd_vec_kernel, dim3(grid_for(total / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)du, N, H, W, U, C1, C2, (bf16_t*)dx1, (bf16_t*)dx2);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  hipLaunchKernelGGL(up_split_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, du, du_dt,
                     N, H, W, U, C1, C2, dx1, dx1_dt, dx2, dx2_dt);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}
