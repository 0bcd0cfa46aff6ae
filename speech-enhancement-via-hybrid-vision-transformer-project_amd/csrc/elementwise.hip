// Small memory-bound kernels around the hot path (gfx950): dtype casts, conv
// weight (re)packing for the implicit GEMMs, dropout/drop-path gradient
// scaling, tanh backward, column reductions (bias / pos-embed gradients) and
// split-K slab reduction.
#include <algorithm>

#include "common.h"

namespace hvit {

static int grid_for(long n, int per_thread = 1) {
  long g = (n / per_thread + 255) / 256;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  return (int)g;
}

#define GRID_STRIDE(i, total) \
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < (total); i += (long)gridDim.x * blockDim.x)

__global__ void cast_kernel(const void* s, int sdt, void* d, int ddt, long n) {
  GRID_STRIDE(i, n) st_dt(d, i, ld_dt(s, i, sdt), ddt);
}

// mode 0: out[co][ky][kx][ci] = w[co][ci][ky][kx]
// mode 1: out[ci][ky][kx][co] = w[co][ci][KS-1-ky][KS-1-kx]   (dgrad, flipped)
__global__ void conv_pack_kernel(const float* w, int Cout, int Cin, int KS, int mode, void* out, int odt) {
  long total = (long)Cout * Cin * KS * KS;
  GRID_STRIDE(i, total) {
    int kx = i % KS;
    long t = i / KS;
    int ky = t % KS;
    t /= KS;
    int ci = t % Cin;
    int co = t / Cin;
    float v = w[i];
    long o;
    if (mode == 0) o = (((long)co * KS + ky) * KS + kx) * Cin + ci;
    else o = (((long)ci * KS + (KS - 1 - ky)) * KS + (KS - 1 - kx)) * Cout + co;
    st_dt(out, o, v, odt);
  }
}

// Eval-mode BatchNorm folded into the conv (components.py:55-85 in eval):
// relu(bn(conv(x, w))) = relu(conv(x, w * sc) + sh), sc = gamma * invstd,
// sh = beta - mean * sc; packed mode-0 weights and the f32 bias
__global__ void bn_fold_kernel(const float* w, int Cout, int Cin, int KS, const float* mean, const float* invstd,
                               const float* gamma, const float* beta, void* out, int odt, float* bias) {
  const long total = (long)Cout * Cin * KS * KS;
  GRID_STRIDE(i, total) {
    const int kx = i % KS;
    long t = i / KS;
    const int ky = t % KS;
    t /= KS;
    const int ci = t % Cin;
    const int co = t / Cin;
    const float sc = gamma[co] * invstd[co];
    st_dt(out, (((long)co * KS + ky) * KS + kx) * Cin + ci, w[i] * sc, odt);
    if (i < Cout) bias[i] = beta[i] - mean[i] * (gamma[i] * invstd[i]);
  }
}

// dw[co][ci][ky][kx] = dwp[co][ky][kx][ci]
__global__ void conv_unpack_kernel(const float* dwp, int Cout, int Cin, int KS, float* dw) {
  long total = (long)Cout * Cin * KS * KS;
  GRID_STRIDE(i, total) {
    int kx = i % KS;
    long t = i / KS;
    int ky = t % KS;
    t /= KS;
    int ci = t % Cin;
    int co = t / Cin;
    dw[i] = dwp[(((long)co * KS + ky) * KS + kx) * Cin + ci];
  }
}

// out[m][n] = g[m][n] * keep(m*N+n)/(1-p) * rowscale[m / rps]
__global__ void dropout_scale_kernel(const void* g, int gdt, void* out, int odt, long M, int N, uint32_t thr,
                                     float ds, DSeed seed_, uint32_t site, const float* rowscale,
                                     int rps) {
  const unsigned long long seed = seed_;
  long total = M * N;
  GRID_STRIDE(i, total) {
    float v = ld_dt(g, i, gdt);
    if (thr) v = rng_keep(seed, site, (uint64_t)i, thr) ? v * ds : 0.f;
    if (rowscale) v *= rowscale[(i / N) / rps];
    st_dt(out, i, v, odt);
  }
}

// vectorised form: 4 consecutive elements per thread, N % 4 == 0, 32-bit indices
__global__ void dropout_scale4_kernel(const void* g, int gdt, void* out, int odt, int M, int N, uint32_t thr,
                                      float ds, DSeed seed_, uint32_t site, const float* rowscale,
                                      int rps) {
  const unsigned long long seed = seed_;
  const int total4 = M * (N / 4);
  for (int i4 = blockIdx.x * blockDim.x + threadIdx.x; i4 < total4; i4 += gridDim.x * blockDim.x) {
    const int i = i4 * 4;
    f32x4 v;
    if (gdt == HVIT_F32) {
      v = *(const f32x4*)((const float*)g + i);
    } else {
      uint2 u = *(const uint2*)((const bf16_t*)g + i);
      v = (f32x4){__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                  __uint_as_float(u.y & 0xffff0000u)};
    }
    if (thr) {
      v *= keep4_at(rng_key(seed, site), (uint64_t)i, thr, ds);
    }
    if (rowscale) v *= rowscale[(i / N) / rps];
    if (odt == HVIT_F32) {
      *(f32x4*)((float*)out + i) = v;
    } else {
      uint2 u;
      u.x = f2bf2(v[0], v[1]);
      u.y = f2bf2(v[2], v[3]);
      *(uint2*)((bf16_t*)out + i) = u;
    }
  }
}

// dropout_scale4 + column sums of the output (the bias gradient of the GEMM
// that consumes it): a thread's 4 columns never change (grid stride is a
// multiple of N/4, host-checked: (N/4) divides 256), so the sums stay in
// registers; threads of a block sharing columns fold through LDS and the
// block writes its N partial sums to part[block][N] (no same-address atomics:
// with a few hundred workgroups those serialised the pass 3x), which one
// column reduction adds into the caller's colsum.
constexpr int DSC_THREADS = 256, DSC_BLOCKS = 1024;
__global__ __launch_bounds__(DSC_THREADS) void dropout_scale4_colsum_kernel(const void* g, int gdt, void* out, int odt, int M,
                                                                    int N, uint32_t thr, float ds,
                                                                    DSeed seed_, uint32_t site,
                                                                    const float* rowscale, int rps,
                                                                    float* __restrict__ part) {
  const unsigned long long seed = seed_;
  __shared__ f32x4 red[DSC_THREADS];
  const int total4 = M * (N / 4);
  const int stride = gridDim.x * blockDim.x;
  f32x4 cs = {0.f, 0.f, 0.f, 0.f};
  // DS_UNROLL independent 16-byte loads in flight per thread (few, long-lived
  // workgroups keep the atomics per column low)
  constexpr int DS_UNROLL = 8;
  for (int base = blockIdx.x * blockDim.x + threadIdx.x; base < total4; base += DS_UNROLL * stride) {
    f32x4 v[DS_UNROLL];
#pragma unroll
    for (int k = 0; k < DS_UNROLL; ++k) {
      const int i = (base + k * stride) * 4;
      v[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (base + k * stride < total4) {
        if (gdt == HVIT_F32) {
          v[k] = *(const f32x4*)((const float*)g + i);
        } else {
          uint2 u = *(const uint2*)((const bf16_t*)g + i);
          v[k] = (f32x4){__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                         __uint_as_float(u.y & 0xffff0000u)};
        }
      }
    }
#pragma unroll
    for (int k = 0; k < DS_UNROLL; ++k) {
      if (base + k * stride >= total4) break;
      const int i = (base + k * stride) * 4;
      if (thr) {
        v[k] *= keep4_at(rng_key(seed, site), (uint64_t)i, thr, ds);
      }
      if (rowscale) v[k] *= rowscale[(i / N) / rps];
      cs += v[k];
      if (odt == HVIT_F32) {
        *(f32x4*)((float*)out + i) = v[k];
      } else {
        uint2 u;
        u.x = f2bf2(v[k][0], v[k][1]);
        u.y = f2bf2(v[k][2], v[k][3]);
        *(uint2*)((bf16_t*)out + i) = u;
      }
    }
  }
  red[threadIdx.x] = cs;
  __syncthreads();
  const int n4 = N / 4;
  if ((int)threadIdx.x < n4) {
    f32x4 t = red[threadIdx.x];
    for (int k = threadIdx.x + n4; k < DSC_THREADS; k += n4) t += red[k];
    const int c = ((blockIdx.x * blockDim.x + threadIdx.x) % n4) * 4;
    *(f32x4*)(part + (long)blockIdx.x * N + c) = t;  // every block writes all N partials
  }
}

__global__ void tanh_bwd_kernel(const void* dy, int dydt, const float* y, void* dz, int dzdt, long n) {
  GRID_STRIDE(i, n) {
    float t = y[i];
    st_dt(dz, i, ld_dt(dy, i, dydt) * (1.f - t * t), dzdt);
  }
}

// Deterministic column sums (no atomics: the result is bit-identical from run
// to run and between eager launches and graph replays).  out[s*N + n] (+)=
// sum of x[m*ld + n] over the rows m of segment s = blockIdx.y, [s*Ms,
// min((s+1)*Ms, Mt)).  A
// block owns TX column chunks of VEC elements (16-byte loads, or scalar loads
// for unaligned widths) and splits the rows over RY = 256 / TX row groups:
// thread (tx, ty) sums rows ty, ty + RY, ... into four accumulators (four rows
// in flight), folded in a fixed order; the RY partials of a column are then
// added in row-group order through LDS.  The summation order depends only on
// (M, N, TX), which the host derives from the shape.
template <typename T, bool VECLD>
__global__ __launch_bounds__(256) void colsum_det_kernel(const T* __restrict__ x, int Ms, int Mt, int N, long ld,
                                                          int TX, int accumulate, float* __restrict__ out) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float red[256 * VEC];
  const int RY = 256 / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int n = (blockIdx.x * TX + tx) * VEC;
  const long seg_off = (long)blockIdx.y * Ms;
  const int M = min(Ms, Mt - (int)seg_off);  // rows of this segment
  float a0[VEC], a1[VEC], a2[VEC], a3[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) a0[e] = a1[e] = a2[e] = a3[e] = 0.f;
  auto ld_row = [&](long m, float* v) {
    const T* p = x + (seg_off + m) * ld + n;
    if constexpr (VECLD) {
      const u32x4 u = *(const u32x4*)p;
      const T* eu = (const T*)&u;
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[e] = Elem<T>::to_f(eu[e]);
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[e] = n + e < N ? Elem<T>::to_f(p[e]) : 0.f;
    }
  };
  if (n < N) {
    int m = ty;
    for (; m + 3 * RY < M; m += 4 * RY) {
      float v0[VEC], v1[VEC], v2[VEC], v3[VEC];
      ld_row(m, v0);
      ld_row(m + RY, v1);
      ld_row(m + 2 * RY, v2);
      ld_row(m + 3 * RY, v3);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        a0[e] += v0[e];
        a1[e] += v1[e];
        a2[e] += v2[e];
        a3[e] += v3[e];
      }
    }
    for (; m < M; m += RY) {
      float v0[VEC];
      ld_row(m, v0);
#pragma unroll
      for (int e = 0; e < VEC; ++e) a0[e] += v0[e];
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) red[ty * (TX * VEC) + tx * VEC + e] = (a0[e] + a1[e]) + (a2[e] + a3[e]);
  __syncthreads();
  for (int c = threadIdx.x; c < TX * VEC; c += blockDim.x) {
    const int col = blockIdx.x * TX * VEC + c;
    if (col >= N) continue;
    float s = 0.f;
    for (int k = 0; k < RY; ++k) s += red[k * (TX * VEC) + c];
    float* o = out + (long)blockIdx.y * N + col;
    *o = accumulate ? *o + s : s;
  }
}

// out[i] = sum_k ws[k*n + i]; 4 consecutive elements per thread, 4 slabs in flight
__global__ void sum_slabs_kernel(const float* ws, int splits, long n, float* out) {
  GRID_STRIDE(i, n) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += ws[(long)k * n + i];
    out[i] = s;
  }
}

__global__ void sum_slabs4_kernel(const float* ws, int splits, int n4, float* out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const f32x4* p = (const f32x4*)ws + i;
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
    int k = 0;
    for (; k + 8 <= splits; k += 8) {  // eight slabs in flight, the same accumulator order
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(long)(k + u) * n4];
      s0 += v[0];
      s1 += v[1];
      s2 += v[2];
      s3 += v[3];
      s0 += v[4];
      s1 += v[5];
      s2 += v[6];
      s3 += v[7];
    }
    for (; k + 4 <= splits; k += 4) {
      s0 += p[(long)k * n4];
      s1 += p[(long)(k + 1) * n4];
      s2 += p[(long)(k + 2) * n4];
      s3 += p[(long)(k + 3) * n4];
    }
    for (; k < splits; ++k) s0 += p[(long)k * n4];
    ((f32x4*)out)[i] = (s0 + s1) + (s2 + s3);
  }
}

// Multi-tensor weight preparation (one launch per forward per form instead of
// one per weight): f32 master parameters -> bf16/f32 copies (kind 0) or conv
// packings (kind 1: [Cout][KS][KS][Cin], kind 2: flipped [Cin][KS][KS][Cout],
// kind 3: kind 1 with eval BatchNorm folded in, bn_fold_kernel's arithmetic
// with the running statistics -- inference no longer spends an eval-prep and a
// fold launch per conv block).  Casts: the flattened index space split into
// 4-element units (every item's numel is a multiple of 4), a thread locating its
// item in the prefix table; packings: weight_pack_tiled_kernel below.
constexpr int WPREP_MAX = 24;
struct WPrepItem {
  const float* src;
  void* dst;
  int n4;    // numel / 4
  int kind;  // 0 cast, 1 pack mode 0, 2 pack mode 1, 3 pack mode 0 with eval BN folded
  int dt;
  int co, ci, ks;
  const float *gamma, *beta, *rmean, *rvar;
  float* bias;
  float eps;
  int ci_shift;  // log2(ci) when ci is a power of two, else -1
  int co_shift;  // log2(co) when co is a power of two, else -1
};
struct WPrepArgs {
  int count;
  int start[WPREP_MAX + 1];  // prefix sums of n4
  WPrepItem it[WPREP_MAX];
};
static_assert(sizeof(WPrepArgs) <= 4096, "weight_prep: kernel argument size");

__global__ __launch_bounds__(256) void weight_prep_kernel(WPrepArgs a) {  // kind 0: casts
  const int total = a.start[a.count];
  int j = 0;
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < total; u += gridDim.x * blockDim.x) {
    while (u >= a.start[j + 1]) ++j;  // u only grows: the search resumes
    const WPrepItem& w = a.it[j];
    const int l4 = u - a.start[j];
    const f32x4 v = *(const f32x4*)(w.src + 4L * l4);
    if (w.dt == HVIT_F32) {
      *(f32x4*)((float*)w.dst + 4L * l4) = v;
    } else {
      *(uint2*)((bf16_t*)w.dst + 4L * l4) = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
    }
  }
}

// The conv packings tiled through LDS: one workgroup per output channel (kinds
// 1 / 3: destination block [KS][KS][Cin] of that channel, contiguous; its source
// [Cin][KS][KS] block read contiguously) or per input channel (kind 2: the
// flipped [KS][KS][Cout] block; its source rows of KS*KS floats gathered), so
// both the reads and the stores coalesce (the flat form above gathered or
// scattered single elements: ~30 us for the model's 4.3 M conv weights x 2
// packings).  start[] holds prefix sums of blocks; the same arithmetic per
// element as the flat form.
constexpr int WPT_MAXE = 40960;  // floats per block (Cin * KS * KS or Cout * KS * KS): 160 KiB of LDS
__global__ __launch_bounds__(256) void weight_pack_tiled_kernel(WPrepArgs a) {
  extern __shared__ float tile[];  // the launch's largest block
  const int blk = blockIdx.x;
  int j = 0;
  while (blk >= a.start[j + 1]) ++j;  // uniform per workgroup
  const WPrepItem& w = a.it[j];
  const int b = blk - a.start[j];
  const int K2 = w.ks * w.ks;
  const int tid = threadIdx.x;
  if (w.kind != 2) {  // b = output channel
    const int n = w.ci * K2;
    const float* src = w.src + (long)b * n;
    for (int i = tid; i < n; i += 256) tile[i] = src[i];
    __syncthreads();
    float sc = 1.f;
    if (w.kind == 3) {
      sc = w.gamma[b] * rsqrtf(w.rvar[b] + w.eps);
      if (tid == 0) w.bias[b] = w.beta[b] - w.rmean[b] * (w.gamma[b] * rsqrtf(w.rvar[b] + w.eps));
    }
    const long o0 = (long)b * n;
    for (int o = tid; o < n; o += 256) {
      const int ci = w.ci_shift >= 0 ? (o & (w.ci - 1)) : o % w.ci;
      const int t = w.ci_shift >= 0 ? (o >> w.ci_shift) : o / w.ci;  // ky * KS + kx
      float x = tile[ci * K2 + t];
      if (w.kind == 3) x *= sc;
      st_dt(w.dst, o0 + o, x, w.dt);
    }
  } else {  // b = input channel; destination [ky'][kx'][co], ky' = KS-1-ky, kx' = KS-1-kx
    const int n = w.co * K2;
    for (int i = tid; i < n; i += 256) {
      const int co = i / K2, t = i - co * K2;
      tile[i] = w.src[((long)co * w.ci + b) * K2 + t];
    }
    __syncthreads();
    const long o0 = (long)b * n;
    for (int o = tid; o < n; o += 256) {
      const int co = w.co_shift >= 0 ? (o & (w.co - 1)) : o % w.co;
      const int tf = w.co_shift >= 0 ? (o >> w.co_shift) : o / w.co;
      st_dt(w.dst, o0 + o, tile[co * K2 + (K2 - 1 - tf)], w.dt);
    }
  }
}

// Packings whose block does not fit the LDS tile (Cin * KS * KS or Cout * KS
// * KS above WPT_MAXE floats): one thread per destination element, gathering
// from the source directly (start[] holds prefix sums of elements); the tiled
// kernel's arithmetic element for element.
__global__ __launch_bounds__(256) void weight_pack_flat_kernel(WPrepArgs a) {
  const int total = a.start[a.count];
  int j = 0;
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < total; u += gridDim.x * blockDim.x) {
    while (u >= a.start[j + 1]) ++j;  // u only grows: the search resumes
    const WPrepItem& w = a.it[j];
    const int o = u - a.start[j];
    const int K2 = w.ks * w.ks;
    if (w.kind != 2) {  // [Cout][KS][KS][Cin] <- [Cout][Cin][KS][KS]
      const int n = w.ci * K2;
      const int b = o / n, r = o - b * n;
      const int ci = r % w.ci, t = r / w.ci;
      float x = w.src[(long)b * n + ci * K2 + t];
      if (w.kind == 3) {
        x *= w.gamma[b] * rsqrtf(w.rvar[b] + w.eps);
        if (r == 0) w.bias[b] = w.beta[b] - w.rmean[b] * (w.gamma[b] * rsqrtf(w.rvar[b] + w.eps));
      }
      st_dt(w.dst, o, x, w.dt);
    } else {  // flipped [Cin][KS][KS][Cout]
      const int n = w.co * K2;
      const int b = o / n, r = o - b * n;
      const int co = r % w.co, tf = r / w.co;
      st_dt(w.dst, o, w.src[((long)co * w.ci + b) * K2 + (K2 - 1 - tf)], w.dt);
    }
  }
}

__global__ void droppath_scale_kernel(int B, uint32_t thr, float ds, DSeed seed_, uint32_t site,
                                      float* out) {
  const unsigned long long seed = seed_;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) out[b] = rng_keep(seed, site, (uint64_t)b, thr) ? ds : 0.f;
}

// The DropPath multipliers of up to DPS_MAX blocks from one launch:
// blockIdx.y = block j, out[j * B + b] as droppath_scale_kernel with block j's
// (p, seed, site) -- the per-block launches were ~4.6 us each of dispatch for
// 2B floats.
constexpr int DPS_MAX = 32;
struct DpsArgs {
  uint32_t thr[DPS_MAX];
  float ds[DPS_MAX];
  DSeed seed[DPS_MAX];
  uint32_t site[DPS_MAX];
};
__global__ void droppath_scales_kernel(int B, DpsArgs a, float* out) {
  const int j = blockIdx.y;
  const unsigned long long seed = a.seed[j];
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) out[(long)j * B + b] = rng_keep(seed, a.site[j], (uint64_t)b, a.thr[j]) ? a.ds[j] : 0.f;
}

}  // namespace hvit

using namespace hvit;

extern "C" int hvit_cast(const void* src, int src_dt, void* dst, int dst_dt, long long n, void* stream) {
  HVIT_CHECK(src && dst, "hvit_cast: null pointer");
  if (n <= 0) return HVIT_OK;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, src, src_dt, dst,
                     dst_dt, (long)n);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_conv_weight_pack(const float* w, int Cout, int Cin, int KS, int mode, void* out,
                                     int out_dt, void* stream) {
  HVIT_CHECK(w && out, "hvit_conv_weight_pack: null pointer");
  HVIT_CHECK(mode == 0 || mode == 1, "hvit_conv_weight_pack: mode");
  long n = (long)Cout * Cin * KS * KS;
  hipLaunchKernelGGL(conv_pack_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, KS,
                     mode, out, out_dt);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_bn_fold(const float* w, int Cout, int Cin, int KS, const float* mean, const float* invstd,
                            const float* gamma, const float* beta, void* w_packed, int w_dt, float* bias,
                            void* stream) {
  HVIT_CHECK(w && mean && invstd && gamma && beta && w_packed && bias, "hvit_bn_fold: null pointer");
  const long n = (long)Cout * Cin * KS * KS;
  HVIT_CHECK(n >= Cout && Cout > 0, "hvit_bn_fold: bad shape");
  hipLaunchKernelGGL(bn_fold_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, KS, mean,
                     invstd, gamma, beta, w_packed, w_dt, bias);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

// dw[co][ci][ky][kx] = sum_z ws[z * slab + ((co*KS + ky)*KS + kx)*Cin + ci]: a
// packed conv weight gradient's split-K slabs summed straight into the
// Parameter's layout (one pass instead of a slab sum and an unpack).  Threads
// walk the packed order four channels at a time (coalesced 16-byte slab reads,
// the same four-accumulator order as sum_slabs4_kernel) and scatter the four
// sums to their [co][ci][ky][kx] places.
__global__ void sum_slabs_unpack4_kernel(const float* ws, int splits, long slab4, int Cout, int Cin, int KS,
                                         float* dw) {
  const int C4 = Cin / 4, T = KS * KS;
  const long total = (long)Cout * T * C4;
  GRID_STRIDE(i, total) {
    const int c4 = i % C4;
    const long t = i / C4;
    const int tap = t % T;
    const int co = t / T;
    const f32x4* p = (const f32x4*)ws + i;
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
    int k = 0;
    // eight slabs' loads in flight per step (the same four-accumulator order)
    for (; k + 8 <= splits; k += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(long)(k + u) * slab4];
      s0 += v[0];
      s1 += v[1];
      s2 += v[2];
      s3 += v[3];
      s0 += v[4];
      s1 += v[5];
      s2 += v[6];
      s3 += v[7];
    }
    for (; k + 4 <= splits; k += 4) {
      s0 += p[(long)k * slab4];
      s1 += p[(long)(k + 1) * slab4];
      s2 += p[(long)(k + 2) * slab4];
      s3 += p[(long)(k + 3) * slab4];
    }
    for (; k < splits; ++k) s0 += p[(long)k * slab4];
    const f32x4 v = (s0 + s1) + (s2 + s3);
    float* o = dw + ((long)co * Cin + 4 * c4) * T + tap;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[(long)e * T] = v[e];
  }
}

int hvit_sum_slabs_unpack(const float* ws, int splits, long long slab, int Cout, int Cin, int KS, float* dw,
                          float* tmp, hipStream_t st) {
  const long n4 = (long)Cout * KS * KS * (Cin / 4);
  if (Cin % 4 || slab % 4 || ((uintptr_t)ws & 15) || splits >= 64) {
    // (many slabs: the column-reduction form of hvit_sum_slabs into tmp, then unpack)
    if (int rc = hvit_sum_slabs(ws, splits, slab, tmp, st)) return rc;
    return hvit_conv_weight_unpack(tmp, Cout, Cin, KS, dw, st);
  }
  hipLaunchKernelGGL(sum_slabs_unpack4_kernel, dim3(grid_for(n4)), dim3(256), 0, st, ws, splits, (long)(slab / 4),
                     Cout, Cin, KS, dw);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_conv_weight_unpack(const float* dw_packed, int Cout, int Cin, int KS, float* dw,
                                       void* stream) {
  HVIT_CHECK(dw_packed && dw, "hvit_conv_weight_unpack: null pointer");
  long n = (long)Cout * Cin * KS * KS;
  hipLaunchKernelGGL(conv_unpack_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dw_packed, Cout,
                     Cin, KS, dw);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" long long hvit_dropout_colsum_ws_elems(int N) { return (long long)DSC_BLOCKS * (N > 0 ? N : 0); }

extern "C" int hvit_dropout_scale(const void* g, int g_dt, long long M, int N, const hvit_dropout_t* dropout,
                                  const float* rowscale, int rows_per_sample, void* out, int out_dt, float* colsum,
                                  float* ws, long long ws_elems, void* stream) {
  HVIT_CHECK(g && out, "hvit_dropout_scale: null pointer");
  HVIT_CHECK(!rowscale || rows_per_sample > 0, "hvit_dropout_scale: rows_per_sample");
  uint32_t thr = dropout ? drop_threshold(dropout->p) : 0;
  float ds = (dropout && dropout->p > 0.f) ? 1.f / (1.f - dropout->p) : 1.f;
  long total = (long)M * N;
  if (total <= 0) return HVIT_OK;
  if (colsum) {
    if (N % 4 == 0 && N / 4 <= 256 && 256 % (N / 4) == 0 && total < (1L << 31) && aligned16(g) && aligned16(out) &&
        ws && aligned16(ws) && ws_elems >= hvit_dropout_colsum_ws_elems(N)) {
      hipLaunchKernelGGL(dropout_scale4_colsum_kernel, dim3(DSC_BLOCKS), dim3(DSC_THREADS), 0,
                         (hipStream_t)stream, g, g_dt, out, out_dt, (int)M, N, thr, ds,
                         dseed(dropout), dropout ? dropout->site : 0u, rowscale, rows_per_sample,
                         ws);
      HVIT_LAUNCH_CHECK();
      return hvit_reduce_rows(ws, HVIT_F32, DSC_BLOCKS, N, N, 1, colsum, stream);
    }
    // other widths / no workspace: the plain pass, then a column reduction of its output
    if (int rc = hvit_dropout_scale(g, g_dt, M, N, dropout, rowscale, rows_per_sample, out, out_dt, nullptr, nullptr,
                                    0, stream))
      return rc;
    return hvit_reduce_rows(out, out_dt, M, N, N, 1, colsum, stream);
  }
  if (N % 4 == 0 && total < (1L << 31) && aligned16(g) && aligned16(out)) {
    hipLaunchKernelGGL(dropout_scale4_kernel, dim3(grid_for(total, 4)), dim3(256), 0, (hipStream_t)stream, g,
                       g_dt, out, out_dt, (int)M, N, thr, ds, dseed(dropout),
                       dropout ? dropout->site : 0u, rowscale, rows_per_sample);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  hipLaunchKernelGGL(dropout_scale_kernel, dim3(grid_for(total, 4)), dim3(256), 0, (hipStream_t)stream, g, g_dt,
                     out, out_dt, (long)M, N, thr, ds, dseed(dropout),
                     dropout ? dropout->site : 0u, rowscale, rows_per_sample);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_tanh_bwd(const void* dy, int dy_dt, const float* y, long long n, void* dz, int dz_dt,
                             void* stream) {
  HVIT_CHECK(dy && y && dz, "hvit_tanh_bwd: null pointer");
  if (n <= 0) return HVIT_OK;
  hipLaunchKernelGGL(tanh_bwd_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, dy, dy_dt, y, dz,
                     dz_dt, (long)n);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

// Deterministic column sums (colsum_det_kernel) over segments of Ms rows
// (the last one clipped at Mt): out [S = cdiv(Mt, Ms)][N].  The column-chunk
// width TX is the largest of 32 / 16 / 8 / 4 that still gives >= 128
// workgroups, so short-and-wide and tall-and-narrow matrices both spread over
// the chip; the choice depends on the shape only (fixed summation order).
static int colsum_launch(const void* x, int dt, long long Ms, long long Mt, long long N, long long ld, int accumulate,
                         float* out, hipStream_t st) {
  HVIT_CHECK(x && out, "hvit_reduce_rows: null pointer");
  HVIT_CHECK(dt == HVIT_F32 || dt == HVIT_BF16, "hvit_reduce_rows: dtype");
  HVIT_CHECK(Ms > 0 && Mt >= 0 && N >= 0 && ld >= N && Mt < (1LL << 31) && N < (1LL << 31),
             "hvit_reduce_rows: bad shape");
  const long long S = Mt > 0 ? (Mt + Ms - 1) / Ms : 1;  // (no rows: one segment of zeros)
  HVIT_CHECK(S < 65536, "hvit_reduce_rows: too many segments");
  if (S == 0 || N == 0) return HVIT_OK;
  const int es = dt == HVIT_F32 ? 4 : 2, vec = 16 / es;
  const bool vecld = N % vec == 0 && ld % vec == 0 && ((uintptr_t)x & 15) == 0;
  const long nvec = (N + vec - 1) / vec;
  int tx = 32;
  while (tx > 4 && cdiv(nvec, tx) * S < 128) tx /= 2;
  dim3 g((unsigned)cdiv(nvec, tx), (unsigned)S);
#define HVIT_COLSUM(T, V)                                                                                       \
  hipLaunchKernelGGL((colsum_det_kernel<T, V>), g, dim3(256), 0, st, (const T*)x, (int)Ms, (int)Mt, (int)N, (long)ld, \
                     tx, accumulate, out)
  if (dt == HVIT_F32) {
    if (vecld) HVIT_COLSUM(float, true);
    else HVIT_COLSUM(float, false);
  } else {
    if (vecld) HVIT_COLSUM(bf16_t, true);
    else HVIT_COLSUM(bf16_t, false);
  }
#undef HVIT_COLSUM
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

// S segments of M rows each (x rows [s*M, (s+1)*M)) -> out [S][N]
int hvit_reduce_rows_seg(const void* x, int dt, long long S, long long M, long long N, long long ld, int accumulate,
                         float* out, void* stream) {
  if (S <= 0 || M <= 0) return HVIT_OK;
  return colsum_launch(x, dt, M, S * M, N, ld, accumulate, out, (hipStream_t)stream);
}

// Column sums of a tall matrix in two deterministic levels when f32 scratch
// (ws, >= 64 * N floats) allows: 64 row segments -> [64][N] partials -> out.
// Otherwise one level (every row of a column chunk walked by one workgroup).
int hvit_reduce_rows_ws(const void* x, int dt, long long M, long long N, long long ld, int accumulate, float* out,
                        float* ws, long long ws_elems, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  constexpr long long P = 64;
  if (M > 4096 && ws && ws_elems >= P * N) {
    if (int rc = colsum_launch(x, dt, (M + P - 1) / P, M, N, ld, 0, ws, st)) return rc;
    const long long S = (M + (M + P - 1) / P - 1) / ((M + P - 1) / P);
    return colsum_launch(ws, HVIT_F32, S, S, N, N, accumulate, out, st);
  }
  return colsum_launch(x, dt, M > 0 ? M : 1, M, N, ld, accumulate, out, st);
}

extern "C" int hvit_reduce_rows(const void* x, int dt, long long M, long long N, long long ld, int accumulate,
                                float* out, void* stream) {
  return colsum_launch(x, dt, M > 0 ? M : 1, M, N, ld, accumulate, out, (hipStream_t)stream);
}

// out[i] = sum_k ws[k * stride + i], i < n (slabs of `stride` elements)
__global__ void sum_slabs_strided_kernel(const float* ws, int splits, long stride, long n, float* out) {
  GRID_STRIDE(i, n) {
    float s0 = 0.f, s1 = 0.f;
    int k = 0;
    for (; k + 1 < splits; k += 2) {
      s0 += ws[(long)k * stride + i];
      s1 += ws[(long)(k + 1) * stride + i];
    }
    if (k < splits) s0 += ws[(long)k * stride + i];
    out[i] = s0 + s1;
  }
}

// the many-slab form: a granule per wave (side_wave_granule)
__global__ __launch_bounds__(256) void sum_slabs_wave_kernel(const float* ws, int splits, long stride4, long n4,
                                                             float* out) {
  const long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n4) return;  // (whole waves)
  const f32x4 s = side_wave_granule((const f32x4*)ws, stride4, splits, i);
  if ((threadIdx.x & 63) == 0) ((f32x4*)out)[i] = s;
}

// A deferred slab-sum job run as a launch of its own: the same summation order
// as the epilogue side job that would otherwise carry it (gemm.h epi_side: a
// wave per granule from SIDE_WAVE_SPLITS slabs, else even | odd pairs)
int hvit_sum_slabs_strided(const float* ws, int splits, long long stride, long long n, float* out, void* stream) {
  HVIT_CHECK(ws && out && splits > 0 && stride >= n, "hvit_sum_slabs_strided: bad args");
  if (n <= 0) return HVIT_OK;
  if (splits >= SIDE_WAVE_SPLITS && n % 4 == 0 && stride % 4 == 0 && ((uintptr_t)ws & 15) == 0 &&
      ((uintptr_t)out & 15) == 0) {
    hipLaunchKernelGGL(sum_slabs_wave_kernel, dim3((unsigned)cdiv(n / 4, 4)), dim3(256), 0, (hipStream_t)stream, ws,
                       splits, (long)(stride / 4), (long)(n / 4), out);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  hipLaunchKernelGGL(sum_slabs_strided_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, ws, splits,
                     (long)stride, (long)n, out);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_sum_slabs(const float* ws, int splits, long long n, float* out, void* stream) {
  HVIT_CHECK(ws && out && splits > 0, "hvit_sum_slabs: bad args");
  if (n <= 0) return HVIT_OK;
  if (splits >= 64 && n <= 65536) {
    // many short slabs (per-workgroup partials): a column reduction of the
    // [splits][n] matrix spreads the work over all CUs
    return hvit_reduce_rows(ws, HVIT_F32, splits, n, n, 0, out, stream);
  }
  if (n % 4 == 0 && ((uintptr_t)ws & 15) == 0 && ((uintptr_t)out & 15) == 0 && n < (1LL << 31)) {
    hipLaunchKernelGGL(sum_slabs4_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, ws, splits,
                       (int)(n / 4), out);
  } else {
    hipLaunchKernelGGL(sum_slabs_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, ws, splits,
                       (long)n, out);
  }
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_weight_prep(int count, const hvit_wprep_item_t* items, void* stream) {
  HVIT_CHECK(count >= 0 && (count == 0 || items), "hvit_weight_prep: bad args");
  // casts (kind 0) in the flat launch, packings (kinds 1-3) in the tiled one,
  // packings whose block is above the LDS tile in the flat gather
  auto big = [](const hvit_wprep_item_t& it) {
    return (long long)it.cin * it.ks * it.ks > WPT_MAXE || (long long)it.cout * it.ks * it.ks > WPT_MAXE;
  };
  for (int pass = 0; pass < 3; ++pass) {
    WPrepArgs a;
    a.count = 0;
    a.start[0] = 0;
    long maxe = 0;  // the tiled launch's largest block (floats)
    auto flush = [&]() -> int {
      const int total = a.start[a.count];
      if (total > 0) {
        if (pass == 0)
          hipLaunchKernelGGL(weight_prep_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, a);
        else if (pass == 2)
          hipLaunchKernelGGL(weight_pack_flat_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, a);
        else {
          if (maxe * (long)sizeof(float) > 65536)
            (void)hipFuncSetAttribute((const void*)weight_pack_tiled_kernel,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)(maxe * sizeof(float)));
          hipLaunchKernelGGL(weight_pack_tiled_kernel, dim3(total), dim3(256), maxe * sizeof(float),
                             (hipStream_t)stream, a);
        }
        HVIT_LAUNCH_CHECK();
      }
      a.count = 0;
      maxe = 0;
      return HVIT_OK;
    };
    for (int k = 0; k < count; ++k) {
      const hvit_wprep_item_t& it = items[k];
      HVIT_CHECK(it.src && it.dst && it.numel >= 0 && it.numel % 4 == 0 && it.numel < (1LL << 31),
                 "hvit_weight_prep: item %d: null pointer or numel %% 4 != 0", k);
      HVIT_CHECK(it.kind >= 0 && it.kind <= 3, "hvit_weight_prep: item %d: kind", k);
      HVIT_CHECK(it.kind != 3 || (it.gamma && it.beta && it.rmean && it.rvar && it.bias),
                 "hvit_weight_prep: item %d: BN fold needs gamma, beta, rmean, rvar, bias", k);
      HVIT_CHECK(it.kind == 0 || (long long)it.cout * it.cin * it.ks * it.ks == it.numel,
                 "hvit_weight_prep: item %d: conv shape", k);
      HVIT_CHECK(aligned16(it.src) && (it.kind != 0 || aligned16(it.dst)), "hvit_weight_prep: item %d: alignment", k);
      if (pass != (it.kind == 0 ? 0 : big(it) ? 2 : 1)) continue;
      const int cis = (it.cin > 0 && (it.cin & (it.cin - 1)) == 0) ? __builtin_ctz((unsigned)it.cin) : -1;
      const int cos = (it.cout > 0 && (it.cout & (it.cout - 1)) == 0) ? __builtin_ctz((unsigned)it.cout) : -1;
      a.it[a.count] = WPrepItem{it.src,   it.dst,  (int)(it.numel / 4), it.kind, it.dt,   it.cout, it.cin,
                                it.ks,    it.gamma, it.beta,             it.rmean, it.rvar, it.bias, it.eps, cis, cos};
      const int units = pass == 0 ? (int)(it.numel / 4) : pass == 2 ? (int)it.numel : (it.kind == 2 ? it.cin : it.cout);
      if (pass == 1) maxe = std::max(maxe, (long)(it.kind == 2 ? it.cout : it.cin) * it.ks * it.ks);
      a.start[a.count + 1] = a.start[a.count] + units;
      if (++a.count == WPREP_MAX)
        if (int rc = flush()) return rc;
    }
    if (int rc = flush()) return rc;
  }
  return HVIT_OK;
}

extern "C" int hvit_droppath_scales(int B, int n, const hvit_dropout_t* dropouts, float* out, void* stream) {
  HVIT_CHECK(out && dropouts && B > 0 && n > 0 && n <= DPS_MAX, "hvit_droppath_scales: bad args");
  DpsArgs a;
  for (int j = 0; j < n; ++j) {
    const hvit_dropout_t& d = dropouts[j];
    a.thr[j] = drop_threshold(d.p);
    a.ds[j] = d.p > 0.f ? 1.f / (1.f - d.p) : 1.f;
    a.seed[j] = dseed(&d);
    a.site[j] = d.site;
  }
  hipLaunchKernelGGL(droppath_scales_kernel, dim3(cdiv(B, 256), n), dim3(256), 0, (hipStream_t)stream, B, a, out);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_droppath_scale(int B, const hvit_dropout_t* dropout, float* out, void* stream) {
  HVIT_CHECK(out && dropout && B > 0, "hvit_droppath_scale: bad args");
  uint32_t thr = drop_threshold(dropout->p);
  float ds = dropout->p > 0.f ? 1.f / (1.f - dropout->p) : 1.f;
  hipLaunchKernelGGL(droppath_scale_kernel, dim3(cdiv(B, 256)), dim3(256), 0, (hipStream_t)stream, B, thr, ds,
                     dseed(dropout), dropout->site, out);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}
