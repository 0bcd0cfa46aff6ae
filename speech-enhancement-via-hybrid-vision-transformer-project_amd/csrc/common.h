// Common device/host helpers for the HybridViT gfx950 kernels.
//
// Element types: activations and GEMM operands are either f32 (the parity path,
// exact-f32 MFMA) or bf16 (the throughput path, bf16 MFMA, f32 accumulate).
// Statistics, residual stream and weight gradients are always f32.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/hvit.h"

typedef uint16_t bf16_t;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ errors --
void hvit_set_error(const char* fmt, ...);
// deterministic column sums (elementwise.hip): S segments of M rows -> out [S][N];
// and a tall matrix's column sums in two levels through f32 scratch ws (>= 64 * N)
int hvit_reduce_rows_seg(const void* x, int dt, long long S, long long M, long long N, long long ld, int accumulate,
                         float* out, void* stream);
int hvit_reduce_rows_ws(const void* x, int dt, long long M, long long N, long long ld, int accumulate, float* out,
                        float* ws, long long ws_elems, void* stream);
#define HVIT_CHECK(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      hvit_set_error(__VA_ARGS__);            \
      return HVIT_ERR_ARG;                    \
    }                                         \
  } while (0)
#define HVIT_LAUNCH_CHECK()                                              \
  do {                                                                   \
    hipError_t e_ = hipGetLastError();                                   \
    if (e_ != hipSuccess) {                                              \
      hvit_set_error("%s: launch failed: %s", __func__, hipGetErrorString(e_)); \
      return HVIT_ERR_LAUNCH;                                            \
    }                                                                    \
  } while (0)

static inline bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

// ---------------------------------------------------------------- bf16 math --
__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// f32 -> bf16, round-to-nearest-even, NaN stays NaN: the plain conversion
// compiles to the gfx950 v_cvt_pk_bf16_f32 (one instruction per pair)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t f2bf2(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int PER16 = 4;  // elements per 16 bytes
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};
template <> struct Elem<bf16_t> {
  static constexpr int PER16 = 8;
  __device__ __forceinline__ static float to_f(bf16_t v) { return bf2f(v); }
  __device__ __forceinline__ static bf16_t from_f(float v) { return f2bf(v); }
};

template <typename T>
__device__ __forceinline__ float ldf(const T* p, long i) { return Elem<T>::to_f(p[i]); }
template <typename T>
__device__ __forceinline__ void stf(T* p, long i, float v) { p[i] = Elem<T>::from_f(v); }

// runtime-dtype load/store (used by epilogues / elementwise kernels)
__device__ __forceinline__ float ld_dt(const void* p, long i, int dt) {
  return dt == HVIT_F32 ? ((const float*)p)[i] : bf2f(((const bf16_t*)p)[i]);
}
__device__ __forceinline__ void st_dt(void* p, long i, float v, int dt) {
  if (dt == HVIT_F32) ((float*)p)[i] = v;
  else ((bf16_t*)p)[i] = f2bf(v);
}

// ---------------------------------------------------------------- dropout RNG --
// Counter-based, 32-bit per element pair:
//   key       = fold32(splitmix64(seed ^ site << 48))     (once per launch: scalar unit)
//   h(pair)   = lowbias32(key ^ (uint32)(idx >> 1))       (2 multiplies per 2 elements)
//   u16(idx)  = (h >> 16 * (idx & 1)) & 0xffff
//   keep(idx) = u16(idx) >= thr,  thr = round(p * 65536)
// Forward and backward regenerate identical masks from (seed, site, index).  The
// pair counter is 32 bits, so a site's mask is unique over its first 2^33
// elements.  (Round 1 hashed a 64-bit splitmix per 4 elements: ~9 quarter-rate
// 32-bit multiplies per group, which made dropout the largest VALU cost of the
// attention and GEMM epilogues.)  Mirror: tests/conftest.py keep_mask.
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ inline uint32_t rng_key(uint64_t seed, uint32_t site) {
  const uint64_t m = mix64(seed ^ ((uint64_t)site << 48));
  return (uint32_t)(m ^ (m >> 32));
}
__device__ __forceinline__ uint32_t hash32(uint32_t x) {  // lowbias32 (Wellons)
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}
// hash of the pair holding element idx (both 16-bit halves)
__device__ __forceinline__ uint32_t rng_pair(uint32_t key, uint64_t idx) {
  return hash32(key ^ (uint32_t)(idx >> 1));
}
__device__ __forceinline__ float keep_lo(uint32_t h, uint32_t thr, float ds) { return (h & 0xffffu) >= thr ? ds : 0.f; }
__device__ __forceinline__ float keep_hi(uint32_t h, uint32_t thr, float ds) { return (h >> 16) >= thr ? ds : 0.f; }
__device__ __forceinline__ uint32_t rng_u16k(uint32_t key, uint64_t idx) {
  return (rng_pair(key, idx) >> (16 * (uint32_t)(idx & 1))) & 0xffffu;
}
__device__ __forceinline__ bool rng_keep(uint64_t seed, uint32_t site, uint64_t idx, uint32_t thr) {
  return rng_u16k(rng_key(seed, site), idx) >= thr;
}
// multipliers of 4 adjacent elements i0..i0+3 (i0 even): two pair hashes
__device__ __forceinline__ f32x4 keep4_at(uint32_t key, uint64_t i0, uint32_t thr, float ds) {
  const uint32_t h0 = rng_pair(key, i0), h1 = rng_pair(key, i0 + 2);
  return (f32x4){keep_lo(h0, thr, ds), keep_hi(h0, thr, ds), keep_lo(h1, thr, ds), keep_hi(h1, thr, ds)};
}
// Dropout seed as a kernel argument: the host value, XOR the 64-bit word at p
// when p is non-NULL (a device-resident seed the model advances once per
// training forward, so a captured hipGraph draws fresh masks on every replay).
// Resolved once at kernel entry (a scalar load).
struct DSeed {
  unsigned long long s;
  const unsigned long long* p;
  __device__ __forceinline__ operator unsigned long long() const { return p ? (s ^ *p) : s; }
};
static inline DSeed dseed(const hvit_dropout_t* d) {
  return d ? DSeed{d->seed, d->seed_ptr} : DSeed{0ull, nullptr};
}
static inline uint32_t drop_threshold(float p) {
  if (p <= 0.f) return 0;
  double t = (double)p * 65536.0 + 0.5;
  if (t > 65536.0) t = 65536.0;
  return (uint32_t)t;
}

// ----------------------------------------------------------------- GELU(erf) --
// GELU (erf form, as torch.nn.GELU()) without the branchy libm erff: erf by
// Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7), one rcp + one exp; the same
// exp(-x^2/2) also gives the Gaussian density for the derivative.
__device__ __forceinline__ float erf_gauss(float z, float& e) {  // e = exp(-z^2)
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * az);
  e = __expf(-az * az);
  const float poly =
      t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  return copysignf(1.f - poly * e, z);
}
__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return 0.5f * x * (1.f + erf_gauss(x * 0.70710678118654752f, e));
}
__device__ __forceinline__ float gelu_grad(float x) {
  float e;
  const float cdf = 0.5f * (1.f + erf_gauss(x * 0.70710678118654752f, e));
  return cdf + x * (0.39894228040143268f * e);
}
// GELU and its derivative from one erf / exp evaluation
struct GeluGG {
  float g, d;
};
__device__ __forceinline__ GeluGG gelu_gg(float x) {
  float e;
  const float cdf = 0.5f * (1.f + erf_gauss(x * 0.70710678118654752f, e));
  return {x * cdf, cdf + x * (0.39894228040143268f * e)};
}

// The same for 4 values, the arithmetic on packed f32 pairs (v_pk_fma_f32 /
// v_pk_mul_f32: two lanes' worth per issue; rcp / exp stay per element): the
// fc1 forward epilogue evaluates one per output, ~40 % fewer VALU issues than
// four gelu_gg calls.  Same operation sequence per element as gelu_gg.
__device__ __forceinline__ void gelu_gg4(const f32x4& v, f32x4& g, f32x4& d) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x2_t x = {v[2 * h], v[2 * h + 1]};
    const f32x2_t z = x * 0.70710678118654752f;
    const f32x2_t az = {fabsf(z.x), fabsf(z.y)};
    const f32x2_t den = 1.f + 0.3275911f * az;
    const f32x2_t t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
    const f32x2_t q = az * az;
    const f32x2_t e = {__expf(-q.x), __expf(-q.y)};
    const f32x2_t poly =
        t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
    const f32x2_t r = 1.f - poly * e;
    const f32x2_t er = {copysignf(r.x, z.x), copysignf(r.y, z.y)};
    const f32x2_t cdf = 0.5f * (1.f + er);
    const f32x2_t gg = x * cdf;
    const f32x2_t dd = cdf + x * (0.39894228040143268f * e);
    g[2 * h] = gg.x;
    g[2 * h + 1] = gg.y;
    d[2 * h] = dd.x;
    d[2 * h + 1] = dd.y;
  }
}

// ---------------------------------------------------------- wave reductions --
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// n / d for 0 <= n < 2^31 by a multiply-high instead of the ~25-instruction
// integer division sequence (index math in VALU-bound grid-stride loops):
// q = floor(n m / 2^(32+s)), m = ceil(2^(32+s) / d), s = ceil(log2 d).  Exact:
// m = 2^(32+s)/d + e, e < 1, adds n e / 2^(32+s) < 2^-(s+1) < 1/d to n/d.
struct FastDiv {
  uint32_t mlo = 0, mhi = 1;
  int s = 0;
  FastDiv() = default;
  explicit FastDiv(int d) {
    while ((1LL << s) < d) ++s;
    const unsigned __int128 one = 1;
    const unsigned long long m = (unsigned long long)(((one << (32 + s)) + (unsigned)d - 1) / (unsigned)d);
    mlo = (uint32_t)m;
    mhi = (uint32_t)(m >> 32);
  }
  __device__ __forceinline__ int div(int n) const {
    const uint32_t hi = __umulhi((uint32_t)n, mlo) + (mhi ? (uint32_t)n : 0u);
    return (int)(hi >> s);
  }
};

// A slab sum's per-granule form for many slabs (epi_side in gemm.h and
// sum_slabs_wave_kernel: one order for both): granule i (4 floats) of
// sum_k src[k * st + i] by one wave -- slabs k = lane, lane + 64, ... per lane,
// then a butterfly.  Result in every lane.
constexpr int SIDE_WAVE_SPLITS = 64;
__device__ __forceinline__ f32x4 side_wave_granule(const f32x4* src, long st, int splits, long i) {
  const int lane = threadIdx.x & 63;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (int k = lane; k < splits; k += 64) s += src[(long)k * st + i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) s[e] += __shfl_xor(s[e], o, 64);
  }
  return s;
}
