// Fused multi-head self-attention for gfx950 (MultiHeadSelfAttention,
// models/attention.py:65-115 of the reference).
//
// Layouts (no permute copies): qkv is the qkv-Linear output [B, N, 3, H, hd]
// (row pitch 3*D), o is [B, N, H, hd] (= the head-merged [B, N, D] the proj
// Linear consumes), lse is [B, H, N] f32 (natural-log units of scale*q.k).
//
// Forward: one workgroup = (b, h, 64 query rows), four waves x 16 rows.  K and
// V^T tiles of 64 keys are staged in LDS; S = Q K^T and O += P V run on MFMA
// (16x16x32 bf16 or 16x16x4 f32); softmax is online (running max / sum per row,
// 16-lane shuffle reductions), attention dropout is applied to P after the
// normaliser (softmax -> dropout, attention.py:101-102) with a counter-based
// mask regenerated bit-identically in the backward.  The N x N score matrix is
// never written to HBM (except by hvit_mhsa_probs for return_attentions).
//
// Backward (FlashAttention-2 style recompute from lse): a dQ kernel over query
// tiles and a dK/dV kernel over key tiles, both recomputing P; delta =
// rowsum(dO * O) is produced by a small pre-pass.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace hvit {

constexpr int AT_THREADS = 256;
constexpr int AT_TILE = 64;  // query rows per workgroup and keys per tile

template <typename T>
__device__ __forceinline__ f32x4 mma_step(u32x4 a, u32x4 b, f32x4 c) {
  if constexpr (sizeof(T) == 2) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, a),
                                                   __builtin_bit_cast(s16x8, b), c, 0, 0, 0);
  } else {
    f32x4 va = __builtin_bit_cast(f32x4, a), vb = __builtin_bit_cast(f32x4, b);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(va[0], vb[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(va[1], vb[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(va[2], vb[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(va[3], vb[3], c, 0, 0, 0);
    return c;
  }
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Geometry for a row of L elements of T in LDS: 16-byte chunks, MFMA steps.
template <typename T, int L>
struct RowGeo {
  static constexpr int CH = L * (int)sizeof(T) / 16;   // 16-byte chunks per row
  static constexpr int STEPS = (CH + 3) / 4;           // MFMA k-steps (4 chunks each)
  static constexpr int PITCH = L * (int)sizeof(T) + 16;
};

// read fragment (row r, step s) of an LDS image with RowGeo G
template <class G>
__device__ __forceinline__ u32x4 frag(const char* base, int r, int s, int fq) {
  int ch = 4 * s + fq;
  if (ch < G::CH) return *(const u32x4*)(base + r * G::PITCH + ch * 16);
  return (u32x4){0u, 0u, 0u, 0u};
}

// stage rows [row0, row0+64) x HD of a strided global matrix into LDS (k-contig)
template <typename T, int HD>
__device__ __forceinline__ void stage_rows(char* dst, const T* src, long pitch, int row0, int nrows) {
  using G = RowGeo<T, HD>;
  for (int ch = threadIdx.x; ch < AT_TILE * G::CH; ch += AT_THREADS) {
    int r = ch / G::CH, c = ch % G::CH;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (row0 + r < nrows) v = *(const u32x4*)(src + (long)(row0 + r) * pitch + c * (16 / sizeof(T)));
    *(u32x4*)(dst + r * G::PITCH + c * 16) = v;
  }
}
// stage the transpose: dst[d][r] = src[row0 + r][d]   (rows of 64 elements)
template <typename T, int HD>
__device__ __forceinline__ void stage_rows_t(char* dst, const T* src, long pitch, int row0, int nrows) {
  using GS = RowGeo<T, HD>;
  using GT = RowGeo<T, AT_TILE>;
  constexpr int E = 16 / sizeof(T);
  for (int ch = threadIdx.x; ch < AT_TILE * GS::CH; ch += AT_THREADS) {
    int r = ch % AT_TILE, c = ch / AT_TILE;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (row0 + r < nrows) v = *(const u32x4*)(src + (long)(row0 + r) * pitch + c * E);
    const T* e = (const T*)&v;
#pragma unroll
    for (int q = 0; q < E; ++q) *(T*)(dst + (c * E + q) * GT::PITCH + r * sizeof(T)) = e[q];
  }
}

// ---------------------------------------------------------------- forward ---
template <typename T, int HD>
__global__ __launch_bounds__(AT_THREADS) void mhsa_fwd_kernel(const T* __restrict__ qkv, T* __restrict__ o,
                                                             float* __restrict__ lse, int B, int N,
                                                             int H, float scale, uint32_t thr,
                                                             float dscale, DSeed seed_,
                                                             uint32_t site) {
  const unsigned long long seed = seed_;
  using GH = RowGeo<T, HD>;        // rows of hd elements
  using GK = RowGeo<T, AT_TILE>;   // rows of 64 keys
  constexpr int NT = HD / 16;      // output 16-col blocks
  __shared__ __attribute__((aligned(16))) char smem[AT_TILE * GH::PITCH + HD * GK::PITCH + 4 * 16 * GK::PITCH];
  char* Ks = smem;
  char* Vt = Ks + AT_TILE * GH::PITCH;
  char* Ps = Vt + HD * GK::PITCH;

  const int D = H * HD;
  const long pitch = 3L * D;
  const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  char* Pw = Ps + w * 16 * GK::PITCH;
  const T* base = qkv + (long)b * N * pitch;
  const T* qp = base + h * HD;
  const T* kp = base + D + h * HD;
  const T* vp = base + 2 * D + h * HD;

  // Q fragments in registers: row q0 + frow
  const int q0 = qt * AT_TILE + w * 16;
  u32x4 qf[GH::STEPS];
#pragma unroll
  for (int s = 0; s < GH::STEPS; ++s) {
    int ch = 4 * s + fq;
    qf[s] = (u32x4){0u, 0u, 0u, 0u};
    if (ch < GH::CH && q0 + frow < N) qf[s] = *(const u32x4*)(qp + (long)(q0 + frow) * pitch + ch * (16 / sizeof(T)));
  }
  const float c2 = scale * 1.4426950408889634f;  // log2(e)
  float mrow[4], lrow[4];
  f32x4 oacc[NT];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mrow[r] = -INFINITY; lrow[r] = 0.f; }
#pragma unroll
  for (int t = 0; t < NT; ++t) oacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const uint64_t bh = (uint64_t)b * H + h;
  for (int k0 = 0; k0 < N; k0 += AT_TILE) {
    __syncthreads();
    stage_rows<T, HD>(Ks, kp, pitch, k0, N);
    stage_rows_t<T, HD>(Vt, vp, pitch, k0, N);
    __syncthreads();
    // S = Q K^T  (16 rows x 64 keys per wave)
    f32x4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < GH::STEPS; ++st) s[j] = mma_step<T>(qf[st], frag<GH>(Ks, 16 * j + frow, st, fq), s[j]);
    }
    // online softmax; lane holds rows 4fq+r, keys 16j+frow
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = (k0 + 16 * j + frow < N) ? s[j][r] * c2 : -INFINITY;
        s[j][r] = v;
        mx = fmaxf(mx, v);
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
      float mn = fmaxf(mrow[r], mx);
      alpha[r] = __builtin_amdgcn_exp2f(mrow[r] - mn);
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float p = __builtin_amdgcn_exp2f(s[j][r] - mn);
        sum += p;
        s[j][r] = p;
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) sum += __shfl_xor(sum, o2, 64);
      lrow[r] = lrow[r] * alpha[r] + sum;
      mrow[r] = mn;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) oacc[t][r] *= alpha[r];
    // dropout on P, write P to this wave's LDS image [16 rows][64 keys]
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = s[j][r];
        if (thr) {
          int qi = q0 + 4 * fq + r, kj = k0 + 16 * j + frow;
          uint64_t idx = (bh * N + qi) * (uint64_t)N + kj;
          p = rng_keep(seed, site, idx, thr) ? p * dscale : 0.f;
        }
        *(T*)(Pw + (4 * fq + r) * GK::PITCH + (16 * j + frow) * sizeof(T)) = Elem<T>::from_f(p);
      }
    lds_fence();
    // O += P V   (A = P[16][64 keys], B = V^T rows = hd)
#pragma unroll
    for (int st = 0; st < GK::STEPS; ++st) {
      u32x4 pa = frag<GK>(Pw, frow, st, fq);
#pragma unroll
      for (int t = 0; t < NT; ++t) oacc[t] = mma_step<T>(pa, frag<GK>(Vt, 16 * t + frow, st, fq), oacc[t]);
    }
    lds_fence();
  }
  // finalize
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int qi = q0 + 4 * fq + r;
    if (qi >= N) continue;
    float inv = 1.f / lrow[r];
#pragma unroll
    for (int t = 0; t < NT; ++t)
      o[((long)b * N + qi) * D + h * HD + 16 * t + frow] = Elem<T>::from_f(oacc[t][r] * inv);
    if (frow == 0) lse[bh * N + qi] = (mrow[r] + log2f(lrow[r])) * 0.6931471805599453f;
  }
}

// ---------------------------------------------------------- delta pre-pass ---
// delta[b,h,n] = sum_d dO[b,n,h,d] * O[b,n,h,d]
template <typename T, int HD>
__global__ void mhsa_delta_kernel(const T* __restrict__ o, const T* __restrict__ dout, float* __restrict__ delta,
                                  int B, int N, int H) {
  long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // (b, n, h)
  int lane = threadIdx.x & 63;
  long total = (long)B * N * H;
  if (row >= total) return;
  float s = 0.f;
  for (int d = lane; d < HD; d += 64) s += Elem<T>::to_f(o[row * HD + d]) * Elem<T>::to_f(dout[row * HD + d]);
  s = wave_sum(s);
  if (lane == 0) {
    int h = row % H;
    long bn = row / H;
    int n = bn % N;
    int b = bn / N;
    delta[((long)b * H + h) * N + n] = s;
  }
}

// --------------------------------------------------------------- dQ kernel ---
// also serves return_attentions (PROBS): writes dropout(softmax) to probs.
template <typename T, int HD, bool PROBS>
__global__ __launch_bounds__(AT_THREADS) void mhsa_dq_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ delta,
                                                            T* __restrict__ dqkv, float* __restrict__ probs,
                                                            int B, int N, int H, float scale, uint32_t thr,
                                                            float dscale, DSeed seed_, uint32_t site) {
  const unsigned long long seed = seed_;
  using GH = RowGeo<T, HD>;
  using GK = RowGeo<T, AT_TILE>;
  constexpr int NT = HD / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * AT_TILE * GH::PITCH + HD * GK::PITCH + 4 * 16 * GK::PITCH];
  char* Ks = smem;
  char* Vs = Ks + AT_TILE * GH::PITCH;
  char* Kt = Vs + AT_TILE * GH::PITCH;
  char* Ps = Kt + HD * GK::PITCH;

  const int D = H * HD;
  const long pitch = 3L * D;
  const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  char* Pw = Ps + w * 16 * GK::PITCH;
  const T* base = qkv + (long)b * N * pitch;
  const T* qp = base + h * HD;
  const T* kp = base + D + h * HD;
  const T* vp = base + 2 * D + h * HD;
  const T* dop = dout + (long)b * N * D + h * HD;
  const uint64_t bh = (uint64_t)b * H + h;

  const int q0 = qt * AT_TILE + w * 16;
  u32x4 qf[GH::STEPS], df[GH::STEPS];
#pragma unroll
  for (int s = 0; s < GH::STEPS; ++s) {
    int ch = 4 * s + fq;
    qf[s] = df[s] = (u32x4){0u, 0u, 0u, 0u};
    if (ch < GH::CH && q0 + frow < N) {
      qf[s] = *(const u32x4*)(qp + (long)(q0 + frow) * pitch + ch * (16 / sizeof(T)));
      if (!PROBS) df[s] = *(const u32x4*)(dop + (long)(q0 + frow) * D + ch * (16 / sizeof(T)));
    }
  }
  const float c2 = scale * 1.4426950408889634f;
  float lse2[4], dl[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int qi = q0 + 4 * fq + r;
    lse2[r] = qi < N ? lse[bh * N + qi] * 1.4426950408889634f : 0.f;
    dl[r] = (!PROBS && qi < N) ? delta[bh * N + qi] : 0.f;
  }
  f32x4 dq[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) dq[t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < N; k0 += AT_TILE) {
    __syncthreads();
    stage_rows<T, HD>(Ks, kp, pitch, k0, N);
    if (!PROBS) {
      stage_rows<T, HD>(Vs, vp, pitch, k0, N);
      stage_rows_t<T, HD>(Kt, kp, pitch, k0, N);
    }
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = dp[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < GH::STEPS; ++st) {
        s[j] = mma_step<T>(qf[st], frag<GH>(Ks, 16 * j + frow, st, fq), s[j]);
        if (!PROBS) dp[j] = mma_step<T>(df[st], frag<GH>(Vs, 16 * j + frow, st, fq), dp[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int qi = q0 + 4 * fq + r, kj = k0 + 16 * j + frow;
        bool valid = qi < N && kj < N;
        float p = valid ? __builtin_amdgcn_exp2f(s[j][r] * c2 - lse2[r]) : 0.f;
        bool keep = true;
        if (thr && valid) keep = rng_keep(seed, site, (bh * N + qi) * (uint64_t)N + kj, thr);
        if (PROBS) {
          if (valid) probs[(bh * N + qi) * (long)N + kj] = keep ? p * dscale : 0.f;
        } else {
          float g = thr ? (keep ? dp[j][r] * dscale : 0.f) : dp[j][r];
          float ds = p * (g - dl[r]);
          *(T*)(Pw + (4 * fq + r) * GK::PITCH + (16 * j + frow) * sizeof(T)) = Elem<T>::from_f(ds);
        }
      }
    if (PROBS) continue;
    lds_fence();
#pragma unroll
    for (int st = 0; st < GK::STEPS; ++st) {
      u32x4 pa = frag<GK>(Pw, frow, st, fq);
#pragma unroll
      for (int t = 0; t < NT; ++t) dq[t] = mma_step<T>(pa, frag<GK>(Kt, 16 * t + frow, st, fq), dq[t]);
    }
    lds_fence();
  }
  if (PROBS) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int qi = q0 + 4 * fq + r;
    if (qi >= N) continue;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      dqkv[((long)b * N + qi) * pitch + h * HD + 16 * t + frow] = Elem<T>::from_f(dq[t][r] * scale);
  }
}

// -------------------------------------------------------------- dK/dV kernel ---
template <typename T, int HD>
__global__ __launch_bounds__(AT_THREADS) void mhsa_dkv_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ delta,
                                                             T* __restrict__ dqkv, int B, int N, int H,
                                                             float scale, uint32_t thr, float dscale,
                                                             DSeed seed_, uint32_t site) {
  const unsigned long long seed = seed_;
  using GH = RowGeo<T, HD>;
  using GK = RowGeo<T, AT_TILE>;
  constexpr int NT = HD / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * AT_TILE * GH::PITCH + 2 * HD * GK::PITCH +
                                                    4 * 16 * GK::PITCH + 2 * AT_TILE * 4];
  char* Qs = smem;
  char* Ds = Qs + AT_TILE * GH::PITCH;
  char* Qt = Ds + AT_TILE * GH::PITCH;
  char* Dt = Qt + HD * GK::PITCH;
  char* Ps = Dt + HD * GK::PITCH;
  float* Ls = (float*)(Ps + 4 * 16 * GK::PITCH);
  float* Dl = Ls + AT_TILE;

  const int D = H * HD;
  const long pitch = 3L * D;
  const int kt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  char* Pw = Ps + w * 16 * GK::PITCH;
  const T* base = qkv + (long)b * N * pitch;
  const T* qp = base + h * HD;
  const T* kp = base + D + h * HD;
  const T* vp = base + 2 * D + h * HD;
  const T* dop = dout + (long)b * N * D + h * HD;
  const uint64_t bh = (uint64_t)b * H + h;

  const int key0 = kt * AT_TILE + w * 16;
  u32x4 kf[GH::STEPS], vf[GH::STEPS];
#pragma unroll
  for (int s = 0; s < GH::STEPS; ++s) {
    int ch = 4 * s + fq;
    kf[s] = vf[s] = (u32x4){0u, 0u, 0u, 0u};
    if (ch < GH::CH && key0 + frow < N) {
      kf[s] = *(const u32x4*)(kp + (long)(key0 + frow) * pitch + ch * (16 / sizeof(T)));
      vf[s] = *(const u32x4*)(vp + (long)(key0 + frow) * pitch + ch * (16 / sizeof(T)));
    }
  }
  const float c2 = scale * 1.4426950408889634f;
  f32x4 dk[NT], dv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) dk[t] = dv[t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int q0 = 0; q0 < N; q0 += AT_TILE) {
    __syncthreads();
    stage_rows<T, HD>(Qs, qp, pitch, q0, N);
    stage_rows<T, HD>(Ds, dop, D, q0, N);
    stage_rows_t<T, HD>(Qt, qp, pitch, q0, N);
    stage_rows_t<T, HD>(Dt, dop, D, q0, N);
    for (int i = threadIdx.x; i < AT_TILE; i += AT_THREADS) {
      int qi = q0 + i;
      Ls[i] = qi < N ? lse[bh * N + qi] * 1.4426950408889634f : 0.f;
      Dl[i] = qi < N ? delta[bh * N + qi] : 0.f;
    }
    __syncthreads();
    // S^T = K Q^T and dP~^T = V dO^T : lane holds keys 4fq+r, queries 16j+frow
    f32x4 s[4], dp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = dp[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < GH::STEPS; ++st) {
        s[j] = mma_step<T>(kf[st], frag<GH>(Qs, 16 * j + frow, st, fq), s[j]);
        dp[j] = mma_step<T>(vf[st], frag<GH>(Ds, 16 * j + frow, st, fq), dp[j]);
      }
    }
    // P~^T -> Pw ; dS^T kept in s[]
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int qi = q0 + 16 * j + frow;
      float l2 = Ls[16 * j + frow], dlt = Dl[16 * j + frow];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int kj = key0 + 4 * fq + r;
        bool valid = qi < N && kj < N;
        float p = valid ? __builtin_amdgcn_exp2f(s[j][r] * c2 - l2) : 0.f;
        bool keep = true;
        if (thr && valid) keep = rng_keep(seed, site, (bh * N + qi) * (uint64_t)N + kj, thr);
        float pd = thr ? (keep ? p * dscale : 0.f) : p;
        float g = thr ? (keep ? dp[j][r] * dscale : 0.f) : dp[j][r];
        s[j][r] = p * (g - dlt);
        *(T*)(Pw + (4 * fq + r) * GK::PITCH + (16 * j + frow) * sizeof(T)) = Elem<T>::from_f(pd);
      }
    }
    lds_fence();
    // dV += P~^T dO
#pragma unroll
    for (int st = 0; st < GK::STEPS; ++st) {
      u32x4 pa = frag<GK>(Pw, frow, st, fq);
#pragma unroll
      for (int t = 0; t < NT; ++t) dv[t] = mma_step<T>(pa, frag<GK>(Dt, 16 * t + frow, st, fq), dv[t]);
    }
    lds_fence();
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *(T*)(Pw + (4 * fq + r) * GK::PITCH + (16 * j + frow) * sizeof(T)) = Elem<T>::from_f(s[j][r]);
    lds_fence();
    // dK += dS^T Q
#pragma unroll
    for (int st = 0; st < GK::STEPS; ++st) {
      u32x4 pa = frag<GK>(Pw, frow, st, fq);
#pragma unroll
      for (int t = 0; t < NT; ++t) dk[t] = mma_step<T>(pa, frag<GK>(Qt, 16 * t + frow, st, fq), dk[t]);
    }
    lds_fence();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int kj = key0 + 4 * fq + r;
    if (kj >= N) continue;
    T* row = dqkv + ((long)b * N + kj) * pitch + h * HD;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      row[D + 16 * t + frow] = Elem<T>::from_f(dk[t][r] * scale);
      row[2 * D + 16 * t + frow] = Elem<T>::from_f(dv[t][r]);
    }
  }
}

// ============================================================================
// v2 fast path: bf16, head_dim 64, N <= 256 keys (the HybridViT shapes).
//
// The whole K and V (or Q and dO) of one (b, h) live in LDS as row-major
// [row][64] bf16 images (128-B rows, 16-B chunks XOR-swizzled by row & 7), so
// every tile is staged once per workgroup with plain 16-byte copies -- no
// transposed staging.  Scores are computed TRANSPOSED (S^T = K Q^T): the
// 16x16 MFMA accumulator then holds, per lane, 4 consecutive keys of one
// query, which is exactly the B-operand layout of v_mfma_f32_16x16x16_bf16,
// so P^T (and dS^T) feed the next MFMA straight from registers; the other
// operand (V^T, K^T, dO^T, Q^T) is read with ds_read_b64_tr_b16.  A lane's 4
// keys also form one dropout-hash group (one 64-bit hash per 16x16 tile).
// ============================================================================
constexpr int V2_KMAX = 512;  // the largest token count of the register-resident kernels
constexpr int V2_ROWB = 128;  // bytes per 64-element bf16 row
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

__device__ __forceinline__ int v2_off(int row, int chunk) { return row * V2_ROWB + ((chunk ^ (row & 7)) << 4); }

// Same image filled by LDS-DMA (global_load_lds_dwordx4): no registers, no
// per-chunk load->store latency chain.  One wave-instruction writes 1 KiB =
// 8 rows; the destination is lane-linear, so the XOR swizzle moves to the
// source address (lane L fetches logical chunk (L%8) ^ row&7 of row 8p + L/8).
// Rows >= n re-read row n-1 (finite data; every use of those rows is masked or
// multiplied by an exact zero).  `rows` is a multiple of 8.
template <int WAVES>
__device__ __forceinline__ void v2_stage_glds(char* dst, const bf16_t* src, long pitch, int n, int rows) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rl = lane >> 3, cp = lane & 7;
  for (int pc = w; pc < (rows >> 3); pc += WAVES) {
    const int row = pc * 8 + rl;
    const int srow = row < n ? row : n - 1;
    const bf16_t* g = src + (long)srow * pitch + ((cp ^ rl) << 3);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16, 0, 0);
  }
}
// 16x16x32 operand fragment: row `row`, k = 32*s + 8*fq .. +7
__device__ __forceinline__ u32x4 v2_frag(const char* img, int row, int s, int fq) {
  return *(const u32x4*)(img + v2_off(row, 4 * s + fq));
}
// transposed 4-row read: lane (g = lane>>4, i = lane&15) receives
// img[k0 + 4g + 0..3][c0 + i]  (k0 multiple of 16, c0 multiple of 16)
__device__ __forceinline__ v4s_t v2_tr(const char* img, int k0, int c0, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int row = k0 + 4 * g + (li >> 2);
  const int col = c0 + 4 * (li & 3);
  const char* a = img + row * V2_ROWB + (((col >> 3) ^ (row & 7)) << 4) + (col & 7) * 2;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)a);
}
// Per-lane constant parts of the two read patterns (row = 16*j + lane part,
// and row & 7 depends on the lane part only), so a tile read is one LDS
// instruction at base + 2048*j + const.
struct V2Lane {
  int kc[2];  // v2_frag offsets for s = 0, 1 (row = frow)
  int tr[4];  // v2_tr offsets for column block t = 0..3 (rows 4g + li/4)
  __device__ __forceinline__ V2Lane(int lane) {
    const int frow = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) kc[s2] = frow * V2_ROWB + (((4 * s2 + fq) ^ (frow & 7)) << 4);
    const int r0 = 4 * fq + (frow >> 2), cb = (frow & 3) >> 1, inner = (frow & 1) * 8;
#pragma unroll
    for (int t = 0; t < 4; ++t) tr[t] = r0 * V2_ROWB + (((2 * t + cb) ^ (r0 & 7)) << 4) + inner;
  }
};
__device__ __forceinline__ u32x4 v2_fragj(const char* img, const V2Lane& L, int j, int s2) {
  return *(const u32x4*)(img + j * 16 * V2_ROWB + L.kc[s2]);
}
__device__ __forceinline__ v4s_t v2_trj(const char* img, const V2Lane& L, int j, int t) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(img + j * 16 * V2_ROWB + L.tr[t]));
}
__device__ __forceinline__ f32x4 v2_mma32(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, a), __builtin_bit_cast(s16x8, b), c, 0,
                                                 0, 0);
}
// Score tile straight from its MFMAs into a branch (the partial-tile mask):
// hipcc pads the MFMA -> VALU-read distance on the fall-through edge but not
// on the taken one (1-3 wait states in the .s where an 8-pass XDL result needs
// 11), so the wait goes inside a statement that takes the tile as an operand.
__device__ __forceinline__ void v2_settle(f32x4& a) { asm volatile("s_nop 7\n\ts_nop 3" : "+v"(a)); }
// 16x16x32 operand from two transposed 4-row reads (tiles jj and jj + 1):
// k = 8g + e  <->  row 16*(jj + e/4) + 4g + e%4
__device__ __forceinline__ u32x4 v2_cat(v4s_t lo, v4s_t hi) {
  const uint2 a = __builtin_bit_cast(uint2, lo), b = __builtin_bit_cast(uint2, hi);
  return (u32x4){a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ u32x4 v2_trj2(const char* img, const V2Lane& L, int jj, int t) {
  return v2_cat(v2_trj(img, L, jj, t), v2_trj(img, L, jj + 1, t));
}
__device__ __forceinline__ v4s_t v2_pack(f32x4 v) {
  uint2 u;
  u.x = f2bf2(v[0], v[1]);
  u.y = f2bf2(v[2], v[3]);
  return __builtin_bit_cast(v4s_t, u);
}
// dropout multipliers of 4 consecutive keys kj..kj+3 (kj % 4 == 0) of query qi
__device__ __forceinline__ f32x4 v2_keep(uint64_t bh, int N, int qi, int kj, uint32_t thr, float dscale,
                                         unsigned long long seed, uint32_t site) {
  const uint64_t idx = (bh * N + qi) * (uint64_t)N + kj;
  return keep4_at(rng_key(seed, site), idx, thr, dscale);
}

// forward: workgroup = (b, h, 16*WAVES queries); wave = 16 queries x all keys.
// WAVES = 16 covers all N <= 256 queries of a (b, h) in one workgroup, so K
// and V are staged into LDS once per (b, h) instead of once per 64 queries.
// KMAX = 512 (256 < N <= 512, a 4-8 s clip's token count): K and V of all keys
// in LDS (128 KiB) and the keys taken in chunks of 256 with an online softmax
// (running max and sum, the output rescaled when the max grows); for N <= 256
// the one chunk gives exactly the single-pass arithmetic.  The KMAX = 512 form
// runs 8-wave workgroups (at 16 waves the 128-VGPR budget spilled).
// FULL: N == KMAX == 256 (the model's 16x16 token grid), every key tile whole
// and every query in range: no partial-tile masks or tile-count tests.
template <int WAVES, int KMAX, bool FULL = false>
__global__ __launch_bounds__(WAVES * 64) void mhsa_fwd_v2(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o,
                                                         float* __restrict__ lse, int N, int H, float scale,
                                                         uint32_t thr, float dscale, DSeed seed_,
                                                         uint32_t site, uint32_t* __restrict__ kbits) {
  const unsigned long long seed = seed_;
  constexpr int CH = 256;  // keys per softmax chunk (the register-resident score block)
  __shared__ __attribute__((aligned(16))) char smem[2 * KMAX * V2_ROWB];
  char* Ks = smem;
  char* Vs = smem + KMAX * V2_ROWB;
  const int D = H * 64;
  const long pitch = 3L * D;
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  const V2Lane LN(lane);
  const bf16_t* base = qkv + (long)b * N * pitch + h * 64;
  const int NK32 = (N + 31) & ~31;  // staged rows: whole tile pairs
  const int q = blockIdx.x * WAVES * 16 + w * 16 + frow;  // this lane's query
  const bool qin = FULL || q < N;
  u32x4 qf[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    qf[s2] = qin ? *(const u32x4*)(base + (long)q * pitch + 32 * s2 + 8 * fq) : (u32x4){0u, 0u, 0u, 0u};
  v2_stage_glds<WAVES>(Ks, base + D, pitch, N, NK32);
  v2_stage_glds<WAVES>(Vs, base + 2 * D, pitch, N, NK32);
  __syncthreads();
  const float c2 = scale * 1.4426950408889634f;
  const uint64_t bh = (uint64_t)b * H + h;
  const uint64_t BHN = (uint64_t)gridDim.z * H * N;  // keep-bit chunk stride (queries)
  const uint32_t rk = rng_key(seed, site);
  const uint64_t qrow = (bh * N + (qin ? q : 0)) * (uint64_t)N;
  const uint32_t hq = (uint32_t)(qrow >> 1) + 2u * (uint32_t)fq;  // dropout-hash pair index of key 0
  // O^T[d][q] += V^T[d][keys] P^T[keys][q]   (4 d-blocks of 16)
  f32x4 ot[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) ot[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float mxc = -INFINITY, sum = 0.f;
  // one 256-key chunk (C0 = 0 or 256, compile time): its scores, the online
  // softmax update, P V; its keep bits
  auto chunk = [&](auto c0c) {
    constexpr int c0 = decltype(c0c)::value;
    const int nkt = FULL ? CH / 16 : (min(N - c0, CH) + 15) >> 4;  // key tiles of this chunk
    const char* Kc = Ks + c0 * V2_ROWB;
    const char* Vc = Vs + c0 * V2_ROWB;
    // S^T tiles: st[j][r] = raw score(key c0 + 16j + 4fq + r, query q)
    // (keys >= N of the last, partial tile masked to -inf).  VALU diet: the 1/sum
    // and the dropout 1/(1-p) on the 16 outputs instead of the 64
    // probabilities, the dropout mask a select, masking only in a partial tile.
    f32x4 st[CH / 16];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < CH / 16; ++j) {
      if (j < nkt) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        a = v2_mma32(v2_fragj(Kc, LN, j, 0), qf[0], a);
        a = v2_mma32(v2_fragj(Kc, LN, j, 1), qf[1], a);
        v2_settle(a);
        if (!FULL && c0 + 16 * j + 16 > N) {  // wave-uniform: only a partial last tile
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (c0 + 16 * j + 4 * fq + r >= N) a[r] = -INFINITY;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, a[r]);
        st[j] = a;
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    // raw scores kept; the scale folds into the exponent's fma (c2 > 0, so the
    // max commutes with it).  (Round 3 measured this form run-to-run
    // nondeterministic at the bf16-ulp level and scaled every score first: that
    // was the missing MFMA -> VALU wait of v2_settle, not the fma.)
    const float mnew = fmaxf(mxc, mx * c2);  // the running max in log2 units
    if constexpr (c0 > 0) {  // online softmax: rescale what the earlier chunks accumulated
      const float rs = __builtin_amdgcn_exp2f(mxc - mnew);
      sum *= rs;
#pragma unroll
      for (int t = 0; t < 4; ++t) ot[t] *= rs;
    }
    mxc = mnew;
    float csum = 0.f;
#pragma unroll
    for (int j = 0; j < CH / 16; ++j) {
      if (j < nkt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = __builtin_amdgcn_exp2f(fmaf(st[j][r], c2, -mxc));
          st[j][r] = pv;
          csum += pv;
        }
      }
    }
    csum += __shfl_xor(csum, 16, 64);
    csum += __shfl_xor(csum, 32, 64);
    sum += csum;
    // two key tiles per 16x16x32 MFMA: the B operand is this lane's P of tiles
    // 2jp, 2jp + 1 (keys c0 + 16(2jp + e/4) + 4fq + e%4), the A operand the
    // matching transposed reads of V.  A missing odd tile is P = 0 against
    // staged (finite) V rows.
    // keep bits for the backward (kbits non-null): bit 8*jp + 4*e + r of this
    // lane's word pair of chunk c0/256 = keep(q, key c0 + 32*jp + 16*e + 4*fq + r)
    uint32_t kb[2] = {0u, 0u};
#pragma unroll
    for (int jp = 0; jp < CH / 32; ++jp) {
      if (2 * jp < nkt) {
        f32x4 p0 = st[2 * jp];
        f32x4 p1 = (2 * jp + 1 < nkt) ? st[2 * jp + 1] : (f32x4){0.f, 0.f, 0.f, 0.f};
        if (thr) {
          uint32_t b8 = 0u;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            if (2 * jp + e < nkt) {
              // rng_pair(rk, qrow + c0 + 32jp + 16e + 4fq) and (.. + 2) in 32 bits:
              // qrow and the offset are even, so (qrow + off) >> 1 = qrow / 2 + off / 2
              const uint32_t x0 = hq + (uint32_t)(c0 / 2 + 16 * jp + 8 * e);
              const uint32_t h0 = hash32(rk ^ x0), h1 = hash32(rk ^ (x0 + 1u));
              const bool k0 = (h0 & 0xffffu) >= thr, k1 = (h0 >> 16) >= thr;
              const bool k2 = (h1 & 0xffffu) >= thr, k3 = (h1 >> 16) >= thr;
              f32x4& pp = e ? p1 : p0;
              pp[0] = k0 ? pp[0] : 0.f;
              pp[1] = k1 ? pp[1] : 0.f;
              pp[2] = k2 ? pp[2] : 0.f;
              pp[3] = k3 ? pp[3] : 0.f;
              b8 |= ((uint32_t)k0 | ((uint32_t)k1 << 1) | ((uint32_t)k2 << 2) | ((uint32_t)k3 << 3)) << (4 * e);
            }
          }
          kb[jp >> 2] |= b8 << (8 * (jp & 3));
        }
        const u32x4 pb = v2_cat(v2_pack(p0), v2_pack(p1));
#pragma unroll
        for (int t = 0; t < 4; ++t) ot[t] = v2_mma32(v2_trj2(Vc, LN, 2 * jp, t), pb, ot[t]);
      }
    }
    if (qin && kbits && thr)
      *(uint2*)(kbits + (((uint64_t)(c0 / CH) * BHN + bh * N + q) * 4 + fq) * 2) = make_uint2(kb[0], kb[1]);
  };
  chunk(std::integral_constant<int, 0>());
  if constexpr (KMAX > CH) {
    if (N > CH) chunk(std::integral_constant<int, CH>());
  }
  if (qin) {
    const float inv = 1.f / sum;
    const float os = thr ? inv * dscale : inv;
    bf16_t* op = o + ((long)b * N + q) * D + h * 64;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uint2 u;
      u.x = f2bf2(ot[t][0] * os, ot[t][1] * os);
      u.y = f2bf2(ot[t][2] * os, ot[t][3] * os);
      *(uint2*)(op + 16 * t + 4 * fq) = u;
    }
    if (fq == 0) lse[bh * N + q] = (mxc + log2f(sum)) * 0.6931471805599453f;
  }
}

// Column sums over a workgroup's rows of one head's [rows][64] gradient block
// held as acc[t][r] (column d = 16t + 4fq + r, row = the lane's query / key):
// the 16 lanes of a quarter (frow) by xor shuffles, the waves through LDS `red`
// ([WAVES][64] f32), then one plain store per column into out[0..63] (this
// workgroup's partial of the qkv bias gradient, attention.py:55; a later pass
// sums the partials: 32 workgroups adding to one address serialised at L2
// and cost more than the reduction pass they replaced).
template <int WAVES>
__device__ __forceinline__ void v2_colsum64(const f32x4 (&acc)[4], float mul, float* red, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int frow = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // the 16 rows of a quarter are one DPP row: rotate-and-add (row_ror 8,
      // 4, 2, 1) leaves the row sum in every lane, on the VALU (no LDS
      // permutes)
      float v = acc[t][r] * mul;
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
      if (frow == 0) red[w * 64 + 16 * t + 4 * fq + r] = v;
    }
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) s += red[i * 64 + threadIdx.x];
    out[threadIdx.x] = s;
  }
}

// dQ (+ delta = rowsum(dO * O), written for the dK/dV kernel):
// workgroup = (b, h, 16*WAVES queries); K, V images of all keys in LDS
// (KMAX = 512: 128 KiB; the forward's keep bits come in 256-key chunks)
template <int WAVES, int KMAX>
__global__ __launch_bounds__(WAVES * 64) void mhsa_dq_v2(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                        const bf16_t* __restrict__ dout,
                                                        const float* __restrict__ lse, float* __restrict__ delta,
                                                        bf16_t* __restrict__ dqkv, int N, int H, float scale,
                                                        uint32_t thr, float dscale, DSeed seed_,
                                                        uint32_t site, const uint32_t* __restrict__ kbits,
                                                        float* __restrict__ dbias) {
  const unsigned long long seed = seed_;
  __shared__ __attribute__((aligned(16))) char smem[2 * KMAX * V2_ROWB + WAVES * 64 * 4];
  char* Ks = smem;
  char* Vs = smem + KMAX * V2_ROWB;
  const int D = H * 64;
  const long pitch = 3L * D;
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  const V2Lane LN(lane);
  const bf16_t* base = qkv + (long)b * N * pitch + h * 64;
  const int NK = (N + 15) & ~15;
  const int nkt = NK >> 4;
  const int q = blockIdx.x * WAVES * 16 + w * 16 + frow;
  const bool qv = q < N;
  const uint64_t bh = (uint64_t)b * H + h;
  u32x4 qf[2], df[2];
  float dl = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    qf[s2] = df[s2] = (u32x4){0u, 0u, 0u, 0u};
    if (qv) {
      qf[s2] = *(const u32x4*)(base + (long)q * pitch + 32 * s2 + 8 * fq);
      df[s2] = *(const u32x4*)(dout + ((long)b * N + q) * D + h * 64 + 32 * s2 + 8 * fq);
      const u32x4 of = *(const u32x4*)(o + ((long)b * N + q) * D + h * 64 + 32 * s2 + 8 * fq);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        dl += __uint_as_float(df[s2][e] << 16) * __uint_as_float(of[e] << 16) +
              __uint_as_float(df[s2][e] & 0xffff0000u) * __uint_as_float(of[e] & 0xffff0000u);
    }
  }
  dl += __shfl_xor(dl, 16, 64);
  dl += __shfl_xor(dl, 32, 64);
  if (qv && fq == 0) delta[bh * N + q] = dl;
  const float lse2 = qv ? lse[bh * N + q] * 1.4426950408889634f : 0.f;
  // the forward's keep bits of this lane's (query, key quad) positions (mhsa_fwd_v2),
  // one 64-bit word per 256-key chunk
  unsigned long long kb64[KMAX / 256];
#pragma unroll
  for (int c = 0; c < KMAX / 256; ++c) {
    kb64[c] = 0ull;
    if (kbits && thr && qv && 256 * c < N) {
      const uint64_t BHN = (uint64_t)gridDim.z * H * N;
      const uint2 w2 = *(const uint2*)(kbits + (((uint64_t)c * BHN + bh * N + q) * 4 + fq) * 2);
      kb64[c] = (unsigned long long)w2.x | ((unsigned long long)w2.y << 32);
    }
  }
  const int NK32 = (N + 31) & ~31;  // staged rows: whole tile pairs (rows >= N finite, P = 0)
  v2_stage_glds<WAVES>(Ks, base + D, pitch, N, NK32);
  v2_stage_glds<WAVES>(Vs, base + 2 * D, pitch, N, NK32);
  __syncthreads();
  const float c2 = scale * 1.4426950408889634f;
  f32x4 dq[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dq[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // dQ^T[d][q] += K^T[d][keys] dS^T[keys][q]: two key tiles per 16x16x32 MFMA
#pragma unroll 2
  for (int j0 = 0; j0 < nkt; j0 += 2) {
    f32x4 ds2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = j0 + u;
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = s;
      s = v2_mma32(v2_fragj(Ks, LN, j, 0), qf[0], s);
      s = v2_mma32(v2_fragj(Ks, LN, j, 1), qf[1], s);
      dp = v2_mma32(v2_fragj(Vs, LN, j, 0), df[0], dp);
      dp = v2_mma32(v2_fragj(Vs, LN, j, 1), df[1], dp);
      f32x4 keep = {1.f, 1.f, 1.f, 1.f};
      if (thr && kbits) {
        const unsigned long long kw = (KMAX > 256 && (j >> 4)) ? kb64[KMAX / 256 - 1] : kb64[0];
        const uint32_t b4 = (uint32_t)(kw >> (8 * ((j & 15) >> 1) + 4 * (j & 1))) & 0xFu;
#pragma unroll
        for (int r = 0; r < 4; ++r) keep[r] = (b4 >> r) & 1u ? dscale : 0.f;
      } else if (thr) {
        keep = v2_keep(bh, N, qv ? q : 0, (16 * j + 4 * fq) < N ? 16 * j + 4 * fq : 0, thr, dscale, seed, site);
      }
      // queries >= N need no mask (q = dO = 0 there: dS = 1 * (0 - 0)); keys
      // >= N only in a partial last tile (wave-uniform branch)
      f32x4 p;
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = __builtin_amdgcn_exp2f(fmaf(s[r], c2, -lse2));
      if (16 * j + 16 > N) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * j + 4 * fq + r >= N) p[r] = 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) ds2[u][r] = p[r] * fmaf(dp[r], keep[r], -dl);
    }
    const u32x4 db = v2_cat(v2_pack(ds2[0]), v2_pack(ds2[1]));
#pragma unroll
    for (int t = 0; t < 4; ++t) dq[t] = v2_mma32(v2_trj2(Ks, LN, j0, t), db, dq[t]);
  }
  if (qv) {
    bf16_t* dp_out = dqkv + ((long)b * N + q) * pitch + h * 64;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uint2 u;
      u.x = f2bf2(dq[t][0] * scale, dq[t][1] * scale);
      u.y = f2bf2(dq[t][2] * scale, dq[t][3] * scale);
      *(uint2*)(dp_out + 16 * t + 4 * fq) = u;
    }
  }
  // q bias gradient (queries >= N hold dq = 0)
  if (dbias)
    v2_colsum64<WAVES>(dq, scale, (float*)(smem + 2 * KMAX * V2_ROWB),
                       dbias + (long)(b * gridDim.x + blockIdx.x) * 3 * D + h * 64);
}

// dK, dV: workgroup = (b, h, 16*WAVES keys); wave = 16 keys x all queries;
// Q, dO images + lse, delta of all queries in LDS (KMAX = 512: 157 KiB in
// all); the workgroup's keys lie in one 256-key chunk of the keep bits
template <int WAVES, int KMAX>
__global__ __launch_bounds__(WAVES * 64) void mhsa_dkv_v2(const bf16_t* __restrict__ qkv,
                                                         const bf16_t* __restrict__ dout,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                         int N, int H, float scale, uint32_t thr, float dscale,
                                                         DSeed seed_, uint32_t site,
                                                         const uint32_t* __restrict__ kbits,
                                                         float* __restrict__ dbias) {
  const unsigned long long seed = seed_;
  // keep bits transposed in LDS: KbT[word][query], pitch KBP words (a lane's 4
  // query rows of one word are one 16-byte read)
  constexpr int KBP = KMAX + 16;
  constexpr int RED = 2 * KMAX * V2_ROWB + 2 * KMAX * 4 + 8 * KBP * 4;  // colsum scratch offset
  static_assert(RED + 2 * WAVES * 64 * 4 <= 160 * 1024, "mhsa_dkv_v2: LDS");
  __shared__ __attribute__((aligned(16))) char smem[RED + 2 * WAVES * 64 * 4];
  char* Qs = smem;
  char* Ds = smem + KMAX * V2_ROWB;
  float* Ls = (float*)(smem + 2 * KMAX * V2_ROWB);
  float* Dl = Ls + KMAX;
  uint32_t* Kb = (uint32_t*)(Dl + KMAX);  // the forward's keep bits of this (b, h): KbT[fq*2 + half][query]
  const int D = H * 64;
  const long pitch = 3L * D;
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  const V2Lane LN(lane);
  const bf16_t* base = qkv + (long)b * N * pitch + h * 64;
  const int NQ = (N + 15) & ~15;
  const int nqt = NQ >> 4;
  const int key = blockIdx.x * WAVES * 16 + w * 16 + frow;  // this lane's key (B operand column)
  const bool kv = key < N;
  const uint64_t bh = (uint64_t)b * H + h;
  u32x4 kf[2], vf[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    kf[s2] = kv ? *(const u32x4*)(base + D + (long)key * pitch + 32 * s2 + 8 * fq) : (u32x4){0u, 0u, 0u, 0u};
    vf[s2] = kv ? *(const u32x4*)(base + 2 * D + (long)key * pitch + 32 * s2 + 8 * fq) : (u32x4){0u, 0u, 0u, 0u};
  }
  const int NQ32 = (N + 31) & ~31;  // staged rows: whole tile pairs (rows >= N finite, P = 0)
  v2_stage_glds<WAVES>(Qs, base, pitch, N, NQ32);
  v2_stage_glds<WAVES>(Ds, dout + (long)b * N * D + h * 64, D, N, NQ32);
  for (int i = threadIdx.x; i < NQ32; i += WAVES * 64) {
    Ls[i] = i < N ? lse[bh * N + i] * 1.4426950408889634f : 0.f;
    Dl[i] = i < N ? delta[bh * N + i] : 0.f;
  }
  const bool use_kb = kbits && thr;
  const int kchunk = (blockIdx.x * WAVES * 16) >> 8;  // the 256-key chunk of this workgroup's keys
  if (use_kb)
    for (int i = threadIdx.x; i < N * 2; i += WAVES * 64) {
      const u32x4 v = ((const u32x4*)(kbits + ((uint64_t)kchunk * gridDim.z * H * N + bh * N) * 8))[i];
      const int q = i >> 1, w0 = 4 * (i & 1);
#pragma unroll
      for (int e = 0; e < 4; ++e) Kb[(w0 + e) * KBP + q] = v[e];
    }
  // this lane's key inside a query's bit pair (chunk-relative key kl): word fq' * 2 + half, bit position
  const int kl = key & 255;
  const int kbit = 8 * (kl >> 5) + 4 * ((kl >> 4) & 1) + (kl & 3);
  const int kword = ((kl >> 2) & 3) * 2 + (kbit >> 5), kshift = kbit & 31;
  __syncthreads();
  const float c2 = scale * 1.4426950408889634f;
  // accumulators: rows = d (16t + 4fq + r), column = this lane's key
  f32x4 dkt[4], dvt[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dkt[t] = dvt[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int j0 = 0; j0 < nqt; j0 += 2) {
    f32x4 pd2[2], ds2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = j0 + u;
      // S^T-free form: S[q][key] with m = queries 16j + 4fq + r, n = key (lane)
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = s;
      s = v2_mma32(v2_fragj(Qs, LN, j, 0), kf[0], s);
      s = v2_mma32(v2_fragj(Qs, LN, j, 1), kf[1], s);
      dp = v2_mma32(v2_fragj(Ds, LN, j, 0), vf[0], dp);
      dp = v2_mma32(v2_fragj(Ds, LN, j, 1), vf[1], dp);
      // dropout: lane (quad position c = key & 3) hashes query row 16j+4fq+c of
      // its key group (two pair hashes); the quad exchanges the 16-bit slices
      // (4 queries x 4 keys)
      uint32_t hlo = 0u, hhi = 0u;
      if (thr && !use_kb) {
        const int qc = 16 * j + 4 * fq + (frow & 3);
        const uint64_t idx = (bh * N + (qc < N ? qc : 0)) * (uint64_t)N + (key & ~3);
        const uint32_t rk = rng_key(seed, site);
        hlo = rng_pair(rk, idx);      // keys (key & ~3) + 0, 1
        hhi = rng_pair(rk, idx + 2);  // keys (key & ~3) + 2, 3
      }
      // keys >= N (lanes of a partial last key block: k = v = 0 there, S = 0):
      // masked once per lane (kv); queries >= N only in a partial last tile
      // (wave-uniform branch; their Ls / Dl rows are 0)
      const f32x4 l4 = *(const f32x4*)(Ls + 16 * j + 4 * fq);
      const f32x4 d4 = *(const f32x4*)(Dl + 16 * j + 4 * fq);
      u32x4 kw4 = {0u, 0u, 0u, 0u};
      if (use_kb) kw4 = *(const u32x4*)(Kb + kword * KBP + 16 * j + 4 * fq);
      f32x4 p;
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = kv ? __builtin_amdgcn_exp2f(fmaf(s[r], c2, -l4[r])) : 0.f;
      if (16 * j + 16 > N) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * j + 4 * fq + r >= N) p[r] = 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qi = 16 * j + 4 * fq + r;
        float kp = 1.f;
        if (use_kb) {
          kp = ((kw4[r] >> kshift) & 1u) ? dscale : 0.f;  // (rows >= N: p is 0 there)
        } else if (thr) {
          const int src = (lane & ~3) | r;
          const uint32_t lo = __shfl(hlo, src, 64), hi = __shfl(hhi, src, 64);
          const uint32_t word = (key & 2) ? hi : lo;
          const uint32_t u16 = (key & 1) ? (word >> 16) : (word & 0xffffu);
          kp = u16 >= thr ? dscale : 0.f;
        }
        pd2[u][r] = p[r] * kp;
        ds2[u][r] = p[r] * fmaf(dp[r], kp, -d4[r]);
      }
    }
    // dV^T[d][key] += dO^T[d][q] P~[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
    // (two query tiles per 16x16x32 MFMA)
    const u32x4 pb = v2_cat(v2_pack(pd2[0]), v2_pack(pd2[1]));
    const u32x4 sb = v2_cat(v2_pack(ds2[0]), v2_pack(ds2[1]));
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dvt[t] = v2_mma32(v2_trj2(Ds, LN, j0, t), pb, dvt[t]);
      dkt[t] = v2_mma32(v2_trj2(Qs, LN, j0, t), sb, dkt[t]);
    }
  }
  if (kv) {
    bf16_t* row = dqkv + ((long)b * N + key) * pitch + h * 64;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uint2 u;
      u.x = f2bf2(dkt[t][0] * scale, dkt[t][1] * scale);
      u.y = f2bf2(dkt[t][2] * scale, dkt[t][3] * scale);
      *(uint2*)(row + D + 16 * t + 4 * fq) = u;
      u.x = f2bf2(dvt[t][0], dvt[t][1]);
      u.y = f2bf2(dvt[t][2], dvt[t][3]);
      *(uint2*)(row + 2 * D + 16 * t + 4 * fq) = u;
    }
  }
  // k and v bias gradients (keys >= N hold dk = dv = 0)
  if (dbias) {
    float* prow = dbias + (long)(b * gridDim.x + blockIdx.x) * 3 * D;
    v2_colsum64<WAVES>(dkt, scale, (float*)(smem + RED), prow + D + h * 64);
    v2_colsum64<WAVES>(dvt, 1.f, (float*)(smem + RED) + WAVES * 64, prow + 2 * D + h * 64);
  }
}

// ----------------------------------------------------------------------------
// Single-pass backward for N <= 256 (one 8-wave workgroup per (b, h)): P and
// dP are formed once per score tile instead of once in the dQ kernel and again
// in the dK/dV kernel, and Q, dO, K, V are staged once.
//
// Wave w owns keys 32w .. 32w+31 (their K and V rows in registers, dK and dV
// accumulated in registers, the dK/dV kernel's S[q][key] form).  The queries
// go by in pairs of 16-row tiles; at step s wave w takes pair (w + s) mod 8,
// so in every step the 8 waves hold 8 different pairs.  dQ^T += K^T dS^T of
// the wave's 32 keys then goes into the pair's f32 dQ rows in LDS
// (read -> MFMA C operand -> write) without conflicts, a barrier hands the
// rows to the next owner, and every dQ row takes its 8 contributions in the
// fixed order w = p, p - 1, ... (mod 8): deterministic, no atomics.  dS^T for
// that MFMA is the dK MFMA's dS transposed through a per-wave 2 KiB LDS image
// (8-byte writes, ds_read_b64_tr_b16 reads), and K^T comes from a K image
// staged once into the dQ rows' space before they are zeroed.
//
// LDS: Q and dO images 2 x 32 KiB, dQ rows 64 KiB (256 x 64 f32, 16-byte
// chunks XOR-swizzled by row & 15), lse / delta 2 KiB, transposed keep bits
// 8.5 KiB, dS^T images 8 x 2 KiB (also the bias column-sum scratch at the end).
// ----------------------------------------------------------------------------
constexpr int FB_WAVES = 8;
constexpr int FB_KBP = 256 + 16;
constexpr int FB_DS = 256 * V2_ROWB, FB_ACC = 2 * FB_DS, FB_LS = FB_ACC + 256 * 256, FB_DL = FB_LS + 1024,
              FB_KB = FB_DL + 1024, FB_SCR = FB_KB + 8 * FB_KBP * 4, FB_SMEM = FB_SCR + FB_WAVES * 2048;
static_assert(FB_SMEM <= 160 * 1024, "mhsa_bwd_fused: LDS");

// f32 dQ row q, 16-byte chunk c (columns 4c .. 4c + 3)
__device__ __forceinline__ int fb_acc(int q, int c) { return q * 256 + ((c ^ (q & 15)) << 4); }
// dS^T image of one wave: [32 keys][32 queries] bf16, 64-byte rows, 8-byte
// units XOR-swizzled by row & 7
__device__ __forceinline__ int fb_scr(int row, int unit) { return row * 64 + ((unit ^ (row & 7)) << 3); }

// FULL: N == 256 (no row / tile range tests).  DM: the dropout form, 0 none,
// 1 the forward's keep bits, 2 re-hashed (mhsa_dkv_v2's quad exchange).
template <bool FULL, int DM>
__global__ __launch_bounds__(FB_WAVES * 64) void mhsa_bwd_fused(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16_t* __restrict__ dqkv, int N, int H, float scale,
    uint32_t thr, float dscale, DSeed seed_, uint32_t site, const uint32_t* __restrict__ kbits,
    float* __restrict__ dbias) {
  const unsigned long long seed = seed_;
  __shared__ __attribute__((aligned(16))) char smem[FB_SMEM];
  char* Qs = smem;
  char* Ds = smem + FB_DS;
  char* Acc = smem + FB_ACC;
  float* Ls = (float*)(smem + FB_LS);
  float* Dl = (float*)(smem + FB_DL);
  uint32_t* Kb = (uint32_t*)(smem + FB_KB);
  const int D = H * 64;
  const long pitch = 3L * D;
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  char* Scr = smem + FB_SCR + w * 2048;
  const V2Lane LN(lane);
  const bf16_t* base = qkv + (long)b * N * pitch + h * 64;
  const bf16_t* dob = dout + (long)b * N * D + h * 64;
  const int nqt = FULL ? 16 : (N + 15) >> 4;
  const int N32 = FULL ? 256 : (N + 31) & ~31;  // staged rows: whole tile pairs (rows >= N finite copies)
  const uint64_t bh = (uint64_t)b * H + h;
  // Q, dO and (into the dQ rows' space) K images of all rows
  v2_stage_glds<FB_WAVES>(Qs, base, pitch, N, N32);
  v2_stage_glds<FB_WAVES>(Ds, dob, D, N, N32);
  // this wave's keys (two 16-key tiles): K and V rows as MFMA B operands
  u32x4 kf[2][2], vf[2][2];
  bool kv[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = 32 * w + 16 * kt + frow;
    kv[kt] = FULL || key < N;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      kf[kt][s2] = kv[kt] ? *(const u32x4*)(base + D + (long)key * pitch + 32 * s2 + 8 * fq) : (u32x4){0u, 0u, 0u, 0u};
      vf[kt][s2] =
          kv[kt] ? *(const u32x4*)(base + 2 * D + (long)key * pitch + 32 * s2 + 8 * fq) : (u32x4){0u, 0u, 0u, 0u};
    }
  }
  // delta = rowsum(dO * O) (two threads per query): this thread's O half-row and
  // lse now (in flight with the staging), its dO half-row from the staged image
  // after the barrier below (dO is read from HBM once)
  const int qd = threadIdx.x >> 1, hf = threadIdx.x & 1;
  const bool qdv = FULL || qd < N;
  u32x4 orow[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
    orow[c] = qdv ? *(const u32x4*)(o + ((long)b * N + qd) * D + h * 64 + 32 * hf + 8 * c) : (u32x4){0u, 0u, 0u, 0u};
  const float lq = (qdv && hf == 0) ? lse[bh * N + qd] * 1.4426950408889634f : 0.f;
  // the forward's keep bits of this (b, h), transposed: Kb[word][query] (mhsa_dkv_v2's layout)
  constexpr bool use_kb = DM == 1;
  if (use_kb)
    for (int i = threadIdx.x; i < N * 2; i += FB_WAVES * 64) {
      const u32x4 v = ((const u32x4*)(kbits + bh * N * 8))[i];
      const int q = i >> 1, w0 = 4 * (i & 1);
#pragma unroll
      for (int e = 0; e < 4; ++e) Kb[(w0 + e) * FB_KBP + q] = v[e];
    }
  int kword[2], kshift[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kl = 32 * w + 16 * kt + frow;
    const int kbit = 8 * (kl >> 5) + 4 * ((kl >> 4) & 1) + (kl & 3);
    kword[kt] = ((kl >> 2) & 3) * 2 + (kbit >> 5);
    kshift[kt] = kbit & 31;
  }
  __syncthreads();
  {
    float dl = 0.f;
    if (qdv) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const u32x4 x = *(const u32x4*)(Ds + v2_off(qd, 4 * hf + c)), y = orow[c];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          dl += __uint_as_float(x[e] << 16) * __uint_as_float(y[e] << 16) +
                __uint_as_float(x[e] & 0xffff0000u) * __uint_as_float(y[e] & 0xffff0000u);
      }
    }
    dl += __shfl_xor(dl, 1, 64);
    if (hf == 0) {  // (read in the step loop, after the barriers below)
      Dl[qd] = qdv ? dl : 0.f;
      Ls[qd] = lq;
      if (qdv) delta[bh * N + qd] = dl;
    }
  }
  // K^T of this wave's 32 keys as the A operand of dQ^T = K^T dS^T (keys 4g + e, 16 + 4g + e):
  // its K rows written from registers into a 4 KiB image (in the dQ rows' space, before they
  // are zeroed) and read back transposed
  u32x4 kT[4];
  {
    char* Ki = Acc + w * 4096;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) *(u32x4*)(Ki + v2_off(16 * kt + frow, 4 * s2 + fq)) = kf[kt][s2];
    lds_fence();
#pragma unroll
    for (int t = 0; t < 4; ++t) kT[t] = v2_trj2(Ki, LN, 0, t);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256 * 16; i += FB_WAVES * 64) ((f32x4*)Acc)[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  const float c2 = scale * 1.4426950408889634f;
  const uint32_t rk = rng_key(seed, site);
  const bool wact = FULL || 32 * w < N;
  f32x4 dkt[4][2], dvt[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) dkt[t][kt] = dvt[t][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < FB_WAVES; ++s) {
    const int j0 = 2 * ((w + s) & (FB_WAVES - 1));  // first query tile of this step's pair
    if (wact && (FULL || j0 < nqt)) {               // wave-uniform
      f32x4 pd[2][2], dsv[2][2];                    // [query tile][key tile]
#pragma unroll
      for (int bq = 0; bq < 2; ++bq) {
        const int j = j0 + bq;
        if (FULL || j < nqt) {
          const u32x4 qa0 = v2_fragj(Qs, LN, j, 0), qa1 = v2_fragj(Qs, LN, j, 1);
          const u32x4 da0 = v2_fragj(Ds, LN, j, 0), da1 = v2_fragj(Ds, LN, j, 1);
          const f32x4 l4 = *(const f32x4*)(Ls + 16 * j + 4 * fq);
          const f32x4 d4 = *(const f32x4*)(Dl + 16 * j + 4 * fq);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            // S[q][key], dP[q][key]: rows = queries 16j + 4fq + r, column = this lane's key
            f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = sv;
            sv = v2_mma32(qa0, kf[kt][0], sv);
            sv = v2_mma32(qa1, kf[kt][1], sv);
            dp = v2_mma32(da0, vf[kt][0], dp);
            dp = v2_mma32(da1, vf[kt][1], dp);
            const int key = 32 * w + 16 * kt + frow;
            uint32_t hlo = 0u, hhi = 0u;
            if (DM == 2) {  // re-hash (mhsa_dkv_v2's quad exchange)
              const int qc = 16 * j + 4 * fq + (frow & 3);
              const uint64_t idx = (bh * N + (qc < N ? qc : 0)) * (uint64_t)N + (key & ~3);
              hlo = rng_pair(rk, idx);
              hhi = rng_pair(rk, idx + 2);
            }
            u32x4 kw4 = {0u, 0u, 0u, 0u};
            if (DM == 1) kw4 = *(const u32x4*)(Kb + kword[kt] * FB_KBP + 16 * j + 4 * fq);
            f32x4 p;
#pragma unroll
            for (int r = 0; r < 4; ++r)
              p[r] = (FULL || kv[kt]) ? __builtin_amdgcn_exp2f(fmaf(sv[r], c2, -l4[r])) : 0.f;
            if (!FULL && 16 * j + 16 > N) {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (16 * j + 4 * fq + r >= N) p[r] = 0.f;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float kp = 1.f;
              if constexpr (DM == 1) {
                kp = ((kw4[r] >> kshift[kt]) & 1u) ? dscale : 0.f;
              } else if constexpr (DM == 2) {
                const int src = (lane & ~3) | r;
                const uint32_t lo = __shfl(hlo, src, 64), hi = __shfl(hhi, src, 64);
                const uint32_t word = (key & 2) ? hi : lo;
                const uint32_t u16 = (key & 1) ? (word >> 16) : (word & 0xffffu);
                kp = u16 >= thr ? dscale : 0.f;
              }
              if constexpr (DM == 0) {
                pd[bq][kt][r] = p[r];
                dsv[bq][kt][r] = p[r] * (dp[r] - d4[r]);
              } else {
                pd[bq][kt][r] = p[r] * kp;
                dsv[bq][kt][r] = p[r] * fmaf(dp[r], kp, -d4[r]);
              }
            }
          }
        } else {
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) pd[bq][kt] = dsv[bq][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
      // dV^T[d][key] += dO^T[d][q] P~[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]  (the pair's 32 queries)
      u32x4 pb[2], sb[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        pb[kt] = v2_cat(v2_pack(pd[0][kt]), v2_pack(pd[1][kt]));
        sb[kt] = v2_cat(v2_pack(dsv[0][kt]), v2_pack(dsv[1][kt]));
        // dS^T image: row = key (16kt + frow), queries 16bq + 4fq .. +3
#pragma unroll
        for (int bq = 0; bq < 2; ++bq)
          *(v4s_t*)(Scr + fb_scr(16 * kt + frow, 4 * bq + fq)) = v2_pack(dsv[bq][kt]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const u32x4 doT = v2_trj2(Ds, LN, j0, t), qT = v2_trj2(Qs, LN, j0, t);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          dvt[t][kt] = v2_mma32(doT, pb[kt], dvt[t][kt]);
          dkt[t][kt] = v2_mma32(qT, sb[kt], dkt[t][kt]);
        }
      }
      lds_fence();  // this wave's dS^T image written before its transposed reads
      // dQ^T[d][q] += K^T[d][keys] dS^T[keys][q] into the pair's f32 rows (this step's owner)
#pragma unroll
      for (int bq = 0; bq < 2; ++bq) {
        if (FULL || j0 + bq < nqt) {
          const int g = lane >> 4, li = lane & 15;
          v4s_t lo, hi;
          {
            const int row = 4 * g + (li >> 2), unit = 4 * bq + (li & 3);
            lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(Scr + fb_scr(row, unit)));
            hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(Scr + fb_scr(row + 16, unit)));
          }
          const u32x4 bfr = v2_cat(lo, hi);
          const int q = 16 * (j0 + bq) + frow;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            f32x4* a = (f32x4*)(Acc + fb_acc(q, 4 * t + fq));
            *a = v2_mma32(kT[t], bfr, *a);
          }
        }
      }
    }
    __syncthreads();
  }
  // dQ (bf16, x scale): two threads per query row
  {
    const int qd = threadIdx.x >> 1, hf = threadIdx.x & 1;
    if (FULL || qd < N) {
      bf16_t* dst = dqkv + ((long)b * N + qd) * pitch + h * 64 + 32 * hf;
#pragma unroll
      for (int c = 0; c < 8; c += 2) {
        const f32x4 x = *(const f32x4*)(Acc + fb_acc(qd, 8 * hf + c));
        const f32x4 y = *(const f32x4*)(Acc + fb_acc(qd, 8 * hf + c + 1));
        u32x4 u;
        u[0] = f2bf2(x[0] * scale, x[1] * scale);
        u[1] = f2bf2(x[2] * scale, x[3] * scale);
        u[2] = f2bf2(y[0] * scale, y[1] * scale);
        u[3] = f2bf2(y[2] * scale, y[3] * scale);
        *(u32x4*)(dst + 4 * c) = u;
      }
    }
  }
  // q part of the qkv bias gradient's partial row: column sums of the f32 dQ rows (rows >= N are 0)
  float* red = (float*)(smem + FB_SCR);
  if (dbias) {
    const int c = threadIdx.x & 63, g8 = threadIdx.x >> 6;
    float sum = 0.f;
    for (int r = 32 * g8; r < 32 * g8 + 32; ++r) sum += ((const float*)(Acc + fb_acc(r, c >> 2)))[c & 3];
    red[g8 * 64 + c] = sum * scale;
  }
  __syncthreads();  // the dQ rows are read: their space takes the dK / dV rows
  // dK (x scale) and dV rows of this wave's keys through LDS ([32 keys][dK 64 | dV 64] bf16,
  // 16-byte chunks XOR-swizzled by row & 15), then stored as whole 128-byte row segments
  {
    char* Rw = Acc + w * 8192;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int row = 16 * kt + frow;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint2 u;
        u.x = f2bf2(dkt[t][kt][0] * scale, dkt[t][kt][1] * scale);
        u.y = f2bf2(dkt[t][kt][2] * scale, dkt[t][kt][3] * scale);
        *(uint2*)(Rw + row * 256 + (((2 * t + (fq >> 1)) ^ (row & 15)) << 4) + 8 * (fq & 1)) = u;
        u.x = f2bf2(dvt[t][kt][0], dvt[t][kt][1]);
        u.y = f2bf2(dvt[t][kt][2], dvt[t][kt][3]);
        *(uint2*)(Rw + row * 256 + (((8 + 2 * t + (fq >> 1)) ^ (row & 15)) << 4) + 8 * (fq & 1)) = u;
      }
    }
    lds_fence();
    const int c = lane & 15;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 4 * i + (lane >> 4);
      const int key = 32 * w + row;
      const u32x4 v = *(const u32x4*)(Rw + row * 256 + ((c ^ (row & 15)) << 4));
      if (FULL || key < N) *(u32x4*)(dqkv + ((long)b * N + key) * pitch + (c < 8 ? D : 2 * D - 64) + h * 64 + 8 * c) = v;
    }
  }
  // k / v parts of the bias partial row from the register accumulators (keys >= N hold 0)
  if (dbias) {
    float* prow = dbias + (long)b * 3 * D;
    f32x4 sk[4], sv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sk[t] = dkt[t][0] + dkt[t][1];
      sv[t] = dvt[t][0] + dvt[t][1];
    }
    v2_colsum64<FB_WAVES>(sk, scale, red + 2 * FB_WAVES * 64, prow + D + h * 64);
    v2_colsum64<FB_WAVES>(sv, 1.f, red + 4 * FB_WAVES * 64, prow + 2 * D + h * 64);
    if (threadIdx.x < 64) {
      float sq = 0.f;
#pragma unroll
      for (int i = 0; i < FB_WAVES; ++i) sq += red[i * 64 + threadIdx.x];
      prow[h * 64 + threadIdx.x] = sq;
    }
  }
}

static bool v2_ok(int dt, int hd, int N) { return dt == HVIT_BF16 && hd == 64 && N <= V2_KMAX && N % 4 == 0; }
static bool v2_big(int N) { return N > 256; }  // the KMAX = 512 instantiations
// waves per v2 workgroup: 16 = all queries (keys) of a (b, h) in one
// workgroup, K/V (Q/dO) staged once.  Measured: two 8-wave workgroups per
// (b, h) are slower both at B*H = 256 (default, B=32) and at B*H = 192
// (config 5, B=16: 20.6 -> 21.5 us per layer); HVIT_ATTN_WAVES = 4 / 8 / 16
// overrides (A/B only).  The one place the wave count is chosen: the launches
// and the bias-partial row count both use it, so an unsupported value (clamped
// to 4, the template the launches fall back to) cannot size the rows apart
// from the grid.
// (N > 256 takes the KMAX = 512 kernels, instantiated for 16 waves only)
// the single-pass backward (mhsa_bwd_fused) for N <= 256; hvit_gemm_tune(4, 0)
// selects the dQ + dK/dV kernel pair (tests)
int& attn_fused_ref() {
  static int v = 1;
  return v;
}
static bool v2_fused(int N) { return attn_fused_ref() != 0 && !v2_big(N); }
static int v2_waves(int N) {
  (void)N;
  return 16;  // (8-wave workgroups measured slower at B·H = 256 and 192)
}

// ------------------------------------------------------------------- host ---
template <typename T, int HD>
static int mhsa_fwd_t(const void* qkv, void* o, float* lse, float* probs, int B, int N, int H,
                      float scale, const hvit_dropout_t* dr, hipStream_t st) {
  uint32_t thr = dr ? drop_threshold(dr->p) : 0;
  float ds = (dr && dr->p > 0.f) ? 1.f / (1.f - dr->p) : 1.f;
  const DSeed seed = dseed(dr);
  uint32_t site = dr ? dr->site : 0;
  dim3 g(cdiv(N, AT_TILE), H, B);
  hipLaunchKernelGGL((mhsa_fwd_kernel<T, HD>), g, dim3(AT_THREADS), 0, st, (const T*)qkv, (T*)o, lse, B,
                     N, H, scale, thr, ds, seed, site);
  HVIT_LAUNCH_CHECK();
  if (probs) {
    hipLaunchKernelGGL((mhsa_dq_kernel<T, HD, true>), g, dim3(AT_THREADS), 0, st, (const T*)qkv,
                       (const T*)nullptr, lse, (const float*)nullptr, (T*)nullptr, probs, B, N, H,
                       scale, thr, ds, seed, site);
    HVIT_LAUNCH_CHECK();
  }
  return HVIT_OK;
}

template <typename T, int HD>
static int mhsa_bwd_t(const void* qkv, const void* o, const void* dout, const float* lse,
                      float* delta, void* dqkv, int B, int N, int H, float scale,
                      const hvit_dropout_t* dr, hipStream_t st) {
  uint32_t thr = dr ? drop_threshold(dr->p) : 0;
  float ds = (dr && dr->p > 0.f) ? 1.f / (1.f - dr->p) : 1.f;
  const DSeed seed = dseed(dr);
  uint32_t site = dr ? dr->site : 0;
  long rows = (long)B * N * H;
  hipLaunchKernelGGL((mhsa_delta_kernel<T, HD>), dim3(cdiv(rows, 4)), dim3(256), 0, st, (const T*)o,
                     (const T*)dout, delta, B, N, H);
  HVIT_LAUNCH_CHECK();
  dim3 g(cdiv(N, AT_TILE), H, B);
  hipLaunchKernelGGL((mhsa_dq_kernel<T, HD, false>), g, dim3(AT_THREADS), 0, st, (const T*)qkv,
                     (const T*)dout, lse, (const float*)delta, (T*)dqkv, (float*)nullptr, B, N, H,
                     scale, thr, ds, seed, site);
  HVIT_LAUNCH_CHECK();
  hipLaunchKernelGGL((mhsa_dkv_kernel<T, HD>), g, dim3(AT_THREADS), 0, st, (const T*)qkv,
                     (const T*)dout, lse, (const float*)delta, (T*)dqkv, B, N, H, scale, thr, ds,
                     seed, site);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

#define HVIT_HD_DISPATCH(FN, ...)                                              \
  switch (hd) {                                                                \
    case 16: return dt == HVIT_BF16 ? FN<bf16_t, 16>(__VA_ARGS__) : FN<float, 16>(__VA_ARGS__); \
    case 32: return dt == HVIT_BF16 ? FN<bf16_t, 32>(__VA_ARGS__) : FN<float, 32>(__VA_ARGS__); \
    case 64: return dt == HVIT_BF16 ? FN<bf16_t, 64>(__VA_ARGS__) : FN<float, 64>(__VA_ARGS__); \
    default: hvit_set_error("mhsa: head_dim %d unsupported (16, 32, 64)", hd); return HVIT_ERR_ARG; \
  }

}  // namespace hvit

using namespace hvit;

static int mhsa_fwd_impl(int dt, const void* qkv, int B, int N, int H, int hd, float scale,
                         const hvit_dropout_t* dropout, void* o, float* lse, float* probs, uint32_t* keep_bits,
                         void* stream) {
  HVIT_CHECK(qkv && o && lse, "hvit_mhsa_fwd: null pointer");
  HVIT_CHECK(B > 0 && N > 0 && H > 0, "hvit_mhsa_fwd: bad shape B=%d N=%d H=%d", B, N, H);
  HVIT_CHECK(aligned16(qkv) && aligned16(o), "hvit_mhsa_fwd: qkv/o must be 16-byte aligned");
  HVIT_CHECK(dt == HVIT_F32 || dt == HVIT_BF16, "hvit_mhsa_fwd: bad dtype");
  hipStream_t st = (hipStream_t)stream;
  if (v2_ok(dt, hd, N) && !probs) {
    const hvit_dropout_t* dr = dropout;
    const uint32_t thr = dr ? drop_threshold(dr->p) : 0;
    const float ds = (dr && dr->p > 0.f) ? 1.f / (1.f - dr->p) : 1.f;
    const int wv = v2_waves(N);
    auto go = [&](auto kern, int waves) {
      hipLaunchKernelGGL(kern, dim3(cdiv(N, 16 * waves), H, B), dim3(64 * waves), 0, st, (const bf16_t*)qkv,
                         (bf16_t*)o, lse, N, H, scale, thr, ds, dseed(dr), dr ? dr->site : 0u, keep_bits);
    };
    if (v2_big(N)) go(mhsa_fwd_v2<8, 512>, 8);
    else if (wv == 16 && N == 256) go(mhsa_fwd_v2<16, 256, true>, 16);
    else if (wv == 16) go(mhsa_fwd_v2<16, 256>, 16);
    else if (wv == 8) go(mhsa_fwd_v2<8, 256>, 8);
    else go(mhsa_fwd_v2<4, 256>, 4);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  HVIT_HD_DISPATCH(mhsa_fwd_t, qkv, o, lse, probs, B, N, H, scale, dropout, st);
}

// partial rows of the fused bias gradient per sample: one per v2 workgroup
// along the token axis; one per sample otherwise
static long long mhsa_bias_rows_per_sample(int dt, int hd, int N) {
  return v2_ok(dt, hd, N) ? (v2_fused(N) ? 1 : cdiv(N, 16 * v2_waves(N))) : 1;
}

static int mhsa_bwd_impl(int dt, const void* qkv, const void* o, const void* dout, const float* lse, int B, int N,
                         int H, int hd, float scale, const hvit_dropout_t* dropout, const uint32_t* keep_bits,
                         void* dqkv, float* delta_ws, float* dbias, void* stream) {
  HVIT_CHECK(qkv && o && dout && lse && dqkv && delta_ws, "hvit_mhsa_bwd: null pointer");
  HVIT_CHECK(B > 0 && N > 0 && H > 0, "hvit_mhsa_bwd: bad shape");
  HVIT_CHECK(aligned16(qkv) && aligned16(o) && aligned16(dout) && aligned16(dqkv),
             "hvit_mhsa_bwd: tensors must be 16-byte aligned");
  HVIT_CHECK(dt == HVIT_F32 || dt == HVIT_BF16, "hvit_mhsa_bwd: bad dtype");
  hipStream_t st = (hipStream_t)stream;
  if (v2_ok(dt, hd, N)) {
    const hvit_dropout_t* dr = dropout;
    const uint32_t thr = dr ? drop_threshold(dr->p) : 0;
    const float ds = (dr && dr->p > 0.f) ? 1.f / (1.f - dr->p) : 1.f;
    const DSeed seed = dseed(dr);
    const uint32_t site = dr ? dr->site : 0u;
    auto go = [&](auto dqk, auto dkvk, int waves) {
      dim3 g(cdiv(N, 16 * waves), H, B);
      hipLaunchKernelGGL(dqk, g, dim3(64 * waves), 0, st, (const bf16_t*)qkv, (const bf16_t*)o, (const bf16_t*)dout,
                         lse, delta_ws, (bf16_t*)dqkv, N, H, scale, thr, ds, seed, site, keep_bits, dbias);
      hipLaunchKernelGGL(dkvk, g, dim3(64 * waves), 0, st, (const bf16_t*)qkv, (const bf16_t*)dout, lse,
                         (const float*)delta_ws, (bf16_t*)dqkv, N, H, scale, thr, ds, seed, site, keep_bits, dbias);
    };
    if (v2_fused(N)) {
      auto fb = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(1, H, B), dim3(FB_WAVES * 64), 0, st, (const bf16_t*)qkv, (const bf16_t*)o,
                           (const bf16_t*)dout, lse, delta_ws, (bf16_t*)dqkv, N, H, scale, thr, ds, seed, site,
                           keep_bits, dbias);
      };
      const int dm = !thr ? 0 : keep_bits ? 1 : 2;
      if (N == 256) {
        if (dm == 0) fb(mhsa_bwd_fused<true, 0>);
        else if (dm == 1) fb(mhsa_bwd_fused<true, 1>);
        else fb(mhsa_bwd_fused<true, 2>);
      } else {
        if (dm == 0) fb(mhsa_bwd_fused<false, 0>);
        else if (dm == 1) fb(mhsa_bwd_fused<false, 1>);
        else fb(mhsa_bwd_fused<false, 2>);
      }
      HVIT_LAUNCH_CHECK();
      return HVIT_OK;
    }
    const int wv = v2_waves(N);
    if (v2_big(N)) go(mhsa_dq_v2<16, 512>, mhsa_dkv_v2<16, 512>, 16);
    else if (wv == 16) go(mhsa_dq_v2<16, 256>, mhsa_dkv_v2<16, 256>, 16);
    else if (wv == 8) go(mhsa_dq_v2<8, 256>, mhsa_dkv_v2<8, 256>, 8);
    else go(mhsa_dq_v2<4, 256>, mhsa_dkv_v2<4, 256>, 4);
    HVIT_LAUNCH_CHECK();
    return HVIT_OK;
  }
  if (dbias) {  // other shapes: one partial row per sample, a segmented column sum of dqkv (one launch, fixed order)
    const auto rc = [&]() -> int { HVIT_HD_DISPATCH(mhsa_bwd_t, qkv, o, dout, lse, delta_ws, dqkv, B, N, H, scale, dropout, st); }();
    if (rc) return rc;
    const long long C3 = 3LL * H * hd;
    return hvit_reduce_rows_seg(dqkv, dt, B, N, C3, C3, 0, dbias, stream);
  }
  HVIT_HD_DISPATCH(mhsa_bwd_t, qkv, o, dout, lse, delta_ws, dqkv, B, N, H, scale, dropout, st);
}

extern "C" int hvit_mhsa_fwd(int dt, const void* qkv, int B, int N, int H, int hd, float scale,
                             const hvit_dropout_t* dropout, void* o, float* lse, float* probs, void* stream) {
  return mhsa_fwd_impl(dt, qkv, B, N, H, hd, scale, dropout, o, lse, probs, nullptr, stream);
}

extern "C" int hvit_mhsa_bwd(int dt, const void* qkv, const void* o, const void* dout, const float* lse, int B, int N,
                             int H, int hd, float scale, const hvit_dropout_t* dropout, void* dqkv, float* delta_ws,
                             void* stream) {
  return mhsa_bwd_impl(dt, qkv, o, dout, lse, B, N, H, hd, scale, dropout, nullptr, dqkv, delta_ws, nullptr, stream);
}

// keep-bit variants: the forward stores its attention-dropout decisions (one
// bit per (query, key): B*H*N*8 32-bit words per 256-key chunk, chunk-major)
// and the backward reads them instead of re-hashing (bf16, head_dim 64,
// N <= 512, N % 4 == 0; other shapes ignore keep_bits and regenerate the mask)
extern "C" long long hvit_mhsa_keep_bits_elems(int B, int N, int H) {
  return (B > 0 && N > 0 && H > 0) ? (long long)B * H * N * 8 * cdiv(N, 256) : 0;
}
// 1 when the kernels for (dt, N, hd) store / read keep bits (else a keep-bit
// buffer would be allocated for nothing: callers skip it)
extern "C" int hvit_mhsa_keep_bits_used(int dt, int N, int hd) { return v2_ok(dt, hd, N) ? 1 : 0; }

int hvit_attn_tune(int value) {
  const int old = hvit::attn_fused_ref();
  hvit::attn_fused_ref() = value;
  return old;
}

extern "C" int hvit_mhsa_fwd_kb(int dt, const void* qkv, int B, int N, int H, int hd, float scale,
                                const hvit_dropout_t* dropout, void* o, float* lse, unsigned* keep_bits,
                                void* stream) {
  HVIT_CHECK(!keep_bits || ((uintptr_t)keep_bits & 15) == 0, "hvit_mhsa_fwd_kb: keep_bits alignment");
  return mhsa_fwd_impl(dt, qkv, B, N, H, hd, scale, dropout, o, lse, nullptr, keep_bits, stream);
}

extern "C" int hvit_mhsa_bwd_kb(int dt, const void* qkv, const void* o, const void* dout, const float* lse, int B,
                                int N, int H, int hd, float scale, const hvit_dropout_t* dropout,
                                const unsigned* keep_bits, void* dqkv, float* delta_ws, void* stream) {
  HVIT_CHECK(!keep_bits || ((uintptr_t)keep_bits & 15) == 0, "hvit_mhsa_bwd_kb: keep_bits alignment");
  return mhsa_bwd_impl(dt, qkv, o, dout, lse, B, N, H, hd, scale, dropout, keep_bits, dqkv, delta_ws, nullptr, stream);
}

// keep_bits and dbias_rows both optional: dbias_rows (f32
// [hvit_mhsa_bias_rows(B, N, H, hd)][3 * H * hd], overwritten) receives partial
// column sums of dqkv whose sum over rows is the qkv bias gradient, formed
// inside the attention backward (v2 shapes) instead of by a pass over dqkv
extern "C" long long hvit_mhsa_bias_rows(int dt, int B, int N, int H, int hd) {
  (void)H;
  return (B > 0 && N > 0) ? (long long)B * mhsa_bias_rows_per_sample(dt, hd, N) : 0;
}

extern "C" int hvit_mhsa_bwd_db(int dt, const void* qkv, const void* o, const void* dout, const float* lse, int B,
                                int N, int H, int hd, float scale, const hvit_dropout_t* dropout,
                                const unsigned* keep_bits, void* dqkv, float* delta_ws, float* dbias, void* stream) {
  HVIT_CHECK(!keep_bits || ((uintptr_t)keep_bits & 15) == 0, "hvit_mhsa_bwd_db: keep_bits alignment");
  return mhsa_bwd_impl(dt, qkv, o, dout, lse, B, N, H, hd, scale, dropout, keep_bits, dqkv, delta_ws, dbias, stream);
}
