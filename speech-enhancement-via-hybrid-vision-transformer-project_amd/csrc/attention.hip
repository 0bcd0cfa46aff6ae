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
                                                             float dscale, unsigned long long seed,
                                                             uint32_t site) {
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
      alpha[r] = exp2f(mrow[r] - mn);
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float p = exp2f(s[j][r] - mn);
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
                                                            float dscale, unsigned long long seed, uint32_t site) {
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
        float p = valid ? exp2f(s[j][r] * c2 - lse2[r]) : 0.f;
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
                                                             unsigned long long seed, uint32_t site) {
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
        float p = valid ? exp2f(s[j][r] * c2 - l2) : 0.f;
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

// ------------------------------------------------------------------- host ---
template <typename T, int HD>
static int mhsa_fwd_t(const void* qkv, void* o, float* lse, float* probs, int B, int N, int H,
                      float scale, const hvit_dropout_t* dr, hipStream_t st) {
  uint32_t thr = dr ? drop_threshold(dr->p) : 0;
  float ds = (dr && dr->p > 0.f) ? 1.f / (1.f - dr->p) : 1.f;
  unsigned long long seed = dr ? dr->seed : 0;
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
  unsigned long long seed = dr ? dr->seed : 0;
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

extern "C" int hvit_mhsa_fwd(int dt, const void* qkv, int B, int N, int H, int hd, float scale,
                             const hvit_dropout_t* dropout, void* o, float* lse, float* probs,
                             void* stream) {
  HVIT_CHECK(qkv && o && lse, "hvit_mhsa_fwd: null pointer");
  HVIT_CHECK(B > 0 && N > 0 && H > 0, "hvit_mhsa_fwd: bad shape B=%d N=%d H=%d", B, N, H);
  HVIT_CHECK(aligned16(qkv) && aligned16(o), "hvit_mhsa_fwd: qkv/o must be 16-byte aligned");
  HVIT_CHECK(dt == HVIT_F32 || dt == HVIT_BF16, "hvit_mhsa_fwd: bad dtype");
  hipStream_t st = (hipStream_t)stream;
  HVIT_HD_DISPATCH(mhsa_fwd_t, qkv, o, lse, probs, B, N, H, scale, dropout, st);
}

extern "C" int hvit_mhsa_bwd(int dt, const void* qkv, const void* o, const void* dout,
                             const float* lse, int B, int N, int H, int hd, float scale,
                             const hvit_dropout_t* dropout, void* dqkv, float* delta_ws,
                             void* stream) {
  HVIT_CHECK(qkv && o && dout && lse && dqkv && delta_ws, "hvit_mhsa_bwd: null pointer");
  HVIT_CHECK(B > 0 && N > 0 && H > 0, "hvit_mhsa_bwd: bad shape");
  HVIT_CHECK(aligned16(qkv) && aligned16(o) && aligned16(dout) && aligned16(dqkv),
             "hvit_mhsa_bwd: tensors must be 16-byte aligned");
  HVIT_CHECK(dt == HVIT_F32 || dt == HVIT_BF16, "hvit_mhsa_bwd: bad dtype");
  hipStream_t st = (hipStream_t)stream;
  HVIT_HD_DISPATCH(mhsa_bwd_t, qkv, o, dout, lse, delta_ws, dqkv, B, N, H, scale, dropout, st);
}
