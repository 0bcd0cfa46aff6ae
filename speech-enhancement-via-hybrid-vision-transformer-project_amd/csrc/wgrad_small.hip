// Tall-skinny bf16 weight gradient dW[N][K] = sum_m dy[m][n] x[m][k] (+ the
// bias gradient db[n] = sum_m dy[m][n]) for the small linears of the step: the
// to_feature_map head (hybrid_vit.py:153, M = 2048 tokens) and the three 1x1
// skip projections (hybrid_vit.py:158-165, 376-386; M = 8192 .. 131072 pixels,
// N = K = 256 .. 64).  These are HBM-bound reductions over M (2 flops per
// loaded byte at N = K = 64) that the tiled GEMM covered with one or four
// output tiles and hundreds of short split-K slices.
//
// Here a workgroup owns one 64x64 output tile and 256 rows: it requests all
// four 64-row stages of both operands at once (16-byte loads of whole 128-byte
// row segments into registers: one memory latency per workgroup), then passes
// them through LDS stage by stage, each wave accumulating a 32x32 sub-tile
// with v_mfma_f32_16x16x32_bf16.  Operand
// fragments are gathered from the [m][n] / [m][k] LDS images column-wise
// (k of the MFMA = m).  The k = 0 tile column also sums its dy fragments for
// the bias gradient.  Each workgroup writes an f32 slab [dW | db]; one
// column reduction (hvit_sum_slabs) finishes.
#include <algorithm>

#include "common.h"

namespace hvit_ws {

constexpr int TM = 64;      // rows (m) per stage
constexpr int NS = 4;       // stages per workgroup, all loaded up front
constexpr int TILE = 64;    // output tile edge
constexpr int PITCH = 72;   // LDS row pitch (bf16): 144 B rows spread the column gathers over banks

__device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, a), __builtin_bit_cast(s16x8, b), c, 0,
                                                 0, 0);
}

// 8 bf16 of column c, rows r0 .. r0+7, of an LDS image [rows][PITCH]
__device__ __forceinline__ u32x4 gather8(const bf16_t* img, int r0, int c) {
  const bf16_t* p = img + r0 * PITCH + c;
  u32x4 f;
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] = (uint32_t)p[(2 * i) * PITCH] | ((uint32_t)p[(2 * i + 1) * PITCH] << 16);
  return f;
}

__global__ __launch_bounds__(256, 2) void wgrad_small_kernel(const bf16_t* __restrict__ dy,
                                                            const bf16_t* __restrict__ x, int M, int N, int K,
                                                            int rows_per_wg, int with_db, float* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) bf16_t sa[TM * PITCH];
  __shared__ __attribute__((aligned(16))) bf16_t sb[TM * PITCH];
  const int tiles_k = K / TILE;
  const int n0 = (blockIdx.x / tiles_k) * TILE, k0 = (blockIdx.x % tiles_k) * TILE;
  const int m_begin = blockIdx.y * rows_per_wg, m_end = min(M, m_begin + rows_per_wg);
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  // loader: thread -> (row, 8-column group) of a 64x64 stage, two passes of 32
  // rows; all NS stages of the workgroup's rows are requested before the first
  // is used (one memory latency per workgroup, not one per stage)
  const int lr = tid >> 3, lc = (tid & 7) * 8;
  u32x4 ra[NS][2], rb[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int m = m_begin + s * TM + lr + 32 * p;
      const bool ok = m < m_end;
      const long mm = ok ? m : m_begin;
      const u32x4 va = *(const u32x4*)(dy + mm * N + n0 + lc);
      const u32x4 vb = *(const u32x4*)(x + mm * K + k0 + lc);
      const u32x4 z = {0u, 0u, 0u, 0u};
      ra[s][p] = ok ? va : z;
      rb[s][p] = ok ? vb : z;
    }
  // wave sub-tile: n rows [nb, nb + 32), k columns [kb, kb + 32)
  const int nb = 32 * (wv >> 1), kb = 32 * (wv & 1);
  const bool do_db = with_db && k0 == 0 && (wv & 1) == 0;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbs[2] = {0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (m_begin + s * TM >= m_end) break;  // uniform
    if (s > 0) __syncthreads();  // the previous stage's fragments are read
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      *(u32x4*)(sa + (lr + 32 * p) * PITCH + lc) = ra[s][p];
      *(u32x4*)(sb + (lr + 32 * p) * PITCH + lc) = rb[s][p];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < TM / 32; ++ks) {
      const int r0 = ks * 32 + 8 * (l >> 4);
      u32x4 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = gather8(sa, r0, nb + 16 * i + (l & 15));
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = gather8(sb, r0, kb + 16 * j + (l & 15));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
      if (do_db) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            dbs[i] += __uint_as_float(fa[i][e] << 16) + __uint_as_float(fa[i][e] & 0xffff0000u);
      }
    }
  }
  // slab z = blockIdx.y: [N][K] then (with_db) [N]
  float* slab = slabs + (size_t)blockIdx.y * ((size_t)N * K + (with_db ? N : 0));
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + nb + 16 * i + 4 * (l >> 4) + r, k = k0 + kb + 16 * j + (l & 15);
        slab[(size_t)n * K + k] = acc[i][j][r];
      }
  if (do_db) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float v = dbs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (l < 16) slab[(size_t)N * K + n0 + nb + 16 * i + l] = v;
    }
  }
}

// NS stages of rows per workgroup; the split count follows
inline void plan(int M, int N, int K, int& rows, int& splits) {
  (void)N;
  (void)K;
  rows = NS * TM;
  splits = (M + rows - 1) / rows;
}

}  // namespace hvit_ws

using namespace hvit_ws;

// applicable shapes: bf16, N and K multiples of 64, small output, tall M
bool hvit_wgrad_small_ok(int dt, int M, int N, int K) {
  return dt == HVIT_BF16 && N % TILE == 0 && K % TILE == 0 && (long)N * K <= 256L * 512 && M >= 8 * TM &&
         M <= 4096L * NS * TM;
}

long long hvit_wgrad_small_ws(int M, int N, int K) {
  if (N % TILE || K % TILE || M <= 0) return 0;
  int rows, splits;
  plan(M, N, K, rows, splits);
  return (long long)splits * ((long long)N * K + N);
}

int hvit_sum_slabs(const float* ws, int splits, long long n, float* out, void* stream);

// dw [N][K] (and db [N] when db == dw + N*K, or NULL) from the slab reduction
int hvit_wgrad_small(const void* dy, const void* x, int M, int N, int K, float* dw, float* db, float* ws,
                     long long ws_elems, void* stream, hvit_slab_sum_t* job) {
  int rows, splits;
  plan(M, N, K, rows, splits);
  HVIT_CHECK(ws && ws_elems >= (long long)splits * ((long long)N * K + N), "hvit_wgrad_small: workspace too small");
  HVIT_CHECK(!db || db == dw + (long long)N * K, "hvit_wgrad_small: db must follow dw");
  HVIT_CHECK(aligned16(dy) && aligned16(x), "hvit_wgrad_small: alignment");
  dim3 grid((N / TILE) * (K / TILE), splits);
  hipLaunchKernelGGL(wgrad_small_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                     (const bf16_t*)x, M, N, K, rows, db ? 1 : 0, ws);
  HVIT_LAUNCH_CHECK();
  // db sits in each slab right after dW: one reduction covers [dW | db] -- or,
  // with a job, the caller's next GEMM launch sums it (epilogue side job)
  const long long n = (long long)N * K + (db ? N : 0);
  if (job) {
    *job = hvit_slab_sum_t{ws, dw, n, n, splits};
    return HVIT_OK;
  }
  return hvit_sum_slabs(ws, splits, n, dw, stream);
}
