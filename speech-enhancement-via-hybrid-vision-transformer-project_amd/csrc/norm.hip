// LayerNorm (attention.py:152-153, :271) and the BatchNorm2d -> ReLU ->
// Dropout2d -> MaxPool2d tail of ConvBlock / TransposeConvBlock
// (components.py:55-99, :144-192) for gfx950.
//
// LayerNorm: one wave per row, float4 lanes, two-pass mean/variance in
// registers.  Backward writes dx into the f32 residual-gradient stream and
// accumulates dgamma/dbeta per workgroup (64 rows) before one atomic per column.
//
// BatchNorm (train): the producing conv GEMM writes per-128-row-tile
// (mean, M2) partials; bn_finalize merges them (Chan et al.) into the batch
// mean / inverse std and updates running stats (momentum, unbiased variance)
// exactly as torch does.  bn_act_fwd applies normalise + affine + ReLU +
// per-(sample, channel) dropout mask + 2x2 max-pool in one pass over NHWC.
// Backward recomputes the pre-pool activations from z to route the pooled
// gradient to the first maximum of each window (torch's tie rule), then a
// reduce pass (sum g, sum g*xhat per channel) and an apply pass.
#include "common.h"

namespace hvit {

// ------------------------------------------------------------- LayerNorm ---
// Full-wave sum on the VALU: rotate-and-add inside each 16-lane DPP row
// (row_ror 8, 4, 2, 1), then the four row sums read out of lanes 0, 16, 32,
// 48 (the shuffle-based wave_sum is six dependent LDS permutes)
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

template <typename TY, int MAXV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                    const float* __restrict__ b, TY* __restrict__ y,
                                                    float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                    int M, int D, float eps) {
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (long)row * D;
  f32x4 v[MAXV], gv[MAXV], bv[MAXV];
  float s = 0.f;
  // every load issued up front: at B=32 the whole launch is one round of waves
  // (a row per wave), so the time is one row's latency chain, and gamma / beta
  // loaded after the two reductions were a second memory round trip
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    int c = lane * 4 + i * 256;
    v[i] = c < D ? *(const f32x4*)(xr + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
    gv[i] = c < D ? *(const f32x4*)(g + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
    bv[i] = c < D ? *(const f32x4*)(b + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  float mean = wave_sum_dpp(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    int c = lane * 4 + i * 256;
    if (c < D)
#pragma unroll
      for (int e = 0; e < 4; ++e) { float d = v[i][e] - mean; q += d * d; }
  }
  float var = wave_sum_dpp(q) / (float)D;
  float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    int c = lane * 4 + i * 256;
    if (c < D) {  // D % 4 == 0: one vector store
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[i][e] - mean) * rstd * gv[i][e] + bv[i][e];
      if constexpr (sizeof(TY) == 4) {
        *(f32x4*)((float*)y + (long)row * D + c) = o;
      } else {
        uint2 u;
        u.x = f2bf2(o[0], o[1]);
        u.y = f2bf2(o[2], o[3]);
        *(uint2*)((bf16_t*)y + (long)row * D + c) = u;
      }
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// rows per workgroup for the backward: 4 waves x RPW rows, every row of a wave
// in registers before any is reduced.  RPW = 2 (8 rows): at D = 768 four rows
// of x / dy / resid were 144 VGPRs, which left one wave per SIMD -- and at
// BASELINE config 5's M = 4096 only 256 workgroups, one per CU (17.6 % of HBM,
// round 4; 39.7 -> 17.9 us per launch with two); at D = 512 two rows per wave
// measured 22.1 -> 20.6 us per launch in-step (round 5, same-box A/B).
__host__ __device__ constexpr int lnb_rpw(int) { return 2; }
static inline int lnb_rows(int D) { return 4 * lnb_rpw(D); }

template <typename TD>
__device__ __forceinline__ f32x4 load_row4(const TD* p) {
  if constexpr (sizeof(TD) == 4) {
    return *(const f32x4*)p;
  } else {
    const uint2 u = *(const uint2*)p;
    return (f32x4){__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                   __uint_as_float(u.y & 0xffff0000u)};
  }
}

// Dropout (+ DropPath row scale) of the LayerNorm input gradient, fused into
// the backward (DROP): g = dx * keep(row * D + c) / (1 - p) * rowscale[row /
// rps] in g's dtype, and the column sums of g (the bias gradient of the GEMM
// that consumes it) -- hvit_dropout_scale's arithmetic on dx while it is in
// registers.
struct LnDrop {
  uint32_t thr = 0;
  float ds = 1.f;
  DSeed seed{0ull, nullptr};
  uint32_t site = 0;
  const float* rowscale = nullptr;
  int rps = 1;
  void* g = nullptr;
  int g_bf16 = 1;
};

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)) (+ resid);
// dgamma/dbeta partials per workgroup: written to the slab ws[blk][2][D]
// (SLAB; [blk][3][D] with DROP's column sums) and summed by a column
// reduction, else added atomically.
template <typename TD, int MAXV, bool SLAB, bool DROP = false, int RPW = 4>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const TD* __restrict__ dy, const float* __restrict__ x,
                                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                                    const float* __restrict__ g, const float* __restrict__ resid,
                                                    float* __restrict__ dx, float* __restrict__ dgamma,
                                                    float* __restrict__ dbeta, float* __restrict__ ws, int M, int D,
                                                    LnDrop dr = LnDrop()) {
  constexpr int NS = DROP ? 3 : 2;
  __shared__ float red[4][NS][MAXV * 256];
  f32x4 acs[DROP ? MAXV : 1];
  uint32_t dkey = 0;
  if constexpr (DROP) {
    if (dr.thr) dkey = rng_key((unsigned long long)dr.seed, dr.site);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) acs[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f32x4 ag[MAXV], ab[MAXV], gam[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    ag[i] = ab[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int c = lane * 4 + i * 256;
    gam[i] = c < D ? *(const f32x4*)(g + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  // all of the wave's rows are loaded before any is reduced: RPW rows x
  // (x, dy, resid) in flight per wave hide the HBM latency at this occupancy
  const int row0 = blockIdx.x * (4 * RPW) + w * RPW;
  f32x4 xv[RPW][MAXV], dv[RPW][MAXV], rv[RPW][MAXV];
  float mu[RPW], rs[RPW], rsc[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = min(row0 + r, M - 1);  // rows past M re-read the last row; never stored
    mu[r] = mean[row];
    rs[r] = rstd[row];
    rsc[r] = (DROP && dr.rowscale) ? dr.rowscale[row / dr.rps] : 1.f;  // (with the rows: no later round trip)
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane * 4 + i * 256;
      if (c < D) {
        xv[r][i] = *(const f32x4*)(x + (long)row * D + c);
        dv[r][i] = load_row4<TD>(dy + (long)row * D + c);
        rv[r][i] = resid ? *(const f32x4*)(resid + (long)row * D + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
      } else {
        xv[r][i] = dv[r][i] = rv[r][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = row0 + r;
    if (row >= M) break;  // uniform per wave
    f32x4 xh[MAXV], gy[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane * 4 + i * 256;
      if (c < D) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xhat = (xv[r][i][e] - mu[r]) * rs[r];
          xh[i][e] = xhat;
          gy[i][e] = dv[r][i][e] * gam[i][e];
          s1 += gy[i][e];
          s2 += gy[i][e] * xhat;
          ag[i][e] += dv[r][i][e] * xhat;
          ab[i][e] += dv[r][i][e];
        }
      }
    }
    s1 = wave_sum_dpp(s1) / (float)D;
    s2 = wave_sum_dpp(s2) / (float)D;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane * 4 + i * 256;
      if (c < D) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rs[r] * (gy[i][e] - s1 - xh[i][e] * s2);
        o += rv[r][i];
        *(f32x4*)(dx + (long)row * D + c) = o;
        if constexpr (DROP) {
          f32x4 k = {dr.ds, dr.ds, dr.ds, dr.ds};
          if (dr.thr) k = keep4_at(dkey, (uint64_t)row * D + c, dr.thr, dr.ds);
          const f32x4 gv = o * k * rsc[r];
          if (dr.g_bf16) {
            *(uint2*)((bf16_t*)dr.g + (long)row * D + c) = make_uint2(f2bf2(gv[0], gv[1]), f2bf2(gv[2], gv[3]));
          } else {
            *(f32x4*)((float*)dr.g + (long)row * D + c) = gv;
          }
          acs[i] += gv;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane * 4 + i * 256;
    if (c < D) {
      *(f32x4*)&red[w][0][c] = ag[i];
      *(f32x4*)&red[w][1][c] = ab[i];
      if constexpr (DROP) *(f32x4*)&red[w][2][c] = acs[i];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const float a = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
      if (SLAB) ws[(size_t)blockIdx.x * NS * D + k * D + c] = a;
      else atomicAdd((k == 0 ? dgamma : k == 1 ? dbeta : dgamma + 2 * D) + c, a);
    }
  }
}

// dgamma[c] / dbeta[c] = column sums of the slab ws[nblk][2D]; a block owns 64
// columns, its 4 waves split the slab rows, folded through LDS
__global__ __launch_bounds__(256) void ln_slab_sum_kernel(const float* __restrict__ ws, int nblk, int D,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float part[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f;
  if (col < 2 * D) {
    int k = w;
    for (; k + 4 < nblk; k += 8) {
      s0 += ws[(size_t)k * 2 * D + col];
      s1 += ws[(size_t)(k + 4) * 2 * D + col];
    }
    for (; k < nblk; k += 4) s0 += ws[(size_t)k * 2 * D + col];
  }
  part[w][threadIdx.x & 63] = s0 + s1;
  __syncthreads();
  if (w == 0 && col < 2 * D) {
    const float t = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
    if (col < D) dgamma[col] = t;
    else dbeta[col - D] = t;
  }
}

// ------------------------------------------------------------- BatchNorm ---
// partials[t][c] = (mean, M2) over cnt_t rows; cnt_t = tile_rows except the last.
// Two levels, both in a fixed order (deterministic) with coalesced reads and
// short dependent chains (a Chan merge is a division deep):
//  1. bn_merge_chunks: workgroup (64 channels, chunk of BNF_CHUNK tiles), thread
//     (channel, group g) loads tiles g, g + 4, ... of the chunk up front (each
//     tile row of 64 channels is one 512-B read) and Chan-merges them in order;
//     the 4 groups are merged in order through LDS; the chunk's (mean, M2)
//     overwrites the chunk's first tile slot (read only by this workgroup, and
//     only before the merge).
//  2. bn_final: workgroup (64 channels), thread (channel, group g of 16) merges
//     chunks g, g + 16, ... in order, the 16 groups in order through LDS, then the
//     batch statistics and the running-stat update (momentum, unbiased var).
// (Round 4's first form -- 128-tile chunks, one thread per channel walking all
// chunk results -- ran 64-256 workgroups with 32- and 128-deep chains: 13.6 +
// 8.2 us per call; a single level with C-strided loads took ~12 us.)
constexpr int BNF_CHUNK = 32;
constexpr int BNF_G1 = 4;   // tile groups per chunk workgroup (BNF_CHUNK / BNF_G1 tiles per thread)
constexpr int BNF_G2 = 16;  // chunk groups of the final workgroup

__device__ __forceinline__ void chan_merge(float& n, float& mu, float& m2, float nb, float mb, float qb) {
  if (nb <= 0.f) return;
  const float nn = n + nb;
  const float d = mb - mu;
  mu += d * (nb / nn);
  m2 += qb + d * d * (n * nb / nn);
  n = nn;
}

__global__ __launch_bounds__(64 * BNF_G1) void bn_merge_chunks_kernel(float* __restrict__ part, int ntiles,
                                                                      int tile_rows, long M, int C) {
  constexpr int PER = BNF_CHUNK / BNF_G1;
  __shared__ float sn[BNF_G1][64], sm[BNF_G1][64], sq[BNF_G1][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int t0 = blockIdx.y * BNF_CHUNK;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (c < C) {
    float2 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int t = t0 + g + BNF_G1 * i;
      v[i] = t < ntiles ? *(const float2*)(part + ((long)t * C + c) * 2) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const long t = t0 + g + BNF_G1 * i;
      const float nb = t < ntiles ? (float)min((long)tile_rows, M - t * tile_rows) : 0.f;
      chan_merge(n, mu, m2, nb, v[i].x, v[i].y);
    }
  }
  sn[g][cl] = n;
  sm[g][cl] = mu;
  sq[g][cl] = m2;
  __syncthreads();
  if (g == 0 && c < C) {
#pragma unroll
    for (int k = 1; k < BNF_G1; ++k) chan_merge(n, mu, m2, sn[k][cl], sm[k][cl], sq[k][cl]);
    *(float2*)(part + ((long)t0 * C + c) * 2) = make_float2(mu, m2);
  }
}

__global__ __launch_bounds__(64 * BNF_G2) void bn_final_kernel(const float* __restrict__ part, int ntiles,
                                                               int tile_rows, long M, int C,
                                                               float* __restrict__ mean_out,
                                                               float* __restrict__ invstd_out,
                                                               float* __restrict__ rmean, float* __restrict__ rvar,
                                                               float momentum, float eps, long long* nbt) {
  __shared__ float sn[BNF_G2][64], sm[BNF_G2][64], sq[BNF_G2][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int nch = (ntiles + BNF_CHUNK - 1) / BNF_CHUNK;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (c < C)
    for (int k = g; k < nch; k += BNF_G2) {
      const long t0 = (long)k * BNF_CHUNK;
      const float rows = (float)min((long)BNF_CHUNK * tile_rows, M - t0 * tile_rows);
      const float2 v = *(const float2*)(part + (t0 * C + c) * 2);
      chan_merge(n, mu, m2, rows, v.x, v.y);
    }
  sn[g][cl] = n;
  sm[g][cl] = mu;
  sq[g][cl] = m2;
  __syncthreads();
  if (g == 0 && c < C) {
#pragma unroll
    for (int k = 1; k < BNF_G2; ++k) chan_merge(n, mu, m2, sn[k][cl], sm[k][cl], sq[k][cl]);
    const float var = m2 / (float)M;
    mean_out[c] = mu;
    invstd_out[c] = rsqrtf(var + eps);
    if (rmean) {
      const float unb = M > 1 ? m2 / (float)(M - 1) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
}

__global__ void bn_eval_prep_kernel(const float* rmean, const float* rvar, int C, float eps, float* mean_out,
                                    float* invstd_out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) {
    mean_out[c] = rmean[c];
    invstd_out[c] = rsqrtf(rvar[c] + eps);
  }
}


static int grid_for(long n) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace hvit

using namespace hvit;

extern "C" int hvit_layernorm_fwd(const float* x, const float* gamma, const float* beta, int M, int D,
                                  float eps, void* y, int y_dt, float* mean, float* rstd, void* stream) {
  HVIT_CHECK(x && gamma && beta && y && mean && rstd, "hvit_layernorm_fwd: null pointer");
  HVIT_CHECK(D % 4 == 0 && D <= 1024 && D > 0, "hvit_layernorm_fwd: D=%d must be a multiple of 4, <= 1024", D);
  HVIT_CHECK(aligned16(x) && aligned16(gamma) && aligned16(beta) && aligned16(y),
             "hvit_layernorm_fwd: x, gamma, beta, y must be 16-byte aligned");
  if (M <= 0) return HVIT_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 g(cdiv(M, 4));
#define LNF(TY, V) hipLaunchKernelGGL((ln_fwd_kernel<TY, V>), g, dim3(256), 0, st, x, gamma, beta, (TY*)y, mean, rstd, M, D, eps)
  if (y_dt == HVIT_F32) {
    if (D <= 256) LNF(float, 1); else if (D <= 512) LNF(float, 2); else if (D <= 768) LNF(float, 3); else LNF(float, 4);
  } else {
    if (D <= 256) LNF(bf16_t, 1); else if (D <= 512) LNF(bf16_t, 2); else if (D <= 768) LNF(bf16_t, 3); else LNF(bf16_t, 4);
  }
#undef LNF
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" long long hvit_layernorm_bwd_ws_elems(int M, int D) {
  return M > 0 ? (long long)cdiv(M, lnb_rows(D)) * 2 * D : 0;
}

extern "C" int hvit_layernorm_bwd(const void* dy, int dy_dt, const float* x, const float* mean,
                                  const float* rstd, const float* gamma, int M, int D, const float* resid,
                                  float* dx, float* dgamma, float* dbeta, float* ws, long long ws_elems,
                                  int flags, void* stream) {
  HVIT_CHECK(dy && x && mean && rstd && gamma && dx && dgamma && dbeta, "hvit_layernorm_bwd: null pointer");
  HVIT_CHECK(D % 4 == 0 && D <= 1024 && D > 0, "hvit_layernorm_bwd: bad D=%d", D);
  HVIT_CHECK(aligned16(x) && aligned16(dx) && aligned16(gamma) && aligned16(dy) && (!resid || aligned16(resid)),
             "hvit_layernorm_bwd: alignment");
  hipStream_t st = (hipStream_t)stream;
  const int nblk = cdiv(M, lnb_rows(D));
  const bool slab = M > 0 && ws && ws_elems >= hvit_layernorm_bwd_ws_elems(M, D);
  if (!slab && !(flags & HVIT_ACC_ZEROED)) {
    (void)hipMemsetAsync(dgamma, 0, sizeof(float) * D, st);
    (void)hipMemsetAsync(dbeta, 0, sizeof(float) * D, st);
  }
  if (M <= 0) return HVIT_OK;
  dim3 g(nblk);
#define LNB(TD, V)                                                                                                \
  do {                                                                                                            \
    constexpr int R_ = lnb_rpw(V * 256);                                                                          \
    if (slab)                                                                                                     \
      hipLaunchKernelGGL((ln_bwd_kernel<TD, V, true, false, R_>), g, dim3(256), 0, st, (const TD*)dy, x, mean,    \
                         rstd, gamma, resid, dx, dgamma, dbeta, ws, M, D, LnDrop());                              \
    else                                                                                                          \
      hipLaunchKernelGGL((ln_bwd_kernel<TD, V, false, false, R_>), g, dim3(256), 0, st, (const TD*)dy, x, mean,   \
                         rstd, gamma, resid, dx, dgamma, dbeta, ws, M, D, LnDrop());                              \
  } while (0)
  if (dy_dt == HVIT_F32) {
    if (D <= 256) LNB(float, 1); else if (D <= 512) LNB(float, 2); else if (D <= 768) LNB(float, 3); else LNB(float, 4);
  } else {
    if (D <= 256) LNB(bf16_t, 1); else if (D <= 512) LNB(bf16_t, 2); else if (D <= 768) LNB(bf16_t, 3); else LNB(bf16_t, 4);
  }
#undef LNB
  HVIT_LAUNCH_CHECK();
  if (slab) {
    if (dbeta == dgamma + D)  // [dgamma | dbeta] contiguous: one column reduction of the [nblk][2D] slab
      return hvit_reduce_rows(ws, HVIT_F32, nblk, 2 * D, 2 * D, (flags & HVIT_ACC_ZEROED) ? 1 : 0, dgamma, stream);
    hipLaunchKernelGGL(ln_slab_sum_kernel, dim3(cdiv(2 * D, 64)), dim3(256), 0, st, ws, nblk, D, dgamma, dbeta);
    HVIT_LAUNCH_CHECK();
  }
  return HVIT_OK;
}

extern "C" long long hvit_layernorm_bwd_drop_ws_elems(int M, int D) {
  return M > 0 ? (long long)cdiv(M, lnb_rows(D)) * 3 * D : 0;
}

// hvit_layernorm_bwd + the dropout / DropPath scaling of its output (see LnDrop)
extern "C" int hvit_layernorm_bwd_drop(const void* dy, int dy_dt, const float* x, const float* mean,
                                       const float* rstd, const float* gamma, int M, int D, const float* resid,
                                       float* dx, float* acc3, const hvit_dropout_t* dropout, const float* rowscale,
                                       int rows_per_sample, void* g_out, int g_dt, float* ws, long long ws_elems,
                                       int flags, void* stream) {
  HVIT_CHECK(dy && x && mean && rstd && gamma && dx && acc3 && g_out && ws, "hvit_layernorm_bwd_drop: null pointer");
  HVIT_CHECK(D % 4 == 0 && D <= 1024 && D > 0, "hvit_layernorm_bwd_drop: bad D=%d", D);
  HVIT_CHECK(aligned16(x) && aligned16(dx) && aligned16(gamma) && aligned16(dy) && aligned16(g_out) &&
                 (!resid || aligned16(resid)),
             "hvit_layernorm_bwd_drop: alignment");
  HVIT_CHECK(ws_elems >= hvit_layernorm_bwd_drop_ws_elems(M, D), "hvit_layernorm_bwd_drop: workspace too small");
  HVIT_CHECK(!rowscale || rows_per_sample > 0, "hvit_layernorm_bwd_drop: rows_per_sample");
  HVIT_CHECK(g_dt == HVIT_BF16 || g_dt == HVIT_F32, "hvit_layernorm_bwd_drop: g dtype");
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0) return HVIT_OK;
  const int nblk = cdiv(M, lnb_rows(D));
  LnDrop d;
  d.thr = dropout ? drop_threshold(dropout->p) : 0;
  d.ds = (dropout && dropout->p > 0.f) ? 1.f / (1.f - dropout->p) : 1.f;
  d.seed = dseed(dropout);
  d.site = dropout ? dropout->site : 0u;
  d.rowscale = rowscale;
  d.rps = rows_per_sample > 0 ? rows_per_sample : 1;
  d.g = g_out;
  d.g_bf16 = g_dt == HVIT_BF16;
  dim3 g(nblk);
#define LNBD(TD, V)                                                                                              \
  hipLaunchKernelGGL((ln_bwd_kernel<TD, V, true, true, lnb_rpw(V * 256)>), g, dim3(256), 0, st, (const TD*)dy, x,   \
                     mean, rstd, gamma, resid, dx, acc3, acc3 + D, ws, M, D, d)
  if (dy_dt == HVIT_F32) {
    if (D <= 256) LNBD(float, 1); else if (D <= 512) LNBD(float, 2); else if (D <= 768) LNBD(float, 3); else LNBD(float, 4);
  } else {
    if (D <= 256) LNBD(bf16_t, 1); else if (D <= 512) LNBD(bf16_t, 2); else if (D <= 768) LNBD(bf16_t, 3); else LNBD(bf16_t, 4);
  }
#undef LNBD
  HVIT_LAUNCH_CHECK();
  if (flags & HVIT_ACC_DEFER) return HVIT_OK;  // the caller sums the partial rows (a later launch's side job)
  // one column reduction of the [nblk][3D] slab into [dgamma | dbeta | colsum]
  return hvit_reduce_rows(ws, HVIT_F32, nblk, 3 * D, 3 * D, (flags & HVIT_ACC_ZEROED) ? 1 : 0, acc3, stream);
}

extern "C" int hvit_bn_finalize(float* partials, int ntiles, int tile_rows, long long M, int C,
                                float* mean, float* invstd, float* running_mean, float* running_var,
                                long long* num_batches_tracked, float momentum, float eps, void* stream) {
  HVIT_CHECK(partials && mean && invstd, "hvit_bn_finalize: null pointer");
  HVIT_CHECK(M > 0 && C > 0 && ntiles > 0, "hvit_bn_finalize: bad sizes");
  HVIT_CHECK((running_mean == nullptr) == (running_var == nullptr), "hvit_bn_finalize: running stats pair");
  hipStream_t st = (hipStream_t)stream;
  // (the partials buffer is the first level's scratch: overwritten)
  hipLaunchKernelGGL(bn_merge_chunks_kernel, dim3(cdiv(C, 64), cdiv(ntiles, BNF_CHUNK)), dim3(64 * BNF_G1), 0, st,
                     (float*)partials, ntiles, tile_rows, (long)M, C);
  HVIT_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_final_kernel, dim3(cdiv(C, 64)), dim3(64 * BNF_G2), 0, st, partials, ntiles, tile_rows,
                     (long)M, C, mean, invstd, running_mean, running_var, momentum, eps, num_batches_tracked);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_bn_eval_prep(const float* running_mean, const float* running_var, int C, float eps,
                                 float* mean, float* invstd, void* stream) {
  HVIT_CHECK(running_mean && running_var && mean && invstd, "hvit_bn_eval_prep: null pointer");
  hipLaunchKernelGGL(bn_eval_prep_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream,
                     running_mean, running_var, C, eps, mean, invstd);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

