// BatchNorm2d -> ReLU -> Dropout2d -> MaxPool2d(pool) tail of ConvBlock /
// TransposeConvBlock (components.py:67-85, :161-178 of the reference) on NHWC
// activations, gfx950.
//
// One thread owns one pooling window x 16 bytes of channels (8 bf16 / 4 f32),
// so every z / y / dy / dz access is a coalesced 16-byte vector and the window
// is read once.  The backward recomputes relu(bn(z)) for the window, routes the
// pooled gradient to the first maximum in scan order (torch's max_pool2d tie
// rule; positions outside full windows get zero), applies the per-(sample,
// channel) dropout mask and relu', then
//   reduce pass: sums[0][c] = sum g, sums[1][c] = sum g * xhat  (dbeta, dgamma)
//   apply pass : dz = gamma * invstd * (g - sum g / M - xhat * sum g*xhat / M)
// Window / pixel indices stay in 32 bits.
#include <algorithm>

#include "common.h"

namespace hvit {

// partial rows of the backward sums: one per workgroup of the sums kernel
// (plain stores, summed in row order by a deterministic column reduction), so
// the sums grid is capped at BN_PART_ROWS
constexpr int BN_PART_ROWS = 1024;

template <typename T>
struct V16 {  // 16 bytes of T as floats
  static constexpr int N = 16 / sizeof(T);
  __device__ __forceinline__ static void load(const T* p, float* f) {
    u32x4 u = *(const u32x4*)p;
    const T* e = (const T*)&u;
#pragma unroll
    for (int i = 0; i < N; ++i) f[i] = Elem<T>::to_f(e[i]);
  }
  __device__ __forceinline__ static void store(T* p, const float* f) {
    T e[N];
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = Elem<T>::from_f(f[i]);
    *(u32x4*)p = *(const u32x4*)e;
  }
};

struct BnArgs {
  int N, H, W, C, pool;
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  uint32_t thr;
  float dscale;
  uint32_t key;  // rng_key(seed, site) (host-resolved when seedp is NULL)
  const unsigned long long* seedp;  // device seed word (hvit_dropout_t.seed_ptr)
  unsigned long long seed;
  uint32_t site;
  // index divisors: channel groups, full windows (Wo, Ho), all windows (Ww, Hw)
  FastDiv fG, fWo, fHo, fWw, fHw;
  // at kernel entry: fold in the device seed word (one scalar load)
  __device__ __forceinline__ void resolve() {
    if (seedp && thr) key = rng_key(seed ^ *seedp, site);
  }
};

// CV per-channel constants p[c .. c+CV-1] as 16-byte vector loads (c is a
// multiple of CV): scalar loads of them came out serialised one round trip
// each (48 of them in the apply pass), a ~20 us floor on every launch
template <int CV>
__device__ __forceinline__ void load_cv(const float* __restrict__ p, int c, float* out) {
#pragma unroll
  for (int v = 0; v < CV / 4; ++v) {
    const f32x4 x = *(const f32x4*)(p + c + 4 * v);
#pragma unroll
    for (int e = 0; e < 4; ++e) out[4 * v + e] = x[e];
  }
}

// Dropout2d multipliers of channels c .. c+CV-1 of sample n (element index
// n*C + c, a multiple of 4: two pair hashes per four channels)
template <int CV>
__device__ __forceinline__ void drop_mask(const BnArgs& a, int n, int c, float* m) {
  if (!a.thr) {
#pragma unroll
    for (int e = 0; e < CV; ++e) m[e] = 1.f;
    return;
  }
  const uint64_t i0 = (uint64_t)n * a.C + c;
#pragma unroll
  for (int e4 = 0; e4 < CV; e4 += 4) {
    const f32x4 k = keep4_at(a.key, i0 + e4, a.thr, a.dscale);
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e4 + e] = k[e];
  }
}

// forward: y[n, oy, ox, c..] over full windows
template <typename T, typename TO>
__global__ __launch_bounds__(256) void bnact_fwd_kernel(const T* __restrict__ z, TO* __restrict__ y, BnArgs a_) {
  BnArgs a = a_;
  a.resolve();
  constexpr int CV = V16<T>::N;
  const int G = a.C / CV;
  const int Ho = a.H / a.pool, Wo = a.W / a.pool;
  const int total = a.N * Ho * Wo * G;
  // a thread's channel group never changes (256 % G == 0, grid stride % G == 0)
  const int c = ((blockIdx.x * blockDim.x + threadIdx.x) % G) * CV;
  float sc[CV], sh[CV], mu_[CV], is_[CV], ga_[CV], be_[CV];
  load_cv<CV>(a.mean, c, mu_);
  load_cv<CV>(a.invstd, c, is_);
  load_cv<CV>(a.gamma, c, ga_);
  load_cv<CV>(a.beta, c, be_);
#pragma unroll
  for (int e = 0; e < CV; ++e) {
    sc[e] = is_[e] * ga_[e];
    sh[e] = be_[e] - mu_[e] * sc[e];
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int t = a.fG.div(i);
    const int t1 = a.fWo.div(t);
    const int ox = t - t1 * Wo;
    const int n = a.fHo.div(t1);
    const int oy = t1 - n * Ho;
    float best[CV];
#pragma unroll
    for (int e = 0; e < CV; ++e) best[e] = 0.f;  // relu output >= 0
    for (int dy = 0; dy < a.pool; ++dy)
      for (int dx = 0; dx < a.pool; ++dx) {
        float v[CV];
        V16<T>::load(z + ((size_t)(n * a.H + oy * a.pool + dy) * a.W + ox * a.pool + dx) * a.C + c, v);
#pragma unroll
        for (int e = 0; e < CV; ++e) best[e] = fmaxf(best[e], __builtin_fmaf(v[e], sc[e], sh[e]));
      }
    float m[CV];
    drop_mask<CV>(a, n, c, m);
    float o[CV];
#pragma unroll
    for (int e = 0; e < CV; ++e) o[e] = best[e] * m[e];
    TO* dst = y + ((size_t)(n * Ho + oy) * Wo + ox) * a.C + c;
    if constexpr (sizeof(TO) == sizeof(T)) {
      V16<TO>::store(dst, o);
    } else {
#pragma unroll
      for (int e = 0; e < CV; ++e) dst[e] = Elem<TO>::from_f(o[e]);
    }
  }
}

// backward: APPLY = false -> per-channel sums; APPLY = true -> dz.  The
// window values are formed with one explicit fma each (forward, reduce and
// apply alike): equal inputs must give equal values so that a tie routes to
// the first maximum, as torch's max-pool does (compiler-chosen contraction
// made tied bf16 inputs differ by an ulp and move the gradient)
template <typename T, typename TD, bool APPLY>
__global__ __launch_bounds__(256) void bnact_bwd_kernel(const T* __restrict__ z, const TD* __restrict__ dy,
                                                       BnArgs a_, float* __restrict__ sums, int training,
                                                       T* __restrict__ dz) {
  BnArgs a = a_;
  a.resolve();
  constexpr int CV = V16<T>::N;
  constexpr int MAXW = 4;  // pool <= 2
  __shared__ float red[2][256][CV];
  const int G = a.C / CV;
  const int P = a.pool;
  const int Ho = a.H / P, Wo = a.W / P;
  const int Hw = (a.H + P - 1) / P, Ww = (a.W + P - 1) / P;
  const int total = a.N * Hw * Ww * G;
  const float invM = 1.f / (float)(a.N * a.H * a.W);
  float acc1[CV], acc2[CV];
#pragma unroll
  for (int e = 0; e < CV; ++e) acc1[e] = acc2[e] = 0.f;
  // a thread's channel group never changes (256 % G == 0, grid stride % G == 0):
  // per-channel constants are loaded once
  const int c = ((blockIdx.x * blockDim.x + threadIdx.x) % G) * CV;
  // sc, sh: relu(bn(z)) = max(z*sc + sh, 0).  Reduce pass: xhat = (z - mu)*is.
  // Apply pass (training): dz = sc*(g - s1 - xhat*s2) = sc*g + ca + cb*z.
  float sc[CV], sh[CV], mu[CV], is[CV], ca[CV], cb[CV], ga_[CV], be_[CV], s1v[CV], s2v[CV];
  load_cv<CV>(a.mean, c, mu);
  load_cv<CV>(a.invstd, c, is);
  load_cv<CV>(a.gamma, c, ga_);
  load_cv<CV>(a.beta, c, be_);
  load_cv<CV>(sums, c, s1v);        // (reduce pass: zeroed accumulators, unused)
  load_cv<CV>(sums + a.C, c, s2v);
  const bool use_s = APPLY && training;
#pragma unroll
  for (int e = 0; e < CV; ++e) {
    sc[e] = is[e] * ga_[e];
    sh[e] = be_[e] - mu[e] * sc[e];
    const float s1 = use_s ? s1v[e] * invM : 0.f;
    const float s2 = use_s ? s2v[e] * invM : 0.f;
    cb[e] = -sc[e] * s2 * is[e];
    ca[e] = -sc[e] * s1 - cb[e] * mu[e];
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int t = a.fG.div(i);
    const int t1 = a.fWw.div(t);
    const int wx = t - t1 * Ww;
    const int n = a.fHw.div(t1);
    const int wy = t1 - n * Hw;
    // window values
    float zv[MAXW][CV];
    bool inb[MAXW];
#pragma unroll
    for (int q = 0; q < MAXW; ++q) {
      const int y = wy * P + (q >> 1), x = wx * P + (q & 1);
      inb[q] = (q < P * P) && (P == 2 || q == 0) && y < a.H && x < a.W;
      if (inb[q]) V16<T>::load(z + ((size_t)(n * a.H + y) * a.W + x) * a.C + c, zv[q]);
    }
    const bool full = wy < Ho && wx < Wo;
    // routed gradient: gv[e] at window position arg[e] (first maximum), 0 elsewhere
    int arg[CV];
    float gv[CV];
#pragma unroll
    for (int e = 0; e < CV; ++e) {
      arg[e] = 0;
      gv[e] = 0.f;
    }
    if (full) {
      float d[CV], m[CV];
      const TD* dp = dy + ((size_t)(n * Ho + wy) * Wo + wx) * a.C + c;
      if constexpr (sizeof(TD) == sizeof(T)) {
        V16<TD>::load(dp, d);
      } else {
#pragma unroll
        for (int e = 0; e < CV; ++e) d[e] = Elem<TD>::to_f(dp[e]);
      }
      drop_mask<CV>(a, n, c, m);
#pragma unroll
      for (int e = 0; e < CV; ++e) {
        float best = fmaxf(__builtin_fmaf(zv[0][e], sc[e], sh[e]), 0.f);
#pragma unroll
        for (int q = 1; q < MAXW; ++q) {
          if (!inb[q]) continue;
          const float v = fmaxf(__builtin_fmaf(zv[q][e], sc[e], sh[e]), 0.f);
          if (v > best) {
            best = v;
            arg[e] = q;
          }
        }
        gv[e] = best > 0.f ? d[e] * m[e] : 0.f;
      }
    }
    if (!APPLY) {
      if (full) {
#pragma unroll
        for (int e = 0; e < CV; ++e) {
          float zr = zv[0][e];
#pragma unroll
          for (int q = 1; q < MAXW; ++q) zr = arg[e] == q ? zv[q][e] : zr;
          acc1[e] += gv[e];
          acc2[e] += gv[e] * ((zr - mu[e]) * is[e]);
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < MAXW; ++q) {
        if (!inb[q]) continue;
        float o[CV];
#pragma unroll
        for (int e = 0; e < CV; ++e) {
          const float gq = arg[e] == q ? gv[e] : 0.f;
          o[e] = training ? sc[e] * gq + ca[e] + cb[e] * zv[q][e] : sc[e] * gq;
        }
        const int y = wy * P + (q >> 1), x = wx * P + (q & 1);
        V16<T>::store(dz + ((size_t)(n * a.H + y) * a.W + x) * a.C + c, o);
      }
    }
  }
  if (!APPLY) {
    // every thread of a block keeps one channel group (256 % G == 0 and the
    // grid stride is a multiple of G); reduce across the block, one atomic each
#pragma unroll
    for (int e = 0; e < CV; ++e) {
      red[0][threadIdx.x][e] = acc1[e];
      red[1][threadIdx.x][e] = acc2[e];
    }
    __syncthreads();
    if (threadIdx.x < G) {
      float t1[CV], t2[CV];
#pragma unroll
      for (int e = 0; e < CV; ++e) t1[e] = t2[e] = 0.f;
      for (int k = threadIdx.x; k < 256; k += G)
#pragma unroll
        for (int e = 0; e < CV; ++e) {
          t1[e] += red[0][k][e];
          t2[e] += red[1][k][e];
        }
      // this workgroup's partial row (deterministic: no atomics)
      float* slot = sums + 2 * a.C * (1 + blockIdx.x);
      const int cc = threadIdx.x * CV;
#pragma unroll
      for (int e = 0; e < CV; ++e) {
        slot[cc + e] = t1[e];
        slot[a.C + cc + e] = t2[e];
      }
    }
  }
}

// backward reduce pass (both modes): per-channel sums of the routed gradient g
// and of g * xhat over full pooling windows.  Software-pipelined: the next
// window's z taps and dy are loaded (raw) before the current one is reduced,
// so every thread keeps two windows of loads in flight.
template <typename T>
__device__ __forceinline__ float raw_elem(const u32x4& u, int e) {
  if constexpr (sizeof(T) == 2) return __uint_as_float((e & 1) ? (u[e >> 1] & 0xffff0000u) : (u[e >> 1] << 16));
  else return __uint_as_float(u[e]);
}

template <typename T, typename TD>
__global__ __launch_bounds__(256) void bnact_sums_kernel(const T* __restrict__ z, const TD* __restrict__ dy,
                                                        BnArgs a_, float* __restrict__ sums) {
  BnArgs a = a_;
  a.resolve();
  constexpr int CV = V16<T>::N;
  constexpr int MAXW = 4;  // pool <= 2
  __shared__ float red[2][256][CV];
  const int G = a.C / CV;
  const int P = a.pool;
  const int Ho = a.H / P, Wo = a.W / P;
  const int total = a.N * Ho * Wo * G;  // full windows only
  const int c = ((blockIdx.x * blockDim.x + threadIdx.x) % G) * CV;
  float sc[CV], sh[CV], mu[CV], is[CV], acc1[CV], acc2[CV], ga_[CV], be_[CV];
  load_cv<CV>(a.mean, c, mu);
  load_cv<CV>(a.invstd, c, is);
  load_cv<CV>(a.gamma, c, ga_);
  load_cv<CV>(a.beta, c, be_);
#pragma unroll
  for (int e = 0; e < CV; ++e) {
    sc[e] = is[e] * ga_[e];
    sh[e] = be_[e] - mu[e] * sc[e];
    acc1[e] = acc2[e] = 0.f;
  }
  struct Item {
    u32x4 zr[MAXW];
    float d[CV];
    int n;
  };
  auto load = [&](int i, Item& it) {
    if (i >= total) return;
    const int t = a.fG.div(i);
    const int t1 = a.fWo.div(t);
    const int wx = t - t1 * Wo;
    it.n = a.fHo.div(t1);
    const int wy = t1 - it.n * Ho;
#pragma unroll
    for (int q = 0; q < MAXW; ++q)
      if (q < P * P)
        it.zr[q] = *(const u32x4*)(z + ((size_t)(it.n * a.H + wy * P + (q >> 1)) * a.W + wx * P + (q & 1)) * a.C + c);
    const TD* dp = dy + ((size_t)(it.n * Ho + wy) * Wo + wx) * a.C + c;
    if constexpr (sizeof(TD) == sizeof(T)) {
      V16<TD>::load(dp, it.d);
    } else {
#pragma unroll
      for (int e = 0; e < CV; ++e) it.d[e] = Elem<TD>::to_f(dp[e]);
    }
  };
  auto reduce = [&](const Item& it) {
    float m[CV];
    drop_mask<CV>(a, it.n, c, m);
#pragma unroll
    for (int e = 0; e < CV; ++e) {
      float zs = raw_elem<T>(it.zr[0], e);
      float best = fmaxf(__builtin_fmaf(zs, sc[e], sh[e]), 0.f);
#pragma unroll
      for (int q = 1; q < MAXW; ++q) {
        if (q >= P * P) break;
        const float zq = raw_elem<T>(it.zr[q], e);
        const float v = fmaxf(__builtin_fmaf(zq, sc[e], sh[e]), 0.f);
        if (v > best) {  // first maximum wins ties (torch's max-pool routing)
          best = v;
          zs = zq;
        }
      }
      const float gv = best > 0.f ? it.d[e] * m[e] : 0.f;
      acc1[e] += gv;
      acc2[e] += gv * ((zs - mu[e]) * is[e]);
    }
  };
  const int stride = gridDim.x * blockDim.x;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  Item cur;
  load(i, cur);
  for (; i < total; i += stride) {
    Item nxt;
    load(i + stride, nxt);
    reduce(cur);
    cur = nxt;
  }
#pragma unroll
  for (int e = 0; e < CV; ++e) {
    red[0][threadIdx.x][e] = acc1[e];
    red[1][threadIdx.x][e] = acc2[e];
  }
  __syncthreads();
  if (threadIdx.x < G) {
    float t1[CV], t2[CV];
#pragma unroll
    for (int e = 0; e < CV; ++e) t1[e] = t2[e] = 0.f;
    for (int k = threadIdx.x; k < 256; k += G)
#pragma unroll
      for (int e = 0; e < CV; ++e) {
        t1[e] += red[0][k][e];
        t2[e] += red[1][k][e];
      }
    float* slot = sums + 2 * a.C * (1 + blockIdx.x);  // this workgroup's partial row (no atomics)
    const int cc = threadIdx.x * CV;
#pragma unroll
    for (int e = 0; e < CV; ++e) {
      slot[cc + e] = t1[e];
      slot[a.C + cc + e] = t2[e];
    }
  }
}


// grid-stride launches; per-kernel caps measured on the B=32 encoder shapes
// (fewer, longer-lived workgroups stream better here than one item per thread)
static int grid_for(long n, long cap) {
  long g = (n + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}
constexpr long BN_GRID_FWD = 2048, BN_GRID_SUMS = BN_PART_ROWS, BN_GRID_APPLY = 1024;

static int make_args(BnArgs& a, int N, int H, int W, int C, int pool, const float* mean, const float* invstd,
                     const float* gamma, const float* beta, const hvit_dropout_t* dr, int cv) {
  HVIT_CHECK(mean && invstd && gamma && beta, "bn_act: null statistics / affine pointer");
  HVIT_CHECK(aligned16(mean) && aligned16(invstd) && aligned16(gamma) && aligned16(beta),
             "bn_act: statistics / affine vectors must be 16-byte aligned");
  HVIT_CHECK(pool == 1 || pool == 2, "bn_act: pool must be 1 or 2");
  HVIT_CHECK(C > 0 && C % cv == 0 && (C / cv) <= 256 && (256 % (C / cv)) == 0,
             "bn_act: C=%d must be a multiple of %d with C/%d dividing 256", C, cv, cv);
  HVIT_CHECK((long)N * H * W * C < (1L << 31), "bn_act: tensor too large for 32-bit indexing");
  a.N = N; a.H = H; a.W = W; a.C = C; a.pool = pool;
  a.mean = mean; a.invstd = invstd; a.gamma = gamma; a.beta = beta;
  a.thr = dr ? drop_threshold(dr->p) : 0;
  a.dscale = (dr && dr->p > 0.f) ? 1.f / (1.f - dr->p) : 1.f;
  a.key = dr ? rng_key(dr->seed, dr->site) : 0u;
  a.seedp = dr ? dr->seed_ptr : nullptr;
  a.seed = dr ? dr->seed : 0ull;
  a.site = dr ? dr->site : 0u;
  a.fG = FastDiv(C / cv);
  a.fWo = FastDiv(std::max(1, W / pool));
  a.fHo = FastDiv(std::max(1, H / pool));
  a.fWw = FastDiv((W + pool - 1) / pool);
  a.fHw = FastDiv((H + pool - 1) / pool);
  return HVIT_OK;
}

}  // namespace hvit

using namespace hvit;

extern "C" int hvit_bn_act_fwd(int dt, const void* z, int N, int H, int W, int C, const float* mean,
                               const float* invstd, const float* gamma, const float* beta,
                               const hvit_dropout_t* dropout2d, int pool, void* y, int y_dt, void* stream) {
  HVIT_CHECK(z && y, "hvit_bn_act_fwd: null pointer");
  HVIT_CHECK(aligned16(z) && aligned16(y), "hvit_bn_act_fwd: alignment");
  BnArgs a;
  const int cv = dt == HVIT_BF16 ? 8 : 4;
  if (int rc = make_args(a, N, H, W, C, pool, mean, invstd, gamma, beta, dropout2d, cv)) return rc;
  const long total = (long)N * (H / pool) * (W / pool) * (C / cv);
  if (total <= 0) return HVIT_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 g(grid_for(total, BN_GRID_FWD));
  if (dt == HVIT_BF16 && y_dt == HVIT_BF16)
    hipLaunchKernelGGL((bnact_fwd_kernel<bf16_t, bf16_t>), g, dim3(256), 0, st, (const bf16_t*)z, (bf16_t*)y, a);
  else if (dt == HVIT_BF16)
    hipLaunchKernelGGL((bnact_fwd_kernel<bf16_t, float>), g, dim3(256), 0, st, (const bf16_t*)z, (float*)y, a);
  else if (y_dt == HVIT_F32)
    hipLaunchKernelGGL((bnact_fwd_kernel<float, float>), g, dim3(256), 0, st, (const float*)z, (float*)y, a);
  else
    hipLaunchKernelGGL((bnact_fwd_kernel<float, bf16_t>), g, dim3(256), 0, st, (const float*)z, (bf16_t*)y, a);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

template <typename T, typename TD>
static int bnact_bwd_t(const void* z, const void* dy, const BnArgs& a, float* sums, int training, void* dz,
                       hipStream_t st) {
  const int cv = 16 / sizeof(T);
  const int P = a.pool;
  const long total = (long)a.N * ((a.H + P - 1) / P) * ((a.W + P - 1) / P) * (a.C / cv);
  if (total <= 0) return HVIT_OK;
  dim3 g(grid_for(total, BN_GRID_SUMS)), ga(grid_for(total, BN_GRID_APPLY));
  {  // the sums are dbeta / dgamma in both modes; only training-mode dz uses them
    const long tsum = (long)a.N * (a.H / P) * (a.W / P) * (a.C / cv);
    const int gs = tsum > 0 ? grid_for(tsum, BN_GRID_SUMS) : 0;
    if (gs > 0) {
      hipLaunchKernelGGL((bnact_sums_kernel<T, TD>), dim3(gs), dim3(256), 0, st, (const T*)z, (const TD*)dy, a, sums);
      HVIT_LAUNCH_CHECK();
    }
    // sums[0 .. 2C) = the partial rows summed in row order (0 rows: zeros)
    if (int rc = hvit_reduce_rows(sums + 2 * a.C, HVIT_F32, gs, 2 * a.C, 2 * a.C, 0, sums, st)) return rc;
  }
  hipLaunchKernelGGL((bnact_bwd_kernel<T, TD, true>), ga, dim3(256), 0, st, (const T*)z, (const TD*)dy, a, sums,
                     training, (T*)dz);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" long long hvit_bn_act_bwd_sums_elems(int C) { return 2LL * C * (1 + BN_PART_ROWS); }

extern "C" int hvit_bn_act_bwd(int dt, const void* z, int N, int H, int W, int C, const float* mean,
                               const float* invstd, const float* gamma, const float* beta,
                               const hvit_dropout_t* dropout2d, int pool, const void* dy, int dy_dt,
                               int training, void* dz, int dz_dt, float* sums, int flags, void* stream) {
  HVIT_CHECK(z && dy && dz && sums, "hvit_bn_act_bwd: null pointer");
  HVIT_CHECK(dz_dt == dt, "hvit_bn_act_bwd: dz dtype must equal z dtype");
  HVIT_CHECK(aligned16(z) && aligned16(dz) && aligned16(dy), "hvit_bn_act_bwd: alignment");
  BnArgs a;
  const int cv = dt == HVIT_BF16 ? 8 : 4;
  if (int rc = make_args(a, N, H, W, C, pool, mean, invstd, gamma, beta, dropout2d, cv)) return rc;
  hipStream_t st = (hipStream_t)stream;
  (void)flags;  // (the partial rows are plain stores: no zeroed accumulator needed)
  if (dt == HVIT_BF16)
    return dy_dt == HVIT_BF16 ? bnact_bwd_t<bf16_t, bf16_t>(z, dy, a, sums, training, dz, st)
                              : bnact_bwd_t<bf16_t, float>(z, dy, a, sums, training, dz, st);
  return dy_dt == HVIT_BF16 ? bnact_bwd_t<float, bf16_t>(z, dy, a, sums, training, dz, st)
                            : bnact_bwd_t<float, float>(z, dy, a, sums, training, dz, st);
}
