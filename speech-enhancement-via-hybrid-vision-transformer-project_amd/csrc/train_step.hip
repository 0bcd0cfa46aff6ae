// The train-step neighbours of the HybridViT path for gfx950:
//
//  * CombinedLoss (training/losses.py:286-387): w_l1 * L1 + w_mse * MSE +
//    w_stoi * mean_b(1 - cos(flatten(pred_b), flatten(tgt_b))) (STOILoss
//    :109-141, F.normalize eps 1e-12) + w_perc * L1 (PerceptualLoss :270-283),
//    optional log compression log(x + 1e-8) of the L1/MSE inputs (:319-321).
//    One pass over pred/target produces six per-sample sums; the scalar loss,
//    its components and the backward's per-sample constants come from those
//    sums, so the reference's four .item() host syncs (:362-383) and ~20 aten
//    launches become three kernels with no host round trip.
//  * clip_grad_norm_ (trainer.py:170-174, torch.nn.utils) and AdamW
//    (training/optimizer.py:53-61, torch.optim.AdamW semantics): a multi-tensor
//    sum of squares with per-block partials, one finalize block (norm and clip
//    coefficient, deterministic order), and a multi-tensor AdamW update that
//    applies the clip coefficient to the gradient on the fly (gradients are
//    read once, never rewritten) and can also write the bf16 copy of each
//    updated weight that the next forward's GEMMs read.
//
// All of it is HBM-bound streaming: float4 lanes, grid-stride loops, tensor
// lists passed by value (no host->device table copies).
#include <math.h>

#include "common.h"

namespace hvit {

// ---------------------------------------------------------------- loss -----
constexpr int LOSS_SUMS = 6;  // |d|, d^2 (compressed inputs), p.t, p.p, t.t, |p - t| (raw)
constexpr int LOSS_CHUNK = 8192;

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

struct LossCfg {
  float w_l1, w_mse, w_stoi, w_perc;
  int logc;
};

template <bool VEC>
__global__ __launch_bounds__(256) void loss_partial_kernel(const float* __restrict__ pred,
                                                          const float* __restrict__ tgt, long P, int nchunk,
                                                          int logc, float* __restrict__ part) {
  __shared__ float red[4];
  const int b = blockIdx.y;
  const long lo = (long)blockIdx.x * LOSS_CHUNK;
  const long hi = min(P, lo + LOSS_CHUNK);
  const float* pp = pred + (long)b * P;
  const float* tp = tgt + (long)b * P;
  float s[LOSS_SUMS] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto acc = [&](float p, float t) {
    const float pi = logc ? logf(p + 1e-8f) : p;
    const float ti = logc ? logf(t + 1e-8f) : t;
    const float d = pi - ti;
    s[0] += fabsf(d);
    s[1] += d * d;
    s[2] += p * t;
    s[3] += p * p;
    s[4] += t * t;
    s[5] += fabsf(p - t);
  };
  if constexpr (VEC) {
    for (long i = lo + 4 * threadIdx.x; i < hi; i += 4 * 256) {
      const f32x4 p = *(const f32x4*)(pp + i);
      const f32x4 t = *(const f32x4*)(tp + i);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc(p[e], t[e]);
    }
  } else {
    for (long i = lo + threadIdx.x; i < hi; i += 256) acc(pp[i], tp[i]);
  }
#pragma unroll
  for (int k = 0; k < LOSS_SUMS; ++k) {
    const float v = block_sum256(s[k], red);
    if (threadIdx.x == 0) part[((long)b * nchunk + blockIdx.x) * LOSS_SUMS + k] = v;
  }
}

// stats[b][6] = per-sample sums (chunk order fixed); out[5] = total, l1, mse,
// stoi, perceptual
__global__ __launch_bounds__(256) void loss_finalize_kernel(const float* __restrict__ part, int B, int nchunk,
                                                           long P, LossCfg c, float* __restrict__ stats,
                                                           float* __restrict__ out) {
  __shared__ float red[4];
  float a = 0.f, q = 0.f, r = 0.f, st = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    float s[LOSS_SUMS] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nchunk; ++k)
#pragma unroll
      for (int j = 0; j < LOSS_SUMS; ++j) s[j] += part[((long)b * nchunk + k) * LOSS_SUMS + j];
#pragma unroll
    for (int j = 0; j < LOSS_SUMS; ++j) stats[(long)b * LOSS_SUMS + j] = s[j];
    const float np = fmaxf(sqrtf(s[3]), 1e-12f), nt = fmaxf(sqrtf(s[4]), 1e-12f);
    a += s[0];
    q += s[1];
    r += s[5];
    st += 1.f - s[2] / (np * nt);
  }
  a = block_sum256(a, red);
  q = block_sum256(q, red);
  r = block_sum256(r, red);
  st = block_sum256(st, red);
  if (threadIdx.x == 0) {
    const float n = (float)B * (float)P;
    const float l1 = a / n, mse = q / n, stoi = st / (float)B, perc = r / n;
    float tot = 0.f;
    if (c.w_l1 > 0.f) tot += c.w_l1 * l1;
    if (c.w_mse > 0.f) tot += c.w_mse * mse;
    if (c.w_stoi > 0.f) tot += c.w_stoi * stoi;
    if (c.w_perc > 0.f) tot += c.w_perc * perc;
    out[0] = tot;
    out[1] = l1;
    out[2] = mse;
    out[3] = stoi;
    out[4] = perc;
  }
}

__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// dpred = gout * d(total)/d(pred); the per-sample constants come from stats
template <bool VEC>
__global__ __launch_bounds__(256) void loss_bwd_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                                                      int B, long P, LossCfg c, const float* __restrict__ stats,
                                                      const float* __restrict__ gout, float* __restrict__ dpred) {
  const float g = gout ? gout[0] : 1.f;
  const float inv_n = 1.f / ((float)B * (float)P);
  const float kl1 = c.w_l1 > 0.f ? g * c.w_l1 * inv_n : 0.f;
  const float kmse = c.w_mse > 0.f ? g * c.w_mse * 2.f * inv_n : 0.f;
  const float kper = c.w_perc > 0.f ? g * c.w_perc * inv_n : 0.f;
  const float kst = c.w_stoi > 0.f ? -g * c.w_stoi / (float)B : 0.f;
  const long total = (long)B * P;
  auto one = [&](float p, float t, float ca, float cb) {
    float d = 0.f, j = 1.f;
    if (c.logc) {
      d = logf(p + 1e-8f) - logf(t + 1e-8f);
      j = 1.f / (p + 1e-8f);
    } else {
      d = p - t;
    }
    return (kl1 * sgnf(d) + kmse * d) * j + kper * sgnf(p - t) + kst * (ca * t - cb * p);
  };
  // d cos_b / dp = t / (|p| |t|) - cos_b * p / |p|^2   (|p| > eps)
  //              = t / (eps * max(|t|, eps))           (|p| <= eps: normalize clamps)
  auto coefs = [&](long b, float& ca, float& cb) {
    const float* s = stats + b * LOSS_SUMS;
    const float np = sqrtf(s[3]), nt = fmaxf(sqrtf(s[4]), 1e-12f);
    if (np > 1e-12f) {
      ca = 1.f / (np * nt);
      cb = s[2] / (np * nt) / (np * np);
    } else {
      ca = 1.f / (1e-12f * nt);
      cb = 0.f;
    }
  };
  if constexpr (VEC) {
    for (long i = 4 * ((long)blockIdx.x * 256 + threadIdx.x); i < total; i += 4L * gridDim.x * 256) {
      float ca, cb;
      coefs(i / P, ca, cb);  // P % 4 == 0: a float4 never straddles samples
      const f32x4 p = *(const f32x4*)(pred + i);
      const f32x4 t = *(const f32x4*)(tgt + i);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = one(p[e], t[e], ca, cb);
      *(f32x4*)(dpred + i) = o;
    }
  } else {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
      float ca, cb;
      coefs(i / P, ca, cb);
      dpred[i] = one(pred[i], tgt[i], ca, cb);
    }
  }
}

// ------------------------------------------------------- clip + AdamW ------
constexpr int MT_MAX = 60;      // tensors per AdamW launch (kernel arguments by value: 64 B per tensor)
constexpr int SQ_MT_MAX = 128;  // tensors per sum-of-squares / scale launch (24 B per tensor: the whole
                                // HybridViT in one launch; three launches of a third each were tail-bound)
constexpr int SUMSQ_GRID = 1024; // partials per sum-of-squares launch

struct SumsqArgs {
  int count;
  long start[SQ_MT_MAX + 1];  // prefix sums of 4-element units (sum of squares: of SQ_TILE-unit tiles)
  long n[SQ_MT_MAX];
  const float* g[SQ_MT_MAX];
};

// a unit = 4 consecutive elements of one tensor (the last unit of a tensor
// may be partial; tensors that are not 16-byte aligned take scalar loads)
__device__ __forceinline__ f32x4 load_unit(const float* p, long u, long n) {
  const long e = 4 * u;
  if (e + 4 <= n && (((uintptr_t)p) & 15) == 0) return *(const f32x4*)(p + e);
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < 4; ++k)
    if (e + k < n) v[k] = p[e + k];
  return v;
}

// multi-tensor chunking: the tensors' 4-element units are cut into tiles of
// SQ_TILE units (a tensor's last tile may be short); blocks take tiles
// round-robin and find a tile's tensor in the tile prefix table (a uniform
// scalar walk), each thread keeping SQ_TILE / 256 independent loads in flight
constexpr int SQ_TILE = 1024;
__device__ __forceinline__ float sq4(f32x4 v) { return v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]; }

__global__ __launch_bounds__(256) void sumsq_kernel(SumsqArgs a, float* __restrict__ part) {
  __shared__ float red[4];
  const long tiles = a.start[a.count];  // start[] holds tile prefix sums here
  int j = 0;
  float s[SQ_TILE / 256] = {};
  for (long t = blockIdx.x; t < tiles; t += gridDim.x) {
    while (t >= a.start[j + 1]) ++j;
    const float* g = a.g[j];
    const long n = a.n[j];
    const long u0 = (t - a.start[j]) * SQ_TILE + threadIdx.x;
    f32x4 v[SQ_TILE / 256];
#pragma unroll
    for (int k = 0; k < SQ_TILE / 256; ++k) {
      const long u = u0 + k * 256;
      v[k] = 4 * u < n ? load_unit(g, u, n) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < SQ_TILE / 256; ++k) s[k] += sq4(v[k]);
  }
  float tot = 0.f;
#pragma unroll
  for (int k = 0; k < SQ_TILE / 256; ++k) tot += s[k];
  tot = block_sum256(tot, red);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// out[0] = total norm, out[1] = min(max_norm / (norm + 1e-6), 1)
__global__ __launch_bounds__(256) void clip_finalize_kernel(const float* __restrict__ part, int n, float max_norm,
                                                           float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = block_sum256(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s);
    out[0] = norm;
    out[1] = fminf(max_norm / (norm + 1e-6f), 1.f);
  }
}

__global__ __launch_bounds__(256) void scale_kernel(SumsqArgs a, const float* __restrict__ coef) {
  const float c = coef[1];
  const long total = a.start[a.count];
  int j = 0;
  for (long u = (long)blockIdx.x * 256 + threadIdx.x; u < total; u += (long)gridDim.x * 256) {
    while (u >= a.start[j + 1]) ++j;
    float* p = (float*)a.g[j];
    const long e = 4 * (u - a.start[j]), n = a.n[j];
    if (e + 4 <= n && (((uintptr_t)p) & 15) == 0) {
      *(f32x4*)(p + e) = *(const f32x4*)(p + e) * c;
    } else {
      for (int k = 0; k < 4; ++k)
        if (e + k < n) p[e + k] *= c;
    }
  }
}

struct AdamArgs {
  int count;
  long start[MT_MAX + 1];
  long n[MT_MAX];
  float* p[MT_MAX];
  const float* g[MT_MAX];
  float* m[MT_MAX];
  float* v[MT_MAX];
  bf16_t* shadow[MT_MAX];
  const float* step[MT_MAX];  // device step counters (nullable: the host bias corrections)
};

static_assert(sizeof(AdamArgs) + 64 <= 4096, "adamw_kernel: kernel argument size");

struct AdamHyper {
  float lr, beta1, beta2, eps, wd, bc1, bc2_sqrt;
};

// torch.optim.AdamW (ADAMW mode of the fused functor):
//   p *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamHyper& h) {
  p *= 1.f - h.lr * h.wd;
  m = h.beta1 * m + (1.f - h.beta1) * g;
  v = h.beta2 * v + (1.f - h.beta2) * g * g;
  const float denom = sqrtf(v) / h.bc2_sqrt + h.eps;
  p -= (h.lr / h.bc1) * (m / denom);
}

// Tiles of AD_TILE 4-element units (a tensor's last tile may be short) taken
// round-robin by the workgroups: the tile's tensor is uniform across the
// workgroup (scalar prefix walk, bias corrections once per tensor change), and
// every thread issues the loads of its AD_UPT units (4 x 16 B each) before any
// arithmetic, so 8 loads are in flight per thread (one unit per thread per
// iteration left the kernel at ~4.2 TB/s).  Per-element arithmetic unchanged.
constexpr int AD_UPT = 2, AD_TILE = 256 * AD_UPT;

__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a, AdamHyper h0, const float* __restrict__ coef,
                                                    const float* __restrict__ hdev) {
  const float c = coef ? coef[1] : 1.f;
  if (hdev) {  // device hyper-parameters (a captured step replays the CURRENT lr / betas / eps / wd)
    h0.lr = hdev[0];
    h0.beta1 = hdev[1];
    h0.beta2 = hdev[2];
    h0.eps = hdev[3];
    h0.wd = hdev[4];
  }
  const long tiles = a.start[a.count];  // start[] holds tile prefix sums
  int j = 0, jh = -1;
  AdamHyper h = h0;
  for (long t = blockIdx.x; t < tiles; t += gridDim.x) {
    while (t >= a.start[j + 1]) ++j;
    if (j != jh) {  // a new tensor: its bias corrections (device step counter, capturable mode)
      jh = j;
      if (a.step[j]) {
        const float st = *a.step[j];
        h.bc1 = 1.f - powf(h0.beta1, st);
        h.bc2_sqrt = sqrtf(1.f - powf(h0.beta2, st));
      } else {
        h.bc1 = h0.bc1;
        h.bc2_sqrt = h0.bc2_sqrt;
      }
    }
    const long n = a.n[j];
    float *P = a.p[j], *M = a.m[j], *V = a.v[j];
    const float* G = a.g[j];
    bf16_t* S = a.shadow[j];
    const long e0 = 4 * ((t - a.start[j]) * AD_TILE + threadIdx.x);
    f32x4 p[AD_UPT], m[AD_UPT], v[AD_UPT], g[AD_UPT];
#pragma unroll
    for (int k = 0; k < AD_UPT; ++k) {
      const long e = e0 + 4L * 256 * k;
      if (e + 4 <= n) {
        p[k] = *(const f32x4*)(P + e);
        m[k] = *(const f32x4*)(M + e);
        v[k] = *(const f32x4*)(V + e);
        g[k] = *(const f32x4*)(G + e);
      }
    }
#pragma unroll
    for (int k = 0; k < AD_UPT; ++k) {
      const long e = e0 + 4L * 256 * k;
      if (e + 4 <= n) {
        const f32x4 gc = g[k] * c;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float pk = p[k][q], mk = m[k][q], vk = v[k][q];
          adam_elem(pk, gc[q], mk, vk, h);
          p[k][q] = pk;
          m[k][q] = mk;
          v[k][q] = vk;
        }
        *(f32x4*)(P + e) = p[k];
        *(f32x4*)(M + e) = m[k];
        *(f32x4*)(V + e) = v[k];
        if (S) {
          uint2 o;
          o.x = f2bf2(p[k][0], p[k][1]);
          o.y = f2bf2(p[k][2], p[k][3]);
          *(uint2*)(S + e) = o;
        }
      } else if (e < n) {  // a tensor's partial last unit
        for (int q = 0; q < 4; ++q) {
          if (e + q >= n) break;
          float pp = P[e + q], mm = M[e + q], vv = V[e + q];
          adam_elem(pp, G[e + q] * c, mm, vv, h);
          P[e + q] = pp;
          M[e + q] = mm;
          V[e + q] = vv;
          if (S) S[e + q] = f2bf(pp);
        }
      }
    }
  }
}

// Device-resident training counters, advanced on the stream so that a captured
// train step (hipGraph) sees fresh values on every replay:
//  * dropout seed (HybridViT training forward): st[0] = base seed, st[1] =
//    forward counter; each forward's seed goes to its own word `out` (read by
//    every dropout kernel of that forward and its backward through
//    hvit_dropout_t.seed_ptr, so two forwards before one backward keep their
//    own masks);
//  * AdamW step counters (torch.optim.AdamW capturable semantics).
__global__ void rng_advance_kernel(unsigned long long* __restrict__ st, unsigned long long* __restrict__ out) {
  if (threadIdx.x == 0) {
    const unsigned long long c = st[1] + 1ull;
    st[1] = c;
    *out = mix64(st[0] ^ mix64(c));
  }
}
__global__ void step_bump_kernel(float* __restrict__ steps, int n, float inc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) steps[i] += inc;
}

static int grid_for_units(long units, int cap) {
  long g = (units + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace hvit

using namespace hvit;

extern "C" long long hvit_loss_ws_elems(int B, long long P) {
  return B > 0 && P > 0 ? (long long)B * cdiv(P, LOSS_CHUNK) * LOSS_SUMS : 0;
}

extern "C" int hvit_loss_fwd(const float* pred, const float* tgt, int B, long long P, const hvit_loss_cfg_t* cfg,
                             float* ws, long long ws_elems, float* stats, float* out, void* stream) {
  HVIT_CHECK(pred && tgt && cfg && ws && stats && out, "hvit_loss_fwd: null pointer");
  HVIT_CHECK(B > 0 && P > 0, "hvit_loss_fwd: empty input (B=%d, P=%lld)", B, P);
  HVIT_CHECK(B <= 65535, "hvit_loss_fwd: B=%d exceeds the grid", B);
  const int nchunk = cdiv(P, LOSS_CHUNK);
  HVIT_CHECK(ws_elems >= (long long)B * nchunk * LOSS_SUMS, "hvit_loss_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const bool vec = P % 4 == 0 && aligned16(pred) && aligned16(tgt);
  const LossCfg c{cfg->w_l1, cfg->w_mse, cfg->w_stoi, cfg->w_perc, cfg->log_compression};
  if (vec)
    hipLaunchKernelGGL(loss_partial_kernel<true>, dim3(nchunk, B), dim3(256), 0, st, pred, tgt, (long)P, nchunk,
                       c.logc, ws);
  else
    hipLaunchKernelGGL(loss_partial_kernel<false>, dim3(nchunk, B), dim3(256), 0, st, pred, tgt, (long)P, nchunk,
                       c.logc, ws);
  HVIT_LAUNCH_CHECK();
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, st, ws, B, nchunk, (long)P, c, stats, out);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_loss_bwd(const float* pred, const float* tgt, int B, long long P, const hvit_loss_cfg_t* cfg,
                             const float* stats, const float* gout, float* dpred, void* stream) {
  HVIT_CHECK(pred && tgt && cfg && stats && dpred, "hvit_loss_bwd: null pointer");
  HVIT_CHECK(B > 0 && P > 0, "hvit_loss_bwd: empty input");
  hipStream_t st = (hipStream_t)stream;
  const LossCfg c{cfg->w_l1, cfg->w_mse, cfg->w_stoi, cfg->w_perc, cfg->log_compression};
  const long total = (long)B * P;
  const bool vec = P % 4 == 0 && aligned16(pred) && aligned16(tgt) && aligned16(dpred);
  if (vec)
    hipLaunchKernelGGL(loss_bwd_kernel<true>, dim3(grid_for_units(total / 4, 2048)), dim3(256), 0, st, pred, tgt,
                       B, (long)P, c, stats, gout, dpred);
  else
    hipLaunchKernelGGL(loss_bwd_kernel<false>, dim3(grid_for_units(total, 2048)), dim3(256), 0, st, pred, tgt, B,
                       (long)P, c, stats, gout, dpred);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" long long hvit_clip_ws_elems(int count) {
  return count <= 0 ? 0 : (long long)cdiv(count, SQ_MT_MAX) * SUMSQ_GRID;
}

static int fill_sumsq(SumsqArgs& a, const hvit_tensor_t* t, int base, int count, long per = 1) {
  a.count = count;
  a.start[0] = 0;
  for (int k = 0; k < count; ++k) {
    const hvit_tensor_t& x = t[base + k];
    HVIT_CHECK(x.ptr && x.numel >= 0, "hvit: tensor %d: null pointer or negative numel", base + k);
    a.g[k] = (const float*)x.ptr;
    a.n[k] = (long)x.numel;
    const long units = (long)((x.numel + 3) / 4);
    a.start[k + 1] = a.start[k] + (units + per - 1) / per;  // per = units per table entry
  }
  return HVIT_OK;
}

extern "C" int hvit_clip_coef(int count, const hvit_tensor_t* grads, float max_norm, float* ws, long long ws_elems,
                              float* out, void* stream) {
  HVIT_CHECK(count >= 0 && (count == 0 || grads) && out, "hvit_clip_coef: bad args");
  HVIT_CHECK(count == 0 || (ws && ws_elems >= hvit_clip_ws_elems(count)), "hvit_clip_coef: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  int nparts = 0;
  for (int base = 0; base < count; base += SQ_MT_MAX) {
    SumsqArgs a;
    if (int rc = fill_sumsq(a, grads, base, std::min(SQ_MT_MAX, count - base), SQ_TILE)) return rc;
    hipLaunchKernelGGL(sumsq_kernel, dim3(SUMSQ_GRID), dim3(256), 0, st, a, ws + nparts);
    HVIT_LAUNCH_CHECK();
    nparts += SUMSQ_GRID;
  }
  hipLaunchKernelGGL(clip_finalize_kernel, dim3(1), dim3(256), 0, st, ws, nparts, max_norm, out);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_scale_tensors(int count, const hvit_tensor_t* tensors, const float* coef, void* stream) {
  HVIT_CHECK(count >= 0 && (count == 0 || tensors) && coef, "hvit_scale_tensors: bad args");
  for (int base = 0; base < count; base += SQ_MT_MAX) {
    SumsqArgs a;
    if (int rc = fill_sumsq(a, tensors, base, std::min(SQ_MT_MAX, count - base))) return rc;
    hipLaunchKernelGGL(scale_kernel, dim3(grid_for_units(a.start[a.count], 2048)), dim3(256), 0,
                       (hipStream_t)stream, a, coef);
    HVIT_LAUNCH_CHECK();
  }
  return HVIT_OK;
}

extern "C" int hvit_adamw_dev(int count, const hvit_adamw_item_t* items, const hvit_adamw_hyper_t* hp,
                              const float* coef, const float* hyper_dev, void* stream);
extern "C" int hvit_adamw(int count, const hvit_adamw_item_t* items, const hvit_adamw_hyper_t* hp,
                          const float* coef, void* stream) {
  return hvit_adamw_dev(count, items, hp, coef, nullptr, stream);
}

extern "C" int hvit_adamw_dev(int count, const hvit_adamw_item_t* items, const hvit_adamw_hyper_t* hp,
                              const float* coef, const float* hyper_dev, void* stream) {
  HVIT_CHECK(!hyper_dev || ((uintptr_t)hyper_dev & 3) == 0, "hvit_adamw_dev: hyper_dev alignment");
  HVIT_CHECK(count >= 0 && (count == 0 || items) && hp, "hvit_adamw: bad args");
  bool host_bc = false;
  for (int k = 0; k < count; ++k) host_bc = host_bc || !items[k].step;
  HVIT_CHECK(!host_bc || (hp->bc1 > 0.f && hp->bc2 > 0.f), "hvit_adamw: bias corrections must be positive");
  const AdamHyper h{hp->lr, hp->beta1, hp->beta2, hp->eps, hp->weight_decay, host_bc ? hp->bc1 : 1.f,
                    host_bc ? sqrtf(hp->bc2) : 1.f};
  // launches of equal tensor counts (104 HybridViT tensors: 52 + 52, not 60 + 44)
  const int per = count > 0 ? cdiv(count, cdiv(count, MT_MAX)) : MT_MAX;
  for (int base = 0; base < count; base += per) {
    AdamArgs a;
    a.count = std::min(per, count - base);
    a.start[0] = 0;
    for (int k = 0; k < a.count; ++k) {
      const hvit_adamw_item_t& it = items[base + k];
      HVIT_CHECK(it.param && it.grad && it.exp_avg && it.exp_avg_sq && it.numel >= 0,
                 "hvit_adamw: item %d: null pointer", base + k);
      HVIT_CHECK(aligned16(it.param) && aligned16(it.grad) && aligned16(it.exp_avg) && aligned16(it.exp_avg_sq) &&
                     (!it.shadow_bf16 || (((uintptr_t)it.shadow_bf16) & 7) == 0),
                 "hvit_adamw: item %d: alignment (16 B; shadow 8 B)", base + k);
      a.p[k] = it.param;
      a.g[k] = it.grad;
      a.m[k] = it.exp_avg;
      a.v[k] = it.exp_avg_sq;
      a.shadow[k] = (bf16_t*)it.shadow_bf16;
      a.step[k] = it.step;
      a.n[k] = (long)it.numel;
      a.start[k + 1] = a.start[k] + ((long)((it.numel + 3) / 4) + AD_TILE - 1) / AD_TILE;  // tiles
    }
    if (a.start[a.count] == 0) continue;
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)std::min<long>(a.start[a.count], 2048)), dim3(256), 0,
                       (hipStream_t)stream, a, h, coef, hyper_dev);
    HVIT_LAUNCH_CHECK();
  }
  return HVIT_OK;
}

extern "C" int hvit_rng_advance(unsigned long long* state, unsigned long long* seed_out, void* stream) {
  HVIT_CHECK(state && seed_out && (((uintptr_t)state) & 7) == 0 && (((uintptr_t)seed_out) & 7) == 0,
             "hvit_rng_advance: null or misaligned pointer");
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, state, seed_out);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

extern "C" int hvit_step_bump(float* steps, int n, float inc, void* stream) {
  HVIT_CHECK(steps && n >= 0, "hvit_step_bump: bad args");
  if (n == 0) return HVIT_OK;
  hipLaunchKernelGGL(step_bump_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, steps, n, inc);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}
