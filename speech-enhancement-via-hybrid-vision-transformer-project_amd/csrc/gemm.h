// Tiled MFMA GEMM for gfx950 with pluggable operand loaders and fused epilogues.
//
//   C[m][n] = sum_k A(m, k) * B(n, k)         (both operands "row x reduction")
//
// Structure: 256 threads (4 waves, 2x2), BM x BN output tile, 128 bytes of K
// per stage (64 bf16 / 32 f32), two LDS stages and two register stages: the
// global loads for stage t+2 are in flight while stage t runs on the MFMAs and
// stage t+1 waits in registers, so HBM/L2 latency is covered by two stages of
// math (counted vmcnt waits; interior tiles use branch-free loads so the
// compiler can count them).  Per 64-byte k-step each lane feeds one 16-byte
// fragment per 16x16 sub-tile:
//   bf16: one  v_mfma_f32_16x16x32_bf16 (8 k per lane)
//   f32 : four v_mfma_f32_16x16x4_f32   (4 k per lane; the k-slots of the four
//         MFMAs are a permutation of the 16 k's, identical for A and B)
// Operand layouts in LDS:
//   KC (reduction dim contiguous in memory): [rows][128 B], 16-byte chunks
//     XOR-swizzled by (row & 7) -> conflict-free ds_read_b128 / ds_write_b128;
//   MN (rows contiguous in memory: wgrad/dgrad operands), bf16: copied as is,
//     [k][rows] (+32 B pad, 128-B XOR swizzle on k bit 3), and read with
//     ds_read_b64_tr_b16 (hardware transpose) -- no scalar LDS scatter;
//   MN, f32 (parity path): scatter-transposed into the KC layout.
// Implicit-GEMM loaders gather conv taps from NHWC activations on the fly
// (3x3 same conv with optional nearest x2 upsample and two concatenated
// sources; the 4x4/stride-4 patch embedding); each thread keeps a cursor per
// 16-byte chunk (its pixel / tap decomposition) that advances incrementally.
#pragma once
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace hvit {

constexpr int GEMM_THREADS = 256;
constexpr int KSTAGE = 128;  // bytes of K per stage (= KC tile row pitch, no pad)

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ int kc_off(int row, int chunk) { return row * KSTAGE + ((chunk ^ (row & 7)) << 4); }

// ------------------------------------------------------------ loaders --------
// Roles: a = row index of the operand (m for A, n for B), b = reduction index.
// KC loaders return 16 bytes = E elements (a, b..b+E-1); MN loaders return
// E elements (a..a+E-1, b).  A thread's chunks in one stage all share the same
// b (KC) or the same a (MN) -- see TileCfg::map -- so a loader keeps that part
// in one shared state `Sh` and only the varying part in a per-chunk cursor
// `Cur` (keeps 128x128 tiles spill-free).  init() builds both for (a, b);
// step() moves BK along the reduction; fetch<CHECK> reads the current chunk
// (CHECK=false: interior tile, no bounds tests).
template <typename T, bool KC_>
struct LdDense {
  static constexpr bool KC = KC_;
  static constexpr int E = Elem<T>::PER16;
  const T* p;
  long ld;     // KC: elements between rows; !KC: elements between k
  int rows;    // row extent
  int K;       // reduction extent
  bool vok;    // base 16-byte aligned and ld % E == 0 (vector loads legal)
  struct Sh {};
  struct Cur {
    const T* q;  // address of the current chunk
    int a, b;
  };
  __device__ __forceinline__ bool fast() const { return vok; }
  __device__ __forceinline__ void init(Sh&, Cur& c, int a, int b) const {
    c.a = a;
    c.b = b;
    c.q = KC ? p + (long)a * ld + b : p + (long)b * ld + a;
  }
  __device__ __forceinline__ void step_sh(Sh&, int) const {}
  __device__ __forceinline__ void step(Cur& c, int bk) const {
    c.b += bk;
    c.q += KC ? (long)bk : (long)bk * ld;
  }
  template <bool CHECK>
  __device__ __forceinline__ u32x4 fetch(const Sh&, const Cur& c) const {
    if (!CHECK) return *(const u32x4*)c.q;
    const int a = c.a, b = c.b;
    u32x4 r = {0u, 0u, 0u, 0u};
    if (KC) {
      if (a >= rows || b >= K) return r;
      if (vok && b + E <= K) return *(const u32x4*)c.q;
      T tmp[E];
#pragma unroll
      for (int e = 0; e < E; ++e) tmp[e] = (b + e < K) ? c.q[e] : (T)0;
      return *(u32x4*)tmp;
    } else {
      if (b >= K || a >= rows) return r;
      if (vok && a + E <= rows) return *(const u32x4*)c.q;
      T tmp[E];
#pragma unroll
      for (int e = 0; e < E; ++e) tmp[e] = (a + e < rows) ? c.q[e] : (T)0;
      return *(u32x4*)tmp;
    }
  }
};

// Implicit im2col over NHWC sources.  Pixel index p = output pixel (n, oy, ox)
// of a Ho x Wo grid; im2col index k = (ky*KS + kx)*Ctot + c.  The conv input is
// concat(src1[C1], src2[C2]) upsampled (nearest) by U from Hs x Ws.
// KC (fwd / dgrad A operand): a = pixel (per chunk), b = k (shared, advances).
// !KC (wgrad B operand):     a = k (shared),         b = pixel (per chunk, advances).
template <typename T, bool KC_>
struct LdConv {
  static constexpr bool KC = KC_;
  static constexpr int E = Elem<T>::PER16;
  const T* src1;
  const T* src2;
  int C1, C2, Ctot;
  int Hs, Ws, U, Hi, Wi;  // source dims, upsample, conv-input dims
  int KS, S, Pd;          // kernel, stride, pad
  int Ho, Wo;             // output grid
  int P;                  // number of output pixels (N*Ho*Wo)
  int Kt;                 // KS*KS*Ctot
  bool vec_ok;            // C1 % E == 0 && C2 % E == 0 (16-byte gathers)

  __device__ __forceinline__ bool fast() const { return vec_ok; }
  __device__ __forceinline__ float elem_f(int p, int k) const {
    if (p >= P || k >= Kt) return 0.f;
    int hw = Ho * Wo;
    int n = p / hw, rem = p - n * hw;
    int oy = rem / Wo, ox = rem - oy * Wo;
    int tap = k / Ctot, c = k - tap * Ctot;
    int ky = tap / KS, kx = tap - ky * KS;
    int iy = oy * S - Pd + ky, ix = ox * S - Pd + kx;
    if (iy < 0 || ix < 0 || iy >= Hi || ix >= Wi) return 0.f;
    int sy = iy / U, sx = ix / U;
    long pix = ((long)n * Hs + sy) * Ws + sx;
    return c < C1 ? Elem<T>::to_f(src1[pix * C1 + c]) : Elem<T>::to_f(src2[pix * C2 + (c - C1)]);
  }

  struct Sh {  // tap part (ky, kx, c) of the im2col index k
    int k, c, kx, ky;
  };
  struct Cur {  // pixel part (n, oy, ox) of p
    int p, n, oy, ox;
  };
  __device__ __forceinline__ void init(Sh& sh, Cur& cu, int a, int b) const {
    const int p = KC ? a : b, k = KC ? b : a;
    cu.p = p;
    const int hw = Ho * Wo;
    cu.n = p / hw;
    const int rem = p - cu.n * hw;
    cu.oy = rem / Wo;
    cu.ox = rem - cu.oy * Wo;
    sh.k = k;
    const int tap = k / Ctot;
    sh.c = k - tap * Ctot;
    sh.ky = tap / KS;
    sh.kx = tap - sh.ky * KS;
  }
  __device__ __forceinline__ void step_sh(Sh& sh, int bk) const {
    if (!KC) return;
    sh.k += bk;
    sh.c += bk;
    while (sh.c >= Ctot) {
      sh.c -= Ctot;
      if (++sh.kx == KS) {
        sh.kx = 0;
        ++sh.ky;
      }
    }
  }
  __device__ __forceinline__ void step(Cur& cu, int bk) const {
    if (KC) return;
    cu.p += bk;
    cu.ox += bk;
    while (cu.ox >= Wo) {
      cu.ox -= Wo;
      if (++cu.oy == Ho) {
        cu.oy = 0;
        ++cu.n;
      }
    }
  }
  template <bool CHECK>
  __device__ __forceinline__ u32x4 fetch(const Sh& sh, const Cur& cu) const {
    if (!CHECK || vec_ok) {
      // padding taps read a valid address and are zeroed by a select
      const int iy = cu.oy * S - Pd + sh.ky, ix = cu.ox * S - Pd + sh.kx;
      bool ok = (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi;
      if (CHECK) ok = ok && cu.p < P && sh.k < Kt;
      const int sy = ok ? (U == 2 ? (iy >> 1) : iy) : 0, sx = ok ? (U == 2 ? (ix >> 1) : ix) : 0;
      const int pix = ((ok ? cu.n : 0) * Hs + sy) * Ws + sx;
      const int c = ok ? sh.c : 0;
      const T* q = c < C1 ? src1 + (long)pix * C1 + c : src2 + (long)pix * C2 + (c - C1);
      const u32x4 v = *(const u32x4*)q;
      const u32x4 z = {0u, 0u, 0u, 0u};
      return ok ? v : z;
    }
    T tmp[E];
#pragma unroll
    for (int e = 0; e < E; ++e) tmp[e] = Elem<T>::from_f(elem_f(cu.p, sh.k + e));
    return *(u32x4*)tmp;
  }
};

// Fast implicit-im2col A loader (bf16, KC role only) for the common case
// where every K stage (64 channels) lies inside one tap and one source:
// C1 % 64 == 0 and C2 % 64 == 0.  The tap / channel state of a stage is then
// wave-uniform (SGPRs: the stage base is readfirstlane'd), the per-chunk state
// is the pixel's (row base, iy0, ix0), and reads go through buffer loads with a
// 32-bit byte offset: taps in the zero padding, or pixels past the end (row
// base beyond the tensor), get an offset past num_records and read zeros --
// no per-element selects or 64-bit address math.
template <typename T>
struct LdConvF {
  static constexpr bool KC = true;
  static constexpr int E = Elem<T>::PER16;
  const T* src1;
  const T* src2;
  int C1, C2, Ctot;
  int Hs, Ws, Hi, Wi, ushift;  // source dims, conv-input dims, log2(U)
  int KS, S, Pd;
  int Ho, Wo, P, Kt;
  unsigned bytes1, bytes2;     // buffer extents
  int pool2 = 0;               // row order: 0 pixel-major (n, oy, ox); 1 pooling windows (n, oy/2, ox/2, 2x2 position)

  __device__ __forceinline__ bool fast() const { return true; }
  // output pixel of GEMM row p.  pool2: rows 4w .. 4w+3 are the 2x2 window w of the
  // pooled image (window-major, NHWC order of the pooled output), so a 2x2 max-pool
  // is a max over 4 consecutive rows in the epilogue
  __device__ __forceinline__ void pix(int p, int& n, int& oy, int& ox) const {
    if (pool2) {
      const int q = p & 3, w = p >> 2, hw = (Ho >> 1) * (Wo >> 1);
      n = w / hw;
      const int rem = w - n * hw;
      const int wy = rem / (Wo >> 1), wx = rem - wy * (Wo >> 1);
      oy = 2 * wy + (q >> 1);
      ox = 2 * wx + (q & 1);
    } else {
      const int hw = Ho * Wo;
      n = p / hw;
      const int rem = p - n * hw;
      oy = rem / Wo;
      ox = rem - oy * Wo;
    }
  }
  struct Sh {
    int c0, kx, ky;  // stage tap (uniform)
    int klane;       // this thread's channel offset inside the stage
  };
  struct Cur {
    int rb, iy0, ix0;  // n*Hs (source row base), oy*S - Pd, ox*S - Pd
  };
  __device__ __forceinline__ void init(Sh& sh, Cur& cu, int a, int b) const {
    int n, oy, ox;
    pix(a, n, oy, ox);
    cu.rb = n * Hs;
    cu.iy0 = oy * S - Pd;
    cu.ix0 = ox * S - Pd;
    const int kb = __builtin_amdgcn_readfirstlane(b & ~63);
    sh.klane = b & 63;
    const int tap = kb / Ctot;
    sh.c0 = kb - tap * Ctot;
    sh.ky = tap / KS;
    sh.kx = tap - sh.ky * KS;
  }
  __device__ __forceinline__ void step_sh(Sh& sh, int bk) const {
    sh.c0 += bk;
    if (sh.c0 >= Ctot) {
      sh.c0 -= Ctot;
      if (++sh.kx == KS) {
        sh.kx = 0;
        ++sh.ky;
      }
    }
  }
  __device__ __forceinline__ void step(Cur&, int) const {}
  template <bool CHECK>
  __device__ __forceinline__ u32x4 fetch(const Sh& sh, const Cur& cu) const {
    const bool first = sh.c0 < C1;  // uniform
    const int Cx = first ? C1 : C2;
    const int coff = (first ? sh.c0 : sh.c0 - C1) + sh.klane;
    const int iy = cu.iy0 + sh.ky, ix = cu.ix0 + sh.kx;
    const bool ok = (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi;
    const int off = (((cu.rb + (iy >> ushift)) * Ws + (ix >> ushift)) * Cx + coff) * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(first ? src1 : src2), (short)0, (int)(first ? bytes1 : bytes2), 0x00020000);
    const unsigned voff = ok ? (unsigned)off : 0x80000000u;
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
  }
};

// Im2col B loader of the conv weight gradient (MN role: a = im2col index k,
// fixed per chunk for the whole K loop; b = output pixel, advancing).  The
// tap / channel / source of a thread's k are resolved once at init; the pixel
// cursor (row base n*Hs, oy, ox) advances incrementally; addresses use 32-bit
// element offsets from a per-thread base pointer.
template <typename T>
struct LdConvWF {
  static constexpr bool KC = false;
  static constexpr int E = Elem<T>::PER16;
  const T* src1;
  const T* src2;
  int C1, C2, Ctot;
  int Hs, Ws, Hi, Wi, ushift;
  int KS, S, Pd;
  int Ho, Wo, P, Kt;

  __device__ __forceinline__ bool fast() const { return true; }
  struct Sh {
    const T* base;
    int Cx, coff, dy0, dx0;
    bool kok;
  };
  struct Cur {
    int p, rb, oy, ox;
  };
  __device__ __forceinline__ void init(Sh& sh, Cur& cu, int a, int b) const {
    const int tap = a / Ctot, c = a - tap * Ctot;
    const int ky = tap / KS, kx = tap - ky * KS;
    const bool first = c < C1;
    sh.base = first ? src1 : src2;
    sh.Cx = first ? C1 : C2;
    sh.coff = first ? c : c - C1;
    sh.dy0 = ky - Pd;
    sh.dx0 = kx - Pd;
    sh.kok = a < Kt;
    const int hw = Ho * Wo;
    const int n = b / hw, rem = b - n * hw;
    cu.p = b;
    cu.rb = n * Hs;
    cu.oy = rem / Wo;
    cu.ox = rem - cu.oy * Wo;
  }
  __device__ __forceinline__ void step_sh(Sh&, int) const {}
  __device__ __forceinline__ void step(Cur& cu, int bk) const {
    cu.p += bk;
    cu.ox += bk;
    while (cu.ox >= Wo) {
      cu.ox -= Wo;
      if (++cu.oy == Ho) {
        cu.oy = 0;
        cu.rb += Hs;
      }
    }
  }
  template <bool CHECK>
  __device__ __forceinline__ u32x4 fetch(const Sh& sh, const Cur& cu) const {
    const int iy = cu.oy * S + sh.dy0, ix = cu.ox * S + sh.dx0;
    bool ok = (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi;
    if (CHECK) ok = ok && sh.kok && cu.p < P;
    const int off = ok ? ((cu.rb + (iy >> ushift)) * Ws + (ix >> ushift)) * sh.Cx + sh.coff : 0;
    const u32x4 v = *(const u32x4*)(sh.base + off);
    const u32x4 z = {0u, 0u, 0u, 0u};
    return ok ? v : z;
  }
};

// ------------------------------------------------------------ epilogue -------
enum EpiMode { EPI_STORE = 0, EPI_SLAB = 1, EPI_PATCH = 2, EPI_SPLIT2 = 3 };
enum EpiAct { ACT_NONE = 0, ACT_GELU_DUAL = 1, ACT_TANH = 2, ACT_GELU_BWD = 3 };
// compile-time epilogue kind: a lean kernel for plain stores (+bias, BN stats,
// column sums) and for split-K slabs; everything else takes the generic one
// and for the three fused ViT epilogues (fc1 GELU, residual adds, GELU
// backward), which are only chosen when every tile is full and vector-aligned
enum EpiKind { EK_GEN = 0, EK_STORE = 1, EK_SLAB = 2, EK_GELU_DUAL = 3, EK_RESID = 4, EK_GELU_BWD = 5, EK_PATCH = 6 };

struct Epi {
  int mode = EPI_STORE;
  void* out = nullptr;
  int out_dt = HVIT_F32;
  long ldo = 0;
  void* out2 = nullptr;  // GELU_DUAL: activation output; SPLIT2: columns >= split_col
  int out2_dt = HVIT_F32;
  long ldo2 = 0;
  int split_col = 0;
  const float* bias = nullptr;
  const float* rowadd = nullptr;  // v += rowadd[(m % rowadd_mod) * rowadd_ld + n]
  long rowadd_ld = 0;
  int rowadd_mod = 1;
  int act = ACT_NONE;
  const void* aux = nullptr;  // GELU_BWD: pre-activation h[m][n] (gd: gelu'(h) itself)
  int gd = 0;  // GELU_DUAL: out receives gelu'(h) instead of h; GELU_BWD: aux already is gelu'(h)
  int relu = 0;  // v = max(v, 0) after bias (the eval-mode folded BatchNorm + ReLU of the conv blocks)
  int pool2 = 0;  // EK_STORE of a pooled conv (LdConvF::pool2 row order): 2x2 max of each 4-row window, row m/4
  int aux_dt = HVIT_F32;
  long ldaux = 0;
  uint32_t drop_thr = 0;  // dropout keep test (0 = off)
  float drop_scale = 1.f;
  uint32_t drop_key = 0;  // rng_key(seed, site) (host-resolved when drop_seedp is NULL)
  const unsigned long long* drop_seedp = nullptr;  // device seed word (hvit_dropout_t.seed_ptr)
  unsigned long long drop_seed = 0;
  uint32_t drop_site = 0;
  const float* resid = nullptr;  // v = resid[m][n] + rowscale[m / rps] * v
  long ldr = 0;
  const float* rowscale = nullptr;
  int rows_per_sample = 1;
  float* stats = nullptr;   // BN partials [64-row tile][N][2] = (mean, M2)
  float* colsum = nullptr;  // column sums of the final v: partial row per 64-row block ([cdiv(M,64)][N])
  long slab_stride = 0;     // EPI_SLAB: elements between split-K slabs (0: M * ldo)
  unsigned* tickets = nullptr;  // EPI_SLAB (ring kernels): per-tile arrival counters, zeroed; the last
  float* red_out = nullptr;     //   slice of a tile sums the slabs into red_out (ld = ldo) in-kernel
  float* rs_ptr = nullptr;  // row sums of the A operand (wgrad bias grad): rs_ptr[z * rs_stride + m]
  long rs_stride = 0;
  bool vec_ok = false;      // N % 4 == 0, every operand 16-B aligned with ld % 4 == 0
  int xcd_remap = 1;        // XCD-aware block order (see tile_of); 0 = hardware order
  int dma = 1;              // host: LDS-DMA kernels allowed (GemmCoreDma); 0 = register staging only
  // EPI_PATCH: m = token (b, py, px) of Hp x Wp, n = (ky*P + kx)*C + c
  int pP = 0, pC = 0, pHp = 0, pWp = 0, pH = 0, pW = 0;
  // side job (hvit_slab_sum_t): a deferred weight gradient's split-K slabs
  // summed by this launch's workgroups before their own tiles (epi_side)
  const float* sj_src = nullptr;
  float* sj_dst = nullptr;
  long sj_n4 = 0;      // float4 granules
  long sj_stride4 = 0;
  int sj_splits = 0;
};

// dst[i] = sum_z src[z * stride + i] over the side job's granules, spread over
// every workgroup of the launch.  gemm_kernel runs it after its tile's
// epilogue (two or three workgroups per CU, out of phase: the load latency
// overlaps a co-resident workgroup's K loop); the ring kernels after issuing
// their DMA prologue (one workgroup per CU: the latency overlaps the first
// stages' flight).  Any in-flight stores only make a later counted vmcnt wait
// stricter.  Two forms by the job's slab count alone -- so the order is the
// job's, whatever launch carries it, and hvit_sum_slabs_strided (the job run
// as a launch of its own: side stream, M = 0 carriers) is bit-identical:
//  * fewer than SIDE_WAVE_SPLITS slabs (split-K weight-gradient slabs: ~10^5
//    granules, 4-32 slabs): a granule per thread, even | odd slabs paired as
//    sum_slabs_strided_kernel, eight slabs' loads in flight per step;
//  * SIDE_WAVE_SPLITS or more (partial column-sum rows, the tall-skinny weight
//    gradients' slabs: 10^2-10^3 granules x 128-512 slabs): a granule per wave,
//    its slabs over the lanes, then a butterfly, as sum_slabs_wave_kernel.  (One
//    thread walking 128 slabs held its workgroup ~20 us past the others: round
//    4, the fc1 weight gradient carrying the fc1 bias rows.)
// (SIDE_WAVE_SPLITS, side_wave_granule: common.h)
__device__ __forceinline__ void epi_side(const Epi& ep) {
  if (!ep.sj_n4) return;
  const long nwg = (long)gridDim.x * gridDim.y * gridDim.z;
  const long b = blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z);
  const f32x4* src = (const f32x4*)ep.sj_src;
  f32x4* dst = (f32x4*)ep.sj_dst;
  const long st = ep.sj_stride4;
  const int wpb = blockDim.x >> 6;
  if (ep.sj_splits >= SIDE_WAVE_SPLITS) {
    for (long i = b * wpb + (threadIdx.x >> 6); i < ep.sj_n4; i += nwg * wpb) {
      const f32x4 s = side_wave_granule(src, st, ep.sj_splits, i);
      if ((threadIdx.x & 63) == 0) dst[i] = s;
    }
    return;
  }
  const long nthr = nwg * blockDim.x;
  for (long i = b * blockDim.x + threadIdx.x; i < ep.sj_n4; i += nthr) {
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
    int k = 0;
    for (; k + 7 < ep.sj_splits; k += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(long)(k + u) * st + i];
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        s0 += v[u];
        s1 += v[u + 1];
      }
    }
    for (; k + 1 < ep.sj_splits; k += 2) {
      s0 += src[(long)k * st + i];
      s1 += src[(long)(k + 1) * st + i];
    }
    if (k < ep.sj_splits) s0 += src[(long)k * st + i];
    dst[i] = s0 + s1;
  }
}

// 4 adjacent output columns (n .. n+nv-1) of row m: store helpers and the
// fused epilogue math.
// ragged / misaligned fallbacks are out of line: they are rare and would
// otherwise be inlined once per unrolled epilogue row (code size, i-cache)
__device__ __attribute__((noinline)) void store4_slow(void* p, long off, f32x4 v, int nv, int dt) {
  for (int e = 0; e < nv; ++e) st_dt(p, off + e, v[e], dt);
}
__device__ __attribute__((noinline)) f32x4 load4_slow(const void* p, long off, int nv, int dt) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  for (int e = 0; e < nv; ++e) v[e] = ld_dt(p, off + e, dt);
  return v;
}

__device__ __forceinline__ void store4(void* p, long off, const f32x4& v, int nv, int dt) {
  if (dt == HVIT_F32) {
    float* q = (float*)p + off;
    if (nv == 4 && (((uintptr_t)q) & 15) == 0) *(f32x4*)q = v;
    else store4_slow(p, off, v, nv, dt);
  } else {
    bf16_t* q = (bf16_t*)p + off;
    if (nv == 4 && (((uintptr_t)q) & 7) == 0) {
      uint2 u;
      u.x = f2bf2(v[0], v[1]);
      u.y = f2bf2(v[2], v[3]);
      *(uint2*)q = u;
    } else {
      store4_slow(p, off, v, nv, dt);
    }
  }
}

__device__ __forceinline__ f32x4 load4(const void* p, long off, int nv, int dt) {
  if (dt == HVIT_F32) {
    const float* q = (const float*)p + off;
    if (nv == 4 && (((uintptr_t)q) & 15) == 0) return *(const f32x4*)q;
  } else {
    const bf16_t* q = (const bf16_t*)p + off;
    if (nv == 4 && (((uintptr_t)q) & 7) == 0) {
      uint2 u = *(const uint2*)q;
      f32x4 v;
      v[0] = __uint_as_float(u.x << 16);
      v[1] = __uint_as_float(u.x & 0xffff0000u);
      v[2] = __uint_as_float(u.y << 16);
      v[3] = __uint_as_float(u.y & 0xffff0000u);
      return v;
    }
  }
  return load4_slow(p, off, nv, dt);
}

// FAST: caller guarantees 4 in-range columns and 16-byte (f32) / 8-byte (bf16)
// alignment -- plain vector accesses, no per-lane branches
template <bool FAST>
__device__ __forceinline__ void store4v(void* p, long off, const f32x4& v, int nv, int dt) {
  if constexpr (FAST) {
    if (dt == HVIT_F32) {
      *(f32x4*)((float*)p + off) = v;
    } else {
      uint2 u;
      u.x = f2bf2(v[0], v[1]);
      u.y = f2bf2(v[2], v[3]);
      *(uint2*)((bf16_t*)p + off) = u;
    }
  } else {
    store4(p, off, v, nv, dt);
  }
}
template <bool FAST>
__device__ __forceinline__ f32x4 load4v(const void* p, long off, int nv, int dt) {
  if constexpr (FAST) {
    if (dt == HVIT_F32) return *(const f32x4*)((const float*)p + off);
    const uint2 u = *(const uint2*)((const bf16_t*)p + off);
    f32x4 v;
    v[0] = __uint_as_float(u.x << 16);
    v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16);
    v[3] = __uint_as_float(u.y & 0xffff0000u);
    return v;
  } else {
    return load4(p, off, nv, dt);
  }
}

// dropout multipliers of 4 adjacent elements (index i0 = m*N + n, i0 even):
// two pair hashes give the four 16-bit uniforms
__device__ __forceinline__ f32x4 keep4(const Epi& ep, uint32_t key, int m, int n, int N) {
  const uint64_t i0 = (uint64_t)m * (uint64_t)N + (uint64_t)n;
  return keep4_at(key, i0, ep.drop_thr, ep.drop_scale);
}
// the dropout key of a launch: folds in the device seed word (one scalar load)
__device__ __forceinline__ uint32_t epi_key(const Epi& ep) {
  return (ep.drop_seedp && ep.drop_thr) ? rng_key(ep.drop_seed ^ *ep.drop_seedp, ep.drop_site) : ep.drop_key;
}

// Inputs the epilogue reads besides the accumulator, loaded for all of a
// thread's rows BEFORE any of its stores: the compiler cannot reorder a load
// above a store that may alias it, so loading inside the store loop would
// serialise one global-load latency per row.
struct EpiIn {
  f32x4 rowadd, aux, resid;
  float rowscale;
};

template <bool FAST>
__device__ __forceinline__ void epi_load4(const Epi& ep, int m, int n, int nv, bool ok, EpiIn& in) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  in.rowadd =
      (ep.rowadd && ok) ? load4v<FAST>(ep.rowadd, (long)(m % ep.rowadd_mod) * ep.rowadd_ld + n, nv, HVIT_F32) : z;
  in.aux = (ep.act == ACT_GELU_BWD && ok) ? load4v<FAST>(ep.aux, (long)m * ep.ldaux + n, nv, ep.aux_dt) : z;
  in.resid = (ep.resid && ok) ? load4v<FAST>(ep.resid, (long)m * ep.ldr + n, nv, HVIT_F32) : z;
  in.rowscale = (ep.resid && ep.rowscale && ok) ? ep.rowscale[m / ep.rows_per_sample] : 1.f;
}

template <bool FAST>
__device__ __forceinline__ void epi_apply4(const Epi& ep, uint32_t dkey, int m, int n, int nv, int N, f32x4& v,
                                           const f32x4& bias, const EpiIn& in) {
  v += bias;
  if (ep.rowadd) v += in.rowadd;
  float keep[4] = {1.f, 1.f, 1.f, 1.f};
  if (ep.drop_thr) {
    const uint64_t i0 = (uint64_t)m * (uint64_t)N + (uint64_t)n;
    if (FAST || (i0 & 1) == 0) {
      const f32x4 k = keep4_at(dkey, i0, ep.drop_thr, ep.drop_scale);
#pragma unroll
      for (int e = 0; e < 4; ++e) keep[e] = k[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) keep[e] = rng_u16k(dkey, i0 + e) >= ep.drop_thr ? ep.drop_scale : 0.f;
    }
  } else if (ep.drop_scale != 1.f) {
#pragma unroll
    for (int e = 0; e < 4; ++e) keep[e] = ep.drop_scale;
  }
  if (ep.act == ACT_GELU_DUAL) {
    f32x4 g, d;
    gelu_gg4(v, g, d);
#pragma unroll
    for (int e = 0; e < 4; ++e) g[e] *= keep[e];
    if (ep.gd == 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] *= keep[e];
    }
    if (ep.out) store4v<FAST>(ep.out, (long)m * ep.ldo + n, ep.gd ? d : v, nv, ep.out_dt);
    store4v<FAST>(ep.out2, (long)m * ep.ldo2 + n, g, nv, ep.out2_dt);
    return;
  }
  if (ep.act == ACT_TANH) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
  }
  if (ep.relu) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] *= keep[e];
  if (ep.act == ACT_GELU_BWD) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] *= ep.gd ? in.aux[e] : gelu_grad(in.aux[e]);
  }
  if (ep.resid) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = in.resid[e] + in.rowscale * v[e];
  }
  if (ep.mode == EPI_STORE) {
    store4v<FAST>(ep.out, (long)m * ep.ldo + n, v, nv, ep.out_dt);
  } else if (ep.mode == EPI_SPLIT2) {
    for (int e = 0; e < nv; ++e) {
      if (n + e < ep.split_col) st_dt(ep.out, (long)m * ep.ldo + n + e, v[e], ep.out_dt);
      else st_dt(ep.out2, (long)m * ep.ldo2 + (n + e - ep.split_col), v[e], ep.out2_dt);
    }
  } else {  // EPI_PATCH: m = token (b, py, px), n = (ky*P + kx)*C + c
    const int hw = ep.pHp * ep.pWp;
    const int b = m / hw, rem = m - b * hw;
    const int py = rem / ep.pWp, px = rem - py * ep.pWp;
    for (int e = 0; e < nv; ++e) {
      const int nn = n + e;
      const int tap = nn / ep.pC, c = nn - tap * ep.pC;
      const int ky = tap / ep.pP, kx = tap - ky * ep.pP;
      const long o = (((long)b * ep.pH + py * ep.pP + ky) * ep.pW + px * ep.pP + kx) * ep.pC + c;
      st_dt(ep.out, o, v[e], ep.out_dt);
    }
  }
}

// k-major ("MN") bf16 tile, [64 k][R rows] with 2R-byte rows and no padding:
// the 16-byte chunk c of row k sits at chunk c ^ swz(k), swz(k) = 2(k&3) ^
// 8((k>>3)&1) (R = 128 and 256: every row starts a 256-B bank row, so the 8
// rows of one 32-lane half of a transposed read land on 8 distinct even 16-B
// slots) or 2((k>>1)&1) ^ 4((k>>3)&1) (R = 64).  Conflict-free
// for the 16x16x32 operand fragments read with two ds_read_b64_tr_b16 (checked
// exhaustively) and for the ds_write_b128 of 8 lanes filling one row; the same
// layout as the LDS-DMA MN image (DmaImg), which applies the swizzle on the
// source side.
template <int R>
struct MnSwz {
  static_assert(R == 64 || R == 128 || R == 256, "MN tile: 64, 128 or 256 rows");
  static constexpr int ROWB = 2 * R;
  __device__ __forceinline__ static int swz(int k) {
    return R >= 128 ? ((2 * (k & 3)) ^ (8 * ((k >> 3) & 1))) : ((2 * ((k >> 1) & 1)) ^ (4 * ((k >> 3) & 1)));
  }
  __device__ __forceinline__ static int off(int k, int chunk) { return k * ROWB + ((chunk ^ swz(k)) << 4); }
  // 16x16x32 operand fragment of rows rb..rb+15, k-step s: lane (g = l>>4,
  // i = l&15) receives rows rb+i, k = 32s + 8g + 0..7
  __device__ __forceinline__ static u32x4 frag(const char* img, int rb, int s, int lane) {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int k0 = 32 * s + 8 * g + q;
    const int ch = (rb >> 3) + (p >> 1), byte = (p & 1) * 8;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + off(k0, ch) + byte));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + off(k0 + 4, ch) + byte));
    u32x4 r;
    r[0] = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
    r[1] = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
    r[2] = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
    r[3] = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
    return r;
  }
};

// ds_read_b64_tr_b16 through inline asm, for images filled by LDS-DMA: the
// intrinsic carries no memory operand, so the compiler's wait-count pass
// assumes it may alias every in-flight LDS-DMA and drains vmcnt(0) before the
// first transposed read of a stage (which defeats the DMA prefetch).  Reads
// issued this way are invisible to that pass: lgkm_wait0() waits for them
// (lgkmcnt(0)) and lds_pin() pins the fragment registers after the wait.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ uint2 ds_tr16_asm(unsigned addr) {
  uint2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
__device__ __forceinline__ u32x4 tr2_asm(unsigned lo, unsigned hi) {
  const uint2 l = ds_tr16_asm(lo), h = ds_tr16_asm(hi);
  return (u32x4){l.x, l.y, h.x, h.y};
}
template <int NF>
__device__ __forceinline__ void lds_pin(u32x4 (&f)[NF]) {
#pragma unroll
  for (int i = 0; i < NF; ++i) asm volatile("" : "+v"(f[i]));
}
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Epilogue barrier over LDS only: the tile image and reduction scratch are the
// only data shared between waves there.  __syncthreads() is a workgroup
// release/acquire fence as well, which makes every wave wait (vmcnt(0)) for
// all of its output stores to land before the next half can be staged.
__device__ __forceinline__ void epi_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename T, int R, bool KC>
struct TileCfg {
  static constexpr int E = Elem<T>::PER16;
  static constexpr int BK = KSTAGE / sizeof(T);
  static constexpr bool TR = !KC && sizeof(T) == 2;
  static constexpr int BYTES = R * KSTAGE;  // per stage (MN bf16: 64 k x 2R bytes, unpadded)
  static constexpr int CH = R * KSTAGE / 16 / GEMM_THREADS;           // chunks per thread
  // chunk ch -> (row, k) offsets within the stage
  __device__ __forceinline__ static void map(int ch, int& row, int& k) {
    if (KC) {
      row = ch / (KSTAGE / 16);
      k = (ch % (KSTAGE / 16)) * E;
    } else {
      k = ch / (R / E);
      row = (ch % (R / E)) * E;
    }
  }
  __device__ __forceinline__ static void store(char* tile, int ch, const u32x4& v) {
    int row, k;
    map(ch, row, k);
    if (KC) {
      *(u32x4*)(tile + kc_off(row, k / E)) = v;
    } else if (TR) {
      *(u32x4*)(tile + MnSwz<R>::off(k, row / E)) = v;
    } else {  // f32 scatter-transpose into the KC layout
      const T* e = (const T*)&v;
#pragma unroll
      for (int i = 0; i < E; ++i)
        *(T*)(tile + kc_off(row + i, k / E) + (k % E) * sizeof(T)) = e[i];
    }
  }
  __device__ __forceinline__ static u32x4 frag(const char* tile, int rb, int s, int lane) {
    if constexpr (TR) {
      return MnSwz<R>::frag(tile, rb, s, lane);
    } else {
      return *(const u32x4*)(tile + kc_off(rb + (lane & 15), 4 * s + (lane >> 4)));
    }
  }
};

// NRS register stages: stage t + NRS - 1 is in flight (global loads) while
// stage t runs on the MFMAs, so a load has NRS - 1 compute phases to land.
template <typename T, int BM, int BN, class LA, class LB, int NRS = 2>
struct GemmCore {
  static_assert(NRS >= 2 && NRS <= 4, "register stages");
  using TA = TileCfg<T, BM, LA::KC>;
  using TB = TileCfg<T, BN, LB::KC>;
  static constexpr int BK = TA::BK;
  static constexpr int WM = 2, WN = 2;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int CA = TA::CH, CB = TB::CH;
  static constexpr int STEPS = KSTAGE / 64;
  static constexpr int SM_LOOP = 2 * (TA::BYTES + TB::BYTES);

  // the K loop: acc += A[m0.., kbeg..kend) * B[n0.., kbeg..kend)^T
  // RS: also accumulate row sums of the A tile (bf16 k-major A only: the
  // wgrad dy operand, whose row sums over the token reduction are the bias
  // gradient); rs_on is uniform (only the blocks of the first N tile)
  static constexpr int RS_RG = BM / 8, RS_KG = GEMM_THREADS / RS_RG, RS_KPG = BK / RS_KG;
  template <bool CHECK, bool RS = false>
  __device__ __forceinline__ static void run(const LA& la, const LB& lb, char* smem, int m0, int n0, int kbeg,
                                             int kend, f32x4 (&acc)[FM][FN], float* rsacc = nullptr,
                                             bool rs_on = false) {
    char* As = smem;
    char* Bs = smem + 2 * TA::BYTES;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
    if (nk == 0) return;

    typename LA::Sh sa;
    typename LB::Sh sb;
    typename LA::Cur ca[CA];
    typename LB::Cur cb[CB];
    int kofa[CA], kofb[CB];
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      int row, k;
      TA::map(tid + c * GEMM_THREADS, row, k);
      kofa[c] = k;
      la.init(sa, ca[c], m0 + row, kbeg + k);
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      int row, k;
      TB::map(tid + c * GEMM_THREADS, row, k);
      kofb[c] = k;
      lb.init(sb, cb[c], n0 + row, kbeg + k);
    }
    u32x4 ra[NRS][CA], rb[NRS][CB];
    // stage s is fetched with the cursors at kbeg + s*BK; stages beyond the end
    // re-read the last valid stage (keeps the load count static; never used)
    int fetched = 0;
    auto fetch = [&](u32x4(&ra)[CA], u32x4(&rb)[CB]) {
      const int s = fetched;
      if (s > 0 && s < nk) {
        la.step_sh(sa, BK);
        lb.step_sh(sb, BK);
#pragma unroll
        for (int c = 0; c < CA; ++c) la.step(ca[c], BK);
#pragma unroll
        for (int c = 0; c < CB; ++c) lb.step(cb[c], BK);
      }
      const int k0 = kbeg + min(s, nk - 1) * BK;
#pragma unroll
      for (int c = 0; c < CA; ++c)
        ra[c] = (!CHECK || k0 + kofa[c] < kend) ? la.template fetch<CHECK>(sa, ca[c]) : (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
      for (int c = 0; c < CB; ++c)
        rb[c] = (!CHECK || k0 + kofb[c] < kend) ? lb.template fetch<CHECK>(sb, cb[c]) : (u32x4){0u, 0u, 0u, 0u};
      ++fetched;
    };
    auto stash = [&](const u32x4(&ra)[CA], const u32x4(&rb)[CB], int buf) {
#pragma unroll
      for (int c = 0; c < CA; ++c) TA::store(As + buf * TA::BYTES, tid + c * GEMM_THREADS, ra[c]);
#pragma unroll
      for (int c = 0; c < CB; ++c) TB::store(Bs + buf * TB::BYTES, tid + c * GEMM_THREADS, rb[c]);
    };
    auto compute = [&](int buf) {
      const char* at = As + buf * TA::BYTES;
      const char* bt = Bs + buf * TB::BYTES;
#pragma unroll
      for (int s = 0; s < STEPS; ++s) {
        u32x4 fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = TA::frag(at, wm * WTM + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[j] = TB::frag(bt, wn * WTN + j * 16, s, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            if constexpr (sizeof(T) == 2) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  __builtin_bit_cast(s16x8, fa[i]), __builtin_bit_cast(s16x8, fb[j]), acc[i][j], 0, 0, 0);
            } else {
              f32x4 va = __builtin_bit_cast(f32x4, fa[i]);
              f32x4 vb = __builtin_bit_cast(f32x4, fb[j]);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[0], vb[0], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[1], vb[1], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[2], vb[2], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[3], vb[3], acc[i][j], 0, 0, 0);
            }
          }
      }
    };

    auto rowsum = [&](int buf) {
      if constexpr (RS) {
        static_assert(TA::TR, "row sums need the k-major bf16 A tile");
        if (!rs_on) return;
        const char* at = As + buf * TA::BYTES;
        const int rg = tid % RS_RG, kg = tid / RS_RG;
#pragma unroll
        for (int i = 0; i < RS_KPG; ++i) {
          const u32x4 v = *(const u32x4*)(at + MnSwz<BM>::off(kg * RS_KPG + i, rg));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            rsacc[2 * e] += __uint_as_float(v[e] << 16);
            rsacc[2 * e + 1] += __uint_as_float(v[e] & 0xffff0000u);
          }
        }
      }
    };

    // prologue: stages 0 .. NRS-1 -> register slots; stage 0 -> LDS buffer 0
#pragma unroll
    for (int u = 0; u < NRS; ++u) fetch(ra[u], rb[u]);
    stash(ra[0], rb[0], 0);
    __syncthreads();
    for (int t = 0; t < nk; t += NRS) {
#pragma unroll
      for (int u = 0; u < NRS; ++u) {
        // stage t+u is in LDS buffer (t+u)&1 and its slot u is free: refill
        // slot u with stage t+u+NRS, run stage t+u, then move stage t+u+1
        // (slot (u+1) % NRS) into the other buffer
        const int buf = (t + u) & 1;
        fetch(ra[u], rb[u]);
        compute(buf);
        rowsum(buf);
        if (t + u + 1 < nk) stash(ra[(u + 1) % NRS], rb[(u + 1) % NRS], buf ^ 1);
        __syncthreads();
        if (t + u + 1 >= nk) return;
      }
    }
  }
};

// ------------------------------------------------ LDS-DMA K loop (bf16) -----
// For dense bf16 operands on interior tiles the K loop stages both operands
// with LDS-DMA (buffer_load_dwordx4 ... lds): no staging registers, no
// ds_write pass, no VGPR->LDS transfer.  One DMA wave-instruction moves 1 KiB
// into a lane-linear LDS range, so every image is a sequence of 1-KiB pieces
// and the bank swizzle is applied to the per-lane SOURCE address (and undone on
// the read):
//   KC (k contiguous, [rows][64 k]): 128-B rows, chunk ^ (row & 7) -- the
//       register path's layout (kc_off), fragments by ds_read_b128;
//   MN (rows contiguous, [64 k][R rows]): 2R-byte rows, chunk ^ swz(k) with
//       swz(k) = 2(k&3) ^ 8((k>>3)&1) (R = 128) or 2((k>>1)&1) ^ 4((k>>3)&1)
//       (R = 64), fragments by ds_read_b64_tr_b16; both are conflict-free for
//       the 16x16x32 operand reads (checked exhaustively).
// Two LDS buffers, stage t+1's DMA in flight while stage t is on the MFMAs; a
// counted vmcnt (never 0 inside the loop) and raw s_barriers, because
// __syncthreads() would drain the in-flight DMA (cdna_hip_programming.md,
// "Pipelining across barriers").  The epilogue is the register path's.
template <typename X>
struct IsDenseBf16 : std::false_type {};
template <bool KC>
struct IsDenseBf16<LdDense<bf16_t, KC>> : std::true_type {};

template <typename X>
struct IsConvFBf16 : std::false_type {};
template <>
struct IsConvFBf16<LdConvF<bf16_t>> : std::true_type {};

template <int R, bool KC>
struct DmaImg {
  static constexpr int ROWB = KC ? KSTAGE : 2 * R;  // bytes per LDS row
  static constexpr int NCH = ROWB / 16;             // 16-B chunks per row
  static constexpr int BYTES = R * KSTAGE;          // one stage: 64 k x R rows x 2 B
  static constexpr int PIECES = BYTES / 1024;       // DMA wave-instructions per stage
  static constexpr int RPP = 1024 / ROWB;           // LDS rows per piece
  static_assert(KC || R == 64 || R == 128 || R == 256, "MN DMA image: 64, 128 or 256 rows");
  __device__ __forceinline__ static int swz(int k) { return MnSwz<KC ? 128 : R>::swz(k); }
  // byte offset (from the tile's origin element) that `lane` fetches for piece pc
  __device__ __forceinline__ static unsigned src_off(int pc, int lane, long ld) {
    const int row = pc * RPP + lane / NCH;  // KC: operand row; MN: k
    const int pcn = lane % NCH;
    const int c = KC ? (pcn ^ (row & 7)) : (pcn ^ swz(row));
    return (unsigned)(((long)row * ld + c * 8) * 2);
  }
  // 16x16x32 operand fragment of rows rb..rb+15, k-step s (MN: asm transposed
  // reads, see lds_fence; callers wait with lgkm_wait0 + lds_pin)
  __device__ __forceinline__ static u32x4 frag(const char* img, int rb, int s, int lane) {
    if constexpr (KC) {
      return *(const u32x4*)(img + kc_off(rb + (lane & 15), 4 * s + (lane >> 4)));
    } else {
      const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
      const int k0 = 32 * s + 8 * g + q;
      const int ch = (rb >> 3) + (p >> 1), byte = (p & 1) * 8;
      const unsigned base = lds_addr(img) + byte;
      return tr2_asm(base + MnSwz<R>::off(k0, ch), base + MnSwz<R>::off(k0 + 4, ch));
    }
  }
};

template <int BM, int BN, bool KCA, bool KCB, int NB = 2>
struct GemmCoreDma {
  using IA = DmaImg<BM, KCA>;
  using IB = DmaImg<BN, KCB>;
  static constexpr int BK = 64;
  static constexpr int WM = 2, WN = 2;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int PA = IA::PIECES / 4, PB = IB::PIECES / 4;  // pieces per wave per stage
  static constexpr int SM_LOOP = NB * (IA::BYTES + IB::BYTES);
  static_assert(NB >= 1 && NB <= 3, "one to three LDS stage buffers");
  static_assert(IA::PIECES % 4 == 0 && IB::PIECES % 4 == 0, "pieces per stage must split over 4 waves");

  template <class L>
  __device__ __forceinline__ static __amdgpu_buffer_rsrc_t rsrc(const L& l) {
    const long elems = L::KC ? (long)l.rows * l.ld : (long)l.K * l.ld;
    const long bytes = elems * 2;
    return __builtin_amdgcn_make_buffer_rsrc((void*)l.p, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                             0x00020000);
  }

  // A is a dense bf16 matrix or the implicit-im2col conv loader (LdConvF: A
  // rows are output pixels, one 64-channel stage lies in one tap and one
  // source).  For the conv, a lane's row in each of its A pieces is a fixed
  // pixel (source row base, iy0, ix0 kept per piece), its 16-byte chunk a fixed
  // 8-channel offset (the KC source swizzle depends on the lane only), and the
  // stage's tap / channel base is wave-uniform: each stage's per-lane byte
  // offset is a few integer ops, and taps in the zero padding (or past the
  // tensor) get an offset past num_records, which the DMA reads as zeros.
  __device__ __forceinline__ static void run(const LdDense<bf16_t, KCA>& la, const LdDense<bf16_t, KCB>& lb,
                                             char* smem, int m0, int n0, int kbeg, int kend, f32x4 (&acc)[FM][FN]) {
    run_t(la, lb, smem, m0, n0, kbeg, kend, acc);
  }
  __device__ __forceinline__ static void run(const LdConvF<bf16_t>& la, const LdDense<bf16_t, KCB>& lb, char* smem,
                                             int m0, int n0, int kbeg, int kend, f32x4 (&acc)[FM][FN]) {
    run_t(la, lb, smem, m0, n0, kbeg, kend, acc);
  }
  template <class LA>
  __device__ __forceinline__ static void run_t(const LA& la, const LdDense<bf16_t, KCB>& lb, char* smem, int m0,
                                               int n0, int kbeg, int kend, f32x4 (&acc)[FM][FN]) {
    constexpr bool CONV = IsConvFBf16<LA>::value;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int nk = (kend - kbeg) / BK;
    if (nk <= 0) return;
    const __amdgpu_buffer_rsrc_t rb = rsrc(lb);
    const unsigned ob = (unsigned)(KCB ? ((long)n0 * lb.ld + kbeg) * 2 : ((long)kbeg * lb.ld + n0) * 2);
    const unsigned db = (unsigned)(KCB ? BK * 2 : (long)BK * lb.ld * 2);
    unsigned vb[PB];
#pragma unroll
    for (int i = 0; i < PB; ++i) vb[i] = IB::src_off(wid + 4 * i, lane, lb.ld);
    // dense A: per-lane source offsets and a uniform per-stage advance
    __amdgpu_buffer_rsrc_t ra;
    unsigned va[PA], oa = 0, da = 0;
    // conv A: per-piece pixel state, the lane's chunk offset, the stage tap cursor
    int crb[PA], ciy[PA], cix[PA], cl8 = 0, c0 = 0, kx = 0, ky = 0;
    __amdgpu_buffer_rsrc_t ra2;
    if constexpr (CONV) {
      static_assert(KCA, "conv A operand is k-contiguous");
      ra = __builtin_amdgcn_make_buffer_rsrc((void*)la.src1, (short)0, (int)la.bytes1, 0x00020000);
      ra2 = __builtin_amdgcn_make_buffer_rsrc((void*)la.src2, (short)0, (int)la.bytes2, 0x00020000);
      cl8 = ((lane & 7) ^ ((lane >> 3) & 7)) << 3;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int p = m0 + (wid + 4 * i) * IA::RPP + (lane >> 3);
        int n, oy, ox;
        la.pix(p, n, oy, ox);
        crb[i] = n * la.Hs;
        ciy[i] = oy * la.S - la.Pd;
        cix[i] = ox * la.S - la.Pd;
      }
      const int kb = __builtin_amdgcn_readfirstlane(kbeg);
      const int tap = kb / la.Ctot;
      c0 = kb - tap * la.Ctot;
      ky = tap / la.KS;
      kx = tap - ky * la.KS;
    } else {
      ra = rsrc(la);
      oa = (unsigned)(KCA ? ((long)m0 * la.ld + kbeg) * 2 : ((long)kbeg * la.ld + m0) * 2);
      da = (unsigned)(KCA ? BK * 2 : (long)BK * la.ld * 2);
#pragma unroll
      for (int i = 0; i < PA; ++i) va[i] = IA::src_off(wid + 4 * i, lane, la.ld);
    }
    auto issue = [&](int t) {
      char* abuf = smem + (NB >= 2 ? t % NB : 0) * (IA::BYTES + IB::BYTES);
      char* bbuf = abuf + IA::BYTES;
      const unsigned sb = ob + (unsigned)(t < nk ? t : nk - 1) * db;
      if constexpr (CONV) {
        const bool first = c0 < la.C1;  // uniform
        const int Cx = first ? la.C1 : la.C2;
        const int coff = (first ? c0 : c0 - la.C1) + cl8;
#pragma unroll
        for (int i = 0; i < PA; ++i) {
          const int iy = ciy[i] + ky, ix = cix[i] + kx;
          const bool ok = (unsigned)iy < (unsigned)la.Hi && (unsigned)ix < (unsigned)la.Wi;
          const int off = (((crb[i] + (iy >> la.ushift)) * la.Ws + (ix >> la.ushift)) * Cx + coff) * 2;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(first ? ra : ra2,
                                                   (__attribute__((address_space(3))) void*)(abuf + (wid + 4 * i) * 1024),
                                                   16, ok ? (unsigned)off : 0x80000000u, 0, 0, 0);
        }
        c0 += BK;  // next stage's tap cursor (LdConvF::step_sh)
        if (c0 >= la.Ctot) {
          c0 -= la.Ctot;
          if (++kx == la.KS) {
            kx = 0;
            ++ky;
          }
        }
      } else {
        const unsigned sa = oa + (unsigned)(t < nk ? t : nk - 1) * da;
#pragma unroll
        for (int i = 0; i < PA; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(ra,
                                                   (__attribute__((address_space(3))) void*)(abuf + (wid + 4 * i) * 1024),
                                                   16, va[i], sa, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < PB; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(bbuf + (wid + 4 * i) * 1024),
                                                 16, vb[i], sb, 0, 0);
    };
    auto load = [&](const char* at, const char* bt, int s, u32x4 (&fa)[FM], u32x4 (&fb)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = IA::frag(at, wm * WTM + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = IB::frag(bt, wn * WTN + j * 16, s, lane);
    };
    auto mma = [&](const u32x4 (&fa)[FM], const u32x4 (&fb)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, fa[i]),
                                                              __builtin_bit_cast(s16x8, fb[j]), acc[i][j], 0, 0, 0);
    };
    // k-step 0's fragments, then k-step 1's reads in flight under k-step 0's
    // MFMAs (explicit lgkmcnt waits: the MN reads are asm, DmaImg::frag)
    auto compute = [&](int t) {
      const char* at = smem + (NB >= 2 ? t % NB : 0) * (IA::BYTES + IB::BYTES);
      const char* bt = at + IA::BYTES;
      static_assert(BK == 64, "two k-steps per stage");
      u32x4 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
      load(at, bt, 0, fa0, fb0);
      lgkm_wait0();
      lds_pin(fa0);
      lds_pin(fb0);
      load(at, bt, 1, fa1, fb1);
      mma(fa0, fb0);
      lgkm_wait0();
      lds_pin(fa1);
      lds_pin(fb1);
      mma(fa1, fb1);
    };
    constexpr int INFLIGHT = PA + PB;  // this wave's DMA instructions of one stage
    if constexpr (NB == 1) {
      // one stage buffer (the 3-workgroups-per-CU variant): no prefetch inside
      // the workgroup; the co-resident workgroups, out of phase, keep the CU's
      // DMA and matrix cores busy
      for (int t = 0; t < nk; ++t) {
        issue(t);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        compute(t);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      return;
    }
    // Two buffers, one barrier per stage: stage t+1's DMA is issued inside
    // stage t's compute, spread over k-step 0's MFMAs (an LDS-DMA piece costs
    // its wave ~60-180 issue cycles: issued as one block they left the matrix
    // pipe idle), into the buffer every wave released before the barrier that
    // opened stage t (its reads of stage t-1 were waited for before its
    // MFMAs).  The last stage issues a never-read stage (zeros past the
    // operand or the next slice's bytes) into that free buffer, so the loop
    // body is uniform; it is drained before the epilogue reuses LDS.
    // Measured (tools/ring_bench.py probes, 8192x2048, K = 2048): 853 -> 1042
    // TFLOP/s against the two-barrier loop with the DMA issued in a block.
    // Three buffers (NB = 3, round 6: the long-K 128x64 / 64x64 kernels): stage
    // t+2 is issued during stage t, so one stage stays in flight through the
    // wait (a counted vmcnt of one stage's DMA instructions).
    constexpr int MPD = (FM * FN) / INFLIGHT > 0 ? (FM * FN) / INFLIGHT : 1;
    issue(0);
    if constexpr (NB == 3) issue(1);
    for (int t = 0; t < nk; ++t) {
      if constexpr (NB == 3)
        __builtin_amdgcn_s_waitcnt(0x0F70 | (INFLIGHT & 15) | (((INFLIGHT >> 4) & 3) << 14));  // vmcnt(INFLIGHT)
      else
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): stage t landed (for this wave)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();  // ... for every wave; buffer (t + NB - 1) % NB is free
      asm volatile("" ::: "memory");
      const char* at = smem + (t % NB) * (IA::BYTES + IB::BYTES);
      const char* bt = at + IA::BYTES;
      u32x4 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
      load(at, bt, 0, fa0, fb0);
      lgkm_wait0();
      lds_pin(fa0);
      lds_pin(fb0);
      load(at, bt, 1, fa1, fb1);
      issue(t + NB - 1);
      mma(fa0, fb0);
      __builtin_amdgcn_sched_group_barrier(0x100, FM + FN, 0);  // k-step 1 fragment reads first
#pragma unroll
      for (int k = 0; k < INFLIGHT && MPD * (k + 1) <= FM * FN; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, MPD, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);    // one DMA piece
      }
      lgkm_wait0();
      lds_pin(fa1);
      lds_pin(fb1);
      mma(fa1, fb1);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // the trailing stage's DMA
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
};

// Diagnostic build only (-DHVIT_GEMM_STAMPS): per-workgroup wall-clock stamps
// (100 MHz s_memrealtime) at start / after the K loop / at exit, read back with
// hvit_debug_gemm_stamps().  Never enabled in the shipped library.
#ifdef HVIT_GEMM_STAMPS
extern __device__ unsigned long long g_gemm_stamps[65536 * 4];
#define GEMM_STAMP(i)                                                                          \
  do {                                                                                         \
    const unsigned bid_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);      \
    if (threadIdx.x == 0 && bid_ < 65536) g_gemm_stamps[bid_ * 4 + (i)] = wall_clock64();      \
  } while (0)
#else
#define GEMM_STAMP(i) \
  do {                \
  } while (0)
#endif

template <typename X>
struct IsConvWF : std::false_type {};
template <typename T>
struct IsConvWF<LdConvWF<T>> : std::true_type {};
#ifndef HVIT_WF_STAGES
#define HVIT_WF_STAGES 2
#endif
#ifndef HVIT_BIG_OCC
#define HVIT_BIG_OCC 2
#endif
// XCD-aware tile order.  Workgroups are dealt round-robin over the 8 XCDs
// (block b and b + 8 share one XCD's 4 MiB L2), so in hardware order every
// XCD sees tiles from all over the output and re-fetches the same A rows / B
// columns from HBM.  Here the hardware block b is given logical tile
// base(b % 8) + b / 8: each XCD owns one contiguous range of the logical order
// (split-K slice major, then M tiles, N tiles fastest), i.e. a compact block of
// output tiles of one K slice whose operand panels stay L2-resident.  The
// mapping is a bijection for any grid size (q = nwg / 8 blocks per XCD, the
// first nwg % 8 XCDs one more).
struct TileId {
  int mt, nt, z;
};
__device__ __forceinline__ TileId tile_of(int remap) {
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  if (!remap) return {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  const int nwg = gx * gy * gz;
  const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int xcd = b & 7, slot = b >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  const int per = gx * gy;
  const int z = lid / per, rem = lid - z * per;
  const int mt = rem / gy;
  return {mt, rem - mt * gy, z};
}

// DMAK: 0 = register-staged K loop, 2 = LDS-DMA with two stage buffers (two
// workgroups per CU), 1 = LDS-DMA with one stage buffer (three per CU), 3 =
// three stage buffers (long K, 128x64 / 64x64 tiles)
template <typename T, int BM, int BN, class LA, class LB, int EK, bool RS = false, int DMAK = 0>
__global__ __launch_bounds__(GEMM_THREADS, (DMAK == 1 ? 3 : BM >= 128 ? HVIT_BIG_OCC : 2)) void gemm_kernel(LA la, LB lb, int M, int N,
                                                                                            int K, int kps, Epi ep) {
  // the implicit-im2col weight gradient streams both operands from HBM once:
  // deeper register prefetch (its 128x64 tiles have the registers for it)
  using C = GemmCore<T, BM, BN, LA, LB, IsConvWF<LB>::value ? HVIT_WF_STAGES : 2>;
  constexpr int WM = C::WM, WN = C::WN, WTM = C::WTM, WTN = C::WTN, FM = C::FM, FN = C::FN;
  // LDS-DMA K loop (DMAK kernels): dense bf16 operands, no row sums
  constexpr bool DMA =
      sizeof(T) == 2 && (IsDenseBf16<LA>::value || IsConvFBf16<LA>::value) && IsDenseBf16<LB>::value && !RS;
  constexpr int SM_DMA = DMAK ? GemmCoreDma<BM, BN, LA::KC, LB::KC, DMAK == 0 ? 2 : DMAK>::SM_LOOP : 0;
  constexpr int SM_LOOP = DMAK == 1 ? SM_DMA : (C::SM_LOOP > SM_DMA ? C::SM_LOOP : SM_DMA);
  constexpr int SM_EPI = (64 * (BN + 4) + (GEMM_THREADS / (BN / 4)) * BN) * 4;
  // the wide (8-column) epilogue's column-sum scratch follows the 64-row tile image
  constexpr int SM_W8 = DMAK ? (64 * (BN + 4) + (GEMM_THREADS / (BN / 8)) * BN) * 4 : 0;
  constexpr int SM_E = SM_EPI > SM_W8 ? SM_EPI : SM_W8;
  __shared__ __attribute__((aligned(16))) char smem[SM_LOOP > SM_E ? SM_LOOP : SM_E];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const TileId tid3 = tile_of(ep.xcd_remap);
  const uint32_t dkey = epi_key(ep);
  const int m0 = tid3.mt * BM;
  const int n0 = tid3.nt * BN;
  const int kbeg = tid3.z * kps;
  const int kend = min(K, kbeg + kps);
  const int frow = lane & 15, fq = lane >> 4;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // epilogue column ownership (see below); the bias is fetched before the K
  // loop so its latency hides behind the MFMAs
  constexpr int CP = BN + 4;                 // LDS tile pitch (floats)
  constexpr int HALVES = BM / 64;
  constexpr int C4 = BN / 4;                 // 4-column chunks per row
  constexpr int RSTEP = GEMM_THREADS / C4;   // rows advanced per sweep
  constexpr int NR = 64 / RSTEP;             // rows per thread per 64-row half
  const int c4 = tid % C4;
  const int r0 = tid / C4;
  const int n = n0 + c4 * 4;
  const bool nok = n < N;
  const bool full = n + 3 < N;
  const int nv = full ? 4 : N - n;
  const f32x4 bias4 = (ep.bias && nok) ? load4(ep.bias, n, nv, HVIT_F32) : (f32x4){0.f, 0.f, 0.f, 0.f};
  // EK_GELU_BWD with a bf16 h (the train path): this thread's h values for the
  // whole tile (NR rows x 4 columns per half) are loaded here, before the K
  // loop, so their HBM latency hides behind the MFMAs instead of stalling the
  // epilogue (full tiles only: the host guarantees them for this kind)
  constexpr int NPRE = EK == EK_GELU_BWD ? HALVES * NR : 1;
  uint2 hpre[NPRE];
  const bool hpre_on = EK == EK_GELU_BWD && ep.aux_dt == HVIT_BF16;
  if constexpr (EK == EK_GELU_BWD) {
    if (hpre_on) {
#pragma unroll
      for (int hh = 0; hh < HALVES; ++hh)
#pragma unroll
        for (int i = 0; i < NR; ++i)
          hpre[hh * NR + i] =
              *(const uint2*)((const bf16_t*)ep.aux + (long)(m0 + hh * 64 + r0 + i * RSTEP) * ep.ldaux + n);
    }
  }

  // Wide epilogue (DMAK kernels of the ViT kinds): a thread owns 8 adjacent
  // columns, so bf16 rows leave as one 16-byte store per lane (the 8-byte
  // stores of the 4-column layout made the epilogue store-issue bound:
  // measured 5.2 us of a 12 us fc1 tile).  Masks, math and results are the
  // 4-column epilogue's.
  constexpr bool W8 = DMAK && IsDenseBf16<LA>::value && (EK == EK_GELU_DUAL || EK == EK_GELU_BWD || EK == EK_STORE || EK == EK_RESID);
  constexpr int C8 = BN / 8, RS8 = GEMM_THREADS / C8, NR8 = 64 / RS8;
  const int c8 = tid % C8, q0 = tid / C8;
  const int n8 = n0 + c8 * 8;
  f32x4 b8a = {0.f, 0.f, 0.f, 0.f}, b8b = b8a;
  constexpr int NPRE8 = (W8 && EK == EK_GELU_BWD) ? HALVES * NR8 : 1;
  u32x4 hpre8[NPRE8];
  if constexpr (W8) {
    if (ep.bias) {
      b8a = *(const f32x4*)(ep.bias + n8);
      b8b = *(const f32x4*)(ep.bias + n8 + 4);
    }
    if constexpr (EK == EK_GELU_BWD) {
      if (ep.aux_dt == HVIT_BF16) {
#pragma unroll
        for (int hh = 0; hh < HALVES; ++hh)
#pragma unroll
          for (int i = 0; i < NR8; ++i)
            hpre8[hh * NR8 + i] =
                *(const u32x4*)((const bf16_t*)ep.aux + (long)(m0 + hh * 64 + q0 + i * RS8) * ep.ldaux + n8);
      }
    }
  }

  GEMM_STAMP(0);
  const bool interior = m0 + BM <= M && n0 + BN <= N && ((kend - kbeg) % C::BK) == 0 && la.fast() && lb.fast();
  float rsacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool rs_on = RS && tid3.nt == 0;
  if constexpr (DMAK) {
    // host guarantees: every tile interior, dense bf16 operands (only this loop
    // is compiled into the kernel, so it keeps its own register budget)
    static_assert(DMA, "DMA-only kernel needs dense bf16 operands");
    (void)interior;
    GemmCoreDma<BM, BN, LA::KC, LB::KC, DMAK == 0 ? 2 : DMAK>::run(la, lb, smem, m0, n0, kbeg, kend, acc);
  } else {
    if (interior) C::template run<false, RS>(la, lb, smem, m0, n0, kbeg, kend, acc, rsacc, rs_on);
    else C::template run<true, RS>(la, lb, smem, m0, n0, kbeg, kend, acc, rsacc, rs_on);
  }
  if constexpr (RS) {
    if (rs_on) {  // fold the k-groups: red[kg][BM]
      float* red = (float*)smem;
      const int rg = tid % C::RS_RG, kg = tid / C::RS_RG;
#pragma unroll
      for (int e = 0; e < 8; ++e) red[kg * BM + rg * 8 + e] = rsacc[e];
      __syncthreads();
      if (tid < BM && m0 + tid < M) {
        float sum = 0.f;
        for (int k = 0; k < C::RS_KG; ++k) sum += red[k * BM + tid];
        ep.rs_ptr[(long)tid3.z * ep.rs_stride + m0 + tid] = sum;
      }
      __syncthreads();
    }
  }
  GEMM_STAMP(1);
  // Retire every outstanding global load here (the bias, and the K loop's
  // never-consumed tail prefetches) with one explicit wait that the compiler's
  // wait-count pass sees: otherwise it re-emits vmcnt(0) per predicated output
  // row, and on gfx9 vmcnt also counts the epilogue's own stores -- each row
  // would wait for the previous row's store to land.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt untouched

  if constexpr (W8) {
    float* Cs = (float*)smem;
    float cs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto wide8 = [](const f32x4& a, const f32x4& b) {
      u32x4 u;
      u[0] = f2bf2(a[0], a[1]);
      u[1] = f2bf2(a[2], a[3]);
      u[2] = f2bf2(b[0], b[1]);
      u[3] = f2bf2(b[2], b[3]);
      return u;
    };
#pragma unroll
    for (int hh = 0; hh < HALVES; ++hh) {
      if (hh > 0) epi_barrier();
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wm * WTM + i * 16 + fq * 4 + r - hh * 64;
            if (row >= 0 && row < 64) Cs[row * CP + wn * WTN + j * 16 + frow] = acc[i][j][r];
          }
      epi_barrier();
      const int mbase = m0 + hh * 64;
      f32x4 ra[NR8], rb[NR8];
      float rsc[NR8];
      if constexpr (EK == EK_RESID) {
#pragma unroll
        for (int i = 0; i < NR8; ++i) {
          const int m = mbase + q0 + i * RS8;
          ra[i] = *(const f32x4*)((const float*)ep.resid + (long)m * ep.ldr + n8);
          rb[i] = *(const f32x4*)((const float*)ep.resid + (long)m * ep.ldr + n8 + 4);
          rsc[i] = ep.rowscale ? ep.rowscale[m / ep.rows_per_sample] : 1.f;
        }
      }
#pragma unroll
      for (int i = 0; i < NR8; ++i) {
        const int row = q0 + i * RS8;
        const int m = mbase + row;
        f32x4 va = *(const f32x4*)(Cs + row * CP + c8 * 8) + b8a;
        f32x4 vb = *(const f32x4*)(Cs + row * CP + c8 * 8 + 4) + b8b;
        if constexpr (EK == EK_GELU_DUAL) {
          f32x4 ka = {1.f, 1.f, 1.f, 1.f}, kb = ka;
          if (ep.drop_thr) {
            ka = keep4(ep, dkey, m, n8, N);
            kb = keep4(ep, dkey, m, n8 + 4, N);
          }
          f32x4 ga, gb, da, db;
          gelu_gg4(va, ga, da);
          gelu_gg4(vb, gb, db);
          ga *= ka;
          gb *= kb;
          if (ep.gd == 2) {  // GELU_DUAL_DK: the backward's multiplier carries the mask
            da *= ka;
            db *= kb;
          }
          // (no out: the inference form, HVIT_ACT_GELU -- only gelu(v) is stored)
          if (ep.out) *(u32x4*)((bf16_t*)ep.out + (long)m * ep.ldo + n8) = ep.gd ? wide8(da, db) : wide8(va, vb);
          *(u32x4*)((bf16_t*)ep.out2 + (long)m * ep.ldo2 + n8) = wide8(ga, gb);
        } else {
          if (EK != EK_STORE && ep.drop_thr) {
            va *= keep4(ep, dkey, m, n8, N);
            vb *= keep4(ep, dkey, m, n8 + 4, N);
          }
          if constexpr (EK == EK_GELU_BWD) {
            f32x4 ha, hb;
            if (ep.aux_dt == HVIT_BF16) {
              const u32x4 u = hpre8[hh * NR8 + i];
              ha = (f32x4){__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u),
                           __uint_as_float(u[1] << 16), __uint_as_float(u[1] & 0xffff0000u)};
              hb = (f32x4){__uint_as_float(u[2] << 16), __uint_as_float(u[2] & 0xffff0000u),
                           __uint_as_float(u[3] << 16), __uint_as_float(u[3] & 0xffff0000u)};
            } else {
              ha = *(const f32x4*)((const float*)ep.aux + (long)m * ep.ldaux + n8);
              hb = *(const f32x4*)((const float*)ep.aux + (long)m * ep.ldaux + n8 + 4);
            }
            if (ep.gd) {
              va *= ha;
              vb *= hb;
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                va[e] *= gelu_grad(ha[e]);
                vb[e] *= gelu_grad(hb[e]);
              }
            }
          }
          if constexpr (EK == EK_RESID) {
            va = ra[i] + rsc[i] * va;
            vb = rb[i] + rsc[i] * vb;
          }
          if (ep.out_dt == HVIT_BF16) {
            *(u32x4*)((bf16_t*)ep.out + (long)m * ep.ldo + n8) = wide8(va, vb);
          } else {
            *(f32x4*)((float*)ep.out + (long)m * ep.ldo + n8) = va;
            *(f32x4*)((float*)ep.out + (long)m * ep.ldo + n8 + 4) = vb;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            cs8[e] += va[e];
            cs8[4 + e] += vb[e];
          }
        }
      }
    }
    if (ep.colsum) {
      float* red = Cs + 64 * CP;  // [RS8][BN]
      epi_barrier();
#pragma unroll
      for (int e = 0; e < 8; ++e) red[q0 * BN + c8 * 8 + e] = cs8[e];
      epi_barrier();
      if (q0 == 0) {
        // deterministic: the tile's column sums as partial row m0/64 (plain
        // stores; the tile's other 64-row rows get zeros), summed in row order
        // by the caller (hvit_epilogue_t.colsum)
        float t8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float t = 0.f;
          for (int k = 0; k < RS8; ++k) t += red[k * BN + c8 * 8 + e];
          t8[e] = t;
        }
        float* row = ep.colsum + (long)(m0 / 64) * N + n8;
        *(f32x4*)row = (f32x4){t8[0], t8[1], t8[2], t8[3]};
        *(f32x4*)(row + 4) = (f32x4){t8[4], t8[5], t8[6], t8[7]};
#pragma unroll
        for (int r = 1; r < BM / 64; ++r) {
          *(f32x4*)(row + (long)r * N) = (f32x4){0.f, 0.f, 0.f, 0.f};
          *(f32x4*)(row + (long)r * N + 4) = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
    }
    epi_side(ep);
    GEMM_STAMP(2);
    return;
  }

  // ------------------------------------------------------------- epilogue ---
  // The accumulator tile is staged through LDS in 64-row halves (f32, padded
  // rows) and then processed row-contiguously: each thread owns 4 adjacent
  // columns, so bias / residual / aux loads and output stores are vectorised
  // and coalesced, and every acc[][] index stays static (no scratch).  Halves
  // whose rows and columns are all in range take a branch-free row loop.
  static_assert((64 * CP + RSTEP * BN) * 4 <= (int)sizeof(smem), "epilogue tile exceeds LDS");
  static_assert(2 * RSTEP * BN <= 64 * CP, "BN statistics scratch exceeds the tile image");
  float* Cs = (float*)smem;
  float csum[4] = {0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int hh = 0; hh < HALVES; ++hh) {
    if (hh > 0) epi_barrier();
    // write this half's accumulators: wave rows wm*WTM + i*16 + fq*4 + r
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WTM + i * 16 + fq * 4 + r - hh * 64;
          if (row >= 0 && row < 64) Cs[row * CP + wn * WTN + j * 16 + frow] = acc[i][j][r];
        }
    epi_barrier();
    const int mbase = m0 + hh * 64;
    const int rows_here = min(64, M - mbase);
    const bool all_in = mbase + 64 <= M && n0 + BN <= N && ep.vec_ok;  // uniform
    float st_sum[4] = {0.f, 0.f, 0.f, 0.f};
    f32x4 sv[NR];  // BN statistics: this thread's output values (registers, no Cs re-read)

    auto rows = [&](auto pred) {
      constexpr bool PRED = decltype(pred)::value;
      if constexpr (EK == EK_SLAB) {
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int row = r0 + i * RSTEP;
          const int m = mbase + row;
          if (PRED && (m >= M || !nok)) continue;
          const f32x4 v = *(const f32x4*)(Cs + row * CP + c4 * 4);
          float* slab = (float*)ep.out + (long)tid3.z * ep.slab_stride + (long)m * ep.ldo + n;
          if (!PRED || (full && (ep.ldo & 3) == 0)) *(f32x4*)slab = v;
          else store4_slow(slab, 0, v, nv, HVIT_F32);
        }
      } else if constexpr (EK == EK_STORE) {
        // host guarantees N % 4 == 0, ldo % 4 == 0 and an aligned output
        if (ep.pool2) {
          // pooled conv (eval BatchNorm folded, ReLU): window w = rows 4w .. 4w+3 of
          // this half (LdConvF::pool2 order); relu(max + bias) = max of relu(v + bias)
          // (uniform branch; host: bf16 output, every window inside the tile)
#pragma unroll
          for (int i = 0; i < (16 + RSTEP - 1) / RSTEP; ++i) {
            const int wi = r0 + i * RSTEP;
            if (wi >= 16 || 4 * wi >= rows_here || !nok) continue;
            f32x4 v = *(const f32x4*)(Cs + (4 * wi) * CP + c4 * 4);
#pragma unroll
            for (int q = 1; q < 4; ++q) {
              const f32x4 u = *(const f32x4*)(Cs + (4 * wi + q) * CP + c4 * 4);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], u[e]);
            }
            v += bias4;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            uint2 u;
            u.x = f2bf2(v[0], v[1]);
            u.y = f2bf2(v[2], v[3]);
            *(uint2*)((bf16_t*)ep.out + (long)((mbase >> 2) + wi) * ep.ldo + n) = u;
          }
          return;
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int row = r0 + i * RSTEP;
          const int m = mbase + row;
          if (PRED && (m >= M || !nok)) continue;
          f32x4 v = *(const f32x4*)(Cs + row * CP + c4 * 4) + bias4;
          if (ep.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if (ep.out_dt == HVIT_F32) {
            *(f32x4*)((float*)ep.out + (long)m * ep.ldo + n) = v;
          } else {
            uint2 u;
            u.x = f2bf2(v[0], v[1]);
            u.y = f2bf2(v[2], v[3]);
            *(uint2*)((bf16_t*)ep.out + (long)m * ep.ldo + n) = u;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            csum[e] += v[e];
            st_sum[e] += v[e];
          }
          sv[i] = v;
        }
      } else if constexpr (EK == EK_GELU_DUAL) {
        // h = v + b (saved for backward), a = dropout(gelu(h))
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int row = r0 + i * RSTEP;
          const int m = mbase + row;
          const f32x4 v = *(const f32x4*)(Cs + row * CP + c4 * 4) + bias4;
          const f32x4 k = ep.drop_thr ? keep4(ep, dkey, m, n, N) : (f32x4){1.f, 1.f, 1.f, 1.f};
          f32x4 g, d;
          gelu_gg4(v, g, d);
          g *= k;
          if (ep.gd == 2) d *= k;  // GELU_DUAL_DK
          if (ep.out) store4v<true>(ep.out, (long)m * ep.ldo + n, ep.gd ? d : v, 4, ep.out_dt);
          store4v<true>(ep.out2, (long)m * ep.ldo2 + n, g, 4, ep.out2_dt);
        }
      } else if constexpr (EK == EK_RESID) {
        // out = resid + rowscale[m / rps] * dropout(v + b)   (f32 residual stream)
        f32x4 r[NR];
        float rs[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int m = mbase + r0 + i * RSTEP;
          r[i] = *(const f32x4*)((const float*)ep.resid + (long)m * ep.ldr + n);
          rs[i] = ep.rowscale ? ep.rowscale[m / ep.rows_per_sample] : 1.f;
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int row = r0 + i * RSTEP;
          const int m = mbase + row;
          f32x4 v = *(const f32x4*)(Cs + row * CP + c4 * 4) + bias4;
          if (ep.drop_thr) v *= keep4(ep, dkey, m, n, N);
          v = r[i] + rs[i] * v;
          store4v<true>(ep.out, (long)m * ep.ldo + n, v, 4, ep.out_dt);
        }
      } else if constexpr (EK == EK_GELU_BWD) {
        // dh = dropout_mask(v) * gelu'(h)   (+ column sums for the bias grad)
        f32x4 h[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int m = mbase + r0 + i * RSTEP;
          if (hpre_on) {
            const uint2 u = hpre[hh * NR + i];
            h[i] = (f32x4){__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                           __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
          } else {
            h[i] = load4v<true>(ep.aux, (long)m * ep.ldaux + n, 4, ep.aux_dt);
          }
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int row = r0 + i * RSTEP;
          const int m = mbase + row;
          f32x4 v = *(const f32x4*)(Cs + row * CP + c4 * 4) + bias4;
          if (ep.drop_thr) v *= keep4(ep, dkey, m, n, N);
          if (ep.gd) {
            v *= h[i];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= gelu_grad(h[i][e]);
          }
          store4v<true>(ep.out, (long)m * ep.ldo + n, v, 4, ep.out_dt);
#pragma unroll
          for (int e = 0; e < 4; ++e) csum[e] += v[e];
        }
      } else if constexpr (EK == EK_PATCH) {
        // col2im scatter of the patch-embedding dgrad: m = token (b, py, px),
        // n = (ky*P + kx)*C + c.  The host guarantees C % 4 == 0 (a thread's
        // 4 columns share one tap), so the column part of the NHWC offset is
        // per-thread constant and each row is one vector store
        const int tap = n / ep.pC, cch = n - tap * ep.pC;
        const int ky = tap / ep.pP, kx = tap - ky * ep.pP;
        const long colpart = ((long)ky * ep.pW + kx) * ep.pC + cch;
        const int hw = ep.pHp * ep.pWp;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int row = r0 + i * RSTEP;
          const int m = mbase + row;
          const int b = m / hw, rem = m - b * hw;
          const int py = rem / ep.pWp, px = rem - py * ep.pWp;
          const long o = (((long)b * ep.pH + py * ep.pP) * ep.pW + px * ep.pP) * ep.pC + colpart;
          store4v<true>(ep.out, o, *(const f32x4*)(Cs + row * CP + c4 * 4), 4, ep.out_dt);
        }
      } else {
        EpiIn in[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int m = mbase + r0 + i * RSTEP;
          epi_load4<!PRED>(ep, m, n, nv, !PRED || (m < M && nok), in[i]);
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int row = r0 + i * RSTEP;
          const int m = mbase + row;
          if (PRED && (m >= M || !nok)) continue;
          f32x4 v = *(const f32x4*)(Cs + row * CP + c4 * 4);
          epi_apply4<!PRED>(ep, dkey, m, n, PRED ? nv : 4, N, v, bias4, in[i]);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (!PRED || e < nv) {
              csum[e] += v[e];
              st_sum[e] += v[e];
            }
          }
          sv[i] = v;
        }
      }
    };
    if constexpr (EK >= EK_GELU_DUAL) {
      rows(std::false_type());  // host guarantees full, aligned tiles
    } else {
      if (all_in) rows(std::false_type());
      else rows(std::true_type());
    }
    if (ep.stats && rows_here > 0) {
      // per-column (mean, M2) of this 64-row sub-tile.  Each thread holds its
      // rows r0 + i*RSTEP (i < cnt) of 4 columns in registers: local mean and
      // M2 there; the RSTEP partials of a column are then merged by one thread
      // per column (r0 < 4 picks column n + r0), 128 columns in parallel.  Full
      // halves (every partial over NR rows) merge without divisions:
      //   mean = sum(m_k) / RSTEP,  M2 = sum(M2_k) + NR sum((m_k - mean)^2);
      // ragged ones by Chan's pairwise rule.  (A single-wave sequential merge
      // with IEEE divisions cost ~1.5 us per tile, 34 us of the enc1 conv.)
      const bool fullh = rows_here == 64;  // uniform
      const int cnt = fullh ? NR : (rows_here > r0 ? min(NR, (rows_here - r0 + RSTEP - 1) / RSTEP) : 0);
      const float inv = fullh ? 1.f / (float)NR : (cnt ? 1.f / (float)cnt : 0.f);
      float mean[4], q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) mean[e] = st_sum[e] * inv;
#pragma unroll
      for (int i = 0; i < NR; ++i)
        if (fullh || i < cnt)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = sv[i][e] - mean[e];
            q[e] += d * d;
          }
      float* red = Cs;  // [2][RSTEP][BN]; the tile's LDS image is no longer read
      epi_barrier();
      *(f32x4*)(red + r0 * BN + c4 * 4) = (f32x4){mean[0], mean[1], mean[2], mean[3]};
      *(f32x4*)(red + (RSTEP + r0) * BN + c4 * 4) = (f32x4){q[0], q[1], q[2], q[3]};
      epi_barrier();
      if (r0 < 4 && n + r0 < N) {
        const int col = c4 * 4 + r0;
        float mk[RSTEP], qs = 0.f, mu = 0.f, m2 = 0.f;
#pragma unroll
        for (int k = 0; k < RSTEP; ++k) {
          mk[k] = red[k * BN + col];
          qs += red[(RSTEP + k) * BN + col];
        }
        if (fullh) {
#pragma unroll
          for (int k = 0; k < RSTEP; ++k) mu += mk[k];
          mu *= 1.f / (float)RSTEP;
          float dd = 0.f;
#pragma unroll
          for (int k = 0; k < RSTEP; ++k) dd += (mk[k] - mu) * (mk[k] - mu);
          m2 = qs + (float)NR * dd;
        } else {
          float na = 0.f;
          m2 = qs;
#pragma unroll
          for (int k = 0; k < RSTEP; ++k) {
            const int ck = rows_here > k ? min(NR, (rows_here - k + RSTEP - 1) / RSTEP) : 0;
            if (ck == 0) continue;
            const float nn = na + (float)ck, wb = (float)ck / nn;
            const float d = mk[k] - mu;
            mu += d * wb;
            m2 += d * d * (na * wb);
            na = nn;
          }
        }
        const long tile = (m0 / 64) + hh;
        *(float2*)(ep.stats + (tile * N + n + r0) * 2) = make_float2(mu, m2);
      }
    }
  }
  if (ep.colsum) {
    float* red = Cs + 64 * CP;
    epi_barrier();
    for (int e = 0; e < 4; ++e) red[r0 * BN + c4 * 4 + e] = csum[e];
    epi_barrier();
    if (r0 == 0)
      // deterministic partial row m0/64 (zeros in the tile's other 64-row rows)
      for (int e = 0; e < 4; ++e) {
        if (n + e >= N) break;
        float s = 0.f;
        for (int k = 0; k < RSTEP; ++k) s += red[k * BN + c4 * 4 + e];
        float* row = ep.colsum + (long)(m0 / 64) * N + n + e;
        *row = s;
        for (int r = 1; r < BM / 64; ++r)
          if (m0 + 64 * r < M) row[(long)r * N] = 0.f;
      }
  }
  epi_side(ep);
  GEMM_STAMP(2);
}




// host-side launcher --------------------------------------------------------
template <class L>
inline long dense_bytes(const L&) { return 0; }
template <typename T, bool KC>
inline long dense_bytes(const LdDense<T, KC>& l) { return (KC ? (long)l.rows : (long)l.K) * l.ld * (long)sizeof(T); }
template <class X>
struct IsDenseKC : std::false_type {};
template <typename T>
struct IsDenseKC<LdDense<T, true>> : std::true_type {};

// Effective split-K count after rounding each split to whole K-tiles (never
// more than requested).  Callers that reduce slabs must use this count.
template <typename T>
inline int plan_splits(int K, int splits, int* kps_out = nullptr) {
  constexpr int BK = KSTAGE / sizeof(T);
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  if (kps < BK) kps = BK;
  if (kps_out) *kps_out = kps;
  return K > 0 ? (K + kps - 1) / kps : 1;
}

// LDS-DMA stage buffers of the 128x64 / 64x64 kernels on long K loops
// (hvit_gemm_tune(8, v): 3 = three buffers from DEEP_MIN_STAGES stages on, 4 = from 8 stages, 2 = two)
inline int& dma_depth_ref() {
  // same-box A/B (gpurun_out/r6n_dma*): two buffers 4.656-4.660 ms/step, three from 16 stages
  // 4.543-4.551, three from 8 stages 4.509-4.524 (vit_linear_dgrad 0.784 -> 0.728, vit_linear_fwd
  // 0.774 -> 0.741, conv_fwd 0.410 -> 0.388 ms/step)
  static int v = 4;
  return v;
}
inline int dma_depth() { return dma_depth_ref(); }
constexpr int DEEP_MIN_STAGES = 16;

template <typename T, class LA, class LB>
int launch_gemm(LA la, LB lb, int M, int N, int K, int splits, const Epi& ep_in, hipStream_t st,
                int force_tile = 0) {
  Epi ep = ep_in;
  if (ep.slab_stride == 0) ep.slab_stride = (long)M * ep.ldo;
  ep.xcd_remap = 1;
  // the DMA loop addresses operands with 32-bit byte offsets
  ep.dma = dense_bytes(la) < (1L << 31) && dense_bytes(lb) < (1L << 31);
  auto vok = [](const void* p, long ld) { return !p || ((((uintptr_t)p) & 15) == 0 && ld % 4 == 0); };
  ep.vec_ok = N % 4 == 0 && vok(ep.out, ep.ldo) && vok(ep.out2, ep.ldo2) && vok(ep.aux, ep.ldaux) &&
              vok(ep.resid, ep.ldr) && vok(ep.rowadd, ep.rowadd_ld);
  if (M <= 0 || N <= 0) return HVIT_OK;
  int kps = 0;
  splits = plan_splits<T>(K, splits, &kps);
  if (splits > 1 && ep.mode != EPI_SLAB) {
    hvit_set_error("launch_gemm: split-K requires EPI_SLAB");
    return HVIT_ERR_ARG;
  }
  // tile: 128x128 when the grid still fills the chip; 128x64 for narrow
  // outputs (N <= 64: conv layers with 64 channels); else 64x64
  int tile = force_tile;
  if (!tile) {
    // 128x64 also when 128x128 would leave fewer than ~1.5 workgroups per CU
    // or a half-empty last column tile (measured: 2.5 % per train step)
    constexpr int policy = 2;  // (policies 0 / 1 measured slower: DESIGN.md §8)
    const long b128 = (long)cdiv(M, 128) * cdiv(N, 128) * splits;
    const long b12864 = (long)cdiv(M, 128) * cdiv(N, 64) * splits;
    if (N <= 64 && (long)cdiv(M, 128) * splits >= 160) tile = 12864;
    else if (policy >= 1 && N > 64 && b128 < 384 && b12864 >= 384) tile = 12864;
    else if (policy >= 2 && N > 64 && N % 128 != 0 && N % 64 == 0 && b12864 >= 160) tile = 12864;
    else if (N > 64 && b128 >= 160) tile = 128;
    else tile = 64;
  }
  const bool lean_store = ep.mode == EPI_STORE && ep.act == ACT_NONE && !ep.rowadd && !ep.resid && !ep.drop_thr &&
                          ep.drop_scale == 1.f && N % 4 == 0 && ep.ldo % 4 == 0 && ((uintptr_t)ep.out & 15) == 0;
  int ek = ep.mode == EPI_SLAB ? EK_SLAB : (lean_store ? EK_STORE : EK_GEN);
  {
    const int bm = tile == 128 || tile == 12864 ? 128 : 64, bn = tile == 128 ? 128 : 64;
    const bool full_tiles = ep.vec_ok && M % bm == 0 && N % bn == 0 && ep.mode == EPI_STORE && !ep.rowadd &&
                            !ep.stats;
    const bool drop_ok = ep.drop_thr ? N % 4 == 0 : ep.drop_scale == 1.f;
    // lean col2im scatter for the patch-embedding dgrad (no bias / act / dropout)
    const bool patch_lean = ep.mode == EPI_PATCH && ep.pC % 4 == 0 && M % bm == 0 && N % bn == 0 && !ep.bias &&
                            ep.act == ACT_NONE && !ep.drop_thr && ep.drop_scale == 1.f && !ep.resid && !ep.rowadd &&
                            !ep.stats && !ep.colsum && ((uintptr_t)ep.out & 15) == 0;
    if (IsDenseKC<LA>::value && ek == EK_GEN && patch_lean) ek = EK_PATCH;
    if (IsDenseKC<LA>::value && ek == EK_GEN && full_tiles && drop_ok) {
      if (ep.act == ACT_GELU_DUAL && !ep.resid) ek = EK_GELU_DUAL;
      else if (ep.act == ACT_NONE && ep.resid && ep.resid != ep.out) ek = EK_RESID;
      else if (ep.act == ACT_GELU_BWD && !ep.resid && ep.aux) ek = EK_GELU_BWD;
    }
  }
  // A-row sums (bias grad) only exist for the bf16 k-major A operand (wgrad)
  constexpr bool RS_OK = !LA::KC && sizeof(T) == 2;
  if (ep.rs_ptr && !RS_OK) {
    hvit_set_error("launch_gemm: A row sums need a bf16 k-major A operand");
    return HVIT_ERR_ARG;
  }
  // DMA-only kernel: dense bf16 operands, every tile interior (M, N multiples of
  // the tile, every K slice a multiple of 64, vector-aligned operands)
  // (or the implicit-im2col conv A loader, LdConvF: every 64-channel stage in
  // one tap and one source, byte offsets < 2^31 -- conv_fast_ok)
  constexpr bool CONV_A = IsConvFBf16<LA>::value;
  constexpr bool DMA_OK = sizeof(T) == 2 && (IsDenseBf16<LA>::value || CONV_A) && IsDenseBf16<LB>::value;
  bool all_in = false;
  if constexpr (DMA_OK) {
    const int bm = tile == 128 || tile == 12864 ? 128 : 64, bn = tile == 128 ? 128 : 64;
    // both operands k-major (the weight gradients): the register path measured
    // faster (1.04 vs 0.82 ms/step)
    constexpr bool mnmn = false;
    constexpr bool conv_dma = true;
    bool a_ok;
    if constexpr (CONV_A) a_ok = conv_dma;
    else a_ok = la.vok;
    all_in = ep.dma && M % bm == 0 && N % bn == 0 && kps % 64 == 0 && K % kps == 0 && a_ok && lb.vok &&
             !ep.rs_ptr && (LA::KC || LB::KC || mnmn);
  }
  auto go = [&](auto ekc) {
    constexpr int EKc = decltype(ekc)::value;
    auto launch = [&](auto rsc) {
      constexpr bool RSc = decltype(rsc)::value && RS_OK;
      auto kern = [&](auto bmc, auto bnc) {
        constexpr int BMc = decltype(bmc)::value, BNc = decltype(bnc)::value;
        dim3 g(cdiv(M, BMc), cdiv(N, BNc), splits);
        if constexpr (DMA_OK && !RSc) {
          if (all_in) {
            // one-buffer LDS-DMA kernels (3 workgroups per CU, out of phase, so one's
            // epilogue overlaps another's K loop) for the 128x128 forward kinds:
            // vit_linear_fwd 0.732 -> 0.721 ms/step.  Not for GELU_BWD (its h
            // prefetch spills at 168 VGPRs: dgrad 0.737 -> 0.780)
            constexpr bool nb1 = true;
            // conv forward (BN statistics epilogue) too: conv_fwd 0.471 -> 0.447 ms/step;
            // not the conv data gradient (0.346 -> 0.362)
            constexpr bool nb1c = true;
            if constexpr (BMc == 128 && BNc == 128 && (EKc == EK_GELU_DUAL || EKc == EK_STORE)) {
              if (CONV_A ? (nb1c && ep.stats) : nb1) {
                hipLaunchKernelGGL((gemm_kernel<T, BMc, BNc, LA, LB, EKc, false, 1>), g, dim3(GEMM_THREADS), 0, st,
                                   la, lb, M, N, K, kps, ep);
                return;
              }
            }
            if constexpr (!(BMc == 128 && BNc == 128)) {
              // (not the conv data gradients -- implicit im2col of dy, plain store epilogue:
              // conv_dgrad 0.376 -> 0.394 ms/step with three buffers, 72 KiB of LDS leaving
              // two workgroups per CU where the 48 KiB two-buffer kernel keeps three; the
              // patch-embedding forward, with its positional-row epilogue, does take them)
              if (dma_depth() >= 3 && kps / 64 >= (dma_depth() == 4 ? 8 : DEEP_MIN_STAGES) &&
                  (!CONV_A || ep.stats || ep.rowadd)) {
                hipLaunchKernelGGL((gemm_kernel<T, BMc, BNc, LA, LB, EKc, false, 3>), g, dim3(GEMM_THREADS), 0, st,
                                   la, lb, M, N, K, kps, ep);
                return;
              }
            }
            hipLaunchKernelGGL((gemm_kernel<T, BMc, BNc, LA, LB, EKc, false, 2>), g, dim3(GEMM_THREADS), 0, st,
                               la, lb, M, N, K, kps, ep);
            return;
          }
        }
        hipLaunchKernelGGL((gemm_kernel<T, BMc, BNc, LA, LB, EKc, RSc>), g, dim3(GEMM_THREADS), 0, st, la, lb, M, N,
                           K, kps, ep);
      };
      using I = std::integral_constant<int, 128>;
      using J = std::integral_constant<int, 64>;
      if (tile == 128) kern(I(), I());
      else if (tile == 12864) kern(I(), J());
      else kern(J(), J());
    };
    if constexpr (RS_OK && (EKc == EK_SLAB || EKc == EK_STORE)) {
      if (ep.rs_ptr) launch(std::true_type());
      else launch(std::false_type());
    } else {
      launch(std::false_type());
    }
  };
  switch (ek) {
    case EK_SLAB: go(std::integral_constant<int, EK_SLAB>()); break;
    case EK_STORE: go(std::integral_constant<int, EK_STORE>()); break;
    case EK_GELU_DUAL:
      if constexpr (IsDenseKC<LA>::value) go(std::integral_constant<int, EK_GELU_DUAL>());
      break;
    case EK_RESID:
      if constexpr (IsDenseKC<LA>::value) go(std::integral_constant<int, EK_RESID>());
      break;
    case EK_GELU_BWD:
      if constexpr (IsDenseKC<LA>::value) go(std::integral_constant<int, EK_GELU_BWD>());
      break;
    case EK_PATCH:
      if constexpr (IsDenseKC<LA>::value) go(std::integral_constant<int, EK_PATCH>());
      break;
    default: go(std::integral_constant<int, EK_GEN>()); break;
  }
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

}  // namespace hvit
