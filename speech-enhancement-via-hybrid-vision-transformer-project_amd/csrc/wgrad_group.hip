// Grouped ViT weight gradients in one launch (round 6), gfx950.
//
//   dw_p[n, k] = sum_m dy_p[m, n] * x_p[m, k]      p = 0 .. P-1, m < M tokens
//
// The four Linear weight gradients of a TransformerEncoderBlock (attention.py:55,
// 58 qkv / proj; components.py:224,227 fc1 / fc2) are GEMMs with a tiny output
// ([512..2048] x [512..2048]) and a long reduction over the B*N tokens (8,192 at
// B = 32).  Alone, each one fills the 256 CUs only by splitting its K: short
// K slices, f32 partial slabs written and re-read (profiles/r6_wgrad_layout_probe
// .txt: 29-39 us for a 17 GFLOP weight gradient, ~0.16 of the MFMA peak).  None
// of them is read before the optimizer, so the backward queues them
// (functional.WgradGroup) and runs the whole queue here: every output tile is a
// 256x256 block over the FULL token range on the LDS-DMA ring of gemm_ring.h
// (RingCore<256, 256, 2, 4, 2>, both operands token-major: MN images with
// transposed fragment reads), so a tile's K loop is 128 stages long and writes
// its result once.  Six blocks at B = 32 give 288 tiles for 256 CUs:
//   phase A: rounds of G whole tiles, one per workgroup (R = T / G rounds);
//   phase B: the T' = T - R*G remaining tiles split into s = G / T' K pieces,
//            one per workgroup, each an f32 partial in its own slab; the last
//            piece of a tile to arrive (ticket) sums the pieces in piece order.
// The R * G + T' * s workgroups run one job each (about R tiles + one piece
// per CU: balanced to within one piece).  The
// sums are fixed-order (one K loop per tile; pieces summed 0..s-1), so results
// are bit-identical from run to run and between eager launches and replays.
// Logical workgroup w = (block % 8) * (blocks / 8) + block / 8 within a round: an XCD owns a
// contiguous run of tiles (same problem, shared dy / x panels in its L2), and
// phase A's workgroups march through K together.
#include "gemm_host.h"
#include "gemm_ring.h"

namespace hvit_wg {
using namespace hvit;

constexpr int BM = 256, MAXP = 64;  // (every configuration's tiles are BM = 256 rows of dw)

// The weight gradients' K loop with 32-deep stages: both operands token-major
// (MN images, transposed fragment reads), one 16x16x32 MFMA k-step per stage,
// NB stages in the LDS ring so NB - 1 of them (NB - 1 x 32 KiB at 256 x 256)
// are in flight under each stage's MFMAs -- the 64-deep two-stage ring keeps
// one 64 KiB stage in flight and its K loop waited on that stage's landing
// (counters, profiles/r6_wgrad_group_pmc.json: ~41 % of wave cycles in
// s_waitcnt at 31 % MFMA busy).  The images are the first 32 k rows of
// gemm.h's 64-deep MN images (DmaImg / MnSwz: rows are k, so the same source
// swizzle and transposed reads apply).
// B operand geometry: dense token-major rows (P = 0), or the implicit
// im2col of a patch embedding (Conv2d k = stride = P, components.py:275-280):
// token t = (image, py, px) of an Hp x Wp grid, its row (ky, kx, c) =
// x[image, P*py + ky, P*px + kx, c] of an NHWC [*, H, Wimg, C] image.  A
// 32-token stage is 32 / Wp whole patch rows of one image, so a lane's source
// offset inside a stage is fixed and consecutive stages are a constant stride
// apart; a 256-column tile lies inside one ky (P*C % 256 == 0).
struct BGeo {
  short P, Wimg, Wp, C;
  int ext;  // bytes of x (buffer range)
};

template <int BM_, int BN_, int WM, int WN, int NB>
struct Ring32 {
  static constexpr int NW = WM * WN, NT = 64 * NW;
  using IA = DmaImg<BM_, false>;
  using IB = DmaImg<BN_, false>;
  static constexpr int BK = 32;
  static constexpr int ABYTES = IA::BYTES / 2, BBYTES = IB::BYTES / 2;
  static constexpr int WTM = BM_ / WM, WTN = BN_ / WN, FM = WTM / 16, FN = WTN / 16;
  static constexpr int PA = IA::PIECES / 2 / NW, PB = IB::PIECES / 2 / NW;
  static constexpr int INFL = PA + PB;  // this wave's DMA instructions per stage
  static constexpr int STAGE = ABYTES + BBYTES;
  static constexpr int SM = NB * STAGE;
  static_assert(IA::PIECES % (2 * NW) == 0 && IB::PIECES % (2 * NW) == 0, "stage pieces must split over the waves");
  static_assert(NB >= 2 && (NB - 2) * INFL <= 63, "ring depth / vmcnt range");
  static constexpr int MPD = (FM * FN) / INFL > 0 ? (FM * FN) / INFL : 1;
  static_assert(MPD * INFL <= FM * FN, "interleave");

  __device__ __forceinline__ static __amdgpu_buffer_rsrc_t rsrc(const LdDense<bf16_t, false>& l) {
    const long bytes = (long)l.K * l.ld * 2;
    return __builtin_amdgcn_make_buffer_rsrc((void*)l.p, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                             0x00020000);
  }

  __device__ __forceinline__ static void run(const LdDense<bf16_t, false>& la, const LdDense<bf16_t, false>& lb,
                                             const BGeo& bg, char* smem, int m0, int n0, int kbeg, int kend,
                                             f32x4 (&acc)[FM][FN]) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int nk = (kend - kbeg) / BK;
    if (nk <= 0) return;
    const __amdgpu_buffer_rsrc_t ra = rsrc(la);
    const __amdgpu_buffer_rsrc_t rb =
        bg.P ? __builtin_amdgcn_make_buffer_rsrc((void*)lb.p, (short)0, (int)bg.ext, 0x00020000) : rsrc(lb);
    const unsigned oa = (unsigned)(((long)kbeg * la.ld + m0) * 2), da = (unsigned)((long)BK * la.ld * 2);
    unsigned ob, db;
    if (bg.P) {
      const int pc = bg.P * bg.C;
      ob = (unsigned)((((long)(kbeg / bg.Wp) * bg.P * bg.Wimg + (long)(n0 / pc) * bg.Wimg) * bg.C + n0 % pc) * 2);
      db = (unsigned)((long)(BK / bg.Wp) * bg.P * bg.Wimg * bg.C * 2);
    } else {
      ob = (unsigned)(((long)kbeg * lb.ld + n0) * 2);
      db = (unsigned)((long)BK * lb.ld * 2);
    }
    unsigned va[PA], vb[PB];
#pragma unroll
    for (int i = 0; i < PA; ++i) va[i] = IA::src_off(wid + NW * i, lane, la.ld);
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      // IB::src_off with the row (token) offset of the operand's geometry
      const int row = (wid + NW * i) * IB::RPP + lane / IB::NCH;
      const int c = (lane % IB::NCH) ^ IB::swz(row);
      const long roff = bg.P ? ((long)(row / bg.Wp) * bg.P * bg.Wimg + (row % bg.Wp) * bg.P) * bg.C : (long)row * lb.ld;
      vb[i] = (unsigned)((roff + c * 8) * 2);
    }
    // stage t -> ring buffer t % NB; stages past the end re-read the last one
    // into a buffer never read again (a constant DMA count per iteration)
    auto issue = [&](int t) {
      char* abuf = smem + (t % NB) * STAGE;
      char* bbuf = abuf + ABYTES;
      const int ts = t < nk ? t : nk - 1;
      const unsigned sa = oa + (unsigned)ts * da, sb = ob + (unsigned)ts * db;
#pragma unroll
      for (int i = 0; i < PA; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(abuf + (wid + NW * i) * 1024),
                                                 16, va[i], sa, 0, 0);
#pragma unroll
      for (int i = 0; i < PB; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(bbuf + (wid + NW * i) * 1024),
                                                 16, vb[i], sb, 0, 0);
    };
#pragma unroll
    for (int t = 0; t < NB - 1; ++t) issue(t);
    for (int t = 0; t < nk; ++t) {
      // stage t landed for this wave (NB-2 younger stages stay in flight) and,
      // after the barrier, for every wave; every wave has also finished reading
      // stage t-1, whose buffer (t+NB-1) % NB the issue below refills
      __builtin_amdgcn_s_waitcnt(vm_imm((NB - 2) * INFL));
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const char* at = smem + (t % NB) * STAGE;
      const char* bt = at + ABYTES;
      u32x4 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = IA::frag(at, wm * WTM + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = IB::frag(bt, wn * WTN + j * 16, 0, lane);
      issue(t + NB - 1);
      lgkm_wait0();
      lds_pin(fa);
      lds_pin(fb);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, fa[i]),
                                                              __builtin_bit_cast(s16x8, fb[j]), acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(vm_imm(0));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
};

// the K loop of a configuration: gemm_ring.h's 64-deep ring or the 32-deep one
template <int BN, int WM, int WN, int NB, int DEEP>
struct CoreOf {
  using T = RingCore<256, BN, WM, WN, NB, false, false>;
};
template <int BN, int WM, int WN, int NB>
struct CoreOf<BN, WM, WN, NB, 1> {
  using T = Ring32<256, BN, WM, WN, NB>;
};

struct Prob {  // (kernel-argument table: kept small, MAXP of them)
  const bf16_t* dy;
  const bf16_t* x;
  float* dw;
  int ldy, ldx;  // row pitches (elements) of dy [M][ldy] and x [M][ldx]
  int k_in;      // dw [n_out][k_in]
  int tile0;     // first tile of this problem in the launch's tile order
  BGeo bg;       // x's geometry (bg.P = 0: dense rows of pitch ldx)
};

struct Table {
  Prob p[MAXP];
  int np, M;
  int G;               // workgroups per phase-A round (a multiple of 8)
  int GB8;             // phase-B blocks / 8 (grid = R * G + 8 * GB8)
  int R, T;            // whole-tile rounds, tiles
  int rem0, s, pu;     // first phase-B tile, pieces per tile, units (64-token stages) per piece
  float* slabs;        // [G][BM * 256] (a piece's slab holds BM x BN, pitch BN)
  unsigned* tickets;   // one per phase-B tile, zero on entry and on exit
};

__device__ __forceinline__ const Prob& find(const Table& tb, int t) {
  int i = 0;
  while (i + 1 < tb.np && t >= tb.p[i + 1].tile0) ++i;
  return tb.p[i];
}

// tile configurations (hvit_gemm_tune(7, v); all 256 x 256 tiles):
//   0: gemm_ring.h's 64-deep ring, 2 x 4 waves, 2 stages (128 KiB: one stage in flight)
//   2: the 32-deep ring, 2 x 4 waves, 4 stages (128 KiB: three 32 KiB stages in flight)
//   6: the 32-deep ring, 4 x 4 waves (64 x 64 each, 114 VGPRs: four waves per SIMD), 4 stages -- default
// Measured and dropped (tools/wgrad_group_probe.py, 6 blocks at B = 32): 256 x 128 tiles on a 3-stage
// ring 368 vs 356 us (cfg 0); 5 stages 352 vs 333 (cfg 2); half of each stage's fragment reads under
// the other half's MFMAs 336 vs 333; 16 waves with 5 stages 365 vs 350 (cfg 6).
template <int BN, int WM, int WN, int NB, int DEEP>
__global__ __launch_bounds__(64 * WM * WN, 1) void wgrad_group_kernel(Table tb) {
  using Core = typename CoreOf<BN, WM, WN, NB, DEEP>::T;
  constexpr int NT = Core::NT, FM = Core::FM, FN = Core::FN, WTM = Core::WTM, WTN = Core::WTN;
  constexpr int CP = BN + 4;  // LDS tile pitch (floats)
  constexpr int C8 = BN / 8, RS8 = NT / C8, NR8 = 64 / RS8;
  constexpr int SM_E = 64 * CP * 4 + 16;
  __shared__ __attribute__((aligned(16))) char smem[Core::SM > SM_E ? Core::SM : SM_E];

  // one job per workgroup: blocks [0, R*G) are R rounds of whole tiles (phase
  // A, stored straight into dw), the rest one K piece each of a remainder tile
  // (phase B, into the workgroup's slab).  (A loop over a workgroup's jobs kept
  // its values live across the K loop and spilled; the dispatcher hands the
  // next round's blocks to the CUs as they free up, which is the same schedule.)
  const int b = blockIdx.x;
  const bool pb = b >= tb.R * tb.G;
  const int loc = pb ? b - tb.R * tb.G : b % tb.G;
  const int per = pb ? tb.GB8 : tb.G / 8;
  const int w = (loc & 7) * per + (loc >> 3);  // XCD-contiguous logical index
  if (pb && w >= (tb.T - tb.rem0) * tb.s) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int frow = lane & 15, fq = lane >> 4;
  const int c8 = tid % C8, q0 = tid / C8;
  float* Cs = (float*)smem;
  Epi none;  // (no side job)
  {
    const int t = pb ? tb.rem0 + w / tb.s : (b / tb.G) * tb.G + w;
    const Prob& pr = find(tb, t);
    const int lt = t - pr.tile0;
    const int tn = pr.k_in / BN;
    const int m0 = (lt / tn) * BM, n0 = (lt % tn) * BN;
    const int kbeg = pb ? (w % tb.s) * tb.pu * 64 : 0;
    const int kend = pb ? min(tb.M, kbeg + tb.pu * 64) : tb.M;
    float* dst = pb ? tb.slabs + (long)w * (BM * 256) : pr.dw + (long)m0 * pr.k_in + n0;
    const int ldo = pb ? BN : pr.k_in;
    LdDense<bf16_t, false> la, lb;
    la.p = pr.dy; la.ld = pr.ldy; la.rows = 0; la.K = tb.M; la.vok = true;  // (rows: unused by MN images)
    lb.p = pr.x; lb.ld = pr.ldx; lb.rows = 0; lb.K = tb.M; lb.vok = true;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) acc[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if constexpr (DEEP) Core::run(la, lb, pr.bg, smem, m0, n0, kbeg, kend, acc);
    else Core::run(la, lb, smem, m0, n0, kbeg, kend, acc, none);
    // the result staged through LDS in 64-row passes; a thread stores 8
    // adjacent f32 columns per row (two 16-byte stores)
#pragma unroll
    for (int hh = 0; hh < BM / 64; ++hh) {
      if (hh > 0) epi_barrier();
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wm * WTM + i * 16 + fq * 4 + r - hh * 64;
            if (row >= 0 && row < 64) Cs[row * CP + wn * WTN + jj * 16 + frow] = acc[i][jj][r];
          }
      epi_barrier();
#pragma unroll
      for (int i = 0; i < NR8; ++i) {
        const int row = q0 + i * RS8;
        float* d = dst + (long)(hh * 64 + row) * ldo + c8 * 8;
        *(f32x4*)d = *(const f32x4*)(Cs + row * CP + c8 * 8);
        *(f32x4*)(d + 4) = *(const f32x4*)(Cs + row * CP + c8 * 8 + 4);
      }
    }
    if (!pb) return;
    // publish the slab, take a ticket; the last piece to arrive sums all of the
    // tile's slabs in piece order (cdna_hip_programming.md, in-launch split-K
    // reduction, counter form: no piece waits for another, no co-residency)
    const int rt = w / tb.s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)(smem + 64 * CP * 4);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned prev = __hip_atomic_fetch_add(tb.tickets + rt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == (unsigned)(tb.s - 1);
      if (last) __hip_atomic_store(tb.tickets + rt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const float* s0 = tb.slabs + (long)(rt * tb.s) * (BM * 256);
    float* dw = pr.dw + (long)m0 * pr.k_in + n0;
#pragma unroll 2
    for (int i = 0; i < BM / RS8; ++i) {
      const int row = q0 + i * RS8;
      const float* src = s0 + row * BN + c8 * 8;
      f32x4 sa = *(const f32x4*)src, sb = *(const f32x4*)(src + 4);
      for (int z = 1; z < tb.s; ++z) {
        const float* q = src + (long)z * (BM * 256);
        sa += *(const f32x4*)q;
        sb += *(const f32x4*)(q + 4);
      }
      float* d = dw + (long)row * pr.k_in + c8 * 8;
      *(f32x4*)d = sa;
      *(f32x4*)(d + 4) = sb;
    }
  }
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
    n = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  }
  return n;
}

// the launch plan of one chunk of problems (<= MAXP)
static void plan(Table& tb, int T, int M) {
  const int G0 = std::max(8, num_cus() / 8 * 8);  // one 128-KiB-LDS workgroup per CU
  const int ku = M / 64;
  tb.T = T;
  tb.G = G0;
  tb.R = T / G0;
  tb.rem0 = tb.R * G0;
  const int rem = T - tb.rem0;
  tb.s = 0;
  tb.pu = ku;
  tb.GB8 = 0;
  if (rem > 0) {
    int s = std::max(1, std::min(G0 / rem, ku));
    const int pu = (ku + s - 1) / s;
    s = (ku + pu - 1) / pu;
    tb.s = s;
    tb.pu = pu;
    tb.GB8 = (rem * s + 7) / 8;
  }
}

// tile configuration (hvit_gemm_tune(7, v), A/B measurements)
static int& cfg_ref() {
  // (isolated loop, tools/wgrad_group_probe.py, 6 blocks at B = 32: cfg 0 356, cfg 2 333-341 / 361 on a slower box,
  // cfg 6 350 on that box (315 with L2-resident operands); in-step 364 -> 338 us, step 4.630 -> 4.622 ms)
  static int c = 6;
  return c;
}

}  // namespace hvit_wg

using namespace hvit_wg;

int hvit_wgrad_group_tune(int value) {
  const int old = cfg_ref();
  if (value == 0 || value == 2 || value == 6) cfg_ref() = value;
  return old;
}

extern "C" int hvit_linear_wgrad_group_ok(int dt, int M, int n_out, int k_in) {
  return dt == HVIT_BF16 && M > 0 && M % 64 == 0 && n_out > 0 && k_in > 0 && n_out % BM == 0 && k_in % 256 == 0 &&
         (long long)M * std::max(n_out, k_in) * 2 < (1LL << 31);
}

extern "C" long long hvit_linear_wgrad_group_ws(void) { return (long long)num_cus() * BM * 256; }
extern "C" long long hvit_linear_wgrad_group_tickets(void) { return (long long)num_cus(); }

// the patch-embedding B geometry of problem q (P = 0: dense); "" when valid
static const char* patch_geo(const hvit_wgrad_prob_t& q, int M, BGeo& g) {
  g = BGeo{0, 0, 0, 0, 0};
  if (q.patch <= 0) return "";
  const int P = q.patch, H = q.img_h, W = q.img_w, C = q.img_c;
  if (H <= 0 || W <= 0 || C <= 0 || H % P || W % P) return "image H / W must be positive multiples of the patch";
  const int Hp = H / P, Wp = W / P;
  if (q.k_in != P * P * C) return "k_in must be patch * patch * C";
  if (32 % Wp) return "the patch grid width must divide 32";
  if ((Hp * Wp) % 32 || M % (Hp * Wp)) return "tokens per image must be a multiple of 32 dividing M";
  if ((P * C) % 256 || C % 8) return "patch * C must be a multiple of 256 (C of 8)";
  const long long ext = (long long)(M / (Hp * Wp)) * H * W * C * 2;
  if (ext >= (1LL << 31) || W > 32767 || C > 32767 || P > 32767) return "image too large for 32-bit offsets";
  g = BGeo{(short)P, (short)W, (short)Wp, (short)C, (int)ext};
  return "";
}

extern "C" int hvit_linear_wgrad_group_patch_ok(int dt, int M, int n_out, int patch, int img_h, int img_w,
                                                int img_c) {
  if (patch <= 0 || cfg_ref() < 2 || !hvit_linear_wgrad_group_ok(dt, M, n_out, patch * patch * img_c)) return 0;
  hvit_wgrad_prob_t q{};
  q.n_out = n_out;
  q.k_in = patch * patch * img_c;
  q.patch = patch;
  q.img_h = img_h;
  q.img_w = img_w;
  q.img_c = img_c;
  BGeo g;
  return *patch_geo(q, M, g) ? 0 : 1;
}

extern "C" int hvit_linear_wgrad_group(int dt, int M, const hvit_wgrad_prob_t* probs, int nprobs, float* ws,
                                       long long ws_elems, unsigned* tickets, long long n_tickets, void* stream) {
  HVIT_CHECK(probs && nprobs >= 0, "hvit_linear_wgrad_group: null problem table");
  HVIT_CHECK(ws && ws_elems >= hvit_linear_wgrad_group_ws(), "hvit_linear_wgrad_group: workspace too small");
  HVIT_CHECK(tickets && n_tickets >= hvit_linear_wgrad_group_tickets(), "hvit_linear_wgrad_group: tickets");
  HVIT_CHECK(aligned16(ws), "hvit_linear_wgrad_group: workspace alignment");
  const int cfg = cfg_ref();
  for (int i = 0; i < nprobs; ++i) {
    const hvit_wgrad_prob_t& q = probs[i];
    HVIT_CHECK(hvit_linear_wgrad_group_ok(dt, M, q.n_out, q.k_in),
               "hvit_linear_wgrad_group: problem %d (M=%d n_out=%d k_in=%d) needs bf16, M %% 64 == 0, n_out and "
               "k_in multiples of %d",
               i, M, q.n_out, q.k_in, BM);
    HVIT_CHECK(q.dy && q.x && q.dw && aligned16(q.dy) && aligned16(q.x) && aligned16(q.dw),
               "hvit_linear_wgrad_group: problem %d pointers (null or not 16-byte aligned)", i);
    HVIT_CHECK(q.ldy >= q.n_out && q.ldy % 8 == 0 && (q.patch > 0 || (q.ldx >= q.k_in && q.ldx % 8 == 0)),
               "hvit_linear_wgrad_group: problem %d row pitches", i);
    HVIT_CHECK((long long)M * q.ldy * 2 < (1LL << 31) && (q.patch > 0 || (long long)M * q.ldx * 2 < (1LL << 31)),
               "hvit_linear_wgrad_group: problem %d operand too large for 32-bit offsets", i);
    BGeo g;
    const char* why = patch_geo(q, M, g);
    HVIT_CHECK(!*why, "hvit_linear_wgrad_group: problem %d patch geometry: %s", i, why);
    HVIT_CHECK(q.patch <= 0 || cfg >= 2, "hvit_linear_wgrad_group: patch problems need a 32-deep ring configuration");
  }
  hipStream_t st = (hipStream_t)stream;
  constexpr int BN = 256;
  for (int c0 = 0; c0 < nprobs; c0 += MAXP) {
    const int np = std::min(MAXP, nprobs - c0);
    Table tb{};
    int T = 0;
    for (int i = 0; i < np; ++i) {
      const hvit_wgrad_prob_t& q = probs[c0 + i];
      Prob& p = tb.p[i];
      p.dy = (const bf16_t*)q.dy;
      p.x = (const bf16_t*)q.x;
      p.dw = q.dw;
      p.ldy = q.ldy;
      p.ldx = q.patch > 0 ? 0 : q.ldx;
      p.k_in = q.k_in;
      p.tile0 = T;
      patch_geo(q, M, p.bg);
      T += (q.n_out / BM) * (q.k_in / BN);
    }
    tb.np = np;
    tb.M = M;
    tb.slabs = ws;
    tb.tickets = tickets;
    plan(tb, T, M);
    if (T == 0) continue;
    const dim3 grid(tb.R * tb.G + 8 * tb.GB8);
    if (cfg == 2)
      hipLaunchKernelGGL((wgrad_group_kernel<256, 2, 4, 4, 1>), grid, dim3(512), 0, st, tb);
    else if (cfg == 6)
      hipLaunchKernelGGL((wgrad_group_kernel<256, 4, 4, 4, 1>), grid, dim3(1024), 0, st, tb);
    else
      hipLaunchKernelGGL((wgrad_group_kernel<256, 2, 4, 2, 0>), grid, dim3(512), 0, st, tb);
    HVIT_LAUNCH_CHECK();
  }
  return HVIT_OK;
}
