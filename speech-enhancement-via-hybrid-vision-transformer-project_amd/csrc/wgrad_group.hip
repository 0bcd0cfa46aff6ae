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

constexpr int BM = 256, BN = 256, MAXP = 56;
using Core = RingCore<BM, BN, 2, 4, 2, false, false>;

struct Prob {
  const bf16_t* dy;
  const bf16_t* x;
  float* dw;
  int ldy, ldx;     // row pitches (elements) of dy [M][ldy] and x [M][ldx]
  int n_out, k_in;  // dw [n_out][k_in]
  int tn;           // k_in / BN
  int tile0;        // first tile of this problem in the launch's tile order
};

struct Table {
  Prob p[MAXP];
  int np, M;
  int G;               // workgroups per phase-A round (a multiple of 8)
  int GB8;             // phase-B blocks / 8 (grid = R * G + 8 * GB8)
  int R, T;            // whole-tile rounds, tiles
  int rem0, s, pu;     // first phase-B tile, pieces per tile, units (64-token stages) per piece
  float* slabs;        // [G][BM * BN]
  unsigned* tickets;   // one per phase-B tile, zero on entry and on exit
};

__device__ __forceinline__ const Prob& find(const Table& tb, int t) {
  int i = 0;
  while (i + 1 < tb.np && t >= tb.p[i + 1].tile0) ++i;
  return tb.p[i];
}

__global__ __launch_bounds__(512, 1) void wgrad_group_kernel(Table tb) {
  constexpr int NT = Core::NT, FM = Core::FM, FN = Core::FN, WTM = Core::WTM, WTN = Core::WTN;
  constexpr int WN = 4;
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
    const int m0 = (lt / pr.tn) * BM, n0 = (lt % pr.tn) * BN;
    const int kbeg = pb ? (w % tb.s) * tb.pu * 64 : 0;
    const int kend = pb ? min(tb.M, kbeg + tb.pu * 64) : tb.M;
    float* dst = pb ? tb.slabs + (long)w * (BM * BN) : pr.dw + (long)m0 * pr.k_in + n0;
    const int ldo = pb ? BN : pr.k_in;
    LdDense<bf16_t, false> la, lb;
    la.p = pr.dy; la.ld = pr.ldy; la.rows = pr.n_out; la.K = tb.M; la.vok = true;
    lb.p = pr.x; lb.ld = pr.ldx; lb.rows = pr.k_in; lb.K = tb.M; lb.vok = true;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) acc[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
    Core::run(la, lb, smem, m0, n0, kbeg, kend, acc, none);
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
    const float* s0 = tb.slabs + (long)(rt * tb.s) * (BM * BN);
    float* dw = pr.dw + (long)m0 * pr.k_in + n0;
#pragma unroll 2
    for (int i = 0; i < BM / RS8; ++i) {
      const int row = q0 + i * RS8;
      const float* src = s0 + row * BN + c8 * 8;
      f32x4 sa = *(const f32x4*)src, sb = *(const f32x4*)(src + 4);
      for (int z = 1; z < tb.s; ++z) {
        const float* q = src + (long)z * (BM * BN);
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

}  // namespace hvit_wg

using namespace hvit_wg;

extern "C" int hvit_linear_wgrad_group_ok(int dt, int M, int n_out, int k_in) {
  return dt == HVIT_BF16 && M > 0 && M % 64 == 0 && n_out > 0 && k_in > 0 && n_out % BM == 0 && k_in % BN == 0 &&
         (long long)M * std::max(n_out, k_in) * 2 < (1LL << 31);
}

extern "C" long long hvit_linear_wgrad_group_ws(void) { return (long long)num_cus() * BM * BN; }
extern "C" long long hvit_linear_wgrad_group_tickets(void) { return (long long)num_cus(); }

extern "C" int hvit_linear_wgrad_group(int dt, int M, const hvit_wgrad_prob_t* probs, int nprobs, float* ws,
                                       long long ws_elems, unsigned* tickets, long long n_tickets, void* stream) {
  HVIT_CHECK(probs && nprobs >= 0, "hvit_linear_wgrad_group: null problem table");
  HVIT_CHECK(ws && ws_elems >= hvit_linear_wgrad_group_ws(), "hvit_linear_wgrad_group: workspace too small");
  HVIT_CHECK(tickets && n_tickets >= hvit_linear_wgrad_group_tickets(), "hvit_linear_wgrad_group: tickets");
  HVIT_CHECK(aligned16(ws), "hvit_linear_wgrad_group: workspace alignment");
  for (int i = 0; i < nprobs; ++i) {
    const hvit_wgrad_prob_t& q = probs[i];
    HVIT_CHECK(hvit_linear_wgrad_group_ok(dt, M, q.n_out, q.k_in),
               "hvit_linear_wgrad_group: problem %d (M=%d n_out=%d k_in=%d) needs bf16, M %% 64 == 0, n_out and "
               "k_in multiples of %d",
               i, M, q.n_out, q.k_in, BM);
    HVIT_CHECK(q.dy && q.x && q.dw && aligned16(q.dy) && aligned16(q.x) && aligned16(q.dw),
               "hvit_linear_wgrad_group: problem %d pointers (null or not 16-byte aligned)", i);
    HVIT_CHECK(q.ldy >= q.n_out && q.ldx >= q.k_in && q.ldy % 8 == 0 && q.ldx % 8 == 0,
               "hvit_linear_wgrad_group: problem %d row pitches", i);
    HVIT_CHECK((long long)M * q.ldy * 2 < (1LL << 31) && (long long)M * q.ldx * 2 < (1LL << 31),
               "hvit_linear_wgrad_group: problem %d operand too large for 32-bit offsets", i);
  }
  hipStream_t st = (hipStream_t)stream;
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
      p.ldx = q.ldx;
      p.n_out = q.n_out;
      p.k_in = q.k_in;
      p.tn = q.k_in / BN;
      p.tile0 = T;
      T += (q.n_out / BM) * p.tn;
    }
    tb.np = np;
    tb.M = M;
    tb.slabs = ws;
    tb.tickets = tickets;
    plan(tb, T, M);
    if (T == 0) continue;
    hipLaunchKernelGGL(wgrad_group_kernel, dim3(tb.R * tb.G + 8 * tb.GB8), dim3(512), 0, st, tb);
    HVIT_LAUNCH_CHECK();
  }
  return HVIT_OK;
}
