// Conv weight gradient of the 3x3 / stride 1 / pad 1 convs by shifted row
// windows (ConvBlock / TransposeConvBlock convs, components.py:55-62 and
// :149-158, with the decoder's nearest x2 upsample and channel concat).
//
//   dW[co][ky][kx][ci] = sum_{n,oy,ox} dy[n][oy][ox][co] * xin[n][oy+ky-1][ox+kx-1][ci]
//
// A workgroup owns an output tile of 128 (or 64) output channels x one kernel
// row ky x all three kx x 64 input channels (128 x 192) and a contiguous range
// of 64-pixel stages of the pixel reduction.  The three kx taps read the SAME
// input row shifted by one pixel, so a stage stages the dy block [64 px][co]
// and ONE input strip [66 px][64 ci] (several short rows with their halos when
// Wo < 64), and the kx = 0/1/2 operands are windows of that strip at row
// offsets 0/1/2: 24.6 KiB per stage feed 3x the MFMA work of the generic
// implicit-im2col tile (128 x 64, 24 KiB per stage), whose ds_write staging
// and L2->CU traffic bounded it at ~0.45 PFLOP/s.
//
// Both images are filled by LDS-DMA (buffer_load_dwordx4 ... lds, lane-linear
// 1-KiB pieces, the MN bank swizzle applied on the source side: MnSwz), three
// stage buffers deep (stage t+2 in flight while t runs), counted vmcnt and raw
// barriers as in GemmCoreDma.  Input taps in the zero padding and pixels past
// the tensor read as zeros through the buffer range check.  Split-K partials
// go to fp32 slabs summed by hvit_sum_slabs (layout of the generic path:
// dw_packed[co][(ky*3 + kx)*Ctot + ci]).
#include "gemm_host.h"

// a named namespace: kernel templates in an anonymous one leave their host
// launch stubs undefined in the shared library
namespace hvit_rows {

struct RowsArgs {
  const bf16_t* dy;          // [P][Cout]
  const bf16_t* src1;        // [N][Hs][Ws][C1]
  const bf16_t* src2;        // [N][Hs][Ws][C2] (or src1)
  int C1, C2, Ctot, Cout;
  int Hs, Ws, ushift, Hi, Wi, Ho, Wo;
  int stages, sps;           // 64-pixel stages in total / per split
  int tiles, cib_n;          // tiles = (Cout / BM) * 3 * cib_n
  float* out;                // slabs [split][Cout][Kt] (or dw_packed when one split)
  long long slab;            // Cout * Kt
  int Kt;
  unsigned bytes1, bytes2, bytes_dy;
};

constexpr int ROWS_BN = 192;     // 3 kx x 64 ci
constexpr int ROWS_BROWS = 72;   // staged input rows per stage (>= 64 + 2 * (64 / Wo))
constexpr int ROWS_NBUF = 3;

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
}

template <int BM>
__device__ __forceinline__ void rows_body(const RowsArgs& a, char* smem) {
  constexpr int WN = 2, WTM = BM / 2, WTN = ROWS_BN / WN;  // 2 x 2 waves
  constexpr int FM = WTM / 16, FN = WTN / 16;
  using IA = DmaImg<BM, false>;
  constexpr int A_BYTES = IA::BYTES;
  constexpr int B_BYTES = ROWS_BROWS * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int PA = IA::PIECES / 4;                   // A pieces per wave per stage
  constexpr int PB = 3;                                // B pieces per wave (piece 8 on every wave)
  constexpr int INF = PA + PB;                         // DMA instructions per wave per stage
  static_assert(ROWS_BROWS % 8 == 0 && ROWS_BROWS / 8 == 9, "9 input pieces per stage");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware order (gemm.h tile_of): each XCD owns a contiguous range of
  // (split, tile), so the tiles of one split share its L2
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int z = lid / a.tiles, tile = lid - z * a.tiles;
  const int cib = tile % a.cib_n, t2 = tile / a.cib_n;
  const int ky = t2 % 3, cob = t2 / 3;
  const int sbeg = z * a.sps;
  const int nk = min(a.stages, sbeg + a.sps) - sbeg;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    // ---- A: dy block [64 px][BM co] of the tile's output channels
    const bf16_t* abase = a.dy + (long)cob * BM;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        (void*)abase, (short)0, (int)(a.bytes_dy - (unsigned)(cob * BM * 2)), 0x00020000);
    unsigned va[PA];
#pragma unroll
    for (int i = 0; i < PA; ++i) va[i] = IA::src_off(wid + 4 * i, lane, a.Cout);
    const unsigned da = (unsigned)(64 * a.Cout * 2);
    // ---- B: the input strip of the tile's 64 channels (one source)
    const int c0 = cib * 64;
    const bool first = c0 < a.C1;  // uniform
    const int Cx = first ? a.C1 : a.C2, coff = first ? c0 : c0 - a.C1;
    const __amdgpu_buffer_rsrc_t rbs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(first ? a.src1 : a.src2), (short)0, (int)(first ? a.bytes1 : a.bytes2), 0x00020000);
    const bool wide = a.Wo >= 64;
    const int SW = a.Wo + 2, nseg = wide ? 1 : 64 / a.Wo;
    // this lane's rows of its B pieces: segment, column, and the swizzled
    // channel chunk.  Nine pieces per stage: waves 1..3 also issue piece 8
    // (same source, same destination, same bytes), so every wave has the same
    // DMA count per stage and the waits below are uniform immediates (a
    // per-wave count made the compiler drain vmcnt(0) before the LDS reads)
    int bseg[PB], bcol[PB], bch[PB];
    bool bon[PB];
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int piece = i < PB - 1 ? wid + 4 * i : 8;
      const int r = piece * 8 + (lane >> 3);
      const int seg = wide ? 0 : r / SW;
      bseg[i] = seg;
      bcol[i] = wide ? r : r - seg * SW;
      bch[i] = coff + 8 * ((lane & 7) ^ MnSwz<64>::swz(r));
      bon[i] = seg < nseg && bcol[i] < (wide ? 66 : SW);
    }
    auto issue = [&](int t) {
      char* abuf = smem + (t % ROWS_NBUF) * STAGE;
      char* bbuf = abuf + A_BYTES;
      const int st = sbeg + t;
      const unsigned sa = (unsigned)st * da;
#pragma unroll
      for (int i = 0; i < PA; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(abuf + (wid + 4 * i) * 1024),
                                                 16, va[i], sa, 0, 0);
      // stage geometry (uniform): first output row and column of the 64 pixels
      const int p0 = st * 64;
      const int row0 = p0 / a.Wo, ox0 = p0 - row0 * a.Wo;
      const int n = row0 / a.Ho, oy0 = row0 - n * a.Ho;
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int piece = i < PB - 1 ? wid + 4 * i : 8;
        const int iy = oy0 + bseg[i] + ky - 1, ix = ox0 + bcol[i] - 1;
        const bool ok = bon[i] && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
        const unsigned off =
            (unsigned)((((n * a.Hs + (iy >> a.ushift)) * a.Ws + (ix >> a.ushift)) * Cx + bch[i]) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rbs, (__attribute__((address_space(3))) void*)(bbuf + piece * 1024),
                                                 16, ok ? off : 0x80000000u, 0, 0, 0);
      }
    };
    // Per-lane byte offsets of the transposed fragment reads, hoisted out of
    // the loop.  A lane reads rows k = 32s + 8g + q (+4) of a k-major image;
    // the chunk of a 16-row block rb is (rb / 8 + p / 2) ^ swz(row), and rb / 8
    // has no bits in common with p / 2, so the block is applied as an XOR of
    // (rb / 8) << 4 on a per-lane base (swz depends on the row bits 0..3 only).
    // The input strip's rows are k + kx (+ 2 per short row of halo).
    const int lg = lane >> 4, lq = (lane & 15) >> 2, lp = lane & 3;
    const int ch0 = lp >> 1, byte = (lp & 1) * 8;
    unsigned aoff[2], boff[2][3][2];
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
      const int row = 8 * lg + lq + 4 * hi;
      aoff[hi] = (unsigned)(row * IA::ROWB + ((ch0 ^ MnSwz<BM>::swz(row)) << 4) + byte);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int hi = 0; hi < 2; ++hi) {
          const int k = 32 * s2 + 8 * lg + lq + 4 * hi;
          const int row = k + kx + (wide ? 0 : 2 * (k / a.Wo));
          boff[s2][kx][hi] = (unsigned)(row * 128 + ((ch0 ^ MnSwz<64>::swz(row)) << 4) + byte);
        }
    auto load = [&](unsigned at, unsigned bt, int s2, u32x4 (&fa)[FM], u32x4 (&fb)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const unsigned x = (unsigned)(((wm * WTM + i * 16) >> 3) << 4);
        const unsigned ab = at + s2 * 32 * IA::ROWB;
        fa[i] = tr2_asm(ab + (aoff[0] ^ x), ab + (aoff[1] ^ x));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * WTN + j * 16;  // kx / channel block per j and wave half
        const int kx = col >> 6;
        const unsigned x = (unsigned)(((col & 63) >> 3) << 4);
        fb[j] = tr2_asm(bt + (boff[s2][kx][0] ^ x), bt + (boff[s2][kx][1] ^ x));
      }
    };
    auto mma = [&](const u32x4 (&fa)[FM], const u32x4 (&fb)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, fa[i]),
                                                              __builtin_bit_cast(s16x8, fb[j]), acc[i][j], 0, 0, 0);
    };
    const unsigned smem_a = lds_addr(smem);
    // k-step 0's fragments, then k-step 1's reads in flight under k-step 0's MFMAs
    auto compute = [&](int t) {
      const unsigned at = smem_a + (unsigned)((t % ROWS_NBUF) * STAGE);
      const unsigned bt = at + A_BYTES;
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
    issue(0);
    if (nk > 1) issue(1);
    for (int t = 0; t < nk; ++t) {
      if (t + 2 < nk) {
        issue(t + 2);
        wait_vm<2 * INF>();  // stage t landed (this wave's pieces)
      } else if (t + 1 < nk) {
        wait_vm<INF>();
      } else {
        wait_vm<0>();
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's stage-t pieces have landed
      asm volatile("" ::: "memory");
      compute(t);
      __builtin_amdgcn_s_barrier();  // buffer t % 3 is free for stage t + 3 (reads drained in compute)
      asm volatile("" ::: "memory");
    }
  }

  // partial dW straight from the accumulators: lane (g, c) holds rows 4g..4g+3
  // of column c of each 16x16 block
  float* o = a.out + (long long)z * a.slab;
  const int c0 = cib * 64;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn * WTN + j * 16 + (lane & 15);
      const int kx = col >> 6, ci = col & 63;
      const long kt = (long)(ky * 3 + kx) * a.Ctot + c0 + ci;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = cob * BM + wm * WTM + i * 16 + 4 * (lane >> 4) + e;
        o[(long)m * a.Kt + kt] = acc[i][j][e];
      }
    }
}

template <int BM>
__global__ __launch_bounds__(256, 2) void conv_wgrad_rows_kernel(RowsArgs a) {
  constexpr int STAGE = DmaImg<BM, false>::BYTES + ROWS_BROWS * 128;
  __shared__ __attribute__((aligned(1024))) char smem[ROWS_NBUF * STAGE];
  rows_body<BM>(a, smem);
}

// split count: balanced grid (see conv_wgrad_splits), >= 4 stages per split,
// at most 512 workgroups: every split writes and the reduction re-reads a full
// f32 weight slab (~75 MB per conv at 768 workgroups), and two rounds of 256
// long-K workgroups beat three of shorter ones (step 5.233 -> 5.214 ms,
// gpurun_out/r5n, r5o; 384: 5.210 vs 5.169 -- too few workgroups)
int rows_splits(long tiles, int stages) {
  constexpr long maxwg = 512;
  const long maxs = std::max(1, std::min(256, stages / 4));
  int best = 1;
  double bs = -1e30;
  for (long s = 1; s <= maxs; ++s) {
    const long nwg = tiles * s;
    if (nwg > maxwg && s > 1) break;
    const long per = (nwg + 255) / 256;
    double score = (double)nwg / (256.0 * per) - 0.02 * (double)nwg / 256.0;
    if (nwg < 384) score -= 0.5 * (384.0 - (double)nwg) / 384.0;
    if (score > bs + 1e-9) {
      bs = score;
      best = (int)s;
    }
  }
  return best;
}

}  // namespace hvit_rows

using namespace hvit_rows;

// eligibility of the shifted-row path (bf16, 3x3 / stride 1 / pad 1, every
// 64-channel block inside one source, whole 64-pixel stages inside one image,
// 31-bit byte offsets)
bool conv_wgrad_rows_geom_ok(const hvit_conv_geom_t* g) {
  if (g->KS != 3 || g->stride != 1 || g->pad != 1 || (g->U != 1 && g->U != 2)) return false;
  if (g->C1 % 64 || g->C2 % 64 || g->Cout % 64) return false;
  if (!aligned16(g->src1) || (g->src2 && !aligned16(g->src2))) return false;
  const int Ho = g->Hs * g->U, Wo = g->Ws * g->U;
  if (Wo >= 64 ? (Wo % 64 != 0) : (Wo % 16 != 0 || 64 % Wo != 0 || Ho % (64 / Wo) != 0)) return false;
  const long P = (long)g->N * Ho * Wo;
  const long in1 = (long)g->N * g->Hs * g->Ws * g->C1 * 2, in2 = (long)g->N * g->Hs * g->Ws * g->C2 * 2;
  return P * g->Cout * 2 < (1L << 31) && in1 < (1L << 31) && in2 < (1L << 31);
}

bool conv_wgrad_rows_ok(int dt, const hvit_conv_geom_t* g) { return dt == HVIT_BF16 && conv_wgrad_rows_geom_ok(g); }

long long conv_wgrad_rows_ws(const hvit_conv_geom_t* g) {
  const int Ho = g->Hs * g->U, Wo = g->Ws * g->U;
  const int stages = (int)((long)g->N * Ho * Wo / 64);
  const int BM = g->Cout % 128 == 0 ? 128 : 64;
  const long tiles = (long)(g->Cout / BM) * 3 * ((g->C1 + g->C2) / 64);
  const int s = rows_splits(tiles, stages);
  const long long kt = 9LL * (g->C1 + g->C2);
  return s > 1 ? (long long)s * g->Cout * kt : 0;
}

int conv_wgrad_rows(const hvit_conv_geom_t* g, const void* dy, float* dw_packed, float* ws, long long ws_elems,
                    hipStream_t st, ConvSlabs* slabs) {
  RowsArgs a;
  const int Ho = g->Hs * g->U, Wo = g->Ws * g->U;
  a.dy = (const bf16_t*)dy;
  a.src1 = (const bf16_t*)g->src1;
  a.src2 = g->src2 ? (const bf16_t*)g->src2 : (const bf16_t*)g->src1;
  a.C1 = g->C1;
  a.C2 = g->C2;
  a.Ctot = g->C1 + g->C2;
  a.Cout = g->Cout;
  a.Hs = g->Hs;
  a.Ws = g->Ws;
  a.ushift = g->U == 2 ? 1 : 0;
  a.Hi = Ho;
  a.Wi = Wo;
  a.Ho = Ho;
  a.Wo = Wo;
  a.stages = (int)((long)g->N * Ho * Wo / 64);
  const int BM = g->Cout % 128 == 0 ? 128 : 64;
  a.cib_n = a.Ctot / 64;
  a.tiles = (g->Cout / BM) * 3 * a.cib_n;
  int splits = rows_splits(a.tiles, a.stages);
  a.Kt = 9 * a.Ctot;
  a.slab = (long long)g->Cout * a.Kt;
  if (splits > 1 && (!ws || ws_elems < (long long)splits * a.slab)) splits = 1;
  a.sps = (a.stages + splits - 1) / splits;
  splits = (a.stages + a.sps - 1) / a.sps;
  a.out = splits > 1 ? ws : dw_packed;
  a.bytes1 = (unsigned)((long)g->N * g->Hs * g->Ws * g->C1 * 2);
  a.bytes2 = (unsigned)((long)g->N * g->Hs * g->Ws * g->C2 * 2);
  a.bytes_dy = (unsigned)((long)a.stages * 64 * g->Cout * 2);
  const dim3 grid((unsigned)(a.tiles * splits));
  if (BM == 128)
    hvit_rows::conv_wgrad_rows_kernel<128><<<grid, dim3(256), 0, st>>>(a);
  else
    hvit_rows::conv_wgrad_rows_kernel<64><<<grid, dim3(256), 0, st>>>(a);
  HVIT_LAUNCH_CHECK();
  if (splits > 1) {
    if (slabs) {  // the caller reduces them (hvit_conv_wgrad_torch)
      slabs->splits = splits;
      slabs->slab = a.slab;
      return HVIT_OK;
    }
    return hvit_sum_slabs(ws, splits, a.slab, dw_packed, st);
  }
  return HVIT_OK;
}
