// Persistent LDS-DMA GEMM whose epilogue runs under the next tile's K loop
// (gfx950), for the short-K (K = 512) ViT linears with heavy epilogues:
//   qkv forward            (attention.py:55)       y = x W^T + b           bf16
//   fc1 forward + GELU     (components.py:224-226) h' / a = drop(gelu(xW^T + b))
//   fc2 data gradient      (components.py:227 bwd) dh = (dy W2) * keep * gelu'(h), + fc1 bias-grad column sums
//
// Why: at K = 512 a tile's K loop (8 stages of 64) is as long as its epilogue
// (fc1: GELU + dropout VALU and 67 MB of bf16 stores per launch), and the
// one-tile-per-CU kernels of gemm_ring.h / gemm.h run the two back to back
// ("GEMM time split").  Here each workgroup walks a
// sequence of tiles; the accumulators of tile s-1 stay in registers while
// tile s's K loop runs, and stage t of tile s carries chunk t of tile s-1's
// epilogue: its VALU work (GELU, dropout hash, packing) issues between the
// stage's MFMAs and its 16-byte stores leave under the next stages' DMA.
//
// Structure (per workgroup, WM x WN waves, each wave a 64 x 64 output block):
//  * tiles BM x BN = 64WM x 64WN, dealt XCD-contiguously (each XCD owns a
//    contiguous range of row-major tiles, its workgroups take every gx-th);
//  * the operand stages of ALL the workgroup's tiles form one stream through
//    an NB-deep LDS ring (LDS-DMA, counted vmcnt, one raw barrier per stage):
//    the next tile's first stages are in flight under this tile's last ones;
//  * transposed MFMA: D = B-fragment x A-fragment, so a lane's accumulator
//    registers hold 4 consecutive OUTPUT COLUMNS of one output row; the B
//    image is read with its rows permuted (pperm below) so that the lane's
//    registers of fragments 2P and 2P+1 are 8 consecutive columns: every
//    epilogue chunk is one 16-byte store per lane, straight from registers --
//    no LDS staging, no barrier, so it can sit inside the K loop;
//  * every stage issues the same VMEM operations in the same order (side data
//    by LDS-DMA, A/B stages by LDS-DMA, the chunk's stores; the first tile's
//    and the prologue's stores write nothing), so every wait is a compile-time
//    vmcnt count (computed below) and the ring never drains.
// Side data: the bias (qkv, fc1) by one LDS-DMA piece per tile into a
// double-buffered LDS slot; fc2's gelu'(h) per chunk by one LDS-DMA piece per
// wave and stage, one chunk ahead, into per-wave double-buffered slots.
#include "gemm_host.h"
#include "gemm_ring.h"

namespace hvit {
namespace pp {

// a zero bias (launches without one)
__device__ __attribute__((aligned(16))) float g_zero[4096];

// B-fragment row permutation: fragment j, MFMA row ii -> wave-tile column
// 32(j>>1) + 8(ii>>2) + 4(j&1) + (ii&3): lane (g = l>>4) then holds columns
// 32P + 8g + 0..3 (fragment 2P) and 32P + 8g + 4..7 (fragment 2P+1).
__device__ __forceinline__ int pperm(int j, int ii) { return 32 * (j >> 1) + 8 * (ii >> 2) + 4 * (j & 1) + (ii & 3); }

// KC (k-contiguous) B image: [rows][128 B] like DmaImg<R, true>, with the
// 16-byte-chunk swizzle chunk ^ (4((row>>1)&1) | 2((row>>4)&1)) (applied on
// the DMA source side): conflict-free ds_read_b128 for the PERMUTED rows of
// pperm (each ds_read_b128 lane group {0-3,12-15,20-27}, ... then reads 16
// distinct 16-byte slots: for a row parity the 8 lanes' (a = ii>>2, b>>1)
// pairs map one-to-one onto the chunk positions).
struct KcPerm {
  __device__ __forceinline__ static int swz(int row) { return (4 * ((row >> 1) & 1)) | (2 * ((row >> 4) & 1)); }
  template <int R>
  __device__ __forceinline__ static unsigned src_off(int pc, int lane, long ld) {
    const int row = pc * 8 + lane / 8;
    const int c = (lane % 8) ^ swz(row);
    return (unsigned)(((long)row * ld + c * 8) * 2);
  }
  __device__ __forceinline__ static u32x4 frag(const char* img, int rbw, int j, int s, int lane) {
    const int row = rbw + pperm(j, lane & 15);
    const int ch = (4 * s + (lane >> 4)) ^ swz(row);
    return *(const u32x4*)(img + row * KSTAGE + (ch << 4));
  }
};

// MN (rows contiguous, k-major) B image: DmaImg<R, false>'s layout; the
// transposed reads take the permuted columns 4 at a time (each providing
// lane's 8-byte segment starts at a 4-column group), which costs a 2-way bank
// conflict (every lane reads the same 8-byte half of its 16-byte chunk).
template <int R>
__device__ __forceinline__ u32x4 frag_mn_perm(const char* img, int rbw, int j, int s, int lane) {
  const int g = lane >> 4, ii = lane & 15, q = ii >> 2, p = ii & 3;
  const int k0 = 32 * s + 8 * g + q;
  const int c = rbw + 32 * (j >> 1) + 8 * p + 4 * (j & 1);
  const int ch = c >> 3, byte = (c & 7) * 2;
  const unsigned base = lds_addr(img) + byte;
  return tr2_asm(base + MnSwz<R>::off(k0, ch), base + MnSwz<R>::off(k0 + 4, ch));
}

// epilogue kinds of this kernel
enum { K_STORE = 0, K_GELU_DUAL = 1, K_GELU_BWD = 2 };

template <int WM, int WN, int NB, int EKP, bool CS>
struct Cfg {
  static constexpr int NW = WM * WN, NT = 64 * NW, BM = 64 * WM, BN = 64 * WN, FM = 4, FN = 4, BK = 64, NK = 8;
  static constexpr int A_BYTES = BM * KSTAGE, B_BYTES = BN * KSTAGE;
  static constexpr int PA = A_BYTES / 1024 / NW, PB = B_BYTES / 1024 / NW;
  static constexpr int INFL = PA + PB;  // A/B DMA pieces per wave per stage
  static constexpr int STAGE = A_BYTES + B_BYTES;
  // side-data DMA pieces issued in stage t (per wave)
  __host__ __device__ static constexpr int side(int t) { return EKP == K_GELU_BWD ? 1 : (t == 0 ? 1 : 0); }
  // stores per epilogue chunk (per wave): the outputs (+ two colsum stores)
  static constexpr int S = (EKP == K_GELU_DUAL ? 2 : 1) + (CS ? 2 : 0);
  __host__ __device__ static constexpr int vm(int t) { return side(t) + INFL + S; }
  // stage-start wait: everything older than the youngest X(t) VMEM operations
  // has completed <=> the DMA of stage t (issued NB-1 stages earlier, after
  // that stage's side pieces, before its stores) has landed
  __host__ __device__ static constexpr int X(int t) {
    int x = S;
    for (int j = 1; j <= NB - 2; ++j) x += vm((t - NB + 1 + j + 8) & 7);
    return x;
  }
  // gelu'(h) of chunk t (the first op of stage t-1) landed, checked after
  // stage t's A/B DMA issue
  static constexpr int WAUX = 2 * INFL + S + 1;
  static constexpr int SIDE_BYTES = EKP == K_GELU_BWD ? 2 * NW * 1024 : 2 * 1024;
  static constexpr int SMEM = NB * STAGE + SIDE_BYTES;
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert(FM * FN / 2 == NK, "one epilogue chunk per stage");
  static_assert(INFL * (NB + 1) + 3 * S + 4 <= 63, "vmcnt range");
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                           0x00020000);
}
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// compile-time loop (the stage index sets s_waitcnt immediates)
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    static_for<I + 1, N>(f);
  }
}
// every epilogue store is ONE buffer_store_dwordx4 (a compiler-counted builtin:
// the counts below rely on it); lanes that must not write carry an offset
// past num_records (bit 31 set, the low bits kept so no two stores coincide
// and none is merged away)
constexpr unsigned OOB = 0x80000000u;
__device__ __forceinline__ void st16(const u32x4& v, __amdgpu_buffer_rsrc_t r, unsigned off) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}

// 16-lane (DPP row) sum, every lane of the row gets the total; fixed order
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
  return v;
}

// (the body lives in a struct's static member: written directly as the
// __global__ template's body, hipcc's host pass silently dropped the kernels'
// launch stubs -- undefined symbols at load time)
template <int WM, int WN, int NB, bool KCB, int EKP, bool CS>
struct PpKernel {
__device__ __forceinline__ static void run(const LdDense<bf16_t, true>& la, const LdDense<bf16_t, KCB>& lb, int M,
                                           int N, const Epi& ep) {
  using C = Cfg<WM, WN, NB, EKP, CS>;
  constexpr int NW = C::NW, BM = C::BM, BN = C::BN, FM = C::FM, FN = C::FN, BK = C::BK, NK = C::NK;
  constexpr int PA = C::PA, PB = C::PB, STAGE = C::STAGE, S = C::S;
  using IA = DmaImg<BM, true>;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  char* const side_lds = smem + NB * STAGE;

  // deferred split-K slab sums carried by this launch (nothing in flight yet)
  epi_side(ep);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int li = lane & 15, g = lane >> 4;

  // ---- tile schedule: XCD x owns row-major tiles [lo, hi); its workgroups
  // (blockIdx % 8 == x) take every gx-th of them
  const int tn = N / BN, T = (M / BM) * tn;
  const int G = gridDim.x, xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, gx = G >> 3;
  const int q8 = T >> 3, r8 = T & 7;
  const int lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int hi = lo + (xcd < r8 ? q8 + 1 : q8);
  const int ns = lo + slot < hi ? (hi - lo - slot + gx - 1) / gx : 0;
  if (ns == 0) return;

  // ---- operand DMA: per-lane source offsets (fixed), per-stage uniform base
  const __amdgpu_buffer_rsrc_t ra = rsrc_of(la.p, (long)la.rows * la.ld * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc_of(lb.p, (KCB ? (long)lb.rows : (long)lb.K) * lb.ld * 2);
  unsigned va[PA], vb[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) va[i] = IA::src_off(wid + NW * i, lane, la.ld);
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    if constexpr (KCB) vb[i] = KcPerm::src_off<BN>(wid + NW * i, lane, lb.ld);
    else vb[i] = DmaImg<BN, false>::src_off(wid + NW * i, lane, lb.ld);
  }
  const unsigned da = BK * 2, db = KCB ? BK * 2 : (unsigned)(BK * lb.ld * 2);
  auto abase = [&](int m0) { return (unsigned)((long)m0 * la.ld * 2); };
  auto bbase = [&](int n0) { return KCB ? (unsigned)((long)n0 * lb.ld * 2) : (unsigned)(n0 * 2); };
  // ring slot of the next DMA (wbuf) and of the stage being read (rbuf)
  int wbuf = 0, rbuf = 0;
  auto ring_next = [](int x) { return x + 1 == NB ? 0 : x + 1; };
  auto issue_ab = [&](unsigned sa, unsigned sb) {
    char* abuf = smem + wbuf * STAGE;
    char* bbuf = abuf + C::A_BYTES;
#pragma unroll
    for (int i = 0; i < PA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(abuf + (wid + NW * i) * 1024), 16, va[i], sa, 0, 0);
#pragma unroll
    for (int i = 0; i < PB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(bbuf + (wid + NW * i) * 1024), 16, vb[i], sb, 0, 0);
    wbuf = ring_next(wbuf);
  };

  // ---- side data and outputs
  const float* biasp = ep.bias ? ep.bias : g_zero;
  const __amdgpu_buffer_rsrc_t rbias = rsrc_of(biasp, ep.bias ? (long)N * 4 : 4096L * 4);
  const __amdgpu_buffer_rsrc_t raux = EKP == K_GELU_BWD ? rsrc_of(ep.aux, (long)M * ep.ldaux * 2) : rbias;
  // out (bf16 [M][ldo]); GELU_DUAL: out may be absent (inference: gelu only)
  const __amdgpu_buffer_rsrc_t rout = rsrc_of(ep.out ? ep.out : ep.out2, ep.out ? (long)M * ep.ldo * 2 : 0L);
  const __amdgpu_buffer_rsrc_t rout2 = EKP == K_GELU_DUAL ? rsrc_of(ep.out2, (long)M * ep.ldo2 * 2) : rout;
  const long nrows_cs = (M + 63) / 64;
  const __amdgpu_buffer_rsrc_t rcs = CS ? rsrc_of(ep.colsum, nrows_cs * N * 4) : rout;
  // the tile's bias (BN floats; the piece's other lanes read past them: zeros
  // or the next columns, never used) -> bias slot sb (every wave: the same bytes)
  auto issue_bias = [&](int n0, int sb) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rbias, (lds_ptr_t)(side_lds + sb * 1024), 16, (unsigned)(lane * 16),
                                             (unsigned)(n0 * 4), 0, 0);
  };
  // chunk c = P*4 + i of a tile at (m0, n0): this lane's row and first column
  auto crow = [&](int m0, int c) { return m0 + wm * 64 + 16 * (c & 3) + li; };
  auto ccol = [&](int n0, int c) { return n0 + wn * 64 + 32 * (c >> 2) + 8 * g; };
  // gelu'(h) of chunk c -> this wave's aux slot sa (lane-linear 16 bytes)
  auto issue_aux = [&](int m0, int n0, int c, int sa) {
    const unsigned off = (unsigned)(((long)crow(m0, c) * ep.ldaux + ccol(n0, c)) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(raux, (lds_ptr_t)(side_lds + (sa * NW + wid) * 1024), 16, off, 0, 0, 0);
  };
  const uint32_t dkey = epi_key(ep);

  // ---- one epilogue chunk: 8 consecutive columns of one row per lane
  // (acc[i][2P], acc[i][2P+1]); !live (no previous tile) keeps every store
  // but points it past the buffer
  auto chunk = [&](f32x4 (&a)[FM][FN], auto cc, int m0, int n0, int bslot, bool live) {
    constexpr int c = decltype(cc)::value, i = c & 3, P = c >> 2;
    const int m = crow(m0, c), n = ccol(n0, c);
    const unsigned kill = live ? 0u : OOB;
    f32x4 va8 = a[i][2 * P], vb8 = a[i][2 * P + 1];
    if constexpr (EKP == K_STORE || EKP == K_GELU_DUAL) {
      const float* bl = (const float*)(side_lds + bslot * 1024) + wn * 64 + 32 * P + 8 * g;
      va8 += *(const f32x4*)bl;
      vb8 += *(const f32x4*)(bl + 4);
    }
    if constexpr (EKP == K_STORE) {
      st16(pack8(va8, vb8), rout, (unsigned)(((long)m * ep.ldo + n) * 2) | kill);
    } else if constexpr (EKP == K_GELU_DUAL) {
      f32x4 ka = {1.f, 1.f, 1.f, 1.f}, kb = ka;
      if (ep.drop_thr) {
        const uint64_t i0 = (uint64_t)m * (uint64_t)N + (uint64_t)n;
        ka = keep4_at(dkey, i0, ep.drop_thr, ep.drop_scale);
        kb = keep4_at(dkey, i0 + 4, ep.drop_thr, ep.drop_scale);
      }
      f32x4 ga, gb, dda, ddb;
      gelu_gg4(va8, ga, dda);
      gelu_gg4(vb8, gb, ddb);
      ga *= ka;
      gb *= kb;
      if (ep.gd == 2) {  // GELU_DUAL_DK
        dda *= ka;
        ddb *= kb;
      }
      st16(ep.gd ? pack8(dda, ddb) : pack8(va8, vb8), rout, (unsigned)(((long)m * ep.ldo + n) * 2) | kill);
      st16(pack8(ga, gb), rout2, (unsigned)(((long)m * ep.ldo2 + n) * 2) | kill);
    } else {  // K_GELU_BWD: v *= keep * gelu'(h)  (aux = gelu'(h) when gd, else h)
      const u32x4 hu = *(const u32x4*)(side_lds + ((c & 1) * NW + wid) * 1024 + lane * 16);
      f32x4 ha, hb;
      unpack8(hu, ha, hb);
      if (ep.drop_thr) {
        const uint64_t i0 = (uint64_t)m * (uint64_t)N + (uint64_t)n;
        va8 *= keep4_at(dkey, i0, ep.drop_thr, ep.drop_scale);
        vb8 *= keep4_at(dkey, i0 + 4, ep.drop_thr, ep.drop_scale);
      }
      if (ep.gd) {
        va8 *= ha;
        vb8 *= hb;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          va8[e] *= gelu_grad(ha[e]);
          vb8[e] *= gelu_grad(hb[e]);
        }
      }
      st16(pack8(va8, vb8), rout, (unsigned)(((long)m * ep.ldo + n) * 2) | kill);
    }
    if constexpr (CS) {
      // column sums of this wave's 64 rows: the chunk's final values replace
      // its (now dead) accumulators; at i = 3 the four rows of each lane are
      // summed in order, then the 16 lanes of the row group (fixed order);
      // one partial row per 64-row block
      a[i][2 * P] = va8;
      a[i][2 * P + 1] = vb8;
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
      if constexpr (i == 3) {
        s0 = a[0][2 * P] + a[1][2 * P] + a[2][2 * P] + a[3][2 * P];
        s1 = a[0][2 * P + 1] + a[1][2 * P + 1] + a[2][2 * P + 1] + a[3][2 * P + 1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s0[e] = row16_sum(s0[e]);
          s1[e] = row16_sum(s1[e]);
        }
      }
      const unsigned off = (unsigned)((((long)((m0 + wm * 64) >> 6)) * N + n) * 4);
      const unsigned wk = (live && i == 3 && li == 0) ? 0u : OOB;
      st16(__builtin_bit_cast(u32x4, s0), rcs, off | wk);
      st16(__builtin_bit_cast(u32x4, s1), rcs, (off + 16) | wk);
    }
  };

  // ---- prologue: ring stages 0 .. NB-2 in flight, each wrapped in the VMEM
  // pattern of the stage slot that would have issued it (slots 8-NB+1 .. 7 of
  // a tile: their side pieces, the DMA, S stores that write nothing)
  int m0 = (lo + slot) / tn * BM, n0 = (lo + slot) % tn * BN;
  static_for<0, NB - 1>([&](auto pc) {
    constexpr int p = decltype(pc)::value, t = NK - (NB - 1) + p;
    if constexpr (C::side(t) > 0) {
      if constexpr (EKP == K_GELU_BWD) issue_aux(m0, n0, 0, (t + 1) & 1);  // slot of "chunk t+1": never used
      else issue_bias(n0, 1);
    }
    issue_ab(abase(m0) + p * da, bbase(n0) + p * db);
#pragma unroll
    for (int k = 0; k < S; ++k) st16((u32x4){0u, 0u, 0u, 0u}, rout, OOB | (unsigned)(64 * (p * S + k) + lane * 16) << 4);
  });

  f32x4 acc[FM][FN], accP[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) accP[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int pm0 = m0, pn0 = n0;  // the tile whose epilogue runs (accP)

  for (int s = 0; s < ns; ++s) {
    // the next tile (its first stages are issued in this tile's last ones);
    // past the last tile the DMA re-reads this tile's stage 7 (never read)
    const bool more = s + 1 < ns;
    const int idn = lo + slot + (s + 1) * gx;
    const int m0n = more ? idn / tn * BM : m0, n0n = more ? idn % tn * BN : n0;
    const bool live = s > 0;
    static_for<0, NK>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      // stage t landed for this wave, then for every wave (and every wave is
      // done reading the ring slot the DMA below refills)
      __builtin_amdgcn_s_waitcnt(vm_imm(C::X(t)));
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const char* at = smem + rbuf * STAGE;
      const char* bt = at + C::A_BYTES;
      rbuf = ring_next(rbuf);
      u32x4 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
      auto load = [&](int ks, u32x4 (&fa)[FM], u32x4 (&fb)[FN]) {
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = IA::frag(at, wm * 64 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (KCB) fb[j] = KcPerm::frag(bt, wn * 64, j, ks, lane);
          else fb[j] = frag_mn_perm<BN>(bt, wn * 64, j, ks, lane);
        }
      };
      // k-step 1's fragments are read under k-step 0's MFMAs, except in the
      // GELU backward (its gelu'(h) chunk and the transposed-read addresses
      // leave no room for a second fragment set: read after them)
      constexpr bool PRE = EKP != K_GELU_BWD;
      load(0, fa0, fb0);
      lgkm_wait0();
      lds_pin(fa0);
      lds_pin(fb0);
      if constexpr (PRE) load(1, fa1, fb1);
      // side data: gelu'(h) of the next chunk (stage 7: chunk 0 of THIS tile,
      // the next tile's first epilogue chunk); the tile's bias at stage 0
      if constexpr (EKP == K_GELU_BWD) {
        if constexpr (t < NK - 1) issue_aux(pm0, pn0, t + 1, (t + 1) & 1);
        else issue_aux(m0, n0, 0, 0);
      } else if constexpr (t == 0) {
        issue_bias(n0, s & 1);
      }
      // the A/B stage NB-1 ahead (this tile, or the next one's first stages)
      if constexpr (t + NB - 1 < NK) {
        issue_ab(abase(m0) + (t + NB - 1) * da, bbase(n0) + (t + NB - 1) * db);
      } else {
        if (more) issue_ab(abase(m0n) + (t + NB - 1 - NK) * da, bbase(n0n) + (t + NB - 1 - NK) * db);
        else issue_ab(abase(m0) + (NK - 1) * da, bbase(n0) + (NK - 1) * db);
      }
      auto mma = [&](const u32x4 (&fa)[FM], const u32x4 (&fb)[FN], auto zc) {
        constexpr bool zero = decltype(zc)::value;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(s16x8, fb[j]), __builtin_bit_cast(s16x8, fa[i]),
                zero ? (f32x4){0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
      };
      mma(fa0, fb0, std::integral_constant<bool, t == 0>());
      if constexpr (EKP == K_GELU_BWD) {
        // this chunk's gelu'(h) (issued at the start of the previous stage)
        __builtin_amdgcn_s_waitcnt(vm_imm(C::WAUX));
        asm volatile("" ::: "memory");
      }
      if constexpr (!PRE) load(1, fa1, fb1);
      lgkm_wait0();
      lds_pin(fa1);
      lds_pin(fb1);
      mma(fa1, fb1, std::false_type());
      // chunk t of the previous tile's epilogue (its VALU fills the MFMA
      // gaps; its stores are the stage's last VMEM operations)
      chunk(accP, tc, pm0, pn0, (s + 1) & 1, live);
    });
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) accP[i][j] = acc[i][j];
    pm0 = m0;
    pn0 = n0;
    m0 = m0n;
    n0 = n0n;
  }
  // ---- the last tile's epilogue: drain the ring's trailing stages first
  __builtin_amdgcn_s_waitcnt(vm_imm(0));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  static_for<0, NK>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if constexpr (EKP == K_GELU_BWD) {
      if constexpr (c > 0) {
        issue_aux(pm0, pn0, c, c & 1);
        __builtin_amdgcn_s_waitcnt(vm_imm(0));
        asm volatile("" ::: "memory");
      }
    }
    chunk(accP, cc, pm0, pn0, (ns & 1) ? 0 : 1, true);
    if constexpr (EKP == K_GELU_BWD) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  });
}

};

template <int WM, int WN, int NB, bool KCB, int EKP, bool CS>
__global__ __launch_bounds__(64 * WM * WN, 2) void gemm_pp_kernel(LdDense<bf16_t, true> la, LdDense<bf16_t, KCB> lb,
                                                                   int M, int N, Epi ep) {
  PpKernel<WM, WN, NB, KCB, EKP, CS>::run(la, lb, M, N, ep);
}

}  // namespace pp

// ------------------------------------------------------------------ host ----
// Mode (hvit_gemm_tune(3, v) / HVIT_PP): -1 automatic, 0 off, 1 = 256x128
// tiles (8 waves, 3-stage ring, one workgroup per CU), 2 = 128x128 (4 waves,
// 2-stage ring, two workgroups per CU).
int& pp_mode_ref() {
  static int v = getenv("HVIT_PP") ? atoi(getenv("HVIT_PP")) : 0;  // (off until validated on the GPU)
  return v;
}

template <int WM, int WN, int NB, bool KCB, int EKP, bool CS>
static int pp_launch(const LdDense<bf16_t, true>& la, const LdDense<bf16_t, KCB>& lb, int M, int N, const Epi& ep,
                     hipStream_t st) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  const int T = (M / BM) * (N / BN);
  const int per_cu = WM * WN == 8 ? 1 : 2;
  int G = std::min(256 * per_cu, T);
  G = std::max(8, G / 8 * 8);
  hipLaunchKernelGGL((pp::gemm_pp_kernel<WM, WN, NB, KCB, EKP, CS>), dim3(G), dim3(64 * WM * WN), 0, st, la, lb, M,
                     N, ep);
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

template <bool KCB, int EKP, bool CS>
static int pp_dispatch(int mode, const LdDense<bf16_t, true>& la, const LdDense<bf16_t, KCB>& lb, int M, int N,
                       const Epi& ep, hipStream_t st) {
  if (mode == 2) return pp_launch<2, 2, 2, KCB, EKP, CS>(la, lb, M, N, ep, st);
  return pp_launch<4, 2, 3, KCB, EKP, CS>(la, lb, M, N, ep, st);
}

// C = A(M x 512, k-contiguous) x B^T through the persistent kernel when the
// launch qualifies; false sends the caller to the ring / gemm.h kernels.
template <bool KCB>
static bool pp_try(const LdDense<bf16_t, true>& la, const LdDense<bf16_t, KCB>& lb, int M, int N, int K,
                   const Epi& ep, hipStream_t st, int* rc) {
  int mode = pp_mode_ref();
  if (mode == 0) return false;
  // automatic: the K = 512 shapes with at least ~1.5 tiles of 256 x 128 per CU
  // (qkv / fc1 forward, the fc2 data gradient at B >= 24)
  if (mode < 0) mode = (M % 256 == 0 && N % 128 == 0 && (long)(M / 256) * (N / 128) >= 384) ? 1 : 0;
  if (mode == 0) return false;
  const int bm = mode == 2 ? 128 : 256, bn = 128;
  if (K != 512 || M <= 0 || M % bm || N % bn || N > 4096) return false;
  if (!la.vok || !lb.vok || (la.ld & 7) || (lb.ld & 7)) return false;
  if (ep.mode != EPI_STORE || ep.resid || ep.rowadd || ep.stats || ep.rs_ptr || ep.relu || ep.pool2) return false;
  if (ep.out_dt != HVIT_BF16 || (ep.ldo & 7)) return false;
  auto al = [](const void* p) { return !p || (((uintptr_t)p) & 15) == 0; };
  if (!al(ep.out) || !al(ep.out2) || !al(ep.aux) || !al(ep.bias) || !al(ep.colsum)) return false;
  if (dense_bytes(la) >= (1L << 31) || dense_bytes(lb) >= (1L << 31)) return false;
  int ekp;
  if (ep.act == ACT_NONE) {
    if (ep.drop_thr || ep.drop_scale != 1.f || ep.colsum) return false;
    ekp = pp::K_STORE;
  } else if (ep.act == ACT_GELU_DUAL) {
    if (!ep.out2 || ep.out2_dt != HVIT_BF16 || (ep.ldo2 & 7) || ep.colsum) return false;
    if (!ep.drop_thr && ep.drop_scale != 1.f) return false;
    ekp = pp::K_GELU_DUAL;
  } else if (ep.act == ACT_GELU_BWD) {
    if (!ep.aux || ep.aux_dt != HVIT_BF16 || (ep.ldaux & 7) || ep.bias) return false;
    if (!ep.drop_thr && ep.drop_scale != 1.f) return false;
    if ((long)M * ep.ldaux * 2 >= (1L << 31)) return false;
    ekp = pp::K_GELU_BWD;
  } else {
    return false;
  }
  // forward (B k-contiguous): qkv, fc1; data gradient (B k-major): fc2
  if constexpr (KCB) {
    if (ekp == pp::K_STORE) *rc = pp_dispatch<KCB, pp::K_STORE, false>(mode, la, lb, M, N, ep, st);
    else if (ekp == pp::K_GELU_DUAL) *rc = pp_dispatch<KCB, pp::K_GELU_DUAL, false>(mode, la, lb, M, N, ep, st);
    else return false;
  } else {
    if (ekp != pp::K_GELU_BWD) return false;
    if (ep.colsum) *rc = pp_dispatch<KCB, pp::K_GELU_BWD, true>(mode, la, lb, M, N, ep, st);
    else *rc = pp_dispatch<KCB, pp::K_GELU_BWD, false>(mode, la, lb, M, N, ep, st);
  }
  return true;
}

}  // namespace hvit

// entry points used by gemm_linear.hip (forward: B k-contiguous; data
// gradient: B = W^T, k-major)
bool hvit_pp_fwd(const void* x, const void* w, int M, int N, int K, const hvit::Epi& ep, hipStream_t st, int* rc) {
  using namespace hvit;
  return pp_try<true>(dense<bf16_t, true>(x, K, M, K), dense<bf16_t, true>(w, K, N, K), M, N, K, ep, st, rc);
}
bool hvit_pp_dgrad(const void* dy, const void* w, int M, int N, int K, const hvit::Epi& ep, hipStream_t st, int* rc) {
  using namespace hvit;
  // dx[M, K] = dy[M, N] w[N, K]: output columns K, reduction N
  return pp_try<false>(dense<bf16_t, true>(dy, N, M, N), dense<bf16_t, false>(w, K, K, N), M, K, N, ep, st, rc);
}
int hvit_pp_tune(int value) {
  const int old = hvit::pp_mode_ref();
  hvit::pp_mode_ref() = value;
  return old;
}
