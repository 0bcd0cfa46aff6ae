// Ring-pipelined LDS-DMA GEMM for the dense bf16 ViT linears (gfx950).
//
//   C[m][n] = sum_k A(m, k) * B(n, k)     A, B dense bf16, KC (k contiguous) or
//                                         MN (rows contiguous, k-major) operands
//
// The HybridViT linears (attention.py:55,58 qkv / proj, components.py:224,227
// fc1 / fc2; forward, data gradient, weight gradient) are too small for the
// chip to hide L2 latency with the two-stage loop of gemm.h: at one or two
// workgroups per CU a 128x128 tile keeps one 32 KiB stage in flight, and the
// K loop runs at the rate one stage's round trip allows.  Here the stages live
// in an LDS ring of NB buffers: stage t + NB - 1 is issued (buffer_load ... lds,
// one 1 KiB piece per wave-instruction) before the wait for stage t, so NB - 1
// stages are in flight under every stage's MFMAs, and each wait is a counted
// vmcnt that leaves them in flight (raw s_barrier: __syncthreads would drain
// them).  Tiles: BM x BN with WM x WN waves (4 or 8), each wave a WTM x WTN
// block of 16x16x32 bf16 MFMAs; LDS images and their bank swizzles are
// gemm.h's DmaImg (source-side swizzle, conflict-free ds_read_b128 /
// ds_read_b64_tr_b16 fragment reads).
//
// Epilogues (staged through LDS in 64-row passes, 8 adjacent columns per
// thread, 16-byte stores): plain (+bias, bf16 or f32, optional column sums),
// fc1's GELU_DUAL, the residual adds of proj / fc2, fc2's GELU backward (+bias
// grad column sums), and split-K partial slabs.  Every tile is interior (the
// host guarantees M % BM == N % BN == 0, K slices multiples of 64).
#pragma once
#include "gemm.h"

namespace hvit {

// s_waitcnt immediate of vmcnt(v), expcnt / lgkmcnt untouched (gfx9: vmcnt
// bits 3:0 and 15:14)
constexpr int vm_imm(int v) { return 0x0F70 | (v & 15) | (((v >> 4) & 3) << 14); }

template <int BM, int BN, int WM, int WN, int NB, bool KCA, bool KCB>
struct RingCore {
  static constexpr int NW = WM * WN, NT = 64 * NW;
  using IA = DmaImg<BM, KCA>;
  using IB = DmaImg<BN, KCB>;
  static constexpr int BK = 64;
  static constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  static constexpr int PA = IA::PIECES / NW, PB = IB::PIECES / NW;
  static constexpr int INFL = PA + PB;  // this wave's DMA instructions per stage
  static constexpr int STAGE = IA::BYTES + IB::BYTES;
  static constexpr int SM = NB * STAGE;
  static_assert(IA::PIECES % NW == 0 && IB::PIECES % NW == 0, "stage pieces must split over the waves");
  static_assert(NB >= 2 && NB <= 4 && (NB - 2) * INFL <= 63, "ring depth / vmcnt range");
  static_assert(FM >= 1 && FN >= 1, "wave tile");
  static constexpr int MPD = (FM * FN) / INFL > 0 ? (FM * FN) / INFL : 1;  // MFMAs per DMA piece in the interleave
  static_assert(MPD * INFL <= FM * FN, "interleave");

  __device__ __forceinline__ static __amdgpu_buffer_rsrc_t rsrc(const LdDense<bf16_t, true>& l) {
    const long bytes = (long)l.rows * l.ld * 2;
    return __builtin_amdgcn_make_buffer_rsrc((void*)l.p, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                             0x00020000);
  }
  __device__ __forceinline__ static __amdgpu_buffer_rsrc_t rsrc(const LdDense<bf16_t, false>& l) {
    const long bytes = (long)l.K * l.ld * 2;
    return __builtin_amdgcn_make_buffer_rsrc((void*)l.p, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                             0x00020000);
  }

  __device__ __forceinline__ static void run(const LdDense<bf16_t, KCA>& la, const LdDense<bf16_t, KCB>& lb, char* smem,
                                             int m0, int n0, int kbeg, int kend, f32x4 (&acc)[FM][FN],
                                             const Epi& ep) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int nk = (kend - kbeg) / BK;
    if (nk <= 0) {
      epi_side(ep);
      return;
    }
    const __amdgpu_buffer_rsrc_t ra = rsrc(la), rb = rsrc(lb);
    const unsigned oa = (unsigned)(KCA ? ((long)m0 * la.ld + kbeg) * 2 : ((long)kbeg * la.ld + m0) * 2);
    const unsigned da = (unsigned)(KCA ? BK * 2 : (long)BK * la.ld * 2);
    const unsigned ob = (unsigned)(KCB ? ((long)n0 * lb.ld + kbeg) * 2 : ((long)kbeg * lb.ld + n0) * 2);
    const unsigned db = (unsigned)(KCB ? BK * 2 : (long)BK * lb.ld * 2);
    unsigned va[PA], vb[PB];
#pragma unroll
    for (int i = 0; i < PA; ++i) va[i] = IA::src_off(wid + NW * i, lane, la.ld);
#pragma unroll
    for (int i = 0; i < PB; ++i) vb[i] = IB::src_off(wid + NW * i, lane, lb.ld);

    // stage t -> ring buffer t % NB.  Stages past the end re-read the last
    // stage into the buffer that would have held them (never read again), so
    // every iteration issues the same number of DMA instructions and every
    // wait is one constant count.
    auto issue = [&](int t) {
      char* abuf = smem + (t % NB) * STAGE;
      char* bbuf = abuf + IA::BYTES;
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
    // prologue: stages 0 .. NB-2 in flight
#pragma unroll
    for (int t = 0; t < NB - 1; ++t) issue(t);
    // a side job (epi_side) while the prologue stages are in flight
    epi_side(ep);
#ifdef HVIT_GEMM_STAMPS
    unsigned long long wait_cyc = 0, t_w0 = 0;
#endif
    for (int t = 0; t < nk; ++t) {
#ifdef HVIT_GEMM_STAMPS
      t_w0 = __builtin_amdgcn_s_memtime();
#endif
      // stage t landed for this wave (NB-2 younger stages stay in flight) ...
      __builtin_amdgcn_s_waitcnt(vm_imm((NB - 2) * INFL));
      asm volatile("" ::: "memory");
      // ... and for every wave; every wave has also finished reading stage
      // t-1 (its reads were waited for before its MFMAs), so buffer
      // (t-1) % NB = (t+NB-1) % NB may be refilled: one barrier per stage
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#ifdef HVIT_GEMM_STAMPS
      wait_cyc += __builtin_amdgcn_s_memtime() - t_w0;
#endif
      const char* at = smem + (t % NB) * STAGE;
      const char* bt = at + IA::BYTES;
      u32x4 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
      load(at, bt, 0, fa0, fb0);
      lgkm_wait0();
      lds_pin(fa0);
      lds_pin(fb0);
      load(at, bt, 1, fa1, fb1);
      // stage t+NB-1's DMA issue spread over k-step 0's MFMAs
      issue(t + NB - 1);
      mma(fa0, fb0);
      __builtin_amdgcn_sched_group_barrier(0x100, FM + FN, 0);  // the k-step 1 fragment reads first
#pragma unroll
      for (int k = 0; k < INFL; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, MPD, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);    // one DMA piece
      }
      __builtin_amdgcn_sched_group_barrier(0x008, FM * FN - MPD * INFL, 0);
      lgkm_wait0();
      lds_pin(fa1);
      lds_pin(fb1);
      mma(fa1, fb1);
    }
#ifdef HVIT_GEMM_STAMPS
    {  // wave 0's cycles spent in the per-stage wait + barrier (shader clock), slot 3
      const unsigned bid_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
      if (threadIdx.x == 0 && bid_ < 65536) g_gemm_stamps[bid_ * 4 + 3] = wait_cyc;
    }
#endif
    // drain the trailing (never used) DMA and let every wave finish reading
    // before the epilogue reuses the ring
    __builtin_amdgcn_s_waitcnt(vm_imm(0));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
};

// wide epilogue helpers ------------------------------------------------------
__device__ __forceinline__ u32x4 pack8(const f32x4& a, const f32x4& b) {
  u32x4 u;
  u[0] = f2bf2(a[0], a[1]);
  u[1] = f2bf2(a[2], a[3]);
  u[2] = f2bf2(b[0], b[1]);
  u[3] = f2bf2(b[2], b[3]);
  return u;
}
__device__ __forceinline__ void unpack8(const u32x4& u, f32x4& a, f32x4& b) {
  a = (f32x4){__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
              __uint_as_float(u[1] & 0xffff0000u)};
  b = (f32x4){__uint_as_float(u[2] << 16), __uint_as_float(u[2] & 0xffff0000u), __uint_as_float(u[3] << 16),
              __uint_as_float(u[3] & 0xffff0000u)};
}

// EK: EK_STORE (+bias, out bf16 / f32, colsum), EK_GELU_DUAL, EK_RESID,
// EK_GELU_BWD (+colsum), EK_SLAB (f32 split-K partial, slab z = blockIdx's K slice)
template <int BM, int BN, int WM, int WN, int NB, bool KCA, bool KCB, int EK>
__global__ __launch_bounds__(64 * WM * WN, (WM * WN == 4 && NB == 2) ? (BN == 64 ? 3 : 2) : 1) void gemm_ring_kernel(LdDense<bf16_t, KCA> la, LdDense<bf16_t, KCB> lb,
                                                                   int M, int N, int K, int kps, Epi ep) {
  using C = RingCore<BM, BN, WM, WN, NB, KCA, KCB>;
  constexpr int NT = C::NT, FM = C::FM, FN = C::FN, WTM = C::WTM, WTN = C::WTN;
  constexpr int CP = BN + 4;                       // LDS tile pitch (floats)
  constexpr int C8 = BN / 8, RS8 = NT / C8, NR8 = 64 / RS8;
  static_assert(RS8 <= 64 && 64 % RS8 == 0, "epilogue row split");
  constexpr int SM_E = (64 * CP + RS8 * BN) * 4;
  __shared__ __attribute__((aligned(16))) char smem[C::SM > SM_E ? C::SM : SM_E];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: the acc -> LDS rows below branch per wave
  const int wm = wid / WN, wn = wid % WN;
  const TileId t3 = tile_of(ep.xcd_remap);
  GEMM_STAMP(0);
  const int m0 = t3.mt * BM, n0 = t3.nt * BN;
  const int kbeg = t3.z * kps;
  const int kend = min(K, kbeg + kps);
  const int frow = lane & 15, fq = lane >> 4;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  C::run(la, lb, smem, m0, n0, kbeg, kend, acc, ep);
  GEMM_STAMP(1);

  // ------------------------------------------------------------ epilogue ---
  const uint32_t dkey = epi_key(ep);
  const int c8 = tid % C8, q0 = tid / C8;
  const int n8 = n0 + c8 * 8;
  f32x4 b8a = {0.f, 0.f, 0.f, 0.f}, b8b = b8a;
  if (EK != EK_SLAB && ep.bias) {
    b8a = *(const f32x4*)(ep.bias + n8);
    b8b = *(const f32x4*)(ep.bias + n8 + 4);
  }
  float* Cs = (float*)smem;
  float cs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int hh = 0; hh < BM / 64; ++hh) {
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
    const int mbase = m0 + hh * 64;
    // this pass's side inputs, issued before the barrier so their latency
    // overlaps it (loads cannot move above the stores that follow them)
    u32x4 hin[NR8];
    f32x4 ra[NR8], rb[NR8];
    float rsc[NR8];
    if constexpr (EK == EK_GELU_BWD) {
#pragma unroll
      for (int i = 0; i < NR8; ++i) {
        const int m = mbase + q0 + i * RS8;
        if (ep.aux_dt == HVIT_BF16) {
          hin[i] = *(const u32x4*)((const bf16_t*)ep.aux + (long)m * ep.ldaux + n8);
        } else {
          const f32x4 x = *(const f32x4*)((const float*)ep.aux + (long)m * ep.ldaux + n8);
          const f32x4 y = *(const f32x4*)((const float*)ep.aux + (long)m * ep.ldaux + n8 + 4);
          hin[i] = pack8(x, y);  // (f32 h only in tests; bf16-rounded like the bf16 path)
        }
      }
    }
    if constexpr (EK == EK_RESID) {
#pragma unroll
      for (int i = 0; i < NR8; ++i) {
        const int m = mbase + q0 + i * RS8;
        ra[i] = *(const f32x4*)(ep.resid + (long)m * ep.ldr + n8);
        rb[i] = *(const f32x4*)(ep.resid + (long)m * ep.ldr + n8 + 4);
        rsc[i] = ep.rowscale ? ep.rowscale[m / ep.rows_per_sample] : 1.f;
      }
    }
    epi_barrier();
#pragma unroll
    for (int i = 0; i < NR8; ++i) {
      const int row = q0 + i * RS8;
      const int m = mbase + row;
      f32x4 va = *(const f32x4*)(Cs + row * CP + c8 * 8);
      f32x4 vb = *(const f32x4*)(Cs + row * CP + c8 * 8 + 4);
      if constexpr (EK == EK_SLAB) {
        float* slab = (float*)ep.out + (long)t3.z * ep.slab_stride + (long)m * ep.ldo + n8;
        *(f32x4*)slab = va;
        *(f32x4*)(slab + 4) = vb;
        continue;
      }
      va += b8a;
      vb += b8b;
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
        if (ep.out) *(u32x4*)((bf16_t*)ep.out + (long)m * ep.ldo + n8) = ep.gd ? pack8(da, db) : pack8(va, vb);
        *(u32x4*)((bf16_t*)ep.out2 + (long)m * ep.ldo2 + n8) = pack8(ga, gb);
        continue;
      }
      if (EK != EK_STORE && ep.drop_thr) {
        va *= keep4(ep, dkey, m, n8, N);
        vb *= keep4(ep, dkey, m, n8 + 4, N);
      }
      if constexpr (EK == EK_GELU_BWD) {
        f32x4 ha, hb;
        unpack8(hin[i], ha, hb);
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
        *(u32x4*)((bf16_t*)ep.out + (long)m * ep.ldo + n8) = pack8(va, vb);
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
  if constexpr (EK == EK_SLAB) {
    // In-kernel split-K reduction (cdna_hip_programming.md section 5, "In-launch
    // split-K reduction", counter form): every slice publishes its slab (plain
    // stores, each wave's vmcnt(0), barrier, one agent release), then takes a
    // ticket; the slice that draws splits-1 acquires and sums all slabs of the
    // tile into red_out.  Correct for any placement of the slices; no slice
    // waits on another, so no co-residency is assumed.  The reducer resets the
    // ticket for the next call (tickets start zeroed: the caller's zero pool).
    if (ep.tickets) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = (int*)(smem + 64 * CP * 4);  // inside the one LDS array (no second __shared__ object)
      const int splits = gridDim.z;
      const int tile = t3.mt * gridDim.y + t3.nt;
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(ep.tickets + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == (unsigned)(splits - 1);
        if (last) __hip_atomic_store(ep.tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      if (!*flag) return;
      if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      constexpr int RPT = BM / RS8;  // rows per thread over the whole tile
#pragma unroll 2
      for (int i = 0; i < RPT; ++i) {
        const int m = m0 + q0 + i * RS8;
        const float* src = (const float*)ep.out + (long)m * ep.ldo + n8;
        f32x4 sa = *(const f32x4*)src, sb = *(const f32x4*)(src + 4);
        for (int z = 1; z < splits; ++z) {
          const float* q = src + (long)z * ep.slab_stride;
          sa += *(const f32x4*)q;
          sb += *(const f32x4*)(q + 4);
        }
        float* dst = ep.red_out + (long)m * ep.ldo + n8;
        *(f32x4*)dst = sa;
        *(f32x4*)(dst + 4) = sb;
      }
    }
    return;
  }
  if (EK != EK_GELU_DUAL && ep.colsum) {
    float* red = Cs + 64 * CP;  // [RS8][BN]
    epi_barrier();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[q0 * BN + c8 * 8 + e] = cs8[e];
    epi_barrier();
    if (q0 == 0) {
      // deterministic partial row m0/64 (zeros in the tile's other 64-row rows)
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
  GEMM_STAMP(2);
}

// ---------------------------------------------------------------- host -----
// Ring configurations (HVIT_RING selects one for A/B; 0 = the gemm.h path):
//   1: 128x128, 4 waves (2x2), 4-stage ring (128 KiB, one workgroup per CU)
//   2: 128x128, 4 waves, 2-stage ring (64 KiB, two workgroups per CU)
//   3: 256x128, 8 waves (4x2), 3-stage ring (144 KiB)
//   4: 256x256, 8 waves (2x4), 2-stage ring (128 KiB)
//   5: 128x64, 4 waves (2x2), 2-stage ring (48 KiB, three workgroups per CU)
struct RingCfg {
  int bm, bn;
};
inline RingCfg ring_cfg(int c) {
  switch (c) {
    case 3: return {256, 128};
    case 4: return {256, 256};
    case 5: return {128, 64};
    default: return {128, 128};
  }
}

template <bool KCA, bool KCB, int EK>
int launch_ring(int cfg, const LdDense<bf16_t, KCA>& la, const LdDense<bf16_t, KCB>& lb, int M, int N, int K,
                int splits, int kps, const Epi& ep, hipStream_t st) {
  const RingCfg rc = ring_cfg(cfg);
  dim3 g(M / rc.bm, N / rc.bn, splits);
  switch (cfg) {
    case 2:
      hipLaunchKernelGGL((gemm_ring_kernel<128, 128, 2, 2, 2, KCA, KCB, EK>), g, dim3(256), 0, st, la, lb, M, N, K,
                         kps, ep);
      break;
    case 3:
      hipLaunchKernelGGL((gemm_ring_kernel<256, 128, 4, 2, 3, KCA, KCB, EK>), g, dim3(512), 0, st, la, lb, M, N, K,
                         kps, ep);
      break;
    case 4:
      hipLaunchKernelGGL((gemm_ring_kernel<256, 256, 2, 4, 2, KCA, KCB, EK>), g, dim3(512), 0, st, la, lb, M, N, K,
                         kps, ep);
      break;
    case 5:
      hipLaunchKernelGGL((gemm_ring_kernel<128, 64, 2, 2, 2, KCA, KCB, EK>), g, dim3(256), 0, st, la, lb, M, N, K,
                         kps, ep);
      break;
    default:
      hipLaunchKernelGGL((gemm_ring_kernel<128, 128, 2, 2, 4, KCA, KCB, EK>), g, dim3(256), 0, st, la, lb, M, N, K,
                         kps, ep);
      break;
  }
  HVIT_LAUNCH_CHECK();
  return HVIT_OK;
}

// The ring path applies to dense bf16 operands with every tile interior:
// M % BM == N % BN == 0, K slices of whole 64-deep stages, 16-byte aligned
// operands / outputs with ld % 8 == 0, byte extents < 2^31.
template <bool KCA, bool KCB>
bool ring_ok(int cfg, const LdDense<bf16_t, KCA>& la, const LdDense<bf16_t, KCB>& lb, int M, int N, int kps,
             int K, const Epi& ep) {
  if (cfg <= 0) return false;
  const RingCfg rc = ring_cfg(cfg);
  if (M % rc.bm || N % rc.bn || kps % 64 || K % kps) return false;
  if (!la.vok || !lb.vok || !ep.vec_ok) return false;
  if ((ep.ldo & 7) || (ep.out2 && (ep.ldo2 & 7)) || (ep.aux && (ep.ldaux & 7))) return false;
  if (ep.rowadd || ep.stats || ep.rs_ptr || ep.act == ACT_TANH || ep.relu || ep.mode == EPI_SPLIT2 ||
      ep.mode == EPI_PATCH)
    return false;
  auto al = [](const void* p) { return !p || (((uintptr_t)p) & 15) == 0; };
  if (!al(ep.out) || !al(ep.out2) || !al(ep.aux) || !al(ep.resid) || !al(ep.bias)) return false;
  return dense_bytes(la) < (1L << 31) && dense_bytes(lb) < (1L << 31);
}

// the configuration the linear entry points use (-1 automatic; hvit_gemm_tune
// for in-process A/B measurements and the tests)
inline int& ring_cfg_ref() {
  static int c = -1;
  return c;
}
inline int ring_default_cfg() { return ring_cfg_ref(); }

// Automatic choice (knob -1), per operand layout and shape, from the
// in-process A/B of tools/ring_bench.py at the B=32 ViT shapes (gpurun_out /
// profiles r3): the 256x256 eight-wave tile wins where it fills the chip in
// one round (fc1 forward 39.3 -> 34.9 us, fc2 data gradient with the GELU
// backward 49.2 -> 45.2 us); weight gradients (both operands k-major) take the
// 128x128 ring at two workgroups per CU (qkv 33.8 -> 28.9 us) or the 128x64
// one for the small projections (proj 23.9 -> 18.4 us); everything else stays
// on gemm.h's kernels (the three-workgroups-per-CU one-buffer forward and the
// 128x64 tiles for N = 512 measured faster there).
inline int ring_pick(bool kca, bool kcb, int M, int N, int K) {
  if (!kca && !kcb) return (long)M * N <= 512L * 512 ? 5 : (long)M * N < 1024L * 1024 ? 2 : 0;
  if (M % 256 == 0 && N % 256 == 0 && (long)(M / 256) * (N / 256) >= 256 && K <= 1024) return 4;
  return 0;
}

// Dense bf16 GEMM through the ring kernels when they apply (returns false
// otherwise, and the caller takes gemm.h's launch_gemm).
template <bool KCA, bool KCB>
bool try_ring(const LdDense<bf16_t, KCA>& la, const LdDense<bf16_t, KCB>& lb, int M, int N, int K, int splits,
              const Epi& ep_in, hipStream_t st, int* rc_out, int cfg = -1) {
  if (cfg < 0) cfg = ring_default_cfg();
  if (cfg < 0) cfg = ring_pick(KCA, KCB, M, N, K);
  if (cfg == 0) return false;
  Epi ep = ep_in;
  if (ep.slab_stride == 0) ep.slab_stride = (long)M * ep.ldo;
  ep.xcd_remap = 1;
  auto vok = [](const void* p, long ld) { return !p || ((((uintptr_t)p) & 15) == 0 && ld % 8 == 0); };
  ep.vec_ok = N % 8 == 0 && vok(ep.out, ep.ldo) && vok(ep.out2, ep.ldo2) && vok(ep.aux, ep.ldaux) &&
              vok(ep.resid, ep.ldr);
  int kps = 0;
  splits = plan_splits<bf16_t>(K, splits, &kps);
  if (!ring_ok(cfg, la, lb, M, N, kps, K, ep)) return false;
  int ek;
  if (ep.mode == EPI_SLAB) ek = EK_SLAB;
  else if (splits > 1) return false;
  else if (ep.act == ACT_GELU_DUAL && !ep.resid) ek = EK_GELU_DUAL;
  else if (ep.act == ACT_NONE && ep.resid && ep.resid != ep.out) ek = EK_RESID;
  else if (ep.act == ACT_GELU_BWD && !ep.resid && ep.aux) ek = EK_GELU_BWD;
  else if (ep.act == ACT_NONE && !ep.resid) ek = EK_STORE;
  else return false;
  if (ek == EK_STORE && (ep.drop_thr || ep.drop_scale != 1.f)) return false;
  if ((ek == EK_GELU_DUAL || ek == EK_RESID || ek == EK_GELU_BWD) && !ep.drop_thr && ep.drop_scale != 1.f) return false;
  int rc = HVIT_OK;
  switch (ek) {
    case EK_SLAB: rc = launch_ring<KCA, KCB, EK_SLAB>(cfg, la, lb, M, N, K, splits, kps, ep, st); break;
    case EK_STORE: rc = launch_ring<KCA, KCB, EK_STORE>(cfg, la, lb, M, N, K, splits, kps, ep, st); break;
    case EK_GELU_BWD:
      if constexpr (KCA) rc = launch_ring<KCA, KCB, EK_GELU_BWD>(cfg, la, lb, M, N, K, splits, kps, ep, st);
      else return false;
      break;
    case EK_GELU_DUAL:
      if constexpr (KCA && KCB) rc = launch_ring<KCA, KCB, EK_GELU_DUAL>(cfg, la, lb, M, N, K, splits, kps, ep, st);
      else return false;
      break;
    case EK_RESID:
      if constexpr (KCA && KCB) rc = launch_ring<KCA, KCB, EK_RESID>(cfg, la, lb, M, N, K, splits, kps, ep, st);
      else return false;
      break;
    default: return false;
  }
  *rc_out = rc;
  return true;
}

}  // namespace hvit
