// Probe: issue cost of integer hash variants on gfx950 (per element, wave64),
// to price the dropout counter hash (common.h hash32 = lowbias32, two
// v_mul_lo_u32).  Build: hipcc --offload-arch=gfx950 -O3 -o hash_probe hash_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ __forceinline__ unsigned h_lowbias(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; return x ^ (x >> 16);
}
__device__ __forceinline__ unsigned h_mul24(unsigned x) {
  x ^= x >> 16; x = __umul24(x, 0x7feb35u) ^ (__umulhi(x, 0x45d9f3bu)); x ^= x >> 15; x = __umul24(x, 0x846ca6u); return x ^ (x >> 13);
}
__device__ __forceinline__ unsigned h_xs(unsigned x) {
  x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x;
}
template <int V>
__global__ void k(unsigned* out, unsigned key, int iters) {
  unsigned a = threadIdx.x + blockIdx.x * 4096u, b = a + 1, c = a + 2, d = a + 3, acc = 0;
  for (int i = 0; i < iters; ++i) {
    unsigned s = key + i * 4;
    if (V == 0) acc += h_lowbias(a ^ s) + h_lowbias(b ^ s) + h_lowbias(c ^ s) + h_lowbias(d ^ s);
    if (V == 1) acc += h_mul24(a ^ s) + h_mul24(b ^ s) + h_mul24(c ^ s) + h_mul24(d ^ s);
    if (V == 2) acc += h_xs(a ^ s) + h_xs(b ^ s) + h_xs(c ^ s) + h_xs(d ^ s);
    if (V == 3) { float f = __builtin_amdgcn_exp2f((float)(int)(a ^ s) * 1e-9f) + __builtin_amdgcn_exp2f((float)(int)(b ^ s) * 1e-9f) +
                   __builtin_amdgcn_exp2f((float)(int)(c ^ s) * 1e-9f) + __builtin_amdgcn_exp2f((float)(int)(d ^ s) * 1e-9f);
                  acc += __float_as_uint(f); }
    if (V == 4) acc += ((a ^ s) * 0x7feb352du) + ((b ^ s) * 0x7feb352du) + ((c ^ s) * 0x7feb352du) + ((d ^ s) * 0x7feb352du);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main() {
  unsigned* o; (void)hipMalloc(&o, 4u << 22);
  const char* names[] = {"lowbias32 (2 mul_lo)", "mul24 variant", "xorshift32", "exp2 + cvt (reference)", "one mul_lo + xor"};
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int iters = 4096, grid = 2048, blk = 256;
  for (int v = 0; v < 5; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0);
      switch (v) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(grid), dim3(blk), 0, 0, o, 7u, iters); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(grid), dim3(blk), 0, 0, o, 7u, iters); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(grid), dim3(blk), 0, 0, o, 7u, iters); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(grid), dim3(blk), 0, 0, o, 7u, iters); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(grid), dim3(blk), 0, 0, o, 7u, iters); break;
      }
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      const double elems = (double)grid * blk * iters * 4;
      if (rep) printf("%-26s %8.3f ms  %7.3f ps/elem  (%.2f chip-cycles@2GHz per wave-elem per SIMD)\n", names[v], ms,
                      ms * 1e9 / elems, ms * 1e-3 * 2e9 * 1024 / (elems / 64));
    }
  }
  return 0;
}
