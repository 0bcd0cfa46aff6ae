// Probe: semantics of v_cvt_scalef32_pk_fp8_bf16 (scale direction, rounding,
// saturation) on gfx950.  Build: hipcc --offload-arch=gfx950 -o cvt_probe cvt_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include <string.h>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
__global__ void k(const bf16x2* a, const float* sc, unsigned* o, int n) {
  int i = threadIdx.x;
  if (i >= n) return;
  s16x2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16((s16x2){0, 0}, a[i], sc[i], false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, a[i], sc[i] * 2.f, true);
  o[i] = __builtin_bit_cast(unsigned, r);
}
static float e4m3(unsigned b) {
  int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
  float v = e ? ldexpf(1.f + m / 8.f, e - 7) : ldexpf(m / 8.f, -6);
  if (e == 15 && m == 7) v = NAN;
  return s ? -v : v;
}
static unsigned short tobf(float f) { unsigned u; memcpy(&u, &f, 4); return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }
int main() {
  const float xs[][2] = {{1.f, 1.5f}, {3.f, -2.f}, {0.1f, 300.f}, {1000.f, 1.0625f}, {1.1875f, 0.f}, {17.f, 19.f}, {1.f, 1.f}, {5.f, 7.f}};
  const float ss[] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 4.f, 0.25f};
  const int n = 8;
  unsigned short hb[2 * n];
  for (int i = 0; i < n; ++i) { hb[2 * i] = tobf(xs[i][0]); hb[2 * i + 1] = tobf(xs[i][1]); }
  bf16x2* da; float* ds; unsigned* dout;
  hipMalloc(&da, sizeof(hb)); hipMalloc(&ds, sizeof(ss)); hipMalloc(&dout, 4 * n);
  hipMemcpy(da, hb, sizeof(hb), hipMemcpyHostToDevice);
  hipMemcpy(ds, ss, sizeof(ss), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, ds, dout, n);
  unsigned ho[n];
  hipMemcpy(ho, dout, 4 * n, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) {
    printf("x=(%g,%g) scale=%g: lo word (scale) -> %g %g ; hi word (scale*2) -> %g %g  [raw %08x]\n", xs[i][0], xs[i][1],
           ss[i], e4m3(ho[i] & 255), e4m3((ho[i] >> 8) & 255), e4m3((ho[i] >> 16) & 255), e4m3(ho[i] >> 24), ho[i]);
  }
  return 0;
}
