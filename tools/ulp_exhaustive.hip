// Exhaustive accuracy of the two hardware float32 operations the certified
// VSD filter relies on (kern_vsd.hip vsd_filter_px): the largest
// distance, in units in the last place of the correctly rounded result, of
//   v_sqrt_f32 (__builtin_amdgcn_sqrtf) from (float)sqrt((double)x)   for every
//     positive normal float32 x (the filter's argument is >= 1),
//   v_rcp_f32  (__builtin_amdgcn_rcpf)  from (float)(1.0 / (double)x)  for every
//     positive normal x with a normal reciprocal.
// Both references are correctly rounded (double rounding of sqrt / quotient
// from binary64 to binary32 is innocuous: 53 >= 2 * 24 + 2). The filter's
// bound assumes <= 2 ulp for the sqrt and <= 1 ulp for the reciprocal.
//   hipcc --offload-arch=gfx950 -O3 tools/ulp_exhaustive.hip -o tools/ulp_exhaustive
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define CHK(x)                       \
  do {                               \
    if ((x) != hipSuccess) return 2; \
  } while (0)

__global__ void k_ulp(uint32_t hi, unsigned* max_sqrt, unsigned* max_rcp,
                      unsigned long long* n_sqrt, unsigned long long* n_rcp) {
  const uint32_t bits = (hi << 24) | (blockIdx.x * blockDim.x + threadIdx.x);
  const float x = __uint_as_float(bits);
  if (!(x >= 0x1p-126f && x <= 0x1.fffffep127f)) return;  // positive normal
  {
    const float ref = (float)sqrt((double)x);
    const float got = __builtin_amdgcn_sqrtf(x);
    const int d = (int)__float_as_uint(got) - (int)__float_as_uint(ref);
    atomicMax(max_sqrt, (unsigned)(d < 0 ? -d : d));
    atomicAdd(n_sqrt, 1ull);
  }
  if (x < 0x1p126f) {  // normal reciprocal
    const float ref = (float)(1.0 / (double)x);
    const float got = __builtin_amdgcn_rcpf(x);
    const int d = (int)__float_as_uint(got) - (int)__float_as_uint(ref);
    atomicMax(max_rcp, (unsigned)(d < 0 ? -d : d));
    atomicAdd(n_rcp, 1ull);
  }
}

int main() {
  unsigned *ms, *mr;
  unsigned long long *ns, *nr;
  CHK(hipMalloc(&ms, 4));
  CHK(hipMalloc(&mr, 4));
  CHK(hipMalloc(&ns, 8));
  CHK(hipMalloc(&nr, 8));
  CHK(hipMemset(ms, 0, 4));
  CHK(hipMemset(mr, 0, 4));
  CHK(hipMemset(ns, 0, 8));
  CHK(hipMemset(nr, 0, 8));
  for (uint32_t hi = 0; hi < 128; ++hi) {  // sign bit 0: positive floats
    hipLaunchKernelGGL(k_ulp, dim3(1 << 16), dim3(256), 0, 0, hi, ms, mr, ns, nr);
    CHK(hipGetLastError());
  }
  unsigned h_ms = 0, h_mr = 0;
  unsigned long long h_ns = 0, h_nr = 0;
  CHK(hipMemcpy(&h_ms, ms, 4, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(&h_mr, mr, 4, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(&h_ns, ns, 8, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(&h_nr, nr, 8, hipMemcpyDeviceToHost));
  printf("v_sqrt_f32: %llu values, max error %u ulp\n", h_ns, h_ms);
  printf("v_rcp_f32: %llu values, max error %u ulp\n", h_nr, h_mr);
  return (h_ns == 0 || h_nr == 0 || h_ms > 2 || h_mr > 1) ? 1 : 0;
}
