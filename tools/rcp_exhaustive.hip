// Exhaustive check (every float32 bit pattern with a normal, finite value and
// a normal reciprocal) that the short reciprocal sequence used on the k_vsd hot
// path -- hardware v_rcp_f32 + one Newton step with fused multiply-adds -- is
// the correctly rounded 1/x, i.e. bit-identical to the IEEE division the spec
// names. The reference is (float)(1.0 / (double)x): double rounding of a
// quotient from binary64 to binary32 is innocuous (53 >= 2 * 24 + 2).
//   hipcc --offload-arch=gfx950 -O3 tools/rcp_exhaustive.hip -o tools/rcp_exhaustive
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CHK(x) \
  do {        \
    if ((x) != hipSuccess) return 2; \
  } while (0)

__device__ __forceinline__ float rcp_fast(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}

__global__ void k_check(uint32_t hi, unsigned long long* bad, uint32_t* first,
                        unsigned long long* checked) {
  const uint32_t lo = blockIdx.x * blockDim.x + threadIdx.x;  // 2^24 per launch
  const uint32_t bits = (hi << 24) | lo;
  const float x = __uint_as_float(bits);
  const float ax = fabsf(x);
  if (!(ax >= 0x1p-126f && ax < 0x1p126f)) return;  // claim: normal x with normal 1/x
  atomicAdd(checked, 1ull);
  const float ref = (float)(1.0 / (double)x);
  const float got = rcp_fast(x);
  if (__float_as_uint(ref) != __float_as_uint(got)) {
    if (atomicAdd(bad, 1ull) == 0) *first = bits;
  }
}

int main() {
  unsigned long long *bad, *checked;
  uint32_t* first;
  CHK(hipMalloc(&bad, 8));
  CHK(hipMalloc(&checked, 8));
  CHK(hipMalloc(&first, 4));
  CHK(hipMemset(bad, 0, 8));
  CHK(hipMemset(checked, 0, 8));
  CHK(hipMemset(first, 0, 4));
  for (uint32_t hi = 0; hi < 256; ++hi) {
    hipLaunchKernelGGL(k_check, dim3(1 << 16), dim3(256), 0, 0, hi, bad, first, checked);
    CHK(hipGetLastError());
  }
  unsigned long long h_bad = 0, h_checked = 0;
  uint32_t h_first = 0;
  CHK(hipMemcpy(&h_bad, bad, 8, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(&h_checked, checked, 8, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(&h_first, first, 4, hipMemcpyDeviceToHost));
  printf("rcp_fast: %llu values checked, %llu mismatches (first 0x%08x)\n", h_checked, h_bad,
         h_first);
  return h_bad != 0 || h_checked == 0;
}
