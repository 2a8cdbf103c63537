// Calibration of rocprofv3 FETCH_SIZE against a known byte count for the
// access widths our kernels use (MI355X_MICROARCH.md §HBM: only the 16 B/lane
// streaming read is calibrated there). Each kernel streams a 1 GiB buffer
// (well past the 256 MiB Infinity Cache) exactly once:
//   k_read4  : 4 B per lane, consecutive lanes -> consecutive dwords (k_vsd's
//              depth-frame and meshlet-triangle loads)
//   k_read16 : 16 B per lane (meshlet vertex blocks; the guide's calibrated case)
// Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_calib.hip -o /tmp/hbm_calib
//   rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_read -d DIR -o run \
//     --output-format csv -- /tmp/hbm_calib
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_read4(const unsigned* __restrict__ p, size_t n, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x9E3779B9u) out[0] = acc;  // keeps the loads alive
}

__global__ void k_read16(const uint4* __restrict__ p, size_t n, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  void* buf = nullptr;
  unsigned* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_read4, dim3(8192), dim3(256), 0, 0, (const unsigned*)buf, bytes / 4, out);
  hipLaunchKernelGGL(k_read16, dim3(8192), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, out);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("streamed %zu bytes per kernel\n", bytes);
  return 0;
}
