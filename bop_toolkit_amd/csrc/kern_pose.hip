// kern_pose.hip — gfx950 kernels for the point-based pose errors.
//
//   MSSD  pose_error.py:96-118   min_s max_v || T_e p - T_g S_s p ||
//   MSPD  pose_error.py:121-144  min_s max_v || pi(K T_e p) - pi(K T_g S_s p) ||
//   ADD   pose_error.py:147-161  mean_v || T_e p - T_g p ||
//   PROJ  pose_error.py:217-232  mean_v || pi(K T_e p) - pi(K T_g p) ||
//   ADI   pose_error.py:164-184  mean_i min_j || T_e p_j - T_g p_i ||   (exact NN)
//
// All per-vertex math is float64 (fp32 misses the 1e-4 bar).
// One launch covers every (tuple, symmetry) pair of a batch: a 256-thread
// workgroup owns one tuple; inside it, lane (k, g) = (symmetry k of the current
// pass, vertex group g) keeps its composed symmetry transform in VGPRs and
// streams the object's SoA float64 vertices (L2-resident, shared by every
// tuple of that object). The max over vertices is a per-lane running max of
// squared distances (sqrt is monotone, so one sqrt per tuple), reduced through
// LDS; min over symmetries likewise. Reductions run in a fixed order:
// results are deterministic.
#include "bopx_internal.h"

namespace bopx {

constexpr int kPoseThreads = 256;

__device__ __forceinline__ double wave_max(double v) {
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
  for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// 3x4 affine [A | b] applied to p with FMA (tolerance path, not bit-exact path).
__device__ __forceinline__ double aff(const double* A, int row, double x, double y, double z) {
  return fma(A[4 * row + 2], z, fma(A[4 * row + 1], y, fma(A[4 * row + 0], x, A[4 * row + 3])));
}

// P = K [R | t] as 3x4 row-major (misc.py:103).
__device__ __forceinline__ void proj_mat(const double* K, const double* R, const double* t,
                                         double* P) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      P[4 * i + j] = fma(K[3 * i + 2], R[6 + j], fma(K[3 * i + 1], R[3 + j], K[3 * i] * R[j]));
    P[4 * i + 3] = fma(K[3 * i + 2], t[2], fma(K[3 * i + 1], t[1], K[3 * i] * t[0]));
  }
}

template <int MODE>  // 0 = MSSD, 1 = MSPD
__global__ __launch_bounds__(kPoseThreads) void k_sym_error(const ObjDesc* __restrict__ objs,
                                                            const int32_t* __restrict__ slots,
                                                            const double* __restrict__ pe,
                                                            const double* __restrict__ pg,
                                                            const double* __restrict__ Km,
                                                            double* __restrict__ out) {
  __shared__ double s_red[kPoseThreads];
  __shared__ double s_symmax[kPoseThreads];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const ObjDesc o = objs[slots[b]];
  const int nv = o.nv, ns = o.ns;
  double E[12], G[12], K[9];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    E[i] = pe[12 * b + i];
    G[i] = pg[12 * b + i];
  }
  double Pe[12];
  if (MODE == 1) {
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = Km[9 * b + i];
    proj_mat(K, E, E + 9, Pe);
  }
  const double* __restrict__ px = o.pts;
  const double* __restrict__ py = o.pts + nv;
  const double* __restrict__ pz = o.pts + 2 * (int64_t)nv;
  double best = INFINITY;
  for (int s0 = 0; s0 < ns; s0 += kPoseThreads) {
    const int sp = min(ns - s0, kPoseThreads);
    const int ng = kPoseThreads / sp;
    const int k = tid % sp, g = tid / sp;
    double m = -INFINITY;
    if (g < ng) {
      // Compose R_gs = R_g S_R, t_gs = R_g S_t + t_g (pose_error.py:114-115).
      const double* S = o.syms + 12 * (int64_t)(s0 + k);
      double Rgs[9], tgs[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
          Rgs[3 * i + j] = fma(G[3 * i + 2], S[6 + j], fma(G[3 * i + 1], S[3 + j], G[3 * i] * S[j]));
        tgs[i] = fma(G[3 * i + 2], S[11], fma(G[3 * i + 1], S[10], fma(G[3 * i], S[9], G[9 + i])));
      }
      double A[12];
      if (MODE == 0) {
        // Difference-affine form: T_e p - T_gs p = (R_e - R_gs) p + (t_e - t_gs).
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
          for (int j = 0; j < 3; ++j) A[4 * i + j] = E[3 * i + j] - Rgs[3 * i + j];
          A[4 * i + 3] = E[9 + i] - tgs[i];
        }
        for (int v = g; v < nv; v += ng) {
          const double x = px[v], y = py[v], z = pz[v];
          const double dx = aff(A, 0, x, y, z), dy = aff(A, 1, x, y, z), dz = aff(A, 2, x, y, z);
          m = fmax(m, fma(dz, dz, fma(dy, dy, dx * dx)));
        }
      } else {
        proj_mat(K, Rgs, tgs, A);
        for (int v = g; v < nv; v += ng) {
          const double x = px[v], y = py[v], z = pz[v];
          const double ize = 1.0 / aff(Pe, 2, x, y, z);
          const double izg = 1.0 / aff(A, 2, x, y, z);
          const double du = aff(Pe, 0, x, y, z) * ize - aff(A, 0, x, y, z) * izg;
          const double dv = aff(Pe, 1, x, y, z) * ize - aff(A, 1, x, y, z) * izg;
          m = fmax(m, fma(dv, dv, du * du));
        }
      }
    }
    s_red[tid] = m;
    __syncthreads();
    if (tid < sp) {
      double mx = -INFINITY;
      for (int gg = 0; gg < ng; ++gg) mx = fmax(mx, s_red[gg * sp + tid]);
      s_symmax[tid] = mx;
    }
    __syncthreads();
    if (tid < 64) {
      double mn = INFINITY;
      for (int i = tid; i < sp; i += 64) mn = fmin(mn, s_symmax[i]);
      mn = wave_min(mn);
      best = fmin(best, mn);
    }
    __syncthreads();
  }
  if (tid == 0) out[b] = sqrt(best);
}

template <int MODE>  // 0 = ADD, 1 = PROJ
__global__ __launch_bounds__(kPoseThreads) void k_mean_error(const ObjDesc* __restrict__ objs,
                                                             const int32_t* __restrict__ slots,
                                                             const double* __restrict__ pe,
                                                             const double* __restrict__ pg,
                                                             const double* __restrict__ Km,
                                                             double* __restrict__ out) {
  __shared__ double s_part[kPoseThreads / 64];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const ObjDesc o = objs[slots[b]];
  const int nv = o.nv;
  double E[12], G[12], A[12], Pe[12], Pg[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    E[i] = pe[12 * b + i];
    G[i] = pg[12 * b + i];
  }
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) A[4 * i + j] = E[3 * i + j] - G[3 * i + j];
      A[4 * i + 3] = E[9 + i] - G[9 + i];
    }
  } else {
    double K[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = Km[9 * b + i];
    proj_mat(K, E, E + 9, Pe);
    proj_mat(K, G, G + 9, Pg);
  }
  const double* __restrict__ px = o.pts;
  const double* __restrict__ py = o.pts + nv;
  const double* __restrict__ pz = o.pts + 2 * (int64_t)nv;
  double sum = 0.0;
  for (int v = tid; v < nv; v += kPoseThreads) {
    const double x = px[v], y = py[v], z = pz[v];
    if (MODE == 0) {
      const double dx = aff(A, 0, x, y, z), dy = aff(A, 1, x, y, z), dz = aff(A, 2, x, y, z);
      sum += sqrt(fma(dz, dz, fma(dy, dy, dx * dx)));
    } else {
      const double ize = 1.0 / aff(Pe, 2, x, y, z), izg = 1.0 / aff(Pg, 2, x, y, z);
      const double du = aff(Pe, 0, x, y, z) * ize - aff(Pg, 0, x, y, z) * izg;
      const double dv = aff(Pe, 1, x, y, z) * ize - aff(Pg, 1, x, y, z) * izg;
      sum += sqrt(fma(dv, dv, du * du));
    }
  }
  sum = wave_sum(sum);
  if ((tid & 63) == 0) s_part[tid >> 6] = sum;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < kPoseThreads / 64; ++w) t += s_part[w];
    out[b] = t / (double)nv;
  }
}

// ADI: exact nearest neighbour by LDS-tiled brute force. The estimate-pose
// vertex cloud is transformed tile by tile into LDS (SoA float64); every thread
// holds kAdiQ GT-pose query vertices in registers and sweeps the tile
// (broadcast LDS reads). cKDTree returns the exact NN distance, so the result
// matches up to the float64 rounding of the transforms.
constexpr int kAdiTile = 512;
constexpr int kAdiQ = 4;

__global__ __launch_bounds__(kPoseThreads) void k_adi(const ObjDesc* __restrict__ objs,
                                                      const int32_t* __restrict__ slots,
                                                      const double* __restrict__ pe,
                                                      const double* __restrict__ pg,
                                                      double* __restrict__ out) {
  __shared__ double s_e[3][kAdiTile];
  __shared__ double s_part[kPoseThreads / 64];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const ObjDesc o = objs[slots[b]];
  const int nv = o.nv;
  double E[12], G[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    E[i] = pe[12 * b + i];
    G[i] = pg[12 * b + i];
  }
  double Ea[12], Ga[12];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      Ea[4 * i + j] = E[3 * i + j];
      Ga[4 * i + j] = G[3 * i + j];
    }
    Ea[4 * i + 3] = E[9 + i];
    Ga[4 * i + 3] = G[9 + i];
  }
  const double* __restrict__ px = o.pts;
  const double* __restrict__ py = o.pts + nv;
  const double* __restrict__ pz = o.pts + 2 * (int64_t)nv;
  double sum = 0.0;
  for (int q0 = 0; q0 < nv; q0 += kPoseThreads * kAdiQ) {
    double qx[kAdiQ], qy[kAdiQ], qz[kAdiQ], best[kAdiQ];
#pragma unroll
    for (int q = 0; q < kAdiQ; ++q) {
      const int i = q0 + q * kPoseThreads + tid;
      const int ii = i < nv ? i : nv - 1;
      const double x = px[ii], y = py[ii], z = pz[ii];
      qx[q] = aff(Ga, 0, x, y, z);
      qy[q] = aff(Ga, 1, x, y, z);
      qz[q] = aff(Ga, 2, x, y, z);
      best[q] = INFINITY;
    }
    for (int j0 = 0; j0 < nv; j0 += kAdiTile) {
      const int nj = min(kAdiTile, nv - j0);
      __syncthreads();
      for (int j = tid; j < nj; j += kPoseThreads) {
        const double x = px[j0 + j], y = py[j0 + j], z = pz[j0 + j];
        s_e[0][j] = aff(Ea, 0, x, y, z);
        s_e[1][j] = aff(Ea, 1, x, y, z);
        s_e[2][j] = aff(Ea, 2, x, y, z);
      }
      __syncthreads();
      for (int j = 0; j < nj; ++j) {
        const double ex = s_e[0][j], ey = s_e[1][j], ez = s_e[2][j];
#pragma unroll
        for (int q = 0; q < kAdiQ; ++q) {
          const double dx = ex - qx[q], dy = ey - qy[q], dz = ez - qz[q];
          best[q] = fmin(best[q], fma(dz, dz, fma(dy, dy, dx * dx)));
        }
      }
    }
#pragma unroll
    for (int q = 0; q < kAdiQ; ++q)
      if (q0 + q * kPoseThreads + tid < nv) sum += sqrt(best[q]);
  }
  sum = wave_sum(sum);
  if ((tid & 63) == 0) s_part[tid >> 6] = sum;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < kPoseThreads / 64; ++w) t += s_part[w];
    out[b] = t / (double)nv;
  }
}

hipError_t launch_sym_error(int mode, const ObjDesc* objs, int64_t n, const int32_t* slots,
                            const double* pe, const double* pg, const double* K, double* out,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  dim3 grid((unsigned)n), block(kPoseThreads);
  if (mode == 0)
    hipLaunchKernelGGL(k_sym_error<0>, grid, block, 0, s, objs, slots, pe, pg, K, out);
  else
    hipLaunchKernelGGL(k_sym_error<1>, grid, block, 0, s, objs, slots, pe, pg, K, out);
  return hipGetLastError();
}

hipError_t launch_mean_error(int mode, const ObjDesc* objs, int64_t n, const int32_t* slots,
                             const double* pe, const double* pg, const double* K, double* out,
                             hipStream_t s) {
  if (n <= 0) return hipSuccess;
  dim3 grid((unsigned)n), block(kPoseThreads);
  if (mode == 0)
    hipLaunchKernelGGL(k_mean_error<0>, grid, block, 0, s, objs, slots, pe, pg, K, out);
  else
    hipLaunchKernelGGL(k_mean_error<1>, grid, block, 0, s, objs, slots, pe, pg, K, out);
  return hipGetLastError();
}

hipError_t launch_adi(const ObjDesc* objs, int64_t n, const int32_t* slots, const double* pe,
                      const double* pg, double* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_adi, dim3((unsigned)n), dim3(kPoseThreads), 0, s, objs, slots, pe, pg,
                     out);
  return hipGetLastError();
}

}  // namespace bopx
