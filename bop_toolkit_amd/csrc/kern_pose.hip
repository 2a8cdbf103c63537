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
#include <algorithm>
#include <cstdlib>

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

// MSSD / MSPD. Work unit = (tuple b, chunk c of up to kSymChunk symmetries):
// block id = b * nch + c, so the units of a many-symmetry object (e.g. a
// discretised continuous symmetry, S = 314) are spread over the whole grid
// instead of serialising on one CU; units past the object's last chunk exit at
// once. Inside a unit, lane (k, g) = (symmetry k, vertex group g) keeps its
// composed transform in VGPRs and sweeps the vertices, staged 256 at a time in
// LDS (broadcast reads), with independent max chains. The unit's min over symmetries of the max squared
// distance is merged into out[b] with a 64-bit atomicMin on the bits of the
// non-negative double (exact and order-independent: deterministic);
// k_sym_init / k_sym_finish bracket the launch (+inf, then sqrt).
#ifndef BOPX_SYM_CHUNK
#define BOPX_SYM_CHUNK 64
#endif
constexpr int kSymChunk = BOPX_SYM_CHUNK;  // <= 64: a unit's symmetries fit wave 0
// Vertices staged in LDS per round of the exhaustive path (two barriers each).
// Round 4: single-symmetry units no longer stage (direct sweep), so the
// exhaustive path only runs with pruning off or for sets > kPruneSpan, and the
// staging's LDS mostly limited residency: MSSD 1,024 -> 256 is 30.5 -> 12 KB of
// LDS, 5 -> 7 resident blocks per CU, -4 % (profiles/r04/ab_sym2.txt). MSPD
// stages 5 values per vertex and was already at 256.
#ifndef BOPX_SYM_STAGE_MSSD
#define BOPX_SYM_STAGE_MSSD 256
#endif
#ifndef BOPX_SYM_STAGE_MSPD
#define BOPX_SYM_STAGE_MSPD 256
#endif
template <int MODE>
constexpr int kSymStage = MODE ? BOPX_SYM_STAGE_MSPD : BOPX_SYM_STAGE_MSSD;
static_assert(kSymStage<0> % kPoseThreads == 0 && kSymStage<1> % kPoseThreads == 0,
              "whole staging passes");

__global__ void k_sym_init(double* __restrict__ out, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] = INFINITY;
}
__global__ void k_sym_finish(double* __restrict__ out, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] = sqrt(out[i]);
}

// 1/x for the tolerance path: hardware reciprocal (v_rcp_f64) refined by one
// Newton step (relative error squared: ~1 ulp); tests bound MSPD/PROJ at 1e-9
// relative to the reference.
__device__ __forceinline__ double rcp64(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}

// Compose R_gs = R_g S_R, t_gs = R_g S_t + t_g (pose_error.py:114-115).
__device__ __forceinline__ void sym_compose(const double* G, const double* S, double* Rgs,
                                            double* tgs) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      Rgs[3 * i + j] = fma(G[3 * i + 2], S[6 + j], fma(G[3 * i + 1], S[3 + j], G[3 * i] * S[j]));
    tgs[i] = fma(G[3 * i + 2], S[11], fma(G[3 * i + 1], S[10], fma(G[3 * i], S[9], G[9 + i])));
  }
}

// Per-symmetry 3x4 matrix of the error: MSSD the difference-affine form
// T_e p - T_gs p = (R_e - R_gs) p + (t_e - t_gs); MSPD the projection K [R_gs | t_gs].
template <int MODE>
__device__ __forceinline__ void sym_matrix(const double* E, const double* K, const double* G,
                                           const double* S, double* A) {
  double Rgs[9], tgs[3];
  sym_compose(G, S, Rgs, tgs);
  if constexpr (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) A[4 * i + j] = E[3 * i + j] - Rgs[3 * i + j];
      A[4 * i + 3] = E[9 + i] - tgs[i];
    }
  } else {
    proj_mat(K, Rgs, tgs, A);
  }
}

// Squared error of one vertex under one symmetry (the same expressions in the
// exhaustive and the pruned sweep, so both give the same bits). MSPD: (ue, ve)
// is the vertex's projection under the estimate (est_proj).
__device__ __forceinline__ double d2_mssd(const double* A, double x, double y, double z) {
  const double dx = aff(A, 0, x, y, z), dy = aff(A, 1, x, y, z), dz = aff(A, 2, x, y, z);
  return fma(dz, dz, fma(dy, dy, dx * dx));
}
__device__ __forceinline__ double d2_mspd(const double* A, double x, double y, double z, double ue,
                                          double ve) {
  const double izg = rcp64(aff(A, 2, x, y, z));
  const double du = fma(-aff(A, 0, x, y, z), izg, ue);
  const double dv = fma(-aff(A, 1, x, y, z), izg, ve);
  return fma(dv, dv, du * du);
}
__device__ __forceinline__ void est_proj(const double* Pe, double x, double y, double z,
                                         double& ue, double& ve) {
  const double ize = rcp64(aff(Pe, 2, x, y, z));
  ue = aff(Pe, 0, x, y, z) * ize;
  ve = aff(Pe, 1, x, y, z) * ize;
}

// Symmetry pruning (units with >= prune_min symmetries). min_s max_v d2(s, v)
// does not need every max: a symmetry whose max over ANY subset of the vertices
// already exceeds the max of a fully swept symmetry cannot be the minimum. The
// unit (1) bounds every symmetry from below by its max over the object's seed
// vertices (farthest-point samples, runtime.cpp seed_vertices), (2) sweeps the
// lowest-bound symmetry over all vertices with the whole workgroup, then
// (3) lets each wave take the next symmetries in ascending bound order and drop
// one as soon as a partial max exceeds the best completed max (or stop once a
// bound does). The best so far is shared by the unit (LDS) and across the
// chunks of a tuple (the output word, read at the start). Every symmetry that
// can be the minimum is swept in full with the same d2 expressions as the
// exhaustive path and max is exact, so the result is bit-identical to it
// (tests/test_gpu_parity.py compares both).
#ifndef BOPX_SYM_PRUNE_MIN
#define BOPX_SYM_PRUNE_MIN 2
#endif
#ifndef BOPX_SYM_SEEDS
#define BOPX_SYM_SEEDS 128  // seed vertices used of the object's kSymSeeds
#endif
constexpr int kPruneSpan = 320;  // symmetry sets up to this size are pruned by one unit
// vertices per thread and step of the whole-workgroup sweep (step 2; 8 measured
// slower than 4, profiles/r04/ab_sym.txt)
#ifndef BOPX_SYM_SWEEP_U
#define BOPX_SYM_SWEEP_U 4
#endif
constexpr int kSweepU = BOPX_SYM_SWEEP_U;
static_assert(kSweepU % 2 == 0, "pairs of maxima");

// A wave-uniform double computed by VALU, moved to SGPRs (readfirstlane of
// both halves): the sweeps' per-tuple / per-candidate matrices then take no
// VGPRs (VALU reads one SGPR pair per instruction).
__device__ __forceinline__ double uniform_d(double v) {
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                          __builtin_amdgcn_readfirstlane(__double2loint(v)));
}
template <int N>
__device__ __forceinline__ void uniform_n(double* a) {
#pragma unroll
  for (int i = 0; i < N; ++i) a[i] = uniform_d(a[i]);
}

// Make LDS written by other lanes of this wave visible (LDS is in order per wave).
__device__ __forceinline__ void wave_lds_sync_pose() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (round 4: forcing MSPD to 6 waves per SIMD, 77 VGPRs, was 26 % slower than
// the free allocation's 89 / 5 waves; MSSD at 8 waves 22 % slower,
// profiles/r04/ab_sym2.txt)
template <int MODE>  // 0 = MSSD, 1 = MSPD
__global__ __launch_bounds__(kPoseThreads) void k_sym_error(const ObjDesc* __restrict__ objs,
                                                            const int32_t* __restrict__ slots,
                                                            const double* __restrict__ pe,
                                                            const double* __restrict__ pg,
                                                            const double* __restrict__ Km,
                                                            double* __restrict__ out, int nch,
                                                            const int32_t* __restrict__ order,
                                                            int prune_min) {
  __shared__ double s_red[kPoseThreads];
  // A block of kSymStage vertices staged for every symmetry of the unit: x, y, z
  // and, for MSPD, the estimate's projection u_e, v_e.
  __shared__ double s_v[MODE ? 5 : 3][kSymStage<MODE>];
  const int64_t b = order ? (int64_t)order[blockIdx.x / nch] : (int64_t)(blockIdx.x / nch);
  const int c = blockIdx.x % nch;
  const int tid = threadIdx.x;
  const ObjDesc o = objs[slots[b]];
  const int nv = o.nv, ns = o.ns, s0 = c * kSymChunk;
  if (s0 >= ns) return;
  const int sp = min(ns - s0, kSymChunk);
  const int ng = kPoseThreads / sp;
  const int k = tid % sp, g = tid / sp;
  double G[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) G[i] = pg[12 * b + i];
  const gptr<const double> px = (gptr<const double>)o.pts;
  const gptr<const double> py = px + nv;
  const gptr<const double> pz = py + nv;
  // A tuple's whole symmetry set (<= kPruneSpan) is pruned by one unit (chunk
  // 0; the tuple's other chunks exit), larger sets chunk by chunk.
  const bool whole = ns <= kPruneSpan;
  const int span = whole ? ns : sp;
  // A single symmetry needs no bounds: the unit is the full sweep of step (2)
  // alone (round 4; no LDS staging rounds and barriers: the same d2 per vertex
  // and an exact max, so the same double as the exhaustive path).
  const bool single = ns == 1;
  if (span >= prune_min || single) {
    if (whole && c != 0) return;
    static_assert(kSymSeeds <= kPoseThreads && kSymSeeds <= kSymStage<MODE>, "seed staging");
    __shared__ double s_L[kPruneSpan];    // per-symmetry lower bound (max over the seeds)
    __shared__ int s_cand[kPruneSpan];    // symmetries left to sweep
    __shared__ unsigned long long s_best;  // best completed max (bits of a non-negative double)
    __shared__ int s_next, s_ncand, s_k0;
    const int sb = whole ? 0 : s0;  // the unit's first symmetry
    const double* syms = o.syms + 12 * (int64_t)sb;
    const int lane = tid & 63, wave = tid >> 6;
    double E[12], K[9], Pe[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) E[i] = pe[12 * b + i];
    if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 9; ++i) K[i] = Km[9 * b + i];
      proj_mat(K, E, E + 9, Pe);
      uniform_n<12>(Pe);  // per-tuple matrices in SGPRs (MSPD 125 -> 89 VGPRs)
    }
    auto d2v = [&](const double* A, int v) {  // vertex v from global memory
      const double x = px[v], y = py[v], z = pz[v];
      if constexpr (MODE == 0) {
        return d2_mssd(A, x, y, z);
      } else {
        double ue, ve;
        est_proj(Pe, x, y, z, ue, ve);
        return d2_mspd(A, x, y, z, ue, ve);
      }
    };
    auto best_now = [&]() {
      return __longlong_as_double((long long)__hip_atomic_load(&s_best, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP));
    };
    auto publish = [&](double M) {
      const unsigned long long bits = (unsigned long long)__double_as_longlong(M);
      atomicMin(&s_best, bits);
      atomicMin((unsigned long long*)&out[b], bits);
    };
    // (1) bounds over the seed vertices, 64 symmetries at a time, lane (k, g) =
    // (symmetry, seed group)
    const int np = min(o.nseed, BOPX_SYM_SEEDS);
    if (!single && tid < np) {
      const gptr<const double> sd = (gptr<const double>)o.seed;
      const int ns_all = o.nseed;  // SoA stride
      const double x = sd[tid], y = sd[ns_all + tid], z = sd[2 * ns_all + tid];
      s_v[0][tid] = x;
      s_v[1][tid] = y;
      s_v[2][tid] = z;
      if constexpr (MODE == 1) est_proj(Pe, x, y, z, s_v[3][tid], s_v[4][tid]);
    }
    if (tid == 0) {
      // another chunk's result (chunked sets), else +inf
      s_best = __hip_atomic_load((unsigned long long*)&out[b], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      s_next = 0;
      s_ncand = 0;
    }
    __syncthreads();
    for (int kb = 0; kb < (single ? 0 : span); kb += 64) {
      const int bp = min(span - kb, 64), bng = kPoseThreads / bp;
      const int bk = tid % bp, bg = tid / bp;
      double m = -INFINITY;
      if (bg < bng) {
        double A[12];
        sym_matrix<MODE>(E, K, G, syms + 12 * (int64_t)(kb + bk), A);
        for (int j = bg; j < np; j += bng)
          m = fmax(m, MODE == 0 ? d2_mssd(A, s_v[0][j], s_v[1][j], s_v[2][j])
                                : d2_mspd(A, s_v[0][j], s_v[1][j], s_v[2][j], s_v[3][j], s_v[4][j]));
      }
      s_red[tid] = m;
      __syncthreads();
      if (tid < bp) {
        double L = -INFINITY;
        for (int gg = 0; gg < bng; ++gg) L = fmax(L, s_red[gg * bp + tid]);
        s_L[kb + tid] = L;
      }
      __syncthreads();
    }
    // argmin of (bound, index): per thread, then per wave, then over the waves
    if (!single) {
      double L = INFINITY;
      int kk = 0x7FFFFFFF;
      for (int i = tid; i < span; i += kPoseThreads)
        if (s_L[i] < L) {
          L = s_L[i];
          kk = i;
        }
      for (int off = 32; off > 0; off >>= 1) {
        const double oL = __shfl_xor(L, off, 64);
        const int ok = __shfl_xor(kk, off, 64);
        if (oL < L || (oL == L && ok < kk)) {
          L = oL;
          kk = ok;
        }
      }
      if (lane == 0) {
        s_red[wave] = L;
        s_cand[wave] = kk;
      }
      __syncthreads();
      if (tid == 0) {
        double bL = s_red[0];
        int bk = s_cand[0];
        for (int w = 1; w < kPoseThreads / 64; ++w)
          if (s_red[w] < bL || (s_red[w] == bL && s_cand[w] < bk)) {
            bL = s_red[w];
            bk = s_cand[w];
          }
        s_k0 = bk;
      }
      __syncthreads();
    }
    const int k0 = single ? 0 : s_k0;
    if (!single && !(s_L[k0] <= best_now())) return;  // no symmetry of the unit can win
    // (2) the lowest bound, swept by the whole workgroup
    {
      double A[12];
      sym_matrix<MODE>(E, K, G, syms + 12 * (int64_t)k0, A);
      uniform_n<12>(A);
      double m = -INFINITY;
      // kSweepU vertices per thread and step, all their loads in flight
      for (int v0 = 0; v0 < nv; v0 += kSweepU * kPoseThreads) {
        double d[kSweepU];
#pragma unroll
        for (int u = 0; u < kSweepU; ++u) d[u] = d2v(A, min(v0 + u * kPoseThreads + tid, nv - 1));
#pragma unroll
        for (int u = 0; u < kSweepU; u += 2) m = fmax(m, fmax(d[u], d[u + 1]));
      }
      m = wave_max(m);
      if (lane == 0) s_red[wave] = m;
      __syncthreads();
      if (tid == 0) publish(fmax(fmax(s_red[0], s_red[1]), fmax(s_red[2], s_red[3])));
      if (single) return;
      __syncthreads();
    }
    // candidates: the other symmetries whose bound does not exceed the best max
    {
      const double best = best_now();
      for (int i0 = 0; i0 < span; i0 += kPoseThreads) {
        const int i = i0 + tid;
        const bool cand = i < span && i != k0 && s_L[i] <= best;
        const uint64_t bal = __builtin_amdgcn_ballot_w64(cand);
        int base = 0;
        if (lane == 0 && bal) base = atomicAdd(&s_ncand, __popcll(bal));
        base = __builtin_amdgcn_readfirstlane(base);
        if (cand)
          s_cand[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = i;
      }
      __syncthreads();
      // short lists in ascending bound order (wave 0), so that the best
      // candidates tighten the bound first
      const int nc = s_ncand;
      if (nc <= 64 && wave == 0) {
        const int kk = lane < nc ? s_cand[lane] : 0x7FFFFFFF;
        const double L = lane < nc ? s_L[kk] : INFINITY;
        int r = 0;
        for (int j = 0; j < 64; ++j) {
          const double Lj = __shfl(L, j, 64);
          const int kj = __shfl(kk, j, 64);
          r += (Lj < L) || (Lj == L && kj < kk);
        }
        wave_lds_sync_pose();
        if (lane < nc) s_cand[r] = kk;
      }
      __syncthreads();
    }
    // (3) the candidates, one wave each. Single-exit loops with wave-uniform
    // conditions (SGPR claims and ballots).
    const int nc = s_ncand;
    auto claim = [&]() {
      int i = 0;
      if (lane == 0) i = atomicAdd(&s_next, 1);
      return __builtin_amdgcn_readfirstlane(i);
    };
    int idx = claim();
    while (idx < nc) {
      const int kk = __builtin_amdgcn_readfirstlane(s_cand[idx]);
      double best = best_now();
      if (s_L[kk] <= best) {  // (else: the bound has passed the best by now)
        double A[12];
        sym_matrix<MODE>(E, K, G, syms + 12 * (int64_t)kk, A);
        uniform_n<12>(A);
        double m = -INFINITY;
        uint64_t dead = 0;  // a lane's partial max exceeds a completed symmetry's max
        for (int v0 = 0; v0 < nv && dead == 0; v0 += 256) {
          double d[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) d[u] = d2v(A, min(v0 + 64 * u + lane, nv - 1));
          m = fmax(m, fmax(fmax(d[0], d[1]), fmax(d[2], d[3])));
          dead = __builtin_amdgcn_ballot_w64(m > best);
          best = best_now();
        }
        if (dead == 0) {
          m = wave_max(m);
          if (lane == 0) publish(m);
        }
      }
      idx = claim();
    }
    return;
  }
  // Exhaustive path: lane (k, g) = (symmetry, vertex group).
  const double* S = o.syms + 12 * (int64_t)(s0 + k);
  double m0 = -INFINITY, m1 = -INFINITY, m2 = -INFINITY, m3 = -INFINITY;
  if constexpr (MODE == 0) {
    double E[12], A[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) E[i] = pe[12 * b + i];
    sym_matrix<0>(E, nullptr, G, S, A);
    auto d2 = [&](int j) { return d2_mssd(A, s_v[0][j], s_v[1][j], s_v[2][j]); };
    for (int v0 = 0; v0 < nv; v0 += kSymStage<MODE>) {
      const int nb = min(kSymStage<MODE>, nv - v0);
      __syncthreads();
#pragma unroll
      for (int i = tid; i < kSymStage<MODE>; i += kPoseThreads)
        if (i < nb) {
          s_v[0][i] = px[v0 + i];
          s_v[1][i] = py[v0 + i];
          s_v[2][i] = pz[v0 + i];
        }
      __syncthreads();
      if (g < ng) {
        int j = g;
        // A max tree over fresh arithmetic results: only the loop-carried m0
        // needs the IEEE-mode canonicalisation before v_max_f64 (once per 4).
        for (; j + 3 * ng < nb; j += 4 * ng)
          m0 = fmax(m0, fmax(fmax(d2(j), d2(j + ng)), fmax(d2(j + 2 * ng), d2(j + 3 * ng))));
        for (; j < nb; j += ng) m1 = fmax(m1, d2(j));
      }
    }
  } else {
    double K[9], E[12], Pe[12], A[12];
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = Km[9 * b + i];
#pragma unroll
    for (int i = 0; i < 12; ++i) E[i] = pe[12 * b + i];
    proj_mat(K, E, E + 9, Pe);
    sym_matrix<1>(E, K, G, S, A);
    auto d2 = [&](int j) {
      return d2_mspd(A, s_v[0][j], s_v[1][j], s_v[2][j], s_v[3][j], s_v[4][j]);
    };
    for (int v0 = 0; v0 < nv; v0 += kSymStage<MODE>) {
      const int nb = min(kSymStage<MODE>, nv - v0);
      __syncthreads();
#pragma unroll
      for (int i = tid; i < kSymStage<MODE>; i += kPoseThreads)
        if (i < nb) {
          const double x = px[v0 + i], y = py[v0 + i], z = pz[v0 + i];
          s_v[0][i] = x;
          s_v[1][i] = y;
          s_v[2][i] = z;
          est_proj(Pe, x, y, z, s_v[3][i], s_v[4][i]);
        }
      __syncthreads();
      if (g < ng) {
        int j = g;
        for (; j + ng < nb; j += 2 * ng) m0 = fmax(m0, fmax(d2(j), d2(j + ng)));
        if (j < nb) m2 = fmax(m2, d2(j));
      }
    }
  }
  s_red[tid] = fmax(fmax(m0, m1), fmax(m2, m3));
  __syncthreads();
  if (tid < 64) {  // sp <= 64: the unit's symmetries live in wave 0
    double mn = INFINITY;
    if (tid < sp) {
      double mx = -INFINITY;
      for (int gg = 0; gg < ng; ++gg) mx = fmax(mx, s_red[gg * sp + tid]);
      mn = mx;
    }
    mn = wave_min(mn);
    if (tid == 0)
      atomicMin((unsigned long long*)&out[b], (unsigned long long)__double_as_longlong(mn));
  }
}

template <int MODE>  // 0 = ADD, 1 = PROJ
__global__ __launch_bounds__(kPoseThreads) void k_mean_error(const ObjDesc* __restrict__ objs,
                                                             const int32_t* __restrict__ slots,
                                                             const double* __restrict__ pe,
                                                             const double* __restrict__ pg,
                                                             const double* __restrict__ Km,
                                                             double* __restrict__ out,
                                                             const int32_t* __restrict__ order) {
  __shared__ double s_part[kPoseThreads / 64];
  const int64_t b = order ? (int64_t)order[blockIdx.x] : (int64_t)blockIdx.x;
  const int tid = threadIdx.x;
  const ObjDesc o = objs[slots[b]];
  const int nv = o.nv;
  double E[12], G[12], A[12], Pe[12], Pg[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    E[i] = pe[12 * b + i];
    G[i] = pg[12 * b + i];
  }
  if constexpr (MODE == 0) {
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
//
// Small batches (fewer tuples than the chip has workgroup slots) split each
// tuple's estimate cloud into point ranges, one workgroup per (tuple, range):
// every range's per-query minimum squared distance is merged with a 64-bit
// atomicMin on the non-negative double bits (exact, order-independent), and
// k_adi_finish forms the mean. Both paths sum the NN distances in the same
// fixed structure (adi_chunk_sum per 1,024-query chunk, chunks in order), so
// a tuple's ADI is the same double whatever the split.
constexpr int kAdiTile = 512;
constexpr int kAdiQ = 4;
constexpr int kAdiChunk = kPoseThreads * kAdiQ;  // queries per sweep

// Sum of one chunk's NN distances: per thread its kAdiQ queries in order, the
// wave's lanes by the xor butterfly, the waves in order. Same value in every
// thread. s_part: kPoseThreads / 64 doubles.
__device__ __forceinline__ double adi_chunk_sum(const double (&best)[kAdiQ], int q0, int nv,
                                                double* s_part) {
  const int tid = threadIdx.x;
  double v = 0.0;
#pragma unroll
  for (int q = 0; q < kAdiQ; ++q)
    if (q0 + q * kPoseThreads + tid < nv) v += sqrt(best[q]);
  v = wave_sum(v);
  __syncthreads();  // previous chunk's readers are done with s_part
  if ((tid & 63) == 0) s_part[tid >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kPoseThreads / 64; ++w) t += s_part[w];
  return t;
}

// SPLIT = false: one workgroup per tuple, writes out[b].
// SPLIT = true: workgroup (tuple, part) sweeps estimate points of range `part`
// of nsplit and merges per-query minima into best2[b * stride + i].
template <bool SPLIT>
__global__ __launch_bounds__(kPoseThreads) void k_adi(const ObjDesc* __restrict__ objs,
                                                      const int32_t* __restrict__ slots,
                                                      const double* __restrict__ pe,
                                                      const double* __restrict__ pg,
                                                      double* __restrict__ out,
                                                      const int32_t* __restrict__ order,
                                                      int nsplit, int64_t stride,
                                                      double* __restrict__ best2, int nq) {
  __shared__ double s_e[3][kAdiTile];
  __shared__ double s_part[kPoseThreads / 64];
  // SPLIT: workgroup (tuple u, estimate-point range part, query chunk class qc);
  // query chunks qc, qc + nq, ... (nq > 1 only for batches too small to fill
  // the chip with point ranges alone)
  const int64_t cell = SPLIT ? (int64_t)blockIdx.x / nq : (int64_t)blockIdx.x;
  const int qc = SPLIT ? (int)((int64_t)blockIdx.x - cell * nq) : 0;
  const int64_t u = SPLIT ? cell / nsplit : (int64_t)blockIdx.x;
  const int part = SPLIT ? (int)(cell % nsplit) : 0;
  const int64_t b = order ? (int64_t)order[u] : u;
  const int tid = threadIdx.x;
  const ObjDesc o = objs[slots[b]];
  const int nv = o.nv;
  // this workgroup's estimate points [js, je)
  const int per = SPLIT ? (nv + nsplit - 1) / nsplit : nv;
  const int js = SPLIT ? min(nv, part * per) : 0;
  const int je = SPLIT ? min(nv, js + per) : nv;
  if (SPLIT && js >= je) return;  // workgroup-uniform
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
  double total = 0.0;
  for (int q0 = qc * kAdiChunk; q0 < nv; q0 += (SPLIT ? nq : 1) * kAdiChunk) {
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
    for (int j0 = js; j0 < je; j0 += kAdiTile) {
      const int nj = min(kAdiTile, je - j0);
      __syncthreads();
      for (int j = tid; j < nj; j += kPoseThreads) {
        const double x = px[j0 + j], y = py[j0 + j], z = pz[j0 + j];
        s_e[0][j] = aff(Ea, 0, x, y, z);
        s_e[1][j] = aff(Ea, 1, x, y, z);
        s_e[2][j] = aff(Ea, 2, x, y, z);
      }
      __syncthreads();
      auto d2 = [&](int j, int q) {
        const double dx = s_e[0][j] - qx[q], dy = s_e[1][j] - qy[q], dz = s_e[2][j] - qz[q];
        return fma(dz, dz, fma(dy, dy, dx * dx));
      };
      // pairs: one IEEE canonicalisation of the loop-carried minimum per two points
      int j = 0;
      for (; j + 1 < nj; j += 2) {
#pragma unroll
        for (int q = 0; q < kAdiQ; ++q) best[q] = fmin(best[q], fmin(d2(j, q), d2(j + 1, q)));
      }
      if (j < nj) {
#pragma unroll
        for (int q = 0; q < kAdiQ; ++q) best[q] = fmin(best[q], d2(j, q));
      }
    }
    if constexpr (SPLIT) {
      // fmin never yields NaN here and d2 >= +0, so the bits order like the values
#pragma unroll
      for (int q = 0; q < kAdiQ; ++q) {
        const int i = q0 + q * kPoseThreads + tid;
        if (i < nv)
          atomicMin((unsigned long long*)&best2[b * stride + i],
                    (unsigned long long)__double_as_longlong(best[q]));
      }
    } else {
      total += adi_chunk_sum(best, q0, nv, s_part);
    }
  }
  if (!SPLIT && tid == 0) out[b] = total / (double)nv;
}

__global__ __launch_bounds__(kPoseThreads) void k_adi_finish(const ObjDesc* __restrict__ objs,
                                                             const int32_t* __restrict__ slots,
                                                             int64_t stride,
                                                             const double* __restrict__ best2,
                                                             double* __restrict__ out) {
  __shared__ double s_part[kPoseThreads / 64];
  const int64_t b = blockIdx.x;
  const int nv = objs[slots[b]].nv;
  double total = 0.0;
  for (int q0 = 0; q0 < nv; q0 += kAdiChunk) {
    double best[kAdiQ];
#pragma unroll
    for (int q = 0; q < kAdiQ; ++q) {
      const int i = q0 + q * kPoseThreads + threadIdx.x;
      best[q] = i < nv ? best2[b * stride + i] : 0.0;
    }
    total += adi_chunk_sum(best, q0, nv, s_part);
  }
  if (threadIdx.x == 0) out[b] = total / (double)nv;
}

hipError_t launch_sym_error(int mode, const ObjDesc* objs, int max_ns, int64_t n,
                            const int32_t* slots, const double* pe, const double* pg,
                            const double* K, double* out, const int32_t* order,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // BOPX_SYM_PRUNE: units with at least this many symmetries take the pruned
  // path (<= 0: never, every set sweeps exhaustively chunk by chunk, including
  // the whole-set units of up to kPruneSpan; identical results either way)
  const char* pe_env = getenv("BOPX_SYM_PRUNE");  // read per call (tests compare both paths)
  const int prune_env = pe_env ? atoi(pe_env) : BOPX_SYM_PRUNE_MIN;
  const int prune_min = prune_env > 0 ? prune_env : 0x7FFFFFFF;
  // chunks per tuple: sets of up to kPruneSpan symmetries that are pruned run
  // as one unit, so only the exhaustive sets (< prune_min) and the larger ones
  // need more (round 4: the S = 314 object had made every tuple launch 5
  // blocks, 4 of which exited at once)
  const int need = max_ns <= kPruneSpan ? min(max_ns, prune_min - 1) : max_ns;
  const int nch = (max(need, 1) + kSymChunk - 1) / kSymChunk;
  if ((int64_t)nch * n > 0x7FFFFFFF) return hipErrorInvalidValue;
  const dim3 gfix((unsigned)((n + 255) / 256)), bfix(256);
  hipLaunchKernelGGL(k_sym_init, gfix, bfix, 0, s, out, n);
  dim3 grid((unsigned)(n * nch)), block(kPoseThreads);
  if (mode == 0)
    hipLaunchKernelGGL(k_sym_error<0>, grid, block, 0, s, objs, slots, pe, pg, K, out, nch,
                       order, prune_min);
  else
    hipLaunchKernelGGL(k_sym_error<1>, grid, block, 0, s, objs, slots, pe, pg, K, out, nch,
                       order, prune_min);
  hipLaunchKernelGGL(k_sym_finish, gfix, bfix, 0, s, out, n);
  return hipGetLastError();
}

hipError_t launch_mean_error(int mode, const ObjDesc* objs, int64_t n, const int32_t* slots,
                             const double* pe, const double* pg, const double* K, double* out,
                             const int32_t* order, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  dim3 grid((unsigned)n), block(kPoseThreads);
  if (mode == 0)
    hipLaunchKernelGGL(k_mean_error<0>, grid, block, 0, s, objs, slots, pe, pg, K, out, order);
  else
    hipLaunchKernelGGL(k_mean_error<1>, grid, block, 0, s, objs, slots, pe, pg, K, out, order);
  return hipGetLastError();
}

hipError_t launch_adi(const ObjDesc* objs, int max_nv, int64_t n, const int32_t* slots,
                      const double* pe, const double* pg, double* out, const int32_t* order,
                      hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // BOPX_ADI_SPLIT: ranges per tuple (0 / unset = automatic; tests force values)
  const char* env = getenv("BOPX_ADI_SPLIT");
  int nsplit = env ? atoi(env) : 0;
  if (nsplit <= 0) {
    // fill ~kAdiWorkgroups workgroups, ranges of >= kAdiMinRange points
    constexpr int64_t kAdiWorkgroups = 2048, kAdiMinRange = 128;
    nsplit = (int)std::min<int64_t>((kAdiWorkgroups + n - 1) / n,
                                    (max_nv + kAdiMinRange - 1) / kAdiMinRange);
  }
  nsplit = std::max(1, std::min(nsplit, std::max(max_nv, 1)));
  // query-chunk classes per range (BOPX_ADI_QSPLIT forces): up to the query
  // chunks of the largest object, until ~kAdiQWorkgroups workgroups
  const char* qenv = getenv("BOPX_ADI_QSPLIT");
  int nq = qenv ? atoi(qenv) : 0;
  const int64_t chunks = std::max<int64_t>(1, (max_nv + kAdiChunk - 1) / kAdiChunk);
  if (nq <= 0) {
    constexpr int64_t kAdiQWorkgroups = 1024;
    nq = (int)std::min<int64_t>(chunks, (kAdiQWorkgroups + n * nsplit - 1) / (n * nsplit));
  }
  nq = (int)std::max<int64_t>(1, std::min<int64_t>(nq, chunks));
  // the per-query scratch is n x max_nv doubles: only for small batches
  const int64_t stride = max_nv;
  if (nsplit * (int64_t)nq > 1 &&
      (n * nsplit * nq > 0x7FFFFFFF || n * stride > ((int64_t)1 << 26)))
    nsplit = nq = 1;
  if (nsplit == 1 && nq == 1) {  // (a query split alone still takes the SPLIT path)
    hipLaunchKernelGGL(k_adi<false>, dim3((unsigned)n), dim3(kPoseThreads), 0, s, objs, slots,
                       pe, pg, out, order, 1, (int64_t)0, (double*)nullptr, 1);
    return hipGetLastError();
  }
  double* best2 = nullptr;
  hipError_t e = hipMallocAsync((void**)&best2, (size_t)(n * stride) * sizeof(double), s);
  if (e != hipSuccess) {  // no room for the scratch: one workgroup per tuple (same result)
    (void)hipGetLastError();
    hipLaunchKernelGGL(k_adi<false>, dim3((unsigned)n), dim3(kPoseThreads), 0, s, objs, slots,
                       pe, pg, out, order, 1, (int64_t)0, (double*)nullptr, 1);
    return hipGetLastError();
  }
  // 0xFF bytes: above the bits of every non-negative double (the +inf start)
  e = hipMemsetAsync(best2, 0xFF, (size_t)(n * stride) * sizeof(double), s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_adi<true>, dim3((unsigned)(n * nsplit * nq)), dim3(kPoseThreads), 0, s,
                       objs, slots, pe, pg, out, order, nsplit, stride, best2, nq);
    hipLaunchKernelGGL(k_adi_finish, dim3((unsigned)n), dim3(kPoseThreads), 0, s, objs, slots,
                       stride, (const double*)best2, out);
    e = hipGetLastError();
  }
  const hipError_t f = hipFreeAsync(best2, s);
  return e != hipSuccess ? e : f;
}

// ---------------------------------------------------------------------------
// Object-grouped launch order: order[k] = the tuple the k-th workgroup takes,
// tuples grouped by slot (counting sort, one workgroup; slots outside [0, ns)
// go last). Workgroups are dispatched in blockIdx order, so the resident ones
// then work on one or two objects at a time and re-read the same meshlet and
// vertex blocks from L2 instead of streaming every object's through it. The
// order within an object is whatever the atomics give: every tuple writes only
// its own outputs, so results do not depend on it.
constexpr int kOrderThreads = 1024;

// Sort key of tuple i: its object slot, or, with VSD cost inputs, (cost class
// descending, slot): the class is 2 log2 (half octaves) of the projected bounding-sphere
// area (diameter * f / z)^2 in px^2 at the nearer of the two poses, so the
// expensive tuples start first (LPT over the workgroup slots; a big tuple
// starting last would set the launch's tail) while tuples of one object stay
// adjacent within a class (meshlet data hot in L2).
__device__ __forceinline__ int order_key(const int32_t* __restrict__ slots, int64_t i, int ns,
                                         const OrderCost& oc) {
  const int sl = (unsigned)slots[i] < (unsigned)ns ? slots[i] : ns;
  if (!oc.pe) return oc.slot_rank && sl < ns ? oc.slot_rank[sl] : sl;
  const double z = fmin(oc.pe[12 * i + 11], oc.pg[12 * i + 11]);
  const int64_t fi = oc.frame_idx[i];
  const double f = fmax(oc.cam[4 * fi], oc.cam[4 * fi + 1]);
  const double r = oc.dia[i] * f / z;
  const double area = r * r;
  int cls = kOrderCostClasses - 1;  // behind the camera / non-finite: most expensive
  if (z > 0.0 && area == area && area < 1e18) {
    // half-octave classes: 2 floor(log2 a) + (a >= sqrt(2) 2^floor(log2 a))
    const unsigned ai = (unsigned)fmin(fmax(area, 1.0), 2147483647.0);
    const int e = 31 - __clz(ai);
    cls = min(kOrderCostClasses - 1, 2 * e + (area >= 1.4142135623730951 * (double)(1u << e)));
  }
  return (kOrderCostClasses - 1 - cls) * (ns + 1) + sl;
}

// Sort keys of every tuple, one thread each over the whole grid: the pose,
// frame and camera loads of the keys run in parallel instead of 12 dependent
// rounds per thread of the single sorting workgroup (27 -> ~8 us per launch
// order at 12.5k tuples).
__global__ __launch_bounds__(256) void k_order_keys(const int32_t* __restrict__ slots, int64_t n,
                                                    int ns, OrderCost oc, int32_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) key[i] = order_key(slots, i, ns, oc);
}

__global__ __launch_bounds__(kOrderThreads) void k_order_by_slot(const int32_t* __restrict__ key,
                                                                  int64_t n, int ns, OrderCost oc,
                                                                  int32_t* __restrict__ order) {
  extern __shared__ int s_cnt[];  // one bucket per key
  __shared__ int s_wsum[kOrderThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = oc.pe ? kOrderCostClasses * (ns + 1) : ns + 1;
  for (int i = tid; i < nb; i += kOrderThreads) s_cnt[i] = 0;
  __syncthreads();
  for (int64_t i = tid; i < n; i += kOrderThreads) atomicAdd(&s_cnt[key[i]], 1);
  __syncthreads();
  // exclusive scan: thread t owns buckets [t * per, (t + 1) * per)
  const int per = (nb + kOrderThreads - 1) / kOrderThreads;
  const int lo = min(tid * per, nb), hi = min(lo + per, nb);
  int sum = 0;
  for (int i = lo; i < hi; ++i) sum += s_cnt[i];
  int inc = sum;
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(inc, d, 64);
    if (lane >= d) inc += v;
  }
  if (lane == 63) s_wsum[wave] = inc;
  __syncthreads();
  int run = inc - sum;
  for (int w = 0; w < wave; ++w) run += s_wsum[w];
  for (int i = lo; i < hi; ++i) {
    const int v = s_cnt[i];
    s_cnt[i] = run;
    run += v;
  }
  __syncthreads();
  for (int64_t i = tid; i < n; i += kOrderThreads) order[atomicAdd(&s_cnt[key[i]], 1)] = (int32_t)i;
}

hipError_t launch_order_by_slot(const int32_t* slots, int64_t n, int ns, int32_t* order,
                                int32_t* keys, hipStream_t s, const OrderCost* cost) {
  if (n <= 0) return hipSuccess;
  if (ns < 0 || ns > kOrderMaxSlots) return hipErrorInvalidValue;
  OrderCost oc{};
  if (cost && (!cost->pe || (int64_t)kOrderCostClasses * (ns + 1) <= kOrderMaxSlots + 1))
    oc = *cost;
  const int nb = oc.pe ? kOrderCostClasses * (ns + 1) : ns + 1;
  hipLaunchKernelGGL(k_order_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slots, n,
                     ns, oc, keys);
  hipLaunchKernelGGL(k_order_by_slot, dim3(1), dim3(kOrderThreads), nb * sizeof(int), s, keys, n,
                     ns, oc, order);
  return hipGetLastError();
}

hipError_t preload_pose_kernels() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_sym_error<0>));
}

}  // namespace bopx
