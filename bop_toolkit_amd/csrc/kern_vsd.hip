// kern_vsd.hip — fused depth raster + Visible Surface Discrepancy on gfx950.
//
// Reference path (per tuple, pose_error.py:17-93):
//   2 GL renders (renderer_vispy.py:433-538) -> 3 full-frame float64 distance
//   images (misc.py:143-163) -> 2 visibility masks (visibility.py:9-75) ->
//   inter/union counts -> per-tau step (or truncated-linear) cost.
//
// Here ONE launch evaluates a whole batch: one 512-thread workgroup (8 waves)
// per tuple, two workgroups per CU.
//  1. The object's meshlets (<= 64 triangles / 64 vertices each) are culled per
//     pose: the 8 corners of each meshlet OBB are projected (float32, the
//     vertex arithmetic) into a conservative pixel rectangle kept in registers.
//     Their union is the tuple's region of interest (ROI): pixels outside both
//     silhouettes cannot change VSD (masks need d_model > 0, visibility.py:37).
//  2. The ROI is swept in 64x64 screen tiles. Per tile, both q-buffers
//     (est, gt; q = 1/Z, 0 = empty) live in LDS; the (pose, meshlet) entries
//     whose rectangle touches the tile are listed and pulled by the waves in
//     groups of two (dynamic balance). Per group: vertex blocks transformed
//     once into LDS (lane = vertex), bbox test + ballot compaction of the
//     triangles that touch the tile, set-up on full waves (lane = triangle),
//     then (triangle, row) items dealt out one per lane and walked with exact
//     integer edge functions and an LDS atomicMax on the float bits
//     (order-independent z-buffer, raster.h).
//  3. Each wave compacts the tile's covered pixels of its rows into a list and
//     evaluates it with full lanes: test depth from HBM, the three float64
//     distances and the float32 visibility tests in the reference operation
//     order (-ffp-contract=off), integer counters (union, inter, per-tau) in
//     registers.
//  4. Counters are reduced across the workgroup in a fixed order; one thread
//     writes e_k = (cnt_k + comp) / union (1.0 when union == 0).
// The same kernel has a silhouette mode (cus / cou_bb_proj) and a GT-info mode
// (calc_gt_info / calc_gt_masks) that reuse steps 1-2 and replace step 3.
// Results are bit-identical to the reference given identical depth maps.
#include <algorithm>
#include <cfloat>
#include <type_traits>

#include "raster.h"

namespace bopx {

constexpr int kVsdThreads = 512;

// Workload counters for the timing diagnostics (BOPX_VSD_ABLATE bit 2). Not
// part of the C-ABI; read with bopx_debug_vsd_stats.
__device__ unsigned long long g_vsd_stats[16];
// Diagnostic phase clocks (BOPX_VSD_ABLATE bit 3; s_memtime, summed over waves):
// [0] clear+coeffs, [1] list, [2] raster work, [3] raster barrier wait,
// [4] pixel work, [5] pixel barrier wait, [6] pre-loop, [7] epilogue; raster work
// split: [8] vertex staging, [9] bbox test + compaction, [10] set-up, [11] walk.
__device__ unsigned long long g_vsd_time[16];
// Wave-level loop trip counts for the instruction census (bit 2; tools/isa_census.py):
// [0] claim-loop iterations, [1] set-up chunks, [2] row-item windows, [3] walk passes,
// [4] walk column-pair iterations (per pass: the widest row of its lanes),
// [5] pixel compaction rows, [6] pixel-loop iterations, [7] exact-path ballots,
// [8] slow-raster column iterations (widest lane), [9] slow-raster rows (widest lane),
// [10] list_tile calls, [11] tile iterations, [12] set-up chunks with a slow triangle
__device__ unsigned long long g_vsd_wave[16];
// Diagnostics are compiled in only with -DBOPX_VSD_DIAG=1 (tools/vsd_stats.py
// loads such a variant); the product kernel carries none of their state.
#ifndef BOPX_VSD_DIAG
#define BOPX_VSD_DIAG 0
#endif
#define VSD_DIAG(bit) (BOPX_VSD_DIAG && (a.ablate & (bit)))
// lane 0 adds v (wave-uniform) to wave-level counter k (diag builds only; the
// product build has no trace of it, not even a captured variable)
#if BOPX_VSD_DIAG
#define VSD_WAVE(k, v)                                                             \
  do {                                                                             \
    if (VSD_DIAG(4) && lane == 0) atomicAdd(&g_vsd_wave[k], (unsigned long long)(v)); \
  } while (0)
#else
#define VSD_WAVE(k, v) ((void)0)
#endif
#define VSD_STAMP(k)                                              \
  do {                                                            \
    if (VSD_DIAG(8)) {                                            \
      const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
      ph[k] += _t - t_prev;                                       \
      t_prev = _t;                                                \
    }                                                             \
  } while (0)

// Correctly rounded float64 sqrt for s = 0 or s >= 2^-767 (finite): the
// rsq + Goldschmidt sequence of the device library's sqrt, without its input
// scaling (taken only below 2^-767) and inf/zero class fix-ups. Arguments here
// come from float32 depths: s = (pX d)^2 + (pY d)^2 + d^2 >= d^2 >= 2^-298 when
// d != 0, so the result is bit-identical to sqrt(s).
__device__ __forceinline__ double sqrt_depth(double s) {
  const double y = __builtin_amdgcn_rsq(s);
  double g = s * y, h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, s);
  g = fma(d, h, g);
  d = fma(-g, g, s);
  g = fma(d, h, g);
  return s > 0.0 ? g : s;
}

// float64 distance of a float32 depth at pixel (pX, pY) (misc.py:158-161).
__device__ __forceinline__ double dist_of(double pX, double pY, float depth) {
  const double d = (double)depth;
  const double a = pX * d, b = pY * d;
  return sqrt_depth((a * a + b * b) + d * d);
}

// visibility._estimate_visib_mask, bop19 (visibility.py:34-37).
__device__ __forceinline__ bool visib19(double dt, double dm, float delta32, int delta_f64,
                                        double delta64) {
  const float diff = (float)dm - (float)dt;
  const bool le = delta_f64 ? ((double)diff <= delta64) : (diff <= delta32);
  return (le || dt == 0.0) && dm > 0.0;
}

// visib19 with the float32 threshold VsdArgs::dthr (runtime.cpp visib_thr32):
// (float)diff <= dthr is the same test for every float32 diff as the float32
// or float64 comparison against delta that visib19 selects.
__device__ __forceinline__ bool visib19t(double dt, double dm, float dthr) {
  const float diff = (float)dm - (float)dt;
  return ((diff <= dthr) || dt == 0.0) && dm > 0.0;
}

// ---------------------------------------------------------------------------
// Certified float32 filter of the per-pixel VSD decisions (round 4).
//
// The reference decides, per pixel, two visibility tests (visibility.py:35-37:
// float32 difference of float64 distances vs delta) and, for intersection
// pixels, n_tau step thresholds (pose_error.py:80-81: float64 |dist_g - dist_e|
// vs tau, here dd >= T_k). The float64 distances (misc.py:158-161) cost three
// IEEE sqrt sequences per pixel; yet the decisions are almost never close to
// their thresholds. The filter evaluates them in float32 from
//   s = sqrt(1 + pX^2 + pY^2)  (hardware sqrt of A[col] + B[row], float32),
//   g = rcp(q_g) s, e = rcp(q_e) s, t = |d_test| s  (hardware reciprocal),
// each within 12u of the float32 rounding of the reference's float64 distance
// (u = 2^-24; s within 6.5u, the reciprocal within 3u of rcp_rn; DESIGN.md §5
// derives the bounds), so the visibility difference is within 14u (g + t) of
// the reference's and the step distance |g - e| within 12u (g + e) of the
// reference's float64 one.
// Every decision is taken from float32 only when it is outside a margin of
// 64u x the distances involved (+ 2^-100 for the subnormal range): visibility
// when |(g - t) - delta| > E, a threshold when lo = dd - E_d and hi = dd + E_d
// fall on the same side of it. Otherwise (and for any non-finite or > 2^100
// value) the lane redoes the pixel with the exact float64 sequence. The
// counters are integers, so the results are bit-identical to the exact path
// (tests/test_gpu_parity.py, the fuzz tests; the diag build counts the pixels
// that take the exact path).
constexpr float kFilterRel = 0x1p-18f;   // 64u
constexpr float kFilterAbs = 0x1p-100f;  // subnormal-range absolute errors
constexpr float kFilterMax = 0x1p100f;   // larger values: exact path

// float32 coefficients of one column / row: A = pX^2, B = 1 + pY^2 (pX, pY the
// float64 misc.py:137-138 values, rounded to float32)
__device__ __forceinline__ float filt_a(double pX) {
  const float x = (float)pX;
  return x * x;
}
__device__ __forceinline__ float filt_b(double pY) {
  const float y = (float)pY;
  return 1.0f + y * y;
}

// Exact per-pixel VSD step decisions (the float64 reference sequence):
// visibility of gt / est and the step distance (only meaningful when both are
// visible). pX, pY: float64 coefficients; qe / qg: q bits (0 = no fragment).
__device__ __forceinline__ void vsd_exact_px(double pX, double pY, uint32_t qe, uint32_t qg,
                                             float dtest, float dthr, bool& vg, bool& ve,
                                             double& dd) {
  const float de = qe ? rcp_rn(__uint_as_float(qe)) : 0.0f;
  const float dg = qg ? rcp_rn(__uint_as_float(qg)) : 0.0f;
  const double dist_t = dist_of(pX, pY, dtest);
  const double dist_g = qg ? dist_of(pX, pY, dg) : 0.0;
  const double dist_e = qe ? dist_of(pX, pY, de) : 0.0;
  vg = visib19t(dist_t, dist_g, dthr);
  ve = visib19t(dist_t, dist_e, dthr) || (vg && dist_e > 0.0);  // visibility.py:74
  dd = fabs(dist_g - dist_e);
}

// Float32 pass of the filter. s2 = A[col] + B[row]. Returns vg / ve, the step
// distance bracket [lo, hi] of |dist_g - dist_e| and whether the visibility
// decisions (or the magnitudes) need the exact path.
__device__ __forceinline__ bool vsd_filter_px(float s2, uint32_t qe, uint32_t qg, float dtest,
                                              float dthr, bool& vg, bool& ve, float& lo,
                                              float& hi) {
  const float s = __builtin_amdgcn_sqrtf(s2);
  const float g = qg ? __builtin_amdgcn_rcpf(__uint_as_float(qg)) * s : 0.0f;
  const float e = qe ? __builtin_amdgcn_rcpf(__uint_as_float(qe)) * s : 0.0f;
  const float t = fabsf(dtest) * s;
  const bool dtz = dtest == 0.0f;  // dist_t == 0
  const float gt = g + t, et = e + t, ge = g + e;
  const float xg = (g - t) - dthr, xe = (e - t) - dthr;
  const bool cg = fabsf(xg) > __builtin_fmaf(gt, kFilterRel, kFilterAbs);
  const bool ce = fabsf(xe) > __builtin_fmaf(et, kFilterRel, kFilterAbs);
  // bitwise forms: no short-circuit branches in the pixel loop
  const bool hg = qg != 0u, he = qe != 0u;
  vg = hg & (dtz | (xg < 0.0f));
  ve = he & (dtz | (xe < 0.0f) | vg);
  const float dd = fabsf(g - e), ed = __builtin_fmaf(ge, kFilterRel, kFilterAbs);
  lo = dd - ed;
  hi = dd + ed;
  return !(gt + e < kFilterMax) | (hg & !dtz & !cg) | (he & !dtz & !vg & !ce);
}

// float32 form of a step threshold T for the filter: T <= 0 passes every
// distance (-inf), otherwise RN(T) (NaN and +inf stay).
__device__ __forceinline__ float filt_thr(double T) { return T <= 0.0 ? -INFINITY : (float)T; }

// Step cost of normalised distances (pose_error.py:66-68,80-81):
// RN(dd / diameter) >= tau is monotone in dd >= 0 for a finite diameter > 0,
// so it is dd >= T for the least double T that passes it. T is found once per
// (tuple, tau) with the reference's own IEEE division: from the guess
// tau * diameter (a few ulps off at most) by ulp steps, else by bisection over
// the ordered bit patterns of the finite non-negative doubles.
__device__ __forceinline__ double dbl_of(uint64_t b) { return __longlong_as_double((long long)b); }

__device__ double step_threshold(double tau, double diam) {
  constexpr uint64_t kMaxBits = 0x7FEFFFFFFFFFFFFFull;  // DBL_MAX
  auto pass = [&](uint64_t b) { return dbl_of(b) / diam >= tau; };
  const double x = tau * diam;
  if (x >= 0.0 && x <= DBL_MAX) {
    uint64_t b = (uint64_t)__double_as_longlong(x);
    if (pass(b)) {
      for (int i = 0; i < 4; ++i, --b)
        if (b == 0 || !pass(b - 1)) return dbl_of(b);
    } else {
      for (int i = 0; i < 4 && b < kMaxBits; ++i)
        if (pass(++b)) return dbl_of(b);
    }
  }
  if (!pass(kMaxBits)) return INFINITY;  // no finite distance passes
  if (pass(0)) return 0.0;
  uint64_t lo = 0, hi = kMaxBits;  // pass(lo) false, pass(hi) true
  while (hi - lo > 1) {
    const uint64_t mid = lo + ((hi - lo) >> 1);
    if (pass(mid)) hi = mid;
    else lo = mid;
  }
  return dbl_of(hi);
}

// Conservative pixel rectangle of one meshlet bounding box (8 object-space
// corners, runtime.cpp obb_corners) under a pose. Any corner with Z <= 0 (or a
// non-finite projection) gives the whole image.
//
// Also classifies the entry for the back-face occlusion test (VsdArgs::cull 3):
// back = every triangle faces away from the camera (normal cone + bounding
// sphere, runtime.cpp meshlet_cone; a heuristic: it only picks which entries
// are tested), and qb = an upper bound of every fragment q = 1/Z the meshlet
// can produce under this pose (the test's threshold; this one must be exact):
//   * every vertex lies in the box, so its exact camera Z >= the smallest exact
//     corner Z; the float32 evaluations of both (vertex in r_vertex, corner
//     here) are within 6 u (|x| + |y| + |z| + |t_z|) of exact (u = 2^-24, |R_ij|
//     <= m = max(1, |R_2j|)), and the L1 norm over the box peaks at a corner:
//     zlo = zmin - 2^-19 (m rho1 + |t_z|) bounds every vertex Z from below
//     (2.6x margin);
//   * a vertex 1/Z is rcp_rn(Z) <= (1 + 2^-24) / zlo and every fragment q <=
//     (1 + 2^-8) x its triangle's largest vertex 1/Z (spec v5, raster.h), so
//     qb = rcp_rn(zlo) (1 + 2^-7) bounds them all (rounding included).
// back is false (never tested) when some corner is not in front of the camera.
__device__ __forceinline__ short4 meshlet_rect(gptr<const float> mb, const float* Rf,
                                               const Cam32& c, int W, int H, float& zmin,
                                               float& qb, bool& back) {
  float umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
  bool full = false;
  zmin = INFINITY;
  // the 96 B of corners in six 16-B loads + cone and sphere, all in flight
  // before the first use
  f32x4 cb[kMletFloats / 4];
#pragma unroll
  for (int k = 0; k < kMletFloats / 4; ++k) cb[k] = *(gptr<const f32x4>)(mb + 4 * k);
  {
    const f32x4 cone = cb[6], sph = cb[7];
    const float X = ((Rf[0] * sph.x + Rf[1] * sph.y) + Rf[2] * sph.z) + Rf[9];
    const float Y = ((Rf[3] * sph.x + Rf[4] * sph.y) + Rf[5] * sph.z) + Rf[10];
    const float Z = ((Rf[6] * sph.x + Rf[7] * sph.y) + Rf[8] * sph.z) + Rf[11];
    const float ax = (Rf[0] * cone.x + Rf[1] * cone.y) + Rf[2] * cone.z;
    const float ay = (Rf[3] * cone.x + Rf[4] * cone.y) + Rf[5] * cone.z;
    const float az = (Rf[6] * cone.x + Rf[7] * cone.y) + Rf[8] * cone.z;
    const float va = (X * ax + Y * ay) + Z * az, vv = (X * X + Y * Y) + Z * Z;
    const float s = sqrtf(fmaxf(vv - va * va, 0.0f));
    const float sina = sqrtf(fmaxf(1.0f - cone.w * cone.w, 0.0f));
    back = cone.w > 0.0f && va * cone.w - s * sina > sph.w;
  }
  float cf[24];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    cf[4 * k] = cb[k].x;
    cf[4 * k + 1] = cb[k].y;
    cf[4 * k + 2] = cb[k].z;
    cf[4 * k + 3] = cb[k].w;
  }
  float rho1 = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float x = cf[3 * k], y = cf[3 * k + 1], z = cf[3 * k + 2];
    rho1 = fmaxf(rho1, (fabsf(x) + fabsf(y)) + fabsf(z));
    const float X = ((Rf[0] * x + Rf[1] * y) + Rf[2] * z) + Rf[9];
    const float Y = ((Rf[3] * x + Rf[4] * y) + Rf[5] * z) + Rf[10];
    const float Z = ((Rf[6] * x + Rf[7] * y) + Rf[8] * z) + Rf[11];
    zmin = fminf(zmin, Z);
    if (!(Z > 0.0f)) {
      full = true;
    } else {
      const float iz = rcp_rn(Z);
      const float u = (c.fx * X) * iz + c.cx, v = (c.fy * Y) * iz + c.cy;
      umin = fminf(umin, u);
      umax = fmaxf(umax, u);
      vmin = fminf(vmin, v);
      vmax = fmaxf(vmax, v);
    }
  }
  {
    // |R_2j| may exceed 1 for a non-rotation input: scale the L1 bound by it
    const float m = fmaxf(fmaxf(fabsf(Rf[6]), fabsf(Rf[7])), fmaxf(fabsf(Rf[8]), 1.0f));
    const float zlo = zmin - 0x1p-19f * (m * rho1 + fabsf(Rf[11]));
    qb = rcp_rn(zlo > 0.0f ? zlo : 1.0f) * 1.0078125f;  // (1 + 2^-7) / zlo
    back = back && !full && zlo > 0.0f && qb < 0x1p100f;
  }
  if (full || !(umin == umin) || !(vmin == vmin) || !(umax == umax) || !(vmax == vmax)) {
    back = false;
    return make_short4(0, 0, (short)(W - 1), (short)(H - 1));
  }
  // Column c is sampled at c + 0.5 and covered only if that centre is inside a
  // triangle, i.e. within [min, max] of the snapped vertex u (snap error
  // 1/512 px). The corners bound the vertices exactly; their float32
  // projection and the vertices' differ by ~1e-3 px at most: 1/16 px of slack.
  const float fx0 = ceilf(umin - 0.5f - 0.0625f), fx1 = floorf(umax - 0.5f + 0.0625f);
  const float fy0 = ceilf(vmin - 0.5f - 0.0625f), fy1 = floorf(vmax - 0.5f + 0.0625f);
  if (fx1 < 0.0f || fy1 < 0.0f || fx0 > (float)(W - 1) || fy0 > (float)(H - 1))
    return make_short4(1, 1, 0, 0);  // empty
  const int x0 = (int)fmaxf(fx0, 0.0f), y0 = (int)fmaxf(fy0, 0.0f);
  const int x1 = (int)fminf(fx1, (float)(W - 1)), y1 = (int)fminf(fy1, (float)(H - 1));
  return make_short4((short)x0, (short)y0, (short)x1, (short)y1);
}

// Max over the 64 lanes of non-negative floats (full exec): DPP butterflies
// inside each row of 16 lanes, then the four row maxima in SALU. No LDS
// round trips (a __shfl_xor reduction is six dependent ds_bpermute).
__device__ __forceinline__ float wave_max_nonneg_f32(float x) {
  int v = __float_as_int(x);  // non-negative floats order like their bits
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false));  // row_ror 4
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false));  // row_ror 8
  const int m = max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
                    max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
  return __int_as_float(m);
}

// True iff every pixel of the tile rectangle [x0, x1] x [y0, y1] (tile-relative,
// wave-uniform, x1 - x0 < 64) holds q bits >= qb in the q tile `dep`. Lanes
// cover 64 / w rows per step, eight steps per LDS round trip; early exit on the
// first failing round.
// A tile rectangle [x0, x1] x [y0, y1] (tile-relative) swept in 8 x 8 pixel
// blocks, lane = (row lane >> 3, column lane & 7) inside a block; a lane past
// the rectangle re-reads its last row / column (harmless for a minimum).
struct Region {
  int x0, x1, y0, y1, nbx, nb;
};

__device__ __forceinline__ Region make_region(uint32_t word, int tw, int th) {
  Region g;
  g.x0 = (int)((word >> 12) & 31u) * 2;
  g.x1 = min((int)((word >> 17) & 31u) * 2 + 1, tw - 1);
  g.y0 = (int)((word >> 22) & 31u) * 2;
  g.y1 = min((int)((word >> 27) & 31u) * 2 + 1, th - 1);
  g.nbx = (g.x1 - g.x0 + 8) >> 3;
  g.nb = g.nbx * ((g.y1 - g.y0 + 8) >> 3);
  return g;
}

// Smallest q bits this lane reads in blocks [b0, b0 + 8) of the region (LDS
// reads issued back to back, one wait at the use).
__device__ __forceinline__ uint32_t region_min8(const uint32_t* dep, const Region& g, int b0,
                                                int lane) {
  uint32_t v[8];
  // block (bx, by) stepped incrementally (wave-uniform, SALU); past the last
  // block the last one is re-read
  int by = (unsigned)b0 / (unsigned)g.nbx, bx = b0 - by * g.nbx;
  const int lr = lane >> 3, lc = lane & 7;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int r = min(g.y0 + 8 * by + lr, g.y1);
    const int c = min(g.x0 + 8 * bx + lc, g.x1);
    v[k] = dep[__mul24(r, kTileStride) + c];
    if (b0 + k + 1 < g.nb) {
      if (++bx == g.nbx) {
        bx = 0;
        ++by;
      }
    }
  }
  return min(min(min(v[0], v[1]), min(v[2], v[3])), min(min(v[4], v[5]), min(v[6], v[7])));
}

// True iff every pixel of the region from block b0 on holds q bits >= qb.
__device__ __forceinline__ bool region_covered(const uint32_t* dep, const Region& g, int b0,
                                               uint32_t qb, int lane) {
  for (int b = b0; b < g.nb; b += 8)
    if (__builtin_amdgcn_ballot_w64(region_min8(dep, g, b, lane) < qb) != 0) return false;
  return true;
}

// Max over the lanes of a non-negative int (diagnostics only: not optimised)
__device__ __forceinline__ int diag_wave_max(int v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
  return v;
}

// Inclusive prefix sum over the 64 lanes (full exec), all in DPP: row_shr 1, 2,
// 4, 8 inside each row of 16 lanes, then row_bcast 15 / 31 carry the row totals
// into the rows above. No LDS round trips (the __shfl_up scan is six dependent
// ds_bpermute + lgkmcnt waits per call).
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Make LDS written by other lanes of this wave visible (LDS is in order per wave;
// the fences stop the compiler from moving accesses across).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Load base[byte_off] for a wave-uniform base and a 32-bit per-lane byte
// offset: global_load with an SGPR base (saddr) and no 64-bit address math.
template <class T>
__device__ __forceinline__ T ld_off(gptr<const T> base, uint32_t byte_off) {
  return *(gptr<const T>)((gptr<const char>)base + byte_off);
}

constexpr int kVsdWaves = kVsdThreads / 64;
#ifndef BOPX_VSD_WALK_UNMASKED  // A/B switch: the unmasked walk for every class
#define BOPX_VSD_WALK_UNMASKED 0
#endif
constexpr int kRowWin = 256;  // row items numbered per window (start flags)
// covered-pixel list of a wave: its rows w, w + kVsdWaves, ... of the tile
constexpr int kPixPerWave = (kTileH + kVsdWaves - 1) / kVsdWaves * kTileW;
// Row records of the walk live in LDS (s_rec, 24 KiB per workgroup), written
// compacted by rank and read as three 16-B LDS reads (ds_read_b128; the
// compiler's b96 + 3 x read2_b32 split was 2 % slower). Row item -> record
// lookup: one start flag per record + ballot / mbcnt. Measured and rejected
// (DESIGN.md §5-6): records kept in registers and fetched with ds_bpermute
// (1 % slower at 2 workgroups per CU, spills at 3), the next pass's record read
// ahead of the walk (+17 %), static round-robin entry assignment (+3 %).
static_assert(kRowWin == 4 * 64, "start flags are cleared one dword per lane");
static_assert(sizeof(RRow) * 64 >= 2 * kPixPerWave, "pixel lists overlay the raster records");
static_assert(kVsdThreads % kTileW == 0, "pixel-pass rows are wave-uniform");
// (pose, meshlet) entries staged together per wave step (1: +3 %, 3: LDS over
// the two-workgroup budget, round 2)
constexpr int kGroup = 2;
// worst case (RPT) of meshlet rectangles per thread
constexpr int kRectsPerThread = (2 * kMaxMeshlets + kVsdThreads - 1) / kVsdThreads;
// Wave-private scratch: the staged vertex blocks and compacted triangle refs of
// an entry group during the raster, the tile's column / row coefficients
// (float64 and float32) during the pixel pass.
constexpr int kStageBytes = kGroup * kMeshletVerts * (int)sizeof(RVtx) + kGroup * kMeshletTris * 4;
constexpr int kCoefBytes = 8 * (kTileW + kTileH) + 4 * (kTileW + kTileH);
constexpr int kWaveScr = kStageBytes > kCoefBytes ? kStageBytes : kCoefBytes;
// Waves that claim the last entry groups of a tile run at issue priority 3
// until the raster-end barrier (the tile's critical path; the sibling
// workgroup's waves yield to them): -0.3 % (round 1).
constexpr int kVsdPrio = 3;
// Entry queue order and occlusion culling: per pose, the (pose, meshlet) entries
// whose nearest OBB corner lies in the near half of that pose's depth range are
// dealt first (front of s_list), the far ones after them (back of s_list,
// growing down). A far entry, once its vertex block is staged, is skipped when
// every pixel of its rectangle inside the tile already holds q >= (1 + 2^-8) x
// the largest 1/Z of its vertices: spec v5 bounds every fragment of the meshlet
// by that (raster.h), and q-buffer values only grow, so a value read while other
// waves still write is a lower bound of the final one. The result is
// bit-identical with or without the test (VsdArgs::cull, BOPX_VSD_CULL=0).
// Back-face occlusion test (VsdArgs::cull == 3; automatic for objects of many
// meshlets). Its claim-loop block is compiled in for every instantiation: the
// second loop latch (`continue` of a fully occluded group) also gives the
// whole claim loop a better register allocation (114 VGPRs without spills
// instead of 128 + 5 spilled, -2.9 % with the test off, round 2).
// Queue order (VsdArgs::qorder, wave-uniform): 0 = near entries first (depth),
// 1 = entries overlapping the tile by >= a quarter of its area first (longest
// first for the raster-end barrier: 1,024 px on the 64x64 tile, round-1 LPT
// order, 2 % faster without the occlusion test); the occlusion test applies to
// far entries either way. The z-buffer is order-independent (atomicMax on the
// q bits), so both orders give bit-identical results
// (test_fused_vsd_occlusion_cull_exact runs both).
constexpr int kLptOverlap = kTileW * kTileH / 4;
// BOPX_VSD_CULL unset: back-face occlusion test for objects above this many meshlets
constexpr int kCullAutoMeshlets = 256;
constexpr int kCullAutoDensity = 12;  // ... and at least this many meshlets per ROI tile

// Each wave's first entry group of a tile is pre-assigned (no claim round trip
// for it): -0.9 % (same-box A/B, round 2); the rest are claimed from s_next,
// which starts at NW * kGroup.

// COST: 0 = step, 1 = tlinear, kCostCover = silhouette overlap, kCostGtInfo = GT stats.
// NT (step cost): thresholds compared per pixel (>= n_tau; 10 for the BOP taus).
// RPT: meshlet rectangles held per thread (1, 2 or 4): the launch picks the
// smallest that covers 2 x the most meshlets of any registered object, so
// objects of up to 16k triangles keep 6 fewer VGPRs live through the tile loop.
// RPT 0 (objects of more than kMaxMeshlets meshlets, no size limit): the
// rectangles are not kept but recomputed per tile, kListLen entries per round,
// each round listed and rasterised into the same q tiles before the pixel pass.
template <int COST, int RPT, int NT>
// two workgroups per CU (4 waves per SIMD: VGPRs <= 128)
__global__ __launch_bounds__(kVsdThreads, 2 * kVsdThreads / 256)
void k_vsd(VsdArgs a) {
  constexpr int NTH = kVsdThreads;  // threads of the workgroup
  constexpr int NW = NTH / 64;      // its waves
  constexpr int kPixPW = (kTileH + NW - 1) / NW * kTileW;   // pixel-list entries per wave
  // q = 1/Z bits, 0 = empty; rows padded by one dword so lanes that walk the
  // same column on consecutive rows (row-split) hit different LDS banks.
  __shared__ uint32_t s_dep[2][kTileStride * kTileH];
  __shared__ __attribute__((aligned(16))) uint8_t s_wscr[NW][kWaveScr];
  __shared__ RRow s_rec[NW][64];          // set-up triangles of the current chunk
  // record start flags of a window of row items
  __shared__ __attribute__((aligned(4))) uint8_t s_own[NW][kRowWin];
  // Tile entry queue. RPT <= 2 (objects of <= 512 meshlets): 32-bit words
  // entry | far << 11 | rectangle in the tile at 2-px granularity (x0/2, x1/2,
  // y0/2, y1/2: 5 bits each from bit 12) for the occlusion test; RPT 4: 16-bit
  // entry indices, no occlusion test (the list would not fit the LDS budget).
  // row-walk atomics (raster.h r_walk_row_max): unmasked for the 1-rectangle
  // objects, masked above (round 2: -0.9 % / -1.2 % on the two classes)
  constexpr bool kWalkMasked = RPT != 1 && !BOPX_VSD_WALK_UNMASKED;
  constexpr bool kStream = RPT == 0;
  constexpr int kR = kStream ? 4 : RPT;  // rectangles per thread and round
  constexpr bool kCull = RPT >= 1 && RPT <= 2;
  constexpr int kListLen = kR * NTH;  // >= 2 * nm (launch_vsd) unless kStream
  using ListT = typename std::conditional<kCull, uint32_t, uint16_t>::type;
  // list-ahead (objects of <= 256 meshlets, round 3: -0.8 %): two queues,
  // the next tile's listed by each wave in the current tile's raster tail
  constexpr bool kAhead = !kStream && RPT == 1;
  constexpr int kQueues = kAhead ? 2 : 1;
  __shared__ __attribute__((aligned(4))) ListT s_lists[kQueues][kListLen];
  // Back-face occlusion test (cull 3): per entry, its fragment bound qb as an
  // 8-bit code below the pose's largest bound: qb <= s_qhi[pose] 2^(-code/64).
  __shared__ uint8_t s_qb[kCull ? kListLen : 4];
  __shared__ float s_qhi[2];
  __shared__ float s_zr[2][2];  // per pose: depth range of the meshlet corners (min, max)
  __shared__ int s_nexts[kQueues];
  __shared__ __attribute__((aligned(16))) float s_pose[2][12];
  __shared__ __attribute__((aligned(16))) float s_pose_pk[2][12];  // r_vertex_pk order
  __shared__ int s_roi[4];
  __shared__ int s_nlists[kQueues];
  __shared__ int s_nsmalls[kQueues];
  __shared__ double s_thr[kMaxTaus];  // step-cost thresholds (T_k, +inf past n_tau)
  // Final per-wave partial counters reuse the depth tiles (after the tile loop).
  uint32_t(*s_cnt)[2 + kMaxTaus] = reinterpret_cast<uint32_t(*)[2 + kMaxTaus]>(&s_dep[0][0]);
  double(*s_lin)[kMaxTaus] = reinterpret_cast<double(*)[kMaxTaus]>(&s_dep[1][0]);

  // tile-parallel mode: workgroup (tuple kb, split sp); tuples from
  // a.split_from on take a.split workgroups each, earlier ones one (S = 1)
  const int64_t n0 = a.split_from;
  const bool tail = a.split > 1 && (int64_t)blockIdx.x >= n0;
  const int S = tail ? a.split : 1;
  const int64_t j = tail ? ((int64_t)blockIdx.x - n0) / S : 0;  // split-tuple index
  const int64_t kb = tail ? n0 + j : (int64_t)blockIdx.x;
  const int sp = tail ? (int)((int64_t)blockIdx.x - n0 - j * S) : 0;
  const int64_t b = a.order ? (int64_t)a.order[kb] : kb;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  RVtx* const w_stage = reinterpret_cast<RVtx*>(&s_wscr[wave][0]);
  uint32_t* const w_tri =
      reinterpret_cast<uint32_t*>(&s_wscr[wave][kGroup * kMeshletVerts * sizeof(RVtx)]);
  double* const w_pX = reinterpret_cast<double*>(&s_wscr[wave][0]);
  double* const w_pY = w_pX + kTileW;
  float* const w_fA = reinterpret_cast<float*>(w_pY + kTileH);  // filter: pX^2, 1 + pY^2
  float* const w_fB = w_fA + kTileW;
  unsigned long long ph[16] = {}, t_prev = 0;
  if (VSD_DIAG(8)) t_prev = __builtin_amdgcn_s_memtime();
  const ObjDesc o = a.objs[a.slots[b]];
  // Capacity guard: this instantiation's entry queue and rectangle registers
  // hold kListLen entries (launch_vsd_rpt_any picks RPT from the context's
  // largest object; the host refuses to launch when that maximum is stale,
  // runtime.cpp launch_dev). An object beyond them can only come from a
  // descriptor table changed under a queued launch: the workgroup then runs
  // with no meshlets (no queue / LDS index out of range) and writes NaN errors
  // (render mode: no fragments). A select, not an early return: an extra exit
  // costs this kernel 8 VGPRs and spills.
  constexpr bool kOneP = COST == kCostGtInfo || COST == kCostRender;
  const bool over = !kStream && (kOneP ? o.nm : 2 * o.nm) > kListLen;
  const int W = a.width, H = a.height, nm = over ? 0 : o.nm;
  // Object arrays live in global memory: address-space-1 views give
  // global_load (vmcnt only) instead of flat_load for pointers read from memory.
  // vertex blocks are float32x4 at a 16-B stride; only x, y, z are loaded
  // (global_load_dwordx3), so no register is held by the padding word
  const gptr<const f32x3> g_mvtx3 = (gptr<const f32x3>)o.mlet_vtx;
  const gptr<const uint32_t> g_mtri = (gptr<const uint32_t>)o.mlet_tri;
  const gptr<const float> g_mlet = (gptr<const float>)o.mlet;
  const int64_t fidx = a.frame_idx[b];
  // test depth: img_w x img_h frames; the raster canvas (W x H) may be larger
  // with the image at (ox, oy) (GT-info mode, calc_gt_info.py:66-73)
  const int IW = a.img_w, IH = a.img_h, ox = a.ox, oy = a.oy;
  const gptr<const float> frame = (gptr<const float>)(a.frames + fidx * (int64_t)IW * IH);
  const double fx = a.cam[4 * fidx + 0], fy = a.cam[4 * fidx + 1];
  const double cx = a.cam[4 * fidx + 2], cy = a.cam[4 * fidx + 3];
  Cam32 c32;
  c32.fx = (float)fx;
  c32.fy = (float)fy;
  c32.cx = (float)(cx + (double)ox);  // the renderer receives cx + offset (float64)
  c32.cy = (float)(cy + (double)oy);
  if (tid < 12) {
    const float pe = (float)a.pose_est[12 * b + tid], pg = (float)a.pose_gt[12 * b + tid];
    s_pose[0][tid] = pe;
    s_pose[1][tid] = pg;
    // pair order {R0,R3, R1,R4, R2,R5, t0,t1, R6,R7,R8, t2}: element tid's slot
    const int d = (int)((0xb76a98531420ull >> (4 * tid)) & 15u);
    s_pose_pk[0][d] = pe;
    s_pose_pk[1][d] = pg;
  }
  const double diam = COST == 0 && a.normalized ? a.diameters[b] : 1.0;
  // Step cost: per-pixel dd >= T_k. Normalised by a finite diameter > 0 with
  // no NaN tau, T_k = step_threshold; otherwise T_k = tau_k and the pixel
  // pass divides dd by the diameter itself (`divide`, pathological inputs).
  bool divide = false;
  if constexpr (COST == 0) {
    bool fast = a.normalized && diam > 0.0 && diam <= DBL_MAX;
    for (int k = 0; k < a.n_tau; ++k) fast = fast && a.taus[k] == a.taus[k];
    divide = a.normalized && !fast;
    if (tid < NT) {
      double T = INFINITY;
      if (tid < a.n_tau) T = fast ? step_threshold(a.taus[tid], diam) : a.taus[tid];
      s_thr[tid] = T;
    }
  }
  if (tid == 0) {
    for (int q = 0; q < kQueues; ++q) {  // tile queue counters (reset again per tile)
      s_nlists[q] = 0;
      s_nsmalls[q] = 0;
      s_nexts[q] = (NW * kGroup);
    }
    s_roi[0] = s_roi[1] = 0x7FFFFFFF;
    s_roi[2] = s_roi[3] = -1;
    s_zr[0][0] = s_zr[1][0] = INFINITY;
    s_zr[0][1] = s_zr[1][1] = 0.0f;
    s_qhi[0] = s_qhi[1] = 0.0f;
  }
  __syncthreads();
  // back-face occlusion test: forced (3) or automatic (-1) for objects of many
  // meshlets, where overdraw per tile is high enough for the skipped entries to
  // pay for the test (tools/gpu_cull_size.sh, configs[3] workload, same box,
  // 2 reps, k_vsd time cull on vs off: 10k triangles +3.2 %, 15k +0.9 %,
  // 20k -1.1 %, 25k -2.0 %, 30k -3.2 %; T-LESS-like configs[4] -2.8 %); the
  // on-screen density condition is applied once the ROI is known (below)
  // (tools/gpu_cull_density.sh: 30k triangles at 1.5x size -1.4 %, 2x +1 %;
  // 10k triangles at 0.5x / 0.7x size still +1.8 % / +1.2 %)
  const bool cull_maybe = kCull && (a.cull == 3 || (a.cull < 0 && nm > kCullAutoMeshlets));
  // GT-info and render modes list only the second pose's entries (nm .. 2 nm - 1):
  // the rectangle registers and queue words hold them from 0 (entry = ebase + local
  // index), so an object needs nm rectangle slots instead of 2 nm (launch_vsd_rpt_any)
  constexpr bool kOnePose = (COST == kCostGtInfo || COST == kCostRender) && !kStream;
  const int ebase = kOnePose ? nm : 0;

  // 1. per-pose meshlet rectangles (kept in registers: entry tid + 512 j) + ROI,
  // and each entry's nearest corner depth (queue order, see kLptOverlap above).
  short4 rect[kR];
  float zmin[kR];
  float qbv[kR];            // fragment bound per entry (back-face test)
  uint32_t back_bits = 0;   // bit j: entry tid + 512 j is back-facing
  float qh[2] = {0.0f, 0.0f};  // per pose: largest bound of a back-facing entry
  int roi[4] = {INT32_MAX, INT32_MAX, -1, -1};
  float zr[4] = {INFINITY, -INFINITY, INFINITY, -INFINITY};  // pose 0 min, max; pose 1
  // (kStream: every entry, the rectangles are only reduced into the ROI here)
  for (int i0 = 0; i0 < (kStream ? 2 * nm : 1); i0 += kListLen)
#pragma unroll
  for (int j = 0; j < kR; ++j) {
    const int i = (kStream ? i0 : ebase) + tid + j * NTH;
    rect[j] = make_short4(1, 1, 0, 0);
    zmin[j] = -INFINITY;
    qbv[j] = 0.0f;
    if (i < 2 * nm && !((COST == kCostGtInfo || COST == kCostRender) && i < nm)) {  // GT-info: gt pose only
      const int r = i >= nm, m = i - r * nm;
      bool bk = false;
      rect[j] = meshlet_rect(g_mlet + kMletFloats * (int64_t)m, s_pose[r], c32, W, H, zmin[j],
                             qbv[j], bk);
      if (rect[j].x <= rect[j].z && rect[j].y <= rect[j].w) {
        if (bk) {
          back_bits |= 1u << j;
          qh[r] = fmaxf(qh[r], qbv[j]);
        }
        roi[0] = min(roi[0], (int)rect[j].x);
        roi[1] = min(roi[1], (int)rect[j].y);
        roi[2] = max(roi[2], (int)rect[j].z);
        roi[3] = max(roi[3], (int)rect[j].w);
        if (zmin[j] > 0.0f) {  // finite (every corner in front of the camera)
          zr[2 * r] = fminf(zr[2 * r], zmin[j]);
          zr[2 * r + 1] = fmaxf(zr[2 * r + 1], zmin[j]);
        }
      }
    }
  }
  if constexpr (kCull) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float o = __shfl_xor(zr[k], off, 64);
        zr[k] = (k & 1) ? fmaxf(zr[k], o) : fminf(zr[k], o);
      }
    }
    // positive floats (or +-inf) order like their int bits: LDS int atomics
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int* z = reinterpret_cast<int*>(&s_zr[0][0]) + k;
        if (k & 1) atomicMax(z, __float_as_int(fmaxf(zr[k], 0.0f)));
        else atomicMin(z, __float_as_int(zr[k]));
      }
    }
    if (cull_maybe) {
      qh[0] = wave_max_nonneg_f32(qh[0]);
      qh[1] = wave_max_nonneg_f32(qh[1]);
      if (lane == 0) {
        atomicMax(reinterpret_cast<int*>(&s_qhi[0]), __float_as_int(qh[0]));
        atomicMax(reinterpret_cast<int*>(&s_qhi[1]), __float_as_int(qh[1]));
      }
    }
  }
  // wave reduction, then one LDS atomic per wave and bound
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    roi[0] = min(roi[0], __shfl_xor(roi[0], off, 64));
    roi[1] = min(roi[1], __shfl_xor(roi[1], off, 64));
    roi[2] = max(roi[2], __shfl_xor(roi[2], off, 64));
    roi[3] = max(roi[3], __shfl_xor(roi[3], off, 64));
  }
  if (lane == 0 && roi[2] >= 0) {
    atomicMin(&s_roi[0], roi[0]);
    atomicMin(&s_roi[1], roi[1]);
    atomicMax(&s_roi[2], roi[2]);
    atomicMax(&s_roi[3], roi[3]);
  }
  // Both q tiles start at 0 once per tuple; afterwards the pixel pass zeroes
  // every pixel it reads (the only ones the raster can have written), so the
  // tiles are clean for the next tile without a separate clearing pass.
  for (int i = tid; i < 2 * kTileStride * kTileH; i += NTH) (&s_dep[0][0])[i] = 0u;
  __syncthreads();
  // render mode: the ROI its q buffer was sized for (launch_pose_roi, the same
  // rule), so every write lands inside the buffer
  int4 rroi = make_int4(0, 0, -1, -1);
  if constexpr (COST == kCostRender) rroi = a.rois[b];
  const int rx0 = COST == kCostRender ? rroi.x : s_roi[0];
  const int ry0 = COST == kCostRender ? rroi.y : s_roi[1];
  const int rx1 = COST == kCostRender ? rroi.z : s_roi[2];
  const int ry1 = COST == kCostRender ? rroi.w : s_roi[3];
  // automatic mode also asks for meshlets dense on screen: >= kCullAutoDensity
  // per ROI tile (a 30k-triangle object drawn large, 10 per tile, loses 1 %)
  const int roi_tiles = rx0 <= rx1 && ry0 <= ry1
                            ? ((rx1 - rx0 + kTileW) / kTileW) * ((ry1 - ry0 + kTileH) / kTileH)
                            : 0;
  const bool cull_back = cull_maybe && (a.cull == 3 || nm >= kCullAutoDensity * roi_tiles);
  // far half of each pose's depth range (wave-uniform thresholds)
  uint32_t far_bits = 0;
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = ebase + tid + j * NTH;
    const int r = i >= nm;
    const float zmid = 0.5f * (s_zr[r][0] + s_zr[r][1]);
    far_bits |= (uint32_t)(zmin[j] > zmid) << j;
  }
  if (cull_back) {
    // back-facing entries take the "far" bit (tested, queued last); their
    // bound as a conservative code: 2^(-code/64) >= qb / qhi (log/exp2 errors
    // ~1e-6 against the 0.05 / 64 slack), clamped to [0, 255] (still >= qb)
    far_bits = back_bits;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int i = tid + j * NTH;
      if ((back_bits >> j) & 1u) {
        const float qhi = s_qhi[ebase + i >= nm];
        const float cf = floorf(64.0f * (__log2f(qhi) - __log2f(qbv[j])) - 0.05f);
        s_qb[i] = (uint8_t)fminf(fmaxf(cf, 0.0f), 255.0f);
      }
    }
  }
  // float32 step thresholds of the filter (wave-uniform, SGPRs); the exact
  // path reads the float64 ones from s_thr
  float thr32[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k)
    thr32[k] = __int_as_float(
        __builtin_amdgcn_readfirstlane(__float_as_int(COST == 0 ? filt_thr(s_thr[k]) : 0.0f)));
  const bool filter = COST == 0 && !divide;

  uint32_t c_union = 0, c_inter = 0, c_valid = 0;
  // cover mode: est / gt silhouette bboxes (x0, y0, x1, y1), empty = (INT_MAX, INT_MAX, -1, -1)
  int bb[8] = {INT32_MAX, INT32_MAX, -1, -1, INT32_MAX, INT32_MAX, -1, -1};
  // step cost: two 16-bit per-tau counters per register (a lane evaluates at
  // most kTileW * kTileH / NTH pixels per tile, <= kVsdMaxTiles tiles)
  uint32_t c_tau[(NT + 1) / 2];
  double lin[kMaxTaus];
#pragma unroll
  for (int k = 0; k < kMaxTaus; ++k) {
    if (k < (NT + 1) / 2) c_tau[k] = 0;
    lin[k] = 0.0;
  }

  if (rx0 <= rx1 && ry0 <= ry1) {
    const int ntx = (rx1 - rx0 + kTileW) / kTileW, nty = (ry1 - ry0 + kTileH) / kTileH;
    if (VSD_DIAG(4) && tid == 0) atomicAdd(&g_vsd_stats[0], (unsigned long long)(ntx * nty));
    VSD_STAMP(6);
    // 2a. list the (pose, meshlet) entries touching tile tt into queue qb (the
    // q tiles are already zero, see the pixel pass): each thread its kR
    // rectangles (kStream: round e0, recomputed)
    auto list_tile = [&](int tt, int qb, int e0) {
      VSD_WAVE(10, 1);
      const int lx0 = rx0 + (tt % ntx) * kTileW, ly0 = ry0 + (tt / ntx) * kTileH;
      const int lx1 = min(lx0 + kTileW - 1, rx1), ly1 = min(ly0 + kTileH - 1, ry1);
#pragma unroll
      for (int j = 0; j < kR; ++j) {
        short4 rc;
        if constexpr (kStream) {  // recomputed (round e0, entry e0 + tid + 512 j)
          const int i = e0 + tid + j * NTH;
          rc = make_short4(1, 1, 0, 0);
          if (i < 2 * nm && !((COST == kCostGtInfo || COST == kCostRender) && i < nm)) {
            const int r = i >= nm, m = i - r * nm;
            float zm, qq;
            bool bk;
            rc = meshlet_rect(g_mlet + kMletFloats * (int64_t)m, s_pose[r], c32, W, H, zm, qq, bk);
          }
        } else {
          rc = rect[j];
        }
        if (rc.x <= lx1 && rc.z >= lx0 && rc.y <= ly1 && rc.w >= ly0 && rc.x <= rc.z &&
            rc.y <= rc.w) {
          const uint32_t far = (far_bits >> j) & 1u;
          ListT word = (ListT)(tid + j * NTH);
          if constexpr (kCull) {
            const uint32_t x0 = (uint32_t)(max((int)rc.x, lx0) - lx0) >> 1;
            const uint32_t x1 = (uint32_t)(min((int)rc.z, lx1) - lx0) >> 1;
            const uint32_t y0 = (uint32_t)(max((int)rc.y, ly0) - ly0) >> 1;
            const uint32_t y1 = (uint32_t)(min((int)rc.w, ly1) - ly0) >> 1;
            word |= (far << 11) | (x0 << 12) | (x1 << 17) | (y0 << 22) | (y1 << 27);
          }
          bool front = !far;
          if (a.qorder && !cull_back) {
            const int ow = min((int)rc.z, lx1) - max((int)rc.x, lx0) + 1;
            const int oh = min((int)rc.w, ly1) - max((int)rc.y, ly0) + 1;
            front = ow * oh >= kLptOverlap;
          }
          if (front)
            s_lists[qb][atomicAdd(&s_nlists[qb], 1)] = word;
          else
            s_lists[qb][kListLen - 1 - atomicAdd(&s_nsmalls[qb], 1)] = word;
        }
      }
    };
    // 2b. one tile's raster into the q tile pair D, claims from queue qb
    auto raster_tile = [&](const int t, const int it, const int qb,
                           uint32_t(*const D)[kTileStride * kTileH]) {
      const int tx0 = rx0 + (t % ntx) * kTileW, ty0 = ry0 + (t / ntx) * kTileH;
      const int tx1 = min(tx0 + kTileW - 1, rx1), ty1 = min(ty0 + kTileH - 1, ry1);
      VSD_WAVE(11, 1);
      ListT* const s_list = s_lists[qb];
      int* const p_nlist = &s_nlists[qb];
      int* const p_nsmall = &s_nsmalls[qb];
      int* const p_next = &s_nexts[qb];
      // The queue counters were reset behind the previous tile's raster-end
      // barrier (or before the loop). list-ahead: this tile was listed in the
      // previous tile's raster tail (the first one here), no barrier of its own.
      // kStream: one round per kListLen entries (a single round otherwise)
      for (int e0 = 0; e0 < (kStream ? 2 * nm : 1); e0 += kListLen) {
      if (kStream && e0 > 0) __syncthreads();  // every wave is done with the last round's queue
      if (!kAhead || kStream) {
        if (tid == 0) {
          *p_nlist = 0;
          *p_nsmall = 0;
          *p_next = (NW * kGroup);
        }
        __syncthreads();
      }
      VSD_STAMP(0);
      if (!kAhead || it == 0) {
        list_tile(t, qb, e0);
        __syncthreads();
      }
      VSD_STAMP(1);
      // 2b. rasterise. Waves pull groups of kGroup (pose, meshlet) entries from a
      // shared counter (dynamic balance). Per group: the wave transforms the
      // three fixed-stride vertex blocks once (lane = vertex) into LDS, tests
      // every triangle's bbox against the tile, compacts the hits (ballot rank)
      // and only then sets up and rasterises them, one triangle per lane.
      const int nnear = __builtin_amdgcn_readfirstlane(*p_nlist);
      const int nl = __builtin_amdgcn_readfirstlane(VSD_DIAG(1) ? 0 : *p_nlist + *p_nsmall);
      // each wave's first group is pre-assigned (wave-th group of the queue),
      // the rest are claimed from s_next, which starts past them
      for (int claimed = 0;; claimed = 1) {
        int base = wave * kGroup;
        if (claimed) {
          if (lane == 0) base = atomicAdd(p_next, kGroup);
          base = __builtin_amdgcn_readfirstlane(base);
        }
        VSD_STAMP(12);
        VSD_WAVE(0, 1);
        if (base >= nl) break;
        if (base + kGroup * NW >= nl) __builtin_amdgcn_s_setprio(kVsdPrio);
        f32x3 v[kGroup];
        uint32_t pk[kGroup];
        int pose[kGroup];
        int ent[kGroup];
        uint32_t word[kGroup];
        // both queue words in flight before the first wait (distinct registers)
        uint32_t wv[kGroup];
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
          const int q = min(base + g, nl - 1);
          wv[g] = (uint32_t)s_list[q < nnear ? q : kListLen - 1 - (q - nnear)];
        }
#pragma unroll
        for (int g = 0; g < kGroup; ++g) word[g] = __builtin_amdgcn_readfirstlane(wv[g]);
        int mlt[kGroup];
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
          ent[g] = (kStream ? e0 : 0) + (int)(word[g] & 0x7FFu);  // queue index (s_qb)
          const int e = ebase + ent[g];
          pose[g] = e >= nm ? 1 : 0;  // uniform (SGPR): e came through readfirstlane
          mlt[g] = e - pose[g] * nm;
        }
        // Back-face occlusion test (cull 3), before any of the entry's data is
        // fetched: skipped when every pixel of its rectangle in the tile already
        // holds q >= its fragment bound. q values only grow, so a value read
        // while other waves still write is a lower bound of the final one.
        uint32_t dead = 0;  // wave-uniform: bit g = entry g skipped
        if constexpr (kCull) {
          if (cull_back) {
#pragma unroll
            for (int g = 0; g < kGroup; ++g) {
              if (base + g >= nl) {
                dead |= 1u << g;
              } else if ((word[g] >> 11) & 1u) {
                const float qbd = s_qhi[pose[g]] *
                                  __builtin_amdgcn_exp2f(-(float)s_qb[ent[g]] * (1.0f / 64.0f));
                const Region rg = make_region(word[g], tx1 - tx0 + 1, ty1 - ty0 + 1);
                if (region_covered(D[pose[g]], rg, 0, __float_as_uint(qbd), lane)) {
                  dead |= 1u << g;
                  if (VSD_DIAG(4) && lane == 0) atomicAdd(&g_vsd_stats[9], 1ull);
                }
              }
            }
            if (dead == (1u << kGroup) - 1u) continue;  // nothing left to draw
          }
        }
        // all loads of the group in flight before the first use
#pragma unroll
        for (int g = 0; g < kGroup; ++g)
          v[g] = ld_off(g_mvtx3 + mlt[g] * kMeshletVerts, (uint32_t)lane * 16u);
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
          pk[g] = ld_off(g_mtri + mlt[g] * kMeshletTris, (uint32_t)lane * 4u);  // entry is valid
          // (clamped duplicate or occluded: no triangles)
          if (base + g >= nl || ((dead >> g) & 1u)) pk[g] = 0xFFFFFFFFu;
        }
        // occlusion test of far entries, part 1: the q reads of the region's
        // first 8 steps go out now, behind the vertex loads, and are compared
        // once the vertex 1/Z maximum is known (after the staging)
        uint32_t qmin[kGroup];
        bool test[kGroup];
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
          qmin[g] = 0xFFFFFFFFu;
          test[g] = false;
          if constexpr (kCull) {
            test[g] = (a.cull == 1 || a.cull == 2) && ((word[g] >> 11) & 1u) && base + g < nl;
            if (test[g])
              qmin[g] = region_min8(D[pose[g]],
                                    make_region(word[g], tx1 - tx0 + 1, ty1 - ty0 + 1), 0, lane);
          }
        }
        if (VSD_DIAG(8)) {  // diagnostics: time the vertex-block loads alone
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          VSD_STAMP(13);
        }
        float izl[kGroup];  // this lane's vertex 1/Z (0 for an invalid vertex)
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
          // 3 x ds_read_b128 of the pose in pair order (X and Y in packed ops)
          const RVtx rv = r_vertex_pk(&s_pose_pk[pose[g]][0], c32, v[g].x, v[g].y, v[g].z);
          w_stage[g * kMeshletVerts + lane] = rv;
          izl[g] = rv.iz;
        }
        wave_lds_sync();
        VSD_STAMP(8);
        if constexpr (kCull) {
          // occlusion test of the far entries (see kLptOverlap above)
#pragma unroll
          for (int g = 0; g < kGroup; ++g) {
            if (test[g]) {
              const uint32_t qb =
                  __float_as_uint(wave_max_nonneg_f32(izl[g]) * 1.00390625f);  // (1 + 2^-8) izmax
              if (__builtin_amdgcn_ballot_w64(qmin[g] < qb) == 0) {
                // first 8 blocks covered; a larger region continues from block 8
                const Region rg = make_region(word[g], tx1 - tx0 + 1, ty1 - ty0 + 1);
                if (rg.nb <= 8 || region_covered(D[pose[g]], rg, 8, qb, lane)) {
                  if (a.cull == 1) pk[g] = 0xFFFFFFFFu;  // no triangle of it can change the tile
                  if (VSD_DIAG(4) && lane == 0) atomicAdd(&g_vsd_stats[9], 1ull);
                }
              }
            }
          }
          VSD_STAMP(14);
        }
        int cnt = 0;
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
          // branch-free: a lane without a triangle (pk = ~0) tests vertex 0 three
          // times and is masked out, so the hit mask feeds the ballot directly
          const bool has = pk[g] != 0xFFFFFFFFu;
          const uint32_t pkg = has ? pk[g] : 0u;
          const RVtx* sg = &w_stage[g * kMeshletVerts];
          const bool hit = has & r_touches(sg[pkg & 255u], sg[(pkg >> 8) & 255u],
                                           sg[(pkg >> 16) & 255u], tx0, tx1, ty0, ty1);
          const unsigned long long bal = __ballot(hit);
          if (hit)
            w_tri[cnt + __popcll(bal & ((1ull << lane) - 1ull))] =
                (pk[g] & 0xFFFFFFu) | ((uint32_t)g << 24) | ((uint32_t)pose[g] << 26);
          cnt += __popcll(bal);
        }
        wave_lds_sync();
        if (VSD_DIAG(4) && lane == 0) atomicAdd(&g_vsd_stats[1], (unsigned long long)kGroup);
        VSD_STAMP(9);
        for (int c0 = 0; c0 < (VSD_DIAG(64) ? 0 : cnt); c0 += 64) {
          VSD_WAVE(1, 1);
          // Set-up, one triangle per lane.
          RTri T;
          bool ok = false;
          int r = 0, cc0 = 0, cc1 = -1, rr0 = 0, rr1 = -1;
          if (c0 + lane < cnt) {
            const uint32_t ref = w_tri[c0 + lane];
            const RVtx* sg = &w_stage[((ref >> 24) & 3u) * kMeshletVerts];
            r = (int)(ref >> 26);
            ok = r_setup_touching(sg[ref & 255u], sg[(ref >> 8) & 255u], sg[(ref >> 16) & 255u],
                                  T);  // passed r_touches in the compaction
            if (ok) {
              cc0 = max(T.c0, tx0);
              cc1 = min(T.c1, tx1);
              rr0 = max(T.r0, ty0);
              rr1 = min(T.r1, ty1);
            }
          }
          VSD_STAMP(10);
          if VSD_DIAG(4) {
            if (ok) {
              atomicAdd(&g_vsd_stats[2], 1ull);
              atomicAdd(&g_vsd_stats[3], (unsigned long long)(cc1 - cc0 + 1) * (rr1 - rr0 + 1));
            }
            if (ok && T.small && T.regular)
              atomicAdd(&g_vsd_stats[4], (unsigned long long)(rr1 - rr0 + 1));
          }
          // extent >= 128 px (int64 edges) or an irregular sliver (clamped q):
          // walked by its own lane with the full spec arithmetic (r_raster)
          const bool fast = T.small & T.regular;
          if VSD_DIAG(4) {
            if (ok && !fast) {
              atomicAdd(&g_vsd_stats[10], 1ull);
              atomicAdd(&g_vsd_stats[11], (unsigned long long)(cc1 - cc0 + 1) * (rr1 - rr0 + 1));
              if (!T.small) atomicAdd(&g_vsd_stats[13], 1ull);
            }
            if (lane == 0 && __builtin_amdgcn_ballot_w64(ok && !fast) != 0)
              atomicAdd(&g_vsd_stats[12], 1ull);
#if BOPX_VSD_DIAG
            const bool slow = ok && !fast;
            const int sr = diag_wave_max(slow ? rr1 - rr0 + 1 : 0);
            const int sc = diag_wave_max(slow ? (rr1 - rr0 + 1) * (cc1 - cc0 + 1) : 0);
            VSD_WAVE(8, sc);
            VSD_WAVE(9, sr);
            VSD_WAVE(12, sr > 0);
#endif
          }
          if (ok && !fast) {
            uint32_t* dep = D[r];
            r_raster(T, cc0, cc1, rr0, rr1, [&](int col, int row, float q) {
              if VSD_DIAG(4) atomicAdd(&g_vsd_stats[5], 1ull);
              atomicMax(&dep[(row - ty0) * kTileStride + (col - tx0)], __float_as_uint(q));
            });
          }
          // Row items: publish one record per small triangle, number its rows
          // (wave prefix sum), then deal the rows out one per lane.
          const bool rows = ok && fast;
          const int h = rows ? rr1 - rr0 + 1 : 0;
          const int inc = wave_incl_scan(h);
          const int first = inc - h;
          const int nrow = __builtin_amdgcn_readlane(inc, 63);
          // records compacted by rank among the row-owning lanes (ascending first)
          const uint64_t rbal = __builtin_amdgcn_ballot_w64(rows);
          if (rows)
            r_make_row(T, cc0, cc1, rr0, tx0, ty0, r, first,
                       s_rec[wave][__builtin_amdgcn_mbcnt_hi(
                           (uint32_t)(rbal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rbal, 0u))]);
          int rec_last = -1;  // the last record started before the current pass
          for (int wb = 0; wb < (VSD_DIAG(32) ? 0 : nrow); wb += kRowWin) {
            VSD_WAVE(2, 1);
            wave_lds_sync();  // records written / previous window's owners consumed
            // one start flag per record instead of one owner byte per row item
            reinterpret_cast<uint32_t*>(&s_own[wave][0])[lane] = 0u;
            wave_lds_sync();
            // transposed: item i's flag at byte 4 (i % 64) + i / 64, so one dword
            // read per lane holds its flags for the window's four passes
            if (rows && first >= wb && first < wb + kRowWin)
              s_own[wave][(((first - wb) & 63) << 2) | ((first - wb) >> 6)] = 1u;
            wave_lds_sync();
            const int wn = min(nrow - wb, kRowWin);
            // item p's record: the last one that starts at or before p, i.e. the
            // start flags up to p (ballot + mbcnt) past those of earlier passes
            const uint32_t fl4 = reinterpret_cast<const uint32_t*>(&s_own[wave][0])[lane];
            for (int p0 = 0; p0 < wn; p0 += 64) {
              const int p = p0 + lane;
              const bool valid = p < wn;
              const uint64_t M = __builtin_amdgcn_ballot_w64(((fl4 >> (p0 >> 3)) & 0xFFu) != 0u) &
                                 __builtin_amdgcn_ballot_w64(valid);
              // flags at or below the lane: bit 0 (scalar) + those of M >> 1 below it
              const uint64_t Mh = M >> 1;
              const int owner = rec_last + (int)(M & 1u) +
                                (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(Mh >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)Mh, 0u));
              rec_last += __popcll(M);
              VSD_WAVE(3, 1);
#if BOPX_VSD_DIAG
              if VSD_DIAG(4) {
                const int wl = valid ? (int)(s_rec[wave][owner].meta >> 25) + 1 : 0;
                VSD_WAVE(4, diag_wave_max((wl + 1) >> 1));
              }
#endif
              if (valid) {
                // the 48-B record as three 16-B LDS reads
                RRow rec;
                {
                  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                  const u32x4* src = reinterpret_cast<const u32x4*>(&s_rec[wave][owner]);
                  u32x4* dst = reinterpret_cast<u32x4*>(&rec);
                  const u32x4 r0 = src[0], r1 = src[1], r2 = src[2];
                  dst[0] = r0;
                  dst[1] = r1;
                  dst[2] = r2;
                }
                const int fr =
                    VSD_DIAG(16) ? r_walk_row_max<true, kWalkMasked>(rec, wb + p - (int)(rec.pyf & 0xFFFFu),
                                                        D[0])
                                 : r_walk_row_max<false, kWalkMasked>(rec, wb + p - (int)(rec.pyf & 0xFFFFu),
                                                  D[0]);
                if VSD_DIAG(4) atomicAdd(&g_vsd_stats[5], (unsigned long long)fr);
              }
            }
          }
          VSD_STAMP(11);
          wave_lds_sync();  // records are rewritten by the next chunk
        }
        wave_lds_sync();  // the staging area is rewritten by the next group
      }
      }  // rounds (kStream)
    };
    auto touch_rows = [&](const int t) -> float {
      // Touch the test-depth lines of this wave's pixel rows (w, w + 8, ...)
      // while it waits for the other waves at the raster-end barrier: the
      // pixel pass then reads them from L2 instead of HBM. The empty asm below
      // consumes the value (the only wait for these loads).
      const int tx0 = rx0 + (t % ntx) * kTileW, ty0 = ry0 + (t / ntx) * kTileH;
      const int tx1 = min(tx0 + kTileW - 1, rx1), ty1 = min(ty0 + kTileH - 1, ry1);
      const gptr<const float> tframe = frame + ((int64_t)ty0 * IW + tx0);
      float touch = 0.0f;
      if constexpr (COST == 0 || COST == 1) {
        if (lane < 3 * (kTileH / NW)) {
          const int row = ty0 + wave + NW * (lane / 3), k = lane % 3;
          const int col = k == 0 ? tx0 : (k == 1 ? min(tx0 + 32, tx1) : tx1);
          if (row <= ty1)
            touch = ld_off(tframe, (uint32_t)(__mul24(row - ty0, IW) + (col - tx0)) * 4u);
        }
      }
      (void)ty1;
      return touch;
    };
    auto coeffs = [&](const int t) {
      const int tx0 = rx0 + (t % ntx) * kTileW, ty0 = ry0 + (t / ntx) * kTileH;
      // float64 distance coefficients of the tile's columns / rows (misc.py:137-138),
      // per wave into its scratch (its staging area is dead until the next
      // tile), computed before the raster-end barrier while other waves finish
      for (int i = lane; i < kTileW; i += 64) {
        const double pX = ((double)(tx0 + i - ox) - cx) / fx;
        w_pX[i] = pX;
        if constexpr (COST == 0) w_fA[i] = filt_a(pX);
      }
      for (int i = lane; i < kTileH; i += 64) {
        const double pY = ((double)(ty0 + i - oy) - cy) / fy;
        w_pY[i] = pY;
        if constexpr (COST == 0) w_fB[i] = filt_b(pY);
      }
    };
    // 3. one tile's pixel pass over the q tile pair D (this wave's rows)
    auto pixel_tile = [&](const int t, uint32_t(*const D)[kTileStride * kTileH]) {
      const int tx0 = rx0 + (t % ntx) * kTileW, ty0 = ry0 + (t / ntx) * kTileH;
      const int tx1 = min(tx0 + kTileW - 1, rx1), ty1 = min(ty0 + kTileH - 1, ry1);
      const gptr<const float> tframe = frame + ((int64_t)ty0 * IW + tx0);
      // 3. per-pixel distances, visibility masks, counters. Each wave first
      // compacts its covered pixels (rows wave, wave + 8, ...) into its own
      // list (ballot rank; the raster records are dead here), then evaluates
      // the list with full lanes. Wave-private: no block barrier, and the
      // pixel -> lane assignment is fixed (deterministic float64 sums).
      uint16_t* pix = reinterpret_cast<uint16_t*>(&s_rec[0][0]) + wave * kPixPW;
      int npix = 0;
      {
        // lane = column, one wave-uniform tile row per step (rows w, w + 8, ...)
        static_assert(kTileW == 64, "pixel compaction maps lanes to tile columns");
        const int nrow = VSD_DIAG(2) ? 0 : ty1 - ty0 + 1;
        const bool col_in = tx0 + lane <= tx1;
        // column right of a tile cut by the ROI: the row walk may have written
        // it (r_walk_row_max); cleared here (wave-private rows, raster done)
        const int cut = tx1 - tx0 + 1;
        VSD_WAVE(5, nrow > wave ? (nrow - wave + NW - 1) / NW : 0);
        for (int r = wave; r < nrow; r += NW) {
          if (cut < kTileW && lane < 2) D[lane][r * kTileStride + cut] = 0u;
          const int ps = r * kTileStride + lane;
          const bool cov = col_in & ((D[0][ps] | D[1][ps]) != 0u);
          const unsigned long long bal = __ballot(cov);
          if constexpr (COST == kCostRender) {  // the row's covered column span
            if (bal != 0ull && lane == 0) {
              const int64_t ri = a.rowoff[b] + (ty0 + r - ry0);
              atomicMin(&a.smin[ri], tx0 + (int)__builtin_ctzll(bal));
              atomicMax(&a.smax[ri], tx0 + 63 - (int)__builtin_clzll(bal));
            }
          }
          const int rank = (int)__builtin_amdgcn_mbcnt_hi(
              (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          if (cov) pix[npix + rank] = (uint16_t)(r * kTileW + lane);
          npix += __popcll(bal);
        }
      }
      wave_lds_sync();
      // step cost: the certified float32 filter, the exact float64 sequence for
      // the pixels it cannot decide (and for every pixel of a tuple with a
      // pathological diameter / tau, `divide`)
      auto dt_of = [&](int p) {
        return ld_off(tframe, (uint32_t)(__mul24(p >> 6, IW) + (p & 63)) * 4u);
      };
      auto step_exact = [&](int p, uint32_t qe, uint32_t qg, float dtest) {
        bool vg, ve;
        double dd;
        vsd_exact_px(w_pX[p % kTileW], w_pY[p / kTileW], qe, qg, dtest, a.dthr, vg, ve, dd);
        c_union += (vg || ve);
        if (vg && ve) {
          ++c_inter;
          if (divide) {  // rare: a real branch, not a speculated division
            dd /= diam;
            asm volatile("" : "+v"(dd));
          }
#pragma unroll
          for (int k = 0; k < NT; ++k)
            c_tau[k >> 1] += (uint32_t)(dd >= s_thr[k]) << (16 * (k & 1));
        }
      };
      auto vsd_px = [&](int p, uint32_t qe, uint32_t qg, float dtest) {
        if constexpr (COST == 0) {
          if (!filter) {
            step_exact(p, qe, qg, dtest);
            return;
          }
          bool vg, ve;
          float lo, hi;
          bool unc = vsd_filter_px(w_fA[p % kTileW] + w_fB[p / kTileW], qe, qg, dtest, a.dthr,
                                   vg, ve, lo, hi);
          const bool in = vg & ve;
          c_union += vg | ve;
          c_inter += in;
#pragma unroll
          for (int k = 0; k < NT; ++k) {
            const bool ge_lo = in & (lo >= thr32[k]), ge_hi = in & (hi >= thr32[k]);
            c_tau[k >> 1] += (uint32_t)ge_lo << (16 * (k & 1));
            unc |= ge_lo != ge_hi;
          }
          if (__builtin_expect(__builtin_amdgcn_ballot_w64(unc) != 0, 0)) {
            VSD_WAVE(7, 1);
            if (unc) {  // undo the float32 increments, redo the pixel exactly
              if VSD_DIAG(4) atomicAdd(&g_vsd_stats[14], 1ull);
              c_union -= vg | ve;
              c_inter -= in;
#pragma unroll
              for (int k = 0; k < NT; ++k)
                c_tau[k >> 1] -= (uint32_t)(in & (lo >= thr32[k])) << (16 * (k & 1));
              step_exact(p, qe, qg, dtest);
            }
          }
        } else {  // tlinear: float64 sums, exact sequence
          const float de = qe ? rcp_rn(__uint_as_float(qe)) : 0.0f;
          const float dg = qg ? rcp_rn(__uint_as_float(qg)) : 0.0f;
          const double pX = w_pX[p % kTileW];
          const double pY = w_pY[p / kTileW];
          const double dist_t = dist_of(pX, pY, dtest);
          const double dist_g = qg ? dist_of(pX, pY, dg) : 0.0;
          const double dist_e = qe ? dist_of(pX, pY, de) : 0.0;
          const bool vg = visib19t(dist_t, dist_g, a.dthr);
          bool ve = visib19t(dist_t, dist_e, a.dthr);
          ve = ve || (vg && dist_e > 0.0);  // visibility.py:74
          c_union += (vg || ve);
          if (vg && ve) {
            ++c_inter;
            double dd = fabs(dist_g - dist_e);
            if (a.normalized) dd /= a.diameters[b];
#pragma unroll
            for (int k = 0; k < kMaxTaus; ++k) {
              if (k < a.n_tau) {
                const double cst = dd / a.taus[k];
                lin[k] += cst > 1.0 ? 1.0 : cst;
              }
            }
          }
        }
      };
      VSD_WAVE(6, (npix + 63) / 64);
      for (int i = lane; i < npix; i += 64) {
        const int p = pix[i];
        const int row = ty0 + p / kTileW, col = tx0 + p % kTileW;
        const int ps = (p / kTileW) * kTileStride + p % kTileW;
        const uint32_t qe = D[0][ps], qg = D[1][ps];
        D[0][ps] = 0u;  // clean for the next tile (rows are wave-private here)
        D[1][ps] = 0u;
        if VSD_DIAG(4) atomicAdd(&g_vsd_stats[6], 1ull);
        if constexpr (COST == kCostRender) {  // the pose's q into its ROI buffer
          a.qbuf[a.qoff[b] + (int64_t)(row - ry0) * (rx1 - rx0 + 1) + (col - rx0)] = qg;
          continue;
        }
        if constexpr (COST == kCostCover) {  // silhouettes only (cus, cou_bb_proj)
          ++c_union;
          c_inter += (qe != 0u && qg != 0u);
          if (qe) {
            bb[0] = min(bb[0], col);
            bb[1] = min(bb[1], row);
            bb[2] = max(bb[2], col);
            bb[3] = max(bb[3], row);
          }
          if (qg) {
            bb[4] = min(bb[4], col);
            bb[5] = min(bb[5], row);
            bb[6] = max(bb[6], col);
            bb[7] = max(bb[7], row);
          }
          continue;
        }
        if constexpr (COST == kCostGtInfo) {  // calc_gt_info.py:113-158, calc_gt_masks.py:104-125
          ++c_union;  // px_count_all (whole canvas silhouette)
          const int x = col - ox, y = row - oy;
          bb[0] = min(bb[0], x);
          bb[1] = min(bb[1], y);
          bb[2] = max(bb[2], x);
          bb[3] = max(bb[3], y);
          if (x < 0 || y < 0 || x >= IW || y >= IH) continue;
          const double pX = w_pX[p % kTileW], pY = w_pY[p / kTileW];
          const double dist_g = dist_of(pX, pY, rcp_rn(__uint_as_float(qg)));
          const double dist_t = dist_of(pX, pY, frame[(int64_t)y * IW + x]);
          c_valid += dist_t > 0.0;
          const bool vis = visib19t(dist_t, dist_g, a.dthr);
          uint8_t* mk = a.masks ? a.masks + (2 * b) * (int64_t)IW * IH + (int64_t)y * IW + x
                                : nullptr;
          if (mk) mk[0] = 255u;
          if (vis) {
            ++c_inter;  // px_count_visib
            bb[4] = min(bb[4], x);
            bb[5] = min(bb[5], y);
            bb[6] = max(bb[6], x);
            bb[7] = max(bb[7], y);
            if (mk) mk[(int64_t)IW * IH] = 255u;
          }
          continue;
        }
        if constexpr (COST == 0 || COST == 1) vsd_px(p, qe, qg, dt_of(p));
      }
    };
    for (int t = sp, it = 0; t < ntx * nty; t += S, ++it) {
      const int qb = kAhead ? (it & 1) : 0;  // this tile's queue
      raster_tile(t, it, qb, s_dep);
      // list-ahead: this wave's share of the next tile's queue, while the other
      // waves finish rasterising (the raster-end barrier below publishes it)
      if constexpr (kAhead) {
        if (t + S < ntx * nty) list_tile(t + S, qb ^ 1, 0);
      }
      // Touch the test-depth lines of this wave's pixel rows while it waits for
      // the other waves at the raster-end barrier: the pixel pass then reads
      // them from L2 instead of HBM. The empty asm below consumes the value
      // (the only wait for these loads).
      const float touch = touch_rows(t);
      // float64 distance coefficients of the tile's columns / rows, per wave
      // into its scratch (its staging area is dead until the next tile),
      // computed before the raster-end barrier while other waves finish
      coeffs(t);
      VSD_STAMP(2);
      __syncthreads();
      __builtin_amdgcn_s_setprio(0);
      // every wave has read the queue counters (after the list barrier) and is
      // done with s_next: reset them for the next tile (ordered by the
      // pixel-end barrier)
      if (kAhead && tid == 0) {
        s_nlists[qb] = 0;
        s_nsmalls[qb] = 0;
        s_nexts[qb] = NW * kGroup;
      }
      asm volatile("" ::"v"(touch));
      VSD_STAMP(3);
      pixel_tile(t, s_dep);
      VSD_STAMP(4);
      __syncthreads();
      VSD_STAMP(5);
    }
  }

  if constexpr (COST == kCostRender) return;  // the q buffer is the output
  // 4. workgroup reduction (fixed order) and the error formula (pose_error.py:75-91).
  __syncthreads();  // s_cnt / s_lin alias the depth tiles
  c_union = wave_sum_u32(c_union);
  c_inter = wave_sum_u32(c_inter);
  uint32_t tau_sum[kMaxTaus];
#pragma unroll
  for (int k = 0; k < kMaxTaus; ++k) {
    tau_sum[k] = 0;
    if (COST == 0) {
      if (k < NT) tau_sum[k] = wave_sum_u32((c_tau[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
    } else {
      lin[k] = wave_sum_f64(lin[k]);
    }
  }
  if (lane == 0) {
    s_cnt[wave][0] = c_union;
    s_cnt[wave][1] = c_inter;
#pragma unroll
    for (int k = 0; k < kMaxTaus; ++k) {
      s_cnt[wave][2 + k] = tau_sum[k];
      s_lin[wave][k] = lin[k];
    }
  }
  if constexpr (COST == kCostCover || COST == kCostGtInfo) {
    c_valid = wave_sum_u32(c_valid);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      for (int off = 32; off > 0; off >>= 1) {
        const int o = __shfl_xor(bb[k], off, 64);
        bb[k] = (k & 2) ? max(bb[k], o) : min(bb[k], o);
      }
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) s_cnt[wave][2 + k] = (uint32_t)bb[k];
    if (lane == 0) s_cnt[wave][10] = c_valid;
  }
  __syncthreads();
  VSD_STAMP(7);
  if (VSD_DIAG(8) && lane == 0)
    for (int k = 0; k < 16; ++k) atomicAdd(&g_vsd_time[k], ph[k]);
  if (tid == 0) {
    uint64_t un = 0, in = 0;
    for (int w = 0; w < NW; ++w) {
      un += s_cnt[w][0];
      in += s_cnt[w][1];
    }
    if constexpr (COST == kCostCover || COST == kCostGtInfo) {
      // cover: union, inter, 8 bbox values; GT info: all, visib, 8 bbox values, valid
      // tile-parallel mode: the same columns as a partial row (k_vsd_combine)
      double* out = S > 1 ? a.part + (j * S + sp) * kVsdPartCols
                          : a.out + b * (int64_t)(COST == kCostCover ? kCoverCols : kGtInfoCols);
      out[0] = (double)un;
      out[1] = (double)in;
      if (COST == kCostGtInfo) {
        uint64_t valid = 0;
        for (int w = 0; w < NW; ++w) valid += s_cnt[w][10];
        out[10] = (double)valid;
      }
      for (int k = 0; k < 8; ++k) {
        int v = (int)s_cnt[0][2 + k];
        for (int w = 1; w < NW; ++w) {
          const int o = (int)s_cnt[w][2 + k];
          v = (k & 2) ? max(v, o) : min(v, o);
        }
        out[2 + k] = (double)v;
      }
      if (over)  // capacity guard (above)
        for (int k = 0; k < (S > 1 ? kVsdPartCols : COST == kCostCover ? kCoverCols : kGtInfoCols);
             ++k)
          out[k] = __builtin_nan("");
      return;
    }
    if (S > 1) {  // partial row of this split; k_vsd_combine applies the formula
      double* row = a.part + (j * S + sp) * kVsdPartCols;
      row[0] = (double)un;
      row[1] = (double)in;
      for (int k = 0; k < a.n_tau; ++k) {
        uint64_t cnt = 0;
        double sum = 0.0;
        for (int w = 0; w < NW; ++w) {
          cnt += s_cnt[w][2 + k];
          sum += s_lin[w][k];
        }
        row[2 + k] = (double)cnt;
        row[2 + kMaxTaus + k] = sum;
      }
      if (over) row[0] = __builtin_nan("");  // k_vsd_combine: NaN union -> NaN errors
      return;
    }
    double* out = a.out + b * (int64_t)a.n_tau;
    if (a.unions) a.unions[b] = (double)un;
    for (int k = 0; k < a.n_tau; ++k) {
      if (un == 0) {
        out[k] = 1.0;
      } else if (COST == 0) {
        uint64_t cnt = 0;
        for (int w = 0; w < NW; ++w) cnt += s_cnt[w][2 + k];
        out[k] = (double)(cnt + (un - in)) / (double)un;
      } else {
        double sum = 0.0;
        for (int w = 0; w < NW; ++w) sum += s_lin[w][k];
        out[k] = (sum + (double)(un - in)) / (double)un;
      }
      if (over) out[k] = __builtin_nan("");  // capacity guard (above)
    }
    if (over && a.unions) a.unions[b] = __builtin_nan("");
  }
}


hipError_t read_vsd_stats(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vsd_stats), sizeof(g_vsd_stats));
  if (e == hipSuccess)
    e = hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(g_vsd_time), sizeof(g_vsd_time));
  if (e == hipSuccess)
    e = hipMemcpyFromSymbol(out + 32, HIP_SYMBOL(g_vsd_wave), sizeof(g_vsd_wave));
  if (e != hipSuccess || !reset) return e;
  unsigned long long z[16] = {};
  e = hipMemcpyToSymbol(HIP_SYMBOL(g_vsd_stats), z, sizeof(g_vsd_stats));
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_vsd_time), z, sizeof(z));
  return e == hipSuccess ? hipMemcpyToSymbol(HIP_SYMBOL(g_vsd_wave), z, sizeof(z)) : e;
}

constexpr int kBopTaus = 10;  // eval_calc_errors.py:47, np.arange(0.05, 0.51, 0.05)

// Tile-parallel mode, second pass: one workgroup per tuple stages its split
// rows in LDS (one round of loads, not a dependent chain per row), then thread
// k sums tau k's rows in split order (counts exact in float64; tlinear sums in
// a fixed order) and applies pose_error.py:85-91 like the one-workgroup path.
constexpr int kCombineThreads = 256;
__global__ __launch_bounds__(kCombineThreads) void k_vsd_combine(
    int S, int n_tau, int cost_type, const double* __restrict__ part, double* __restrict__ out,
    const int32_t* __restrict__ order, int64_t n0, double* __restrict__ unions) {
  __shared__ double s_row[kVsdMaxSplit * kVsdPartCols];
  const int64_t j = blockIdx.x, kb = n0 + j;  // split tuple j of the launch order
  const int64_t b = order ? (int64_t)order[kb] : kb;
  const double* row = part + j * S * kVsdPartCols;
  for (int i = threadIdx.x; i < S * kVsdPartCols; i += kCombineThreads) s_row[i] = row[i];
  __syncthreads();
  const int k = threadIdx.x;
  if (cost_type == kCostCover || cost_type == kCostGtInfo) {
    // counts summed (exact), bounding boxes min / max (empty = INT_MAX, -1)
    const int cols = cost_type == kCostCover ? kCoverCols : kGtInfoCols;
    if (k >= cols) return;
    double v = s_row[k];
    for (int s = 1; s < S; ++s) {
      const double o = s_row[s * kVsdPartCols + k];
      if (k < 2 || k == 10) v += o;
      else v = ((k - 2) & 2) ? fmax(v, o) : fmin(v, o);
    }
    out[b * cols + k] = v;
    return;
  }
  if (k >= n_tau) return;
  double un = 0.0, in = 0.0, acc = 0.0;
  const int col = (cost_type == 0 ? 2 : 2 + kMaxTaus) + k;
  for (int s = 0; s < S; ++s) {
    un += s_row[s * kVsdPartCols];
    in += s_row[s * kVsdPartCols + 1];
    acc += s_row[s * kVsdPartCols + col];
  }
  out[b * n_tau + k] = un == 0.0 ? 1.0 : (acc + (un - in)) / un;
  if (unions && k == 0) unions[b] = un;
}

// Workgroups per tuple: batches of fewer than kVsdSplitBelow tuples split each
// tuple's ROI tiles over S = clamp(kVsdSplitTarget / n, 4, 16) workgroups, so
// the last tuples' tiles spread over the CUs instead of trailing;
// BOPX_VSD_SPLIT=k forces k (1 = off). Every cost mode (VSD, silhouette
// cover, GT info: each ROI tile and its mask pixels belong to one split). Measured
// (tools/split_sweep.py, wall ms per bopx_vsd_batch call, 5k-vertex object,
// profiles/r02_split/split_sweep.jsonl) — best S per batch size: 32-64 tuples
// 16, 128 8, 192-768 4 (768: S = 1 / 2 / 4 1.06 / 0.90 / 0.86 ms), 1,024 a tie
// (0.92 / 0.91 / 1.03), from 1,536 S = 1 (1.23 / 1.27 / 1.47; the 12,504-tuple
// bench: 9.38 / 10.0 / 11.4 ms for k_vsd).
constexpr int64_t kVsdSplitTarget = 1024;
constexpr int64_t kVsdSplitBelow = 1024;
// Large batches: the last BOPX_VSD_TAIL tuples of the launch order (the
// cheapest under the cost-class order) take kVsdTailSplit workgroups each, so
// the launch's tail drains in smaller pieces.
constexpr int kVsdTailSplit = 4;
static int vsd_split(int64_t n, int cost_type, int64_t& split_from) {
  static const int force = [] {
    const char* e = getenv("BOPX_VSD_SPLIT");
    return e ? atoi(e) : 0;
  }();
  static const int64_t tail = [] {
    const char* e = getenv("BOPX_VSD_TAIL");
    return e ? (int64_t)atoll(e) : (int64_t)0;
  }();
  split_from = 0;
  if (force > 0) return force < kVsdMaxSplit ? force : kVsdMaxSplit;
  if (n >= kVsdSplitBelow) {
    if (tail <= 0) return 1;
    split_from = tail < n ? n - tail : 0;
    return kVsdTailSplit;
  }
  const int64_t s = kVsdSplitTarget / n;
  return (int)(s < 4 ? 4 : s > kVsdMaxSplit ? kVsdMaxSplit : s);
}

template <int RPT>
static void launch_vsd_rpt(const VsdArgs& a, int cost_type, hipStream_t s) {
  dim3 grid((unsigned)(a.split_from + (a.n - a.split_from) * a.split)), block(kVsdThreads);
#if BOPX_VSD_DIAG
  // occupancy experiment (diag builds): unused dynamic LDS per workgroup
  static const unsigned dyn = [] {
    const char* e = getenv("BOPX_VSD_DYNLDS");
    return e ? (unsigned)atoi(e) : 0u;
  }();
#else
  constexpr unsigned dyn = 0;
#endif
  if (cost_type == 0 && a.n_tau <= kBopTaus)
    hipLaunchKernelGGL((k_vsd<0, RPT, kBopTaus>), grid, block, dyn, s, a);
  else if (cost_type == 0)
    hipLaunchKernelGGL((k_vsd<0, RPT, kMaxTaus>), grid, block, 0, s, a);
  else if (cost_type == 1)
    hipLaunchKernelGGL((k_vsd<1, RPT, kMaxTaus>), grid, block, 0, s, a);
  else if (cost_type == kCostCover)
    hipLaunchKernelGGL((k_vsd<kCostCover, RPT, kMaxTaus>), grid, block, 0, s, a);
  else if (cost_type == kCostRender)
    hipLaunchKernelGGL((k_vsd<kCostRender, RPT, kMaxTaus>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((k_vsd<kCostGtInfo, RPT, kMaxTaus>), grid, block, 0, s, a);
}

// rectangle registers per thread (RPT) for the largest registered object
static void launch_vsd_rpt_any(const VsdArgs& a, int cost_type, hipStream_t s) {
  // GT-info / render modes hold only the second pose's rectangles (kOnePose)
  const int need = (cost_type == kCostGtInfo || cost_type == kCostRender ? 1 : 2) * a.max_nm;
  if (need <= kVsdThreads)
    launch_vsd_rpt<1>(a, cost_type, s);
  else if (need <= 2 * kVsdThreads)
    launch_vsd_rpt<2>(a, cost_type, s);
  else if (need <= kRectsPerThread * kVsdThreads)
    launch_vsd_rpt<kRectsPerThread>(a, cost_type, s);
  else
    launch_vsd_rpt<0>(a, cost_type, s);  // rectangles recomputed per tile (any size)
}

hipError_t launch_vsd(const VsdArgs& a_in, int cost_type, hipStream_t s) {
  if (a_in.n <= 0) return hipSuccess;
  VsdArgs a = a_in;
  a.split = vsd_split(a.n, cost_type, a.split_from);
  a.part = nullptr;
  // render mode: the splits write disjoint tiles of the q buffer, nothing to combine
  if (a.split > 1 && cost_type == kCostRender) {
    launch_vsd_rpt_any(a, cost_type, s);
    return hipGetLastError();
  }
  if (a.split > 1) {
    // stream-ordered scratch, freed behind the combine pass; without it the
    // launch keeps one workgroup per tuple
    const size_t bytes =
        (size_t)(a.n - a.split_from) * a.split * kVsdPartCols * sizeof(double);
    if (hipMallocAsync((void**)&a.part, bytes, s) != hipSuccess) {
      (void)hipGetLastError();
      a.part = nullptr;
      a.split = 1;
      a.split_from = 0;
    }
  }
  launch_vsd_rpt_any(a, cost_type, s);
  if (a.split > 1) {
    // the scratch is freed on every path (a failed launch skips the combine)
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_vsd_combine, dim3((unsigned)(a.n - a.split_from)),
                         dim3(kCombineThreads), 0, s, a.split, a.n_tau, cost_type,
                         (const double*)a.part, a.out, a.order, a.split_from, a.unions);
      e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(a.part, s);
    return e != hipSuccess ? e : f;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Shared renders (multi-instance images: an image with k instances of an object
// and k estimates has k^2 (est, gt) tuples; the reference renders both poses
// for every one of them, pose_error.py:42-45 under eval_calc_errors.py:281-290).
// Each distinct pose is rasterised once (k_vsd<kCostRender>) into an HBM q
// buffer over its ROI, then k_vsd_pair runs the VSD pixel pass of every tuple
// on the two cached buffers: 2k renders instead of 2k^2. Same raster, same
// per-pixel arithmetic and integer counts as the fused k_vsd: step-cost results
// are bit-identical to it (tlinear sums change order, ~1e-13).

// ROI of each render: the union of its pose's meshlet rectangles, clipped to
// the image (exactly k_vsd's per-tuple ROI restricted to one pose).
__global__ __launch_bounds__(256) void k_pose_roi(const ObjDesc* __restrict__ objs,
                                                  const int32_t* __restrict__ slots,
                                                  const double* __restrict__ pose,
                                                  const int32_t* __restrict__ frame_idx,
                                                  const double* __restrict__ cam, int W, int H,
                                                  int4* __restrict__ rois) {
  __shared__ float s_rf[12];
  __shared__ int s_r[4];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const ObjDesc o = objs[slots[b]];
  const int64_t fi = frame_idx[b];
  Cam32 c32;
  c32.fx = (float)cam[4 * fi + 0];
  c32.fy = (float)cam[4 * fi + 1];
  c32.cx = (float)(cam[4 * fi + 2] + 0.0);  // k_vsd: cx + ox, ox = 0 here
  c32.cy = (float)(cam[4 * fi + 3] + 0.0);
  if (tid < 12) s_rf[tid] = (float)pose[12 * b + tid];
  if (tid == 0) {
    s_r[0] = s_r[1] = 0x7FFFFFFF;
    s_r[2] = s_r[3] = -1;
  }
  __syncthreads();
  float rf[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) rf[k] = s_rf[k];
  int r[4] = {INT32_MAX, INT32_MAX, -1, -1};
  const gptr<const float> mlet = (gptr<const float>)o.mlet;
  for (int m = tid; m < o.nm; m += 256) {
    float zm, qb;
    bool bk;
    const short4 rc = meshlet_rect(mlet + kMletFloats * (int64_t)m, rf, c32, W, H, zm, qb, bk);
    if (rc.x <= rc.z && rc.y <= rc.w) {
      r[0] = min(r[0], (int)rc.x);
      r[1] = min(r[1], (int)rc.y);
      r[2] = max(r[2], (int)rc.z);
      r[3] = max(r[3], (int)rc.w);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    r[0] = min(r[0], __shfl_xor(r[0], off, 64));
    r[1] = min(r[1], __shfl_xor(r[1], off, 64));
    r[2] = max(r[2], __shfl_xor(r[2], off, 64));
    r[3] = max(r[3], __shfl_xor(r[3], off, 64));
  }
  if (lane == 0 && r[2] >= 0) {
    atomicMin(&s_r[0], r[0]);
    atomicMin(&s_r[1], r[1]);
    atomicMax(&s_r[2], r[2]);
    atomicMax(&s_r[3], r[3]);
  }
  __syncthreads();
  if (tid == 0) rois[b] = s_r[2] >= 0 ? make_int4(s_r[0], s_r[1], s_r[2], s_r[3])
                                      : make_int4(0, 0, -1, -1);  // empty
}

hipError_t launch_pose_roi(const ObjDesc* objs, int64_t n, const int32_t* slots,
                           const double* pose, const int32_t* frame_idx, const double* cam, int W,
                           int H, int4* rois, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pose_roi, dim3((unsigned)n), dim3(256), 0, s, objs, slots, pose, frame_idx,
                     cam, W, H, rois);
  return hipGetLastError();
}

// The VSD pixel pass of one (est, gt) tuple on two cached q buffers: one
// 256-thread workgroup per tuple sweeps the union of the two ROIs, wave w
// taking rows w, w + 4, ... and lanes the columns (a fixed pixel -> lane map:
// deterministic float64 sums), with the fused kernel's per-pixel arithmetic.
constexpr int kPairThreads = 256;
constexpr int kPairWaves = kPairThreads / 64;
constexpr int kPairCols = 1024;  // column coefficients staged in LDS per block of columns
// pixels per lane and step, their loads in flight together (round 3, same box:
// 1 / 2 / 4 / 8 -> 4.3 / 3.85 / 4.03 / 4.4 ms on the multi-instance workload)
constexpr int kPairU = 2;

template <int COST, int NT>
__global__ __launch_bounds__(kPairThreads) void k_vsd_pair(PairArgs a) {
  __shared__ double s_pX[kPairCols];
  __shared__ double s_thr[kMaxTaus];
  __shared__ uint32_t s_cnt[kPairWaves][2 + kMaxTaus];
  __shared__ double s_lin[kPairWaves][kMaxTaus];
  // (an XCD-aware order, consecutive tuples on one XCD's L2, measured 4.27 ->
  // 4.49 ms on the configs[5] 20k-tuple batch: the plain order stays)
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int re = a.est_r[b], rg = a.gt_r[b];
  if ((uint64_t)re >= (uint64_t)a.n_renders || (uint64_t)rg >= (uint64_t)a.n_renders) {
    // bad render index (the _dev entry cannot check on the host): NaN errors
    if (tid < a.n_tau) a.out[b * (int64_t)a.n_tau + tid] = __builtin_nan("");
    if (tid == 0 && a.unions) a.unions[b] = __builtin_nan("");
    return;
  }
  const int4 Re = a.rois[re], Rg = a.rois[rg];
  const int64_t oe = a.qoff[re], og = a.qoff[rg];
  const int we = Re.z - Re.x + 1, wg = Rg.z - Rg.x + 1;
  const int64_t fidx = a.rframe[rg];
  const int W = a.width, H = a.height;
  const gptr<const float> frame = (gptr<const float>)(a.frames + fidx * (int64_t)W * H);
  const gptr<const uint32_t> qbuf = (gptr<const uint32_t>)a.qbuf;
  const double fx = a.cam[4 * fidx + 0], fy = a.cam[4 * fidx + 1];
  const double cx = a.cam[4 * fidx + 2], cy = a.cam[4 * fidx + 3];
  const double diam = COST == 0 && a.normalized ? a.diameters[b] : 1.0;
  bool divide = false;
  if constexpr (COST == 0) {  // step thresholds as in k_vsd
    bool fast = a.normalized && diam > 0.0 && diam <= DBL_MAX;
    for (int k = 0; k < a.n_tau; ++k) fast = fast && a.taus[k] == a.taus[k];
    divide = a.normalized && !fast;
    if (tid < NT) {
      double T = INFINITY;
      if (tid < a.n_tau) T = fast ? step_threshold(a.taus[tid], diam) : a.taus[tid];
      s_thr[tid] = T;
    }
  }
  // union of the two ROIs (an empty ROI has x0 > x1)
  const bool ee = Re.x > Re.z, ge = Rg.x > Rg.z;
  const int ux0 = ee ? Rg.x : (ge ? Re.x : min(Re.x, Rg.x));
  const int uy0 = ee ? Rg.y : (ge ? Re.y : min(Re.y, Rg.y));
  const int ux1 = ee ? Rg.z : (ge ? Re.z : max(Re.z, Rg.z));
  const int uy1 = ee ? Rg.w : (ge ? Re.w : max(Re.w, Rg.w));
  __syncthreads();
  double thr[NT];  // wave-uniform (SGPRs)
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    const double v = COST == 0 ? s_thr[k] : 0.0;
    thr[k] = __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                              __builtin_amdgcn_readfirstlane(__double2loint(v)));
  }
  uint32_t c_union = 0, c_inter = 0;
  uint32_t c_tau[(NT + 1) / 2];
  double lin[kMaxTaus];
#pragma unroll
  for (int k = 0; k < kMaxTaus; ++k) {
    if (k < (NT + 1) / 2) c_tau[k] = 0;
    lin[k] = 0.0;
  }
  for (int cb = ux0; cb <= ux1; cb += kPairCols) {  // blocks of columns (wide images)
    const int cb1 = min(cb + kPairCols - 1, ux1);
    __syncthreads();  // the previous block's coefficients are consumed
    for (int i = tid; i <= cb1 - cb; i += kPairThreads) s_pX[i] = ((double)(cb + i) - cx) / fx;
    __syncthreads();
    for (int row = uy0 + wave; row <= uy1; row += kPairWaves) {
      const bool rin_e = row >= Re.y && row <= Re.w, rin_g = row >= Rg.y && row <= Rg.w;
      // covered columns of the row in either render (spans from the render pass)
      int L = INT32_MAX, R = -1;
      if (rin_e) {
        L = min(L, a.smin[a.rowoff[re] + (row - Re.y)]);
        R = max(R, a.smax[a.rowoff[re] + (row - Re.y)]);
      }
      if (rin_g) {
        L = min(L, a.smin[a.rowoff[rg] + (row - Rg.y)]);
        R = max(R, a.smax[a.rowoff[rg] + (row - Rg.y)]);
      }
      L = __builtin_amdgcn_readfirstlane(max(L, cb));
      R = __builtin_amdgcn_readfirstlane(min(R, cb1));
      if (L > R) continue;
      const double pY = ((double)row - cy) / fy;  // misc.py:137-138, as k_vsd's w_pY
      // kPairU pixels per lane and step: every load of the step in flight
      // before the first use (the loop is latency-bound on the q / test-depth
      // reads otherwise); lane -> pixel map fixed (col = L + lane + 64 i)
      // the exact float64 sequence per pixel (vsd_exact_px; the float32 filter
      // of k_vsd measured +3 % here: this loop waits on its loads, and the
      // filter's registers cost a wave per SIMD, profiles/r04/ab_pair_filter.txt)
      auto vsd_pixel = [&](uint32_t qe, uint32_t qg, float dtest, int col) {
        const double pX = s_pX[col - cb];
        if constexpr (COST == 0) {
          bool vg, ve;
          double dd;
          vsd_exact_px(pX, pY, qe, qg, dtest, a.dthr, vg, ve, dd);
          c_union += (vg || ve);
          if (vg && ve) {
            ++c_inter;
            if (divide) {
              dd /= diam;
              asm volatile("" : "+v"(dd));
            }
#pragma unroll
            for (int k = 0; k < NT; ++k) c_tau[k >> 1] += (uint32_t)(dd >= thr[k]) << (16 * (k & 1));
          }
        } else {  // tlinear: float64 sums
          const float de = qe ? rcp_rn(__uint_as_float(qe)) : 0.0f;
          const float dg = qg ? rcp_rn(__uint_as_float(qg)) : 0.0f;
          const double dist_t = dist_of(pX, pY, dtest);
          const double dist_g = qg ? dist_of(pX, pY, dg) : 0.0;
          const double dist_e = qe ? dist_of(pX, pY, de) : 0.0;
          const bool vg = visib19t(dist_t, dist_g, a.dthr);
          bool ve = visib19t(dist_t, dist_e, a.dthr);
          ve = ve || (vg && dist_e > 0.0);  // visibility.py:74
          c_union += (vg || ve);
          if (vg && ve) {
            ++c_inter;
            double dd = fabs(dist_g - dist_e);
            if (a.normalized) dd /= a.diameters[b];
#pragma unroll
            for (int k = 0; k < kMaxTaus; ++k) {
              if (k < a.n_tau) {
                const double cst = dd / a.taus[k];
                lin[k] += cst > 1.0 ? 1.0 : cst;
              }
            }
          }
        }
      };
      const int64_t re_row = oe + (int64_t)(row - Re.y) * we - Re.x;
      const int64_t rg_row = og + (int64_t)(row - Rg.y) * wg - Rg.x;
      const int64_t f_row = (int64_t)row * W;
      for (int c0 = L + lane; c0 <= R; c0 += 64 * kPairU) {
        uint32_t qe[kPairU], qg[kPairU];
        float dt[kPairU];
#pragma unroll
        for (int u = 0; u < kPairU; ++u) {
          const int col = c0 + 64 * u;
          const bool in = col <= R;
          qe[u] = in && rin_e && col >= Re.x && col <= Re.z ? qbuf[re_row + col] : 0u;
          qg[u] = in && rin_g && col >= Rg.x && col <= Rg.z ? qbuf[rg_row + col] : 0u;
          dt[u] = in ? frame[f_row + col] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kPairU; ++u)
          if ((qe[u] | qg[u]) != 0u) vsd_pixel(qe[u], qg[u], dt[u], c0 + 64 * u);
      }
      // 16-bit per-lane tau counters: a lane sees at most (w/64 + 1)(h/4 + 1)
      // pixels of a w x h union, < 42k for any image within the fused kernel's
      // kVsdMaxTiles (w h <= 2048 x 4096, w, h <= 32767; fill_vsd_args checks it)
    }
  }
  c_union = wave_sum_u32(c_union);
  c_inter = wave_sum_u32(c_inter);
  uint32_t tau_sum[kMaxTaus];
#pragma unroll
  for (int k = 0; k < kMaxTaus; ++k) {
    tau_sum[k] = 0;
    if (COST == 0) {
      if (k < NT) tau_sum[k] = wave_sum_u32((c_tau[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
    } else {
      lin[k] = wave_sum_f64(lin[k]);
    }
  }
  if (lane == 0) {
    s_cnt[wave][0] = c_union;
    s_cnt[wave][1] = c_inter;
#pragma unroll
    for (int k = 0; k < kMaxTaus; ++k) {
      s_cnt[wave][2 + k] = tau_sum[k];
      s_lin[wave][k] = lin[k];
    }
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t un = 0, in = 0;
    for (int w = 0; w < kPairWaves; ++w) {
      un += s_cnt[w][0];
      in += s_cnt[w][1];
    }
    if (a.unions) a.unions[b] = (double)un;
    double* out = a.out + b * (int64_t)a.n_tau;
    for (int k = 0; k < a.n_tau; ++k) {
      if (un == 0) {
        out[k] = 1.0;
      } else if (COST == 0) {
        uint64_t cnt = 0;
        for (int w = 0; w < kPairWaves; ++w) cnt += s_cnt[w][2 + k];
        out[k] = (double)(cnt + (un - in)) / (double)un;
      } else {
        double sum = 0.0;
        for (int w = 0; w < kPairWaves; ++w) sum += s_lin[w][k];
        out[k] = (sum + (double)(un - in)) / (double)un;
      }
    }
  }
}

hipError_t launch_vsd_pair(const PairArgs& a, int cost_type, hipStream_t s) {
  if (a.n <= 0) return hipSuccess;
  const dim3 grid((unsigned)a.n), block(kPairThreads);
  if (cost_type == 0 && a.n_tau <= kBopTaus)
    hipLaunchKernelGGL((k_vsd_pair<0, kBopTaus>), grid, block, 0, s, a);
  else if (cost_type == 0)
    hipLaunchKernelGGL((k_vsd_pair<0, kMaxTaus>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((k_vsd_pair<1, kMaxTaus>), grid, block, 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// VSD given three host-supplied depth maps (foreign renderer path). Each block
// reduces 4096 pixels into one partial row [union, inter, cnt[n_tau], lin[n_tau]]
// (float64, exact for counts); the host sums the rows in order.
constexpr int kDepthsPix = 4096;

int vsd_depths_blocks(int W, int H) {
  return (int)(((int64_t)W * H + kDepthsPix - 1) / kDepthsPix);
}

struct TauArr {
  double v[kMaxTaus];
};

__global__ __launch_bounds__(kVsdThreads) void k_vsd_depths(
    int W, int H, const float* __restrict__ dt, const float* __restrict__ de,
    const float* __restrict__ dg, double fx, double fy, double cx, double cy, float delta32,
    int delta_f64, double delta64, TauArr taus, int n_tau, int normalized, double diameter,
    double* __restrict__ partials) {
  __shared__ double s_p[kVsdThreads / 64][2 + 2 * kMaxTaus];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t npx = (int64_t)W * H;
  double acc[2 + 2 * kMaxTaus];
#pragma unroll
  for (int k = 0; k < 2 + 2 * kMaxTaus; ++k) acc[k] = 0.0;
  for (int j = tid; j < kDepthsPix; j += kVsdThreads) {
    const int64_t i = (int64_t)blockIdx.x * kDepthsPix + j;
    if (i >= npx) break;
    const int row = (int)(i / W), col = (int)(i % W);
    const double pX = ((double)col - cx) / fx, pY = ((double)row - cy) / fy;
    const double dist_t = dist_of(pX, pY, dt[i]);
    const double dist_g = dist_of(pX, pY, dg[i]);
    const double dist_e = dist_of(pX, pY, de[i]);
    const bool vg = visib19(dist_t, dist_g, delta32, delta_f64, delta64);
    bool ve = visib19(dist_t, dist_e, delta32, delta_f64, delta64);
    ve = ve || (vg && dist_e > 0.0);
    acc[0] += (vg || ve) ? 1.0 : 0.0;
    if (vg && ve) {
      acc[1] += 1.0;
      double dd = fabs(dist_g - dist_e);
      if (normalized) dd /= diameter;
#pragma unroll
      for (int k = 0; k < kMaxTaus; ++k) {
        if (k < n_tau) {
          acc[2 + k] += (dd >= taus.v[k]) ? 1.0 : 0.0;
          const double cst = dd / taus.v[k];
          acc[2 + kMaxTaus + k] += cst > 1.0 ? 1.0 : cst;
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 2 + 2 * kMaxTaus; ++k) acc[k] = wave_sum_f64(acc[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 2 + 2 * kMaxTaus; ++k) s_p[wave][k] = acc[k];
  __syncthreads();
  if (tid < 2 + 2 * kMaxTaus) {
    double v = 0.0;
    for (int w = 0; w < kVsdThreads / 64; ++w) v += s_p[w][tid];
    partials[(int64_t)blockIdx.x * (2 + 2 * kMaxTaus) + tid] = v;
  }
}

hipError_t launch_vsd_depths(int W, int H, const float* dt, const float* de, const float* dg,
                             double fx, double fy, double cx, double cy, float delta32,
                             int delta_f64, double delta64, const double* taus_host, int n_tau,
                             int normalized, double diameter, double* partials, int n_blocks,
                             hipStream_t s) {
  TauArr ta;
  for (int k = 0; k < kMaxTaus; ++k) ta.v[k] = k < n_tau ? taus_host[k] : 1.0;
  hipLaunchKernelGGL(k_vsd_depths, dim3(n_blocks), dim3(kVsdThreads), 0, s, W, H, dt, de, dg, fx,
                     fy, cx, cy, delta32, delta_f64, delta64, ta, n_tau, normalized, diameter,
                     partials);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Silhouette overlap of two host-supplied depth maps (foreign renderer path of
// cus / cou_bb_proj, pose_error.py:256-330): mask = depth > 0. One grid-stride
// pass; wave-reduced counts and bboxes merged with 64-bit atomics into
// acc[kCoverCols] (exact, order-independent). acc is set by k_cover_init.
__global__ void k_cover_init(long long* acc) {
  const int k = threadIdx.x;
  if (k < kCoverCols) acc[k] = (k < 2) ? 0 : (((k - 2) & 2) ? -1 : INT32_MAX);
}

__global__ __launch_bounds__(256) void k_cover_depths(int W, int H, const float* __restrict__ de,
                                                      const float* __restrict__ dg,
                                                      long long* __restrict__ acc) {
  long long un = 0, in = 0;
  int bb[8] = {INT32_MAX, INT32_MAX, -1, -1, INT32_MAX, INT32_MAX, -1, -1};
  const int64_t n = (int64_t)W * H;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool me = de[i] > 0.0f, mg = dg[i] > 0.0f;
    if (!(me || mg)) continue;
    const int row = (int)(i / W), col = (int)(i % W);
    ++un;
    in += (me && mg);
    if (me) {
      bb[0] = min(bb[0], col);
      bb[1] = min(bb[1], row);
      bb[2] = max(bb[2], col);
      bb[3] = max(bb[3], row);
    }
    if (mg) {
      bb[4] = min(bb[4], col);
      bb[5] = min(bb[5], row);
      bb[6] = max(bb[6], col);
      bb[7] = max(bb[7], row);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    un += __shfl_xor(un, off, 64);
    in += __shfl_xor(in, off, 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int o = __shfl_xor(bb[k], off, 64);
      bb[k] = (k & 2) ? max(bb[k], o) : min(bb[k], o);
    }
  }
  if ((threadIdx.x & 63) == 0 && un > 0) {
    atomicAdd((unsigned long long*)&acc[0], (unsigned long long)un);
    atomicAdd((unsigned long long*)&acc[1], (unsigned long long)in);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k & 2)
        atomicMax(&acc[2 + k], (long long)bb[k]);
      else
        atomicMin(&acc[2 + k], (long long)bb[k]);
    }
  }
}

hipError_t launch_cover_depths(int W, int H, const float* de, const float* dg, long long* acc,
                               hipStream_t s) {
  hipLaunchKernelGGL(k_cover_init, dim3(1), dim3(64), 0, s, acc);
  const int64_t n = (int64_t)W * H;
  const unsigned blocks = (unsigned)std::min<int64_t>(2048, (n + 255) / 256);
  if (blocks > 0)
    hipLaunchKernelGGL(k_cover_depths, dim3(blocks), dim3(256), 0, s, W, H, de, dg, acc);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// misc.depth_im_to_dist_im_fast (misc.py:143-163), elementwise.
__global__ void k_dist_im(int W, int H, const float* __restrict__ depth, double fx, double fy,
                          double cx, double cy, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)W * H) return;
  const int row = (int)(i / W), col = (int)(i % W);
  out[i] = dist_of(((double)col - cx) / fx, ((double)row - cy) / fy, depth[i]);
}

hipError_t launch_dist_im(int W, int H, const float* depth, double fx, double fy, double cx,
                          double cy, double* out, hipStream_t s) {
  const int64_t n = (int64_t)W * H;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_dist_im, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, H, depth,
                     fx, fy, cx, cy, out);
  return hipGetLastError();
}

// visibility._estimate_visib_mask (+ estimate_visib_mask_est's OR), elementwise.
__global__ void k_visib(int64_t n, const double* __restrict__ dt, const double* __restrict__ dm,
                        const uint8_t* __restrict__ vg, float delta32, int delta_f64,
                        double delta64, int mode, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = dt[i], m = dm[i];
  const float diff = (float)m - (float)t;
  const bool le = delta_f64 ? ((double)diff <= delta64) : (diff <= delta32);
  bool v = mode == 0 ? (le && t > 0.0 && m > 0.0) : ((le || t == 0.0) && m > 0.0);
  if (vg) v = v || (vg[i] && m > 0.0);
  out[i] = v ? 1 : 0;
}

hipError_t launch_visib(int64_t n, const double* dt, const double* dm, const uint8_t* vg,
                        float delta32, int delta_f64, double delta64, int mode, uint8_t* out,
                        hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_visib, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, dt, dm, vg,
                     delta32, delta_f64, delta64, mode, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Batched full-frame renderer: one thread per (instance, triangle), global
// atomicMax q-buffer (max 1/Z). Frames are zero-filled first and converted to
// depth after.
// Frames hold the q-buffer (max 1/Z, 0 = empty) while instances are composited;
// to_background = 1 converts it in place to depth = 1.0f / q (0 stays 0).
__global__ void k_depth_fill(uint32_t* __restrict__ f, int64_t n, int to_background) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (to_background) {
    const uint32_t q = f[i];
    f[i] = q ? __float_as_uint(1.0f / __uint_as_float(q)) : 0u;
  } else {
    f[i] = 0u;
  }
}

hipError_t launch_depth_fill(float* frames, int64_t n_pixels, int to_background,
                             hipStream_t s) {
  if (n_pixels <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_depth_fill, dim3((unsigned)((n_pixels + 255) / 256)), dim3(256), 0, s,
                     (uint32_t*)frames, n_pixels, to_background);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_render_batch(const ObjDesc* __restrict__ objs,
                                                      int64_t inst0,
                                                      const int32_t* __restrict__ slots,
                                                      const double* __restrict__ pose,
                                                      const int32_t* __restrict__ frame_idx,
                                                      const double* __restrict__ cam,
                                                      uint32_t* __restrict__ frames, int W,
                                                      int H) {
  __shared__ float s_pose[12];
  const int64_t inst = inst0 + blockIdx.y;
  const ObjDesc o = objs[slots[inst]];
  if (threadIdx.x < 12) s_pose[threadIdx.x] = (float)pose[12 * inst + threadIdx.x];
  __syncthreads();
  const int tri = blockIdx.x * blockDim.x + threadIdx.x;
  if (tri >= o.nf) return;
  const int64_t f = frame_idx[inst];
  Cam32 c;
  c.fx = (float)cam[4 * f];
  c.fy = (float)cam[4 * f + 1];
  c.cx = (float)cam[4 * f + 2];
  c.cy = (float)cam[4 * f + 3];
  const float4 v0 = o.vtx[o.faces[3 * (int64_t)tri]], v1 = o.vtx[o.faces[3 * (int64_t)tri + 1]],
               v2 = o.vtx[o.faces[3 * (int64_t)tri + 2]];
  RTri T;
  if (!r_setup(r_vertex(s_pose, c, v0.x, v0.y, v0.z), r_vertex(s_pose, c, v1.x, v1.y, v1.z),
               r_vertex(s_pose, c, v2.x, v2.y, v2.z), T, 0, W - 1, 0, H - 1))
    return;
  uint32_t* fr = frames + f * (int64_t)W * H;
  r_raster(T, max(T.c0, 0), min(T.c1, W - 1), max(T.r0, 0), min(T.r1, H - 1),
           [&](int col, int row, float q) {
             atomicMax(&fr[(int64_t)row * W + col], __float_as_uint(q));
           });
}

hipError_t launch_render_batch(const ObjDesc* objs, int max_nf, int64_t n, const int32_t* slots,
                               const double* pose, const int32_t* frame_idx, const double* cam,
                               float* frames, int W, int H, hipStream_t s) {
  const unsigned gx = (unsigned)((max_nf + 255) / 256);
  for (int64_t i0 = 0; i0 < n; i0 += 65535) {
    const unsigned gy = (unsigned)(n - i0 < 65535 ? n - i0 : 65535);
    hipLaunchKernelGGL(k_render_batch, dim3(gx, gy), dim3(256), 0, s, objs, i0, slots, pose,
                       frame_idx, cam, (uint32_t*)frames, W, H);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t preload_vsd_kernels() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_vsd_combine));
}

}  // namespace bopx
