// raster.h — gfx950 triangle depth rasteriser building blocks.
//
// Replaces the OpenGL depth pass of renderer_vispy.py:433-538 /
// renderer_py.py:422-555 (eye-Z depth, pixel-centre sampling, no culling,
// GL_LESS z-test, background 0). The arithmetic follows raster spec v5 of
// DESIGN.md §4 exactly, so results are bit-identical to the CPU twin
// (oracle/bopx_oracle.c: oracle_render_depth) whatever the tiling, culling or
// triangle order:
//   * vertex: float32, no FMA contraction (built with -ffp-contract=off),
//     iz = 1/Z (one IEEE division), u = (fx X) iz + cx, snapped to 1/256 px
//     with round-half-even (v_rndne_f32);
//   * exact integer edge functions with the top-left fill rule (watertight:
//     a pixel centre on a shared edge belongs to exactly one triangle).
//     Triangles whose fixed-point extent is < 2^15 (128 px) step their edge
//     functions incrementally in int32 (|E| < 2^31 is guaranteed there); larger
//     ones evaluate them directly in int64 — the same integers either way;
//   * 1/Z is affine in screen space: q = fma(ga, dx, fma(gb, dy, iz0)) in
//     float32 per fragment (gradients set up once per triangle in float32);
//   * a "regular" triangle (|ga|, |gb| <= 2^64 and 2^10 * 2area >= bw^2 + bh^2 of
//     its snapped bbox) has |q - exact plane| <= 2^-9 dz + 2^-23 izmax (DESIGN.md
//     §4), so q <= (1 + 2^-8) izmax; an irregular one (a sliver) has its q clamped
//     to izmax (fminf). Every fragment is therefore bounded by its triangle's
//     largest vertex 1/Z times (1 + 2^-8): the occlusion test of k_vsd relies on it;
//   * the z-buffer keeps max q with an order-independent atomicMax on the
//     positive-float bits; depth = 1.0f / q_max (= min of the per-fragment
//     depths, RN(1/x) being monotone). 0 bits = no fragment = background.
#pragma once
#include "bopx_internal.h"

namespace bopx {


// Correctly rounded 1/x, bit-identical to the IEEE 1.0f / x the spec names:
// hardware reciprocal plus one fused Newton step. Checked against
// (float)(1.0 / (double)x) for every float32 x with |x| and |1/x| normal
// (tools/rcp_exhaustive.hip: 4,227,858,432 values, no mismatch); other inputs
// take the IEEE division.
// The range test is one unsigned compare on the bits (|x| in [2^-126, 2^126));
// the IEEE path is a wave-uniform branch taken only if some lane needs it.
__device__ __forceinline__ float rcp_rn(float x) {
  const float r0 = __builtin_amdgcn_rcpf(x);
  const float r = __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
  const bool ok = (__float_as_uint(x) & 0x7FFFFFFFu) - 0x00800000u < 0x7E000000u;
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) != 0, 0)) return ok ? r : 1.0f / x;
  return r;
}

struct Cam32 {
  float fx, fy, cx, cy;
};

// 12 bytes (ds_read_b96). Valid vertices have |U| <= 2^22; U = INT32_MIN marks
// a vertex that is not rasterisable (Z <= 0 or outside the guard band).
struct RVtx {
  int32_t U, V;
  float iz;
  __device__ __forceinline__ bool ok() const { return U != INT32_MIN; }
};

// Camera-space transform + projection of one float32 vertex. Rf: R row-major
// (9) then t (3), float32 (GL uniforms are float32, renderer_vispy.py:441-442).
__device__ __forceinline__ RVtx r_vertex(const float* __restrict__ Rf, const Cam32& c,
                                         float x, float y, float z) {
  RVtx o;
  const float X = ((Rf[0] * x + Rf[1] * y) + Rf[2] * z) + Rf[9];
  const float Y = ((Rf[3] * x + Rf[4] * y) + Rf[5] * z) + Rf[10];
  const float Z = ((Rf[6] * x + Rf[7] * y) + Rf[8] * z) + Rf[11];
  // Branch-free: every lane computes the projection, invalid ones are
  // replaced by the sentinel afterwards (same values as an early return).
  const float iz = rcp_rn(Z);  // the one IEEE division per vertex (spec v5)
  const float u = (c.fx * X) * iz + c.cx;
  const float v = (c.fy * Y) * iz + c.cy;
  const bool ok = (int)(Z > 0.0f) & (int)(fabsf(u) <= kGuardBand) & (int)(fabsf(v) <= kGuardBand);
  o.U = ok ? (int32_t)__builtin_rintf((ok ? u : 0.0f) * 256.0f) : INT32_MIN;
  o.V = ok ? (int32_t)__builtin_rintf((ok ? v : 0.0f) * 256.0f) : 0;
  o.iz = ok ? iz : 0.0f;
  return o;
}

// r_vertex with X and Y computed as the two halves of packed float32 ops
// (v_pk_mul_f32 / v_pk_add_f32: the same IEEE operations in the same order,
// no contraction, so the same bits). P: the pose in pair order
// {R0,R3, R1,R4, R2,R5, t0,t1, R6,R7,R8, t2} (16-B aligned).
__device__ __forceinline__ RVtx r_vertex_pk(const float* __restrict__ P, const Cam32& c, float x,
                                            float y, float z) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const float4 p0 = reinterpret_cast<const float4*>(P)[0];
  const float4 p1 = reinterpret_cast<const float4*>(P)[1];
  const float4 p2 = reinterpret_cast<const float4*>(P)[2];
  const f32x2 r03 = {p0.x, p0.y}, r14 = {p0.z, p0.w}, r25 = {p1.x, p1.y}, t01 = {p1.z, p1.w};
  const f32x2 xx = {x, x}, yy = {y, y}, zz = {z, z};
  const f32x2 XY = ((r03 * xx + r14 * yy) + r25 * zz) + t01;
  // Z in scalar ops: the empty asm keeps the SLP vectoriser from pairing its
  // products (the pairs would cost more register copies than they save)
  float zx = p2.x * x, zy = p2.y * y, zz1 = p2.z * z;
  asm("" : "+v"(zx), "+v"(zy), "+v"(zz1));
  const float Z = ((zx + zy) + zz1) + p2.w;
  const float iz = rcp_rn(Z);
  const f32x2 f = {c.fx, c.fy}, cc = {c.cx, c.cy}, izz = {iz, iz};
  const f32x2 uv = (f * XY) * izz + cc;
  const f32x2 uv256 = uv * (f32x2){256.0f, 256.0f};
  RVtx o;
  const bool ok = (int)(Z > 0.0f) & (int)(fabsf(uv.x) <= kGuardBand) & (int)(fabsf(uv.y) <= kGuardBand);
  o.U = ok ? (int32_t)__builtin_rintf(ok ? uv256.x : 0.0f) : INT32_MIN;
  o.V = ok ? (int32_t)__builtin_rintf(ok ? uv256.y : 0.0f) : 0;
  o.iz = ok ? iz : 0.0f;
  return o;
}

__device__ __forceinline__ int64_t r_floor_div256(int64_t a) {
  return a >= 0 ? a / 256 : -((-a + 255) / 256);
}

// A set-up triangle: vertices ordered so that area > 0; edge k is the edge
// opposite vertex k (k=0: b->c, 1: c->a, 2: a->b), E_k(P) = dU*(Py-Vs) - dV*(Px-Us).
struct RTri {
  int32_t U0, V0;           // vertex a (reference point of the 1/Z plane)
  float iz0, ga, gb;        // 1/Z plane
  int32_t Us[3], Vs[3];     // edge start vertices
  int32_t dU[3], dV[3];     // edge vectors
  int32_t tl[3];            // top-left bias (1 = edge owns its centres)
  int32_t c0, c1, r0, r1;   // pixel bbox (unclipped)
  float izmax;              // largest vertex 1/Z (the clamp of irregular triangles)
  bool small;               // int32 incremental path is exact
  bool regular;             // q needs no clamp (spec v5)
};

// Spec v5 regularity (exact integers, the oracle's formula): finite moderate
// gradients and 2^10 * area2 >= bw^2 + bh^2 (area2 = twice the fixed-point area,
// bw / bh = fixed-point bbox extents).
__device__ __forceinline__ bool r_regular(float ga, float gb, int64_t area2, int64_t bw,
                                          int64_t bh) {
  return fabsf(ga) <= 0x1p64f && fabsf(gb) <= 0x1p64f && (area2 << 10) >= bw * bw + bh * bh;
}
// The same for a small triangle (bw, bh < 2^15, area2 < 2^31) in uint32:
// 2^10 a >= s  <=>  a >= ceil(s / 2^10), s = bw^2 + bh^2 < 2^31.
__device__ __forceinline__ bool r_regular_small(float ga, float gb, uint32_t area2, uint32_t bw,
                                                uint32_t bh) {
  // bw, bh < 2^15: full-rate 24-bit multiplies (exact)
  return fmaxf(fabsf(ga), fabsf(gb)) <= 0x1p64f &&
         area2 >= (__umul24(bw, bw) + __umul24(bh, bh) + 1023u) >> 10;
}

// Returns false for triangles with no fragment inside the pixel rectangle
// [x0,x1] x [y0,y1] (invalid vertex, zero area, or bbox outside the rectangle);
// the bbox test runs first so culled triangles skip the float64 set-up.
__device__ __forceinline__ bool r_setup(RVtx a, RVtx b, RVtx c, RTri& t, int x0, int x1, int y0,
                                        int y1) {
  if (!(a.ok() && b.ok() && c.ok())) return false;
  {
    // |U|, |V| <= 2^22 (guard band): floor(x / 256) is an arithmetic shift.
    const int32_t minU = min(a.U, min(b.U, c.U)), maxU = max(a.U, max(b.U, c.U));
    const int32_t minV = min(a.V, min(b.V, c.V)), maxV = max(a.V, max(b.V, c.V));
    t.c0 = (minU + 127) >> 8;  // ceil((minU - 128) / 256)
    t.c1 = (maxU - 128) >> 8;  // floor((maxU - 128) / 256)
    t.r0 = (minV + 127) >> 8;
    t.r1 = (maxV - 128) >> 8;
    if (max(t.c0, x0) > min(t.c1, x1) || max(t.r0, y0) > min(t.r1, y1)) return false;
    t.small = (maxU - minU) < 32768 && (maxV - minV) < 32768;
  }
  float farea;
  int64_t farea_exact;
  bool neg;
  if (t.small) {  // |area| <= 2 * 32767^2 < 2^31; factors < 2^15: exact 24-bit multiplies
    const int32_t area = __mul24(b.U - a.U, c.V - a.V) - __mul24(b.V - a.V, c.U - a.U);
    if (area == 0) return false;
    neg = area < 0;
    farea_exact = neg ? -area : area;
    farea = (float)farea_exact;
  } else {
    const int64_t area = (int64_t)(b.U - a.U) * (c.V - a.V) - (int64_t)(b.V - a.V) * (c.U - a.U);
    if (area == 0) return false;
    neg = area < 0;
    farea_exact = neg ? -area : area;
    farea = (float)(double)farea_exact;
  }
  if (neg) {
    const RVtx tmp = b;
    b = c;
    c = tmp;
  }
  const float inv_area = rcp_rn(farea);
  const float dza = a.iz - c.iz, dzb = b.iz - c.iz;
  t.ga = ((float)(b.V - c.V) * dza + (float)(c.V - a.V) * dzb) * inv_area;
  t.gb = ((float)(c.U - b.U) * dza + (float)(a.U - c.U) * dzb) * inv_area;
  t.U0 = a.U;
  t.V0 = a.V;
  t.iz0 = a.iz;
  t.izmax = fmaxf(a.iz, fmaxf(b.iz, c.iz));
  {
    const int32_t minU = min(a.U, min(b.U, c.U)), maxU = max(a.U, max(b.U, c.U));
    const int32_t minV = min(a.V, min(b.V, c.V)), maxV = max(a.V, max(b.V, c.V));
    t.regular = r_regular(t.ga, t.gb, (int64_t)farea_exact, (int64_t)maxU - minU,
                          (int64_t)maxV - minV);
  }
  const RVtx s[3] = {b, c, a}, e[3] = {c, a, b};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    t.Us[k] = s[k].U;
    t.Vs[k] = s[k].V;
    t.dU[k] = e[k].U - s[k].U;
    t.dV[k] = e[k].V - s[k].V;
    t.tl[k] = (t.dV[k] < 0 || (t.dV[k] == 0 && t.dU[k] > 0)) ? 1 : 0;
  }
  return true;
}

// r_setup for a triangle that already passed r_touches (valid vertices, bbox
// meets the rectangle): the same RTri, false only for a zero area. Built for
// full waves (k_vsd): no early returns, the winding swap is a select, and the
// int64 area of large triangles runs behind a wave-uniform branch.
__device__ __forceinline__ bool r_setup_touching(const RVtx a, const RVtx b0, const RVtx c0,
                                                 RTri& t) {
  const int32_t minU = min(a.U, min(b0.U, c0.U)), maxU = max(a.U, max(b0.U, c0.U));
  const int32_t minV = min(a.V, min(b0.V, c0.V)), maxV = max(a.V, max(b0.V, c0.V));
  t.c0 = (minU + 127) >> 8;
  t.c1 = (maxU - 128) >> 8;
  t.r0 = (minV + 127) >> 8;
  t.r1 = (maxV - 128) >> 8;
  t.small = (maxU - minU) < 32768 && (maxV - minV) < 32768;
  // small: factors < 2^15, exact 24-bit multiplies (other lanes: replaced below)
  const int32_t area32 = __mul24(b0.U - a.U, c0.V - a.V) - __mul24(b0.V - a.V, c0.U - a.U);
  bool neg = area32 < 0, nz = area32 != 0;
  const uint32_t aabs = (uint32_t)(neg ? -area32 : area32);
  float farea = (float)aabs;
  int64_t area64 = 0;
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!t.small) != 0, 0)) {
    if (!t.small) {
      const int64_t area =
          (int64_t)(b0.U - a.U) * (c0.V - a.V) - (int64_t)(b0.V - a.V) * (c0.U - a.U);
      neg = area < 0;
      nz = area != 0;
      area64 = neg ? -area : area;
      farea = (float)(double)area64;
    }
  }
  const RVtx b = neg ? c0 : b0, c = neg ? b0 : c0;
  const float inv_area = rcp_rn(nz ? farea : 1.0f);
  const float dza = a.iz - c.iz, dzb = b.iz - c.iz;
  t.ga = ((float)(b.V - c.V) * dza + (float)(c.V - a.V) * dzb) * inv_area;
  t.gb = ((float)(c.U - b.U) * dza + (float)(a.U - c.U) * dzb) * inv_area;
  t.U0 = a.U;
  t.V0 = a.V;
  t.iz0 = a.iz;
  t.izmax = fmaxf(a.iz, fmaxf(b.iz, c.iz));
  t.regular = r_regular_small(t.ga, t.gb, aabs, (uint32_t)(maxU - minU), (uint32_t)(maxV - minV));
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!t.small) != 0, 0)) {
    if (!t.small)
      t.regular = r_regular(t.ga, t.gb, area64, (int64_t)maxU - minU, (int64_t)maxV - minV);
  }
  const RVtx s[3] = {b, c, a}, e[3] = {c, a, b};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    t.Us[k] = s[k].U;
    t.Vs[k] = s[k].V;
    t.dU[k] = e[k].U - s[k].U;
    t.dV[k] = e[k].V - s[k].V;
    t.tl[k] = (t.dV[k] < 0 || (t.dV[k] == 0 && t.dU[k] > 0)) ? 1 : 0;
  }
  return nz;
}

// Cheap pre-test: all vertices valid and the pixel bbox meets [x0,x1] x [y0,y1]
// (the same bbox r_setup computes; r_setup may still reject zero-area triangles).
__device__ __forceinline__ bool r_touches(RVtx a, RVtx b, RVtx c, int x0, int x1, int y0,
                                          int y1) {
  const int32_t minU = min(a.U, min(b.U, c.U)), maxU = max(a.U, max(b.U, c.U));
  const int32_t minV = min(a.V, min(b.V, c.V)), maxV = max(a.V, max(b.V, c.V));
  // branch-free: an invalid vertex (U = INT32_MIN, V = 0) is the minimum U, so one
  // compare covers the three validity tests, and no term can overflow
  return (int)(minU != INT32_MIN) & (int)(max((minU + 127) >> 8, x0) <= min((maxU - 128) >> 8, x1)) &
         (int)(max((minV + 127) >> 8, y0) <= min((maxV - 128) >> 8, y1));
}

// Spec v5 fragment value: fused plane evaluation, clamped to izmax for an
// irregular triangle (fminf: a NaN becomes izmax).
__device__ __forceinline__ float r_q(const RTri& t, int32_t px, int32_t py) {
  const float q = __builtin_fmaf(t.ga, (float)(px - t.U0),
                                 __builtin_fmaf(t.gb, (float)(py - t.V0), t.iz0));
  return t.regular ? q : fminf(q, t.izmax);
}

// Visit every fragment of t inside the pixel rectangle [cc0,cc1] x [rr0,rr1]
// (already clipped to the triangle bbox); plot(col, row, q) with q > 0.
template <class Plot>
__device__ __forceinline__ void r_raster(const RTri& t, int cc0, int cc1, int rr0, int rr1,
                                         Plot plot) {
  if (cc0 > cc1 || rr0 > rr1) return;
  const int32_t px0 = 256 * cc0 + 128, py0 = 256 * rr0 + 128;
  if (t.small) {
    // uint32 wrap-around arithmetic: exact at every visited pixel (|E| < 2^31),
    // and well-defined one step past the rectangle where the value is unused.
    uint32_t er[3], sx[3], sy[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      er[k] = (uint32_t)t.dU[k] * (uint32_t)(py0 - t.Vs[k]) -
              (uint32_t)t.dV[k] * (uint32_t)(px0 - t.Us[k]) + (uint32_t)t.tl[k];
      sx[k] = (uint32_t)(-256 * t.dV[k]);
      sy[k] = (uint32_t)(256 * t.dU[k]);
    }
    // Nested row/column loops (a flattened single loop measured 1.4x slower:
    // its row-wrap branch diverges every iteration).
    int32_t py = py0;
    for (int row = rr0; row <= rr1; ++row, py += 256) {
      uint32_t e0 = er[0], e1 = er[1], e2 = er[2];
      int32_t px = px0;
      for (int col = cc0; col <= cc1; ++col, px += 256) {
        if (((int32_t)e0 > 0) & ((int32_t)e1 > 0) & ((int32_t)e2 > 0)) {
          const float q = r_q(t, px, py);
          if (q > 0.0f) plot(col, row, q);
        }
        e0 += sx[0];
        e1 += sx[1];
        e2 += sx[2];
      }
      er[0] += sy[0];
      er[1] += sy[1];
      er[2] += sy[2];
    }
  } else {
    for (int row = rr0; row <= rr1; ++row) {
      const int64_t py = 256 * (int64_t)row + 128;
      for (int col = cc0; col <= cc1; ++col) {
        const int64_t px = 256 * (int64_t)col + 128;
        bool in = true;
#pragma unroll
        for (int k = 0; k < 3; ++k)
          in = in && ((int64_t)t.dU[k] * (py - t.Vs[k]) - (int64_t)t.dV[k] * (px - t.Us[k]) +
                      t.tl[k]) > 0;
        if (in) {
          const float q = r_q(t, (int32_t)px, (int32_t)py);
          if (q > 0.0f) plot(col, row, q);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Row items (the k_vsd fast path). A wave's set-up triangles publish one 48-B
// record each in LDS; the wave then hands out (triangle, row) items, one per
// lane, and each lane walks the columns of its row with the same int32
// incremental edge values and q expression as r_raster (identical fragments).
// Balancing rows instead of whole triangles bounds a lane's walk by the widest
// row in the batch instead of the largest bounding box.
struct __attribute__((aligned(16))) RRow {
  uint32_t er[3];      // edge values (+ top-left bias - 1) at (cc0, rr0)
  uint32_t duv[3];     // dU | dV << 16 (int16 each: small triangles)
  float px0u;          // 256*cc0 + 128 - U0 (an integer, |.| < 2^15: exact)
  uint32_t pyf;        // first item | (256*rr0 + 128 - V0) << 16 (|.| < 2^15: small triangles)
  float ga, iz0, gb;   // 1/Z plane (ga first: an even register of the 16-B read)
  uint32_t meta;       // byte offset of (cc0, rr0) in the q-tile pair | (w-1) << 25
};
static_assert(sizeof(RRow) == 48, "RRow is a 48-B LDS record");

// Small triangles only; [cc0,cc1] x [rr0,rr1] inside the 64x64 tile at (x0, y0).
// The row walk's tile address and row start are precomputed here, once per
// triangle, instead of once per walked row: 256*rr0 + 128 - V0 lies between
// minV - maxV and maxV - minV (rr0 within the bbox rows), an int16 for a small
// triangle; the byte offset (pose's tile of the pair, row, column) is < 2^16.
static_assert(2 * kTileStride * kTileH * 4 <= 65536, "q-tile pair byte offsets are 16-bit");
__device__ __forceinline__ void r_make_row(const RTri& t, int cc0, int cc1, int rr0, int x0,
                                           int y0, int pose, int first, RRow& r) {
  const int32_t px0 = 256 * cc0 + 128, py0 = 256 * rr0 + 128;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    // |dU|, |dV|, |p0 - vertex| < 2^15 -> exact 24-bit multiplies
    // biased by -1: a centre is inside iff every walked edge value is >= 0, so
    // the walk reads coverage off the sign bits (no wrap: |E| < 2^31, tl - 1 <= 0)
    r.er[k] = (uint32_t)(__mul24(t.dU[k], py0 - t.Vs[k]) - __mul24(t.dV[k], px0 - t.Us[k]) +
                         (t.tl[k] - 1));
    r.duv[k] = ((uint32_t)t.dU[k] & 0xFFFFu) | ((uint32_t)t.dV[k] << 16);
  }
  r.px0u = (float)(px0 - t.U0);
  r.pyf = (uint32_t)first | ((uint32_t)(py0 - t.V0) << 16);
  r.iz0 = t.iz0;
  r.ga = t.ga;
  r.gb = t.gb;
  r.meta = (uint32_t)(4 * ((pose * kTileH + rr0 - y0) * kTileStride + cc0 - x0)) |
           ((uint32_t)(cc1 - cc0) << 25);
}

// Walk row j of a record into the LDS z-buffer, branch-free: every column issues one
// signed atomicMax of q's bits OR'd with the sign bit of the column's smallest
// (biased) edge value, i.e. a negative no-op on the buffer (0-initialised, only
// ever non-negative) where the pixel centre is outside the triangle: one
// v_and_or_b32 instead of a compare and a select per column. Records are regular
// small triangles only, so q is finite (never NaN): a q <= 0 (including -0.0) has
// a sign bit or is +0 and loses the signed max against the buffer, which is
// exactly the spec's "fragments with q <= 0 are dropped" without a compare. No
// exec-mask branches in the loop body.
// dep: the q-tile pair (row pitch kTileStride); the record's offset picks the pose's
// tile. Returns the fragment count (diagnostics).
// MASKED: only covered centres issue their atomicMax (exec-masked; fewer bank
// conflicts on scattered rows) instead of every column (0 where the centre is
// outside: no exec-mask save / restore). Round 2, same box: unmasked 0.9 %
// faster for 1-rectangle objects, masked 1.2 % faster for the 2-rectangle
// class; skipping a column no lane covers (ballot) was 1.9 % slower.
template <bool kNoAtomics = false, bool MASKED = true>  // kNoAtomics: timing ablation (diag builds)
__device__ __forceinline__ int r_walk_row_max(const RRow& r, int j, uint32_t* dep) {
  // j < 64 always; the mask (a no-op) tells the compiler so, which keeps every
  // multiply below on the full-rate 24-bit path.
  j &= 63;
  const int w = (int)(r.meta >> 25) + 1;
  uint32_t e[3], sx[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int32_t dU256 = (int32_t)(r.duv[k] << 16) >> 8;  // 256 dU, |256 dU| < 2^23
    const int32_t dV = (int32_t)r.duv[k] >> 16;
    e[k] = r.er[k] + (uint32_t)__mul24(dU256, j);
    sx[k] = (uint32_t)__mul24(-256, dV);
  }
  // spec v5: q = fma(ga, dx, fma(gb, dy, iz0)); the row term once per row
  const float qrow = __builtin_fmaf(r.gb, (float)(((int32_t)r.pyf >> 16) + (j << 8)), r.iz0);
  // the column pair's dx (integers below 2^24: += 512 is exact), packed so the
  // two fmas and the step are one v_pk_fma_f32 / v_pk_add_f32 each
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  f32x2 fdx = {r.px0u, r.px0u + 256.0f};
  // ga and qrow in the low halves only: the packed fma reads each low half for
  // both columns (op_sel_hi), so neither is copied into a register pair
  const f32x2 ga_ = {r.ga, r.iz0}, step2 = {512.0f, 512.0f};
  f32x2 qrow_;  // the high half is never read
  qrow_.x = qrow;
  int* d = reinterpret_cast<int*>(reinterpret_cast<char*>(dep) + (r.meta & 0xFFFFu) +
                                 __mul24(j, 4 * kTileStride));
  int frags = 0;
  // Two columns per iteration (independent chains). The second column of the
  // last pair may be one past the rectangle and is not masked: past the
  // triangle's own bbox no pixel centre is inside it; past a tile clip it lands
  // in the padding column (tc0 + w = 64 < kTileStride) or, for a tile cut by
  // the ROI, in the column right of it, which the pixel compaction clears.
  // i < w  <=>  i << 25 <= meta (the offset below bit 25; i <= 64: no wrap)
  for (int i = 0; ((uint32_t)i << 25) <= r.meta; i += 2, fdx += step2) {
    const uint32_t f0 = e[0] + sx[0], f1 = e[1] + sx[1], f2 = e[2] + sx[2];
    const int32_t m0 = min((int32_t)e[0], min((int32_t)e[1], (int32_t)e[2]));
    const int32_t m1 = min((int32_t)f0, min((int32_t)f1, (int32_t)f2));
    f32x2 q;  // {fma(ga, fdx.x, qrow), fma(ga, fdx.y, qrow)}
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(q) : "v"(ga_), "v"(fdx), "v"(qrow_));
    const float q0 = q.x, q1 = q.y;
    frags += (m0 >= 0) + ((i + 1 < w) & (m1 >= 0));  // diagnostics (dead in the product build)
    if constexpr (kNoAtomics) {
      asm volatile("" ::"v"(m0 >= 0 ? q0 : 0.0f), "v"(m1 >= 0 ? q1 : 0.0f), "v"(d + i));
    } else if constexpr (MASKED) {
      if (m0 >= 0) atomicMax(d + i, __float_as_int(q0));
      if (m1 >= 0) atomicMax(d + i + 1, __float_as_int(q1));
    } else {
      atomicMax(d + i, __float_as_int(q0) | (m0 & INT32_MIN));
      atomicMax(d + i + 1, __float_as_int(q1) | (m1 & INT32_MIN));
    }
    e[0] = f0 + sx[0];
    e[1] = f1 + sx[1];
    e[2] = f2 + sx[2];
  }
  return frags;
}

}  // namespace bopx
