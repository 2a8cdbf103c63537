// raster.h — gfx950 triangle depth rasteriser building blocks.
//
// Replaces the OpenGL depth pass of renderer_vispy.py:433-538 /
// renderer_py.py:422-555 (eye-Z depth, pixel-centre sampling, no culling,
// GL_LESS z-test, background 0). The arithmetic follows the raster spec of
// DESIGN.md §4 exactly, so results are bit-identical to the CPU twin
// (oracle/bopx_oracle.c: oracle_render_depth) whatever the tiling, culling or
// triangle order:
//   * vertex: float32, no FMA contraction (built with -ffp-contract=off);
//   * snap to 1/256 px with round-half-even (v_rndne_f32);
//   * exact int64 edge functions with the top-left fill rule (watertight:
//     a pixel centre on a shared edge belongs to exactly one triangle);
//   * depth = area / ((w0/Z0 + w1/Z1) + w2/Z2) in float64 -> float32, combined
//     with an order-independent unsigned atomicMin on the positive-float bits.
#pragma once
#include "bopx_internal.h"

namespace bopx {

struct Cam32 {
  float fx, fy, cx, cy;
};

struct RVtx {
  int32_t U, V;
  float Z;
  bool ok;
};

// Camera-space transform + projection of one float32 vertex. Rf: R row-major
// (9) then t (3), float32 (GL uniforms are float32, renderer_vispy.py:441-442).
__device__ __forceinline__ RVtx r_vertex(const float* __restrict__ Rf, const Cam32& c,
                                         float x, float y, float z) {
  RVtx o;
  float X = ((Rf[0] * x + Rf[1] * y) + Rf[2] * z) + Rf[9];
  float Y = ((Rf[3] * x + Rf[4] * y) + Rf[5] * z) + Rf[10];
  float Z = ((Rf[6] * x + Rf[7] * y) + Rf[8] * z) + Rf[11];
  o.Z = Z;
  o.U = 0;
  o.V = 0;
  o.ok = false;
  if (!(Z > 0.0f)) return o;
  float u = (c.fx * X) / Z + c.cx;
  float v = (c.fy * Y) / Z + c.cy;
  if (!(fabsf(u) <= kGuardBand) || !(fabsf(v) <= kGuardBand)) return o;
  o.U = (int32_t)__builtin_rintf(u * 256.0f);
  o.V = (int32_t)__builtin_rintf(v * 256.0f);
  o.ok = true;
  return o;
}

__device__ __forceinline__ int64_t r_edge(int32_t aU, int32_t aV, int32_t bU, int32_t bV,
                                          int64_t px, int64_t py) {
  return (int64_t)(bU - aU) * (py - aV) - (int64_t)(bV - aV) * (px - aU);
}

__device__ __forceinline__ bool r_top_left(int32_t aU, int32_t aV, int32_t bU, int32_t bV) {
  int32_t dx = bU - aU, dy = bV - aV;
  return dy < 0 || (dy == 0 && dx > 0);
}

__device__ __forceinline__ int64_t r_floor_div256(int64_t a) {
  return a >= 0 ? a / 256 : -((-a + 255) / 256);
}

// A set-up triangle: vertices ordered so that area > 0.
struct RTri {
  int32_t U0, V0, U1, V1, U2, V2;
  int64_t area;
  double iz0, iz1, iz2;
  bool tl0, tl1, tl2;
  int32_t c0, c1, r0, r1;  // pixel bbox (unclipped against any tile)
};

// Returns false for triangles that produce no fragments (invalid vertex, zero area).
__device__ __forceinline__ bool r_setup(RVtx a, RVtx b, RVtx c, RTri& t) {
  if (!(a.ok && b.ok && c.ok)) return false;
  int64_t area = r_edge(a.U, a.V, b.U, b.V, c.U, c.V);
  if (area == 0) return false;
  if (area < 0) {
    RVtx tmp = b;
    b = c;
    c = tmp;
    area = -area;
  }
  t.U0 = a.U; t.V0 = a.V; t.U1 = b.U; t.V1 = b.V; t.U2 = c.U; t.V2 = c.V;
  t.area = area;
  t.iz0 = 1.0 / (double)a.Z;
  t.iz1 = 1.0 / (double)b.Z;
  t.iz2 = 1.0 / (double)c.Z;
  t.tl0 = r_top_left(b.U, b.V, c.U, c.V);
  t.tl1 = r_top_left(c.U, c.V, a.U, a.V);
  t.tl2 = r_top_left(a.U, a.V, b.U, b.V);
  int32_t minU = min(a.U, min(b.U, c.U)), maxU = max(a.U, max(b.U, c.U));
  int32_t minV = min(a.V, min(b.V, c.V)), maxV = max(a.V, max(b.V, c.V));
  t.c0 = (int32_t)(-r_floor_div256(-((int64_t)minU - 128)));
  t.c1 = (int32_t)r_floor_div256((int64_t)maxU - 128);
  t.r0 = (int32_t)(-r_floor_div256(-((int64_t)minV - 128)));
  t.r1 = (int32_t)r_floor_div256((int64_t)maxV - 128);
  return true;
}

// Fragment test + depth at pixel (col, row). Returns +inf bits when not covered.
__device__ __forceinline__ bool r_fragment(const RTri& t, int32_t col, int32_t row, float& z) {
  int64_t px = 256 * (int64_t)col + 128, py = 256 * (int64_t)row + 128;
  int64_t w0 = r_edge(t.U1, t.V1, t.U2, t.V2, px, py);
  int64_t w1 = r_edge(t.U2, t.V2, t.U0, t.V0, px, py);
  int64_t w2 = r_edge(t.U0, t.V0, t.U1, t.V1, px, py);
  bool in = (w0 > 0 || (w0 == 0 && t.tl0)) && (w1 > 0 || (w1 == 0 && t.tl1)) &&
            (w2 > 0 || (w2 == 0 && t.tl2));
  if (!in) return false;
  double den = ((double)w0 * t.iz0 + (double)w1 * t.iz1) + (double)w2 * t.iz2;
  z = (float)((double)t.area / den);
  return true;
}

__device__ __forceinline__ void load_pose32(const double* __restrict__ p, float* Rf) {
  for (int i = 0; i < 12; ++i) Rf[i] = (float)p[i];
}

}  // namespace bopx
