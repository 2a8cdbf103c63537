/*
 * bopx_oracle.c — CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed
 * CPU baseline. The product (bop_toolkit_amd + libbopx.so) never links or calls it.
 *
 * Parity pinning: every function here is checked against golden vectors that
 * tests/golden/gen_golden.py captured by importing the reference
 * (/root/reference/bop_toolkit_lib) in the build container, see
 * tests/test_oracle_golden.py. The depth rasteriser has no reference oracle
 * (vispy/glumpy/bop_renderer are not importable here): its semantics are the
 * spec in DESIGN.md §4 ("raster parity unpinned" vs. the reference renderers;
 * pinned by analytic tests and bit-exactness against the HIP rasteriser).
 *
 * Each function follows the reference formula literally (operation order
 * included where it matters for bit-exactness):
 *   oracle_dist_im      misc.py:143-163   (Precomputer :110-140)
 *   oracle_visib_mask   visibility.py:9-42, 58-75
 *   oracle_vsd_depths   pose_error.py:47-93
 *   oracle_mssd         pose_error.py:96-118 (+ misc.transform_pts_Rt :266-276)
 *   oracle_mspd         pose_error.py:121-144 (+ misc.project_pts :93-107)
 *   oracle_add / _adi   pose_error.py:147-184
 *   oracle_proj         pose_error.py:217-232
 *   oracle_render_depth renderer_py.py:422-555 / renderer_vispy.py:433-538
 *                       semantics (eye-Z, pixel centres, no culling, z-test
 *                       LESS, background 0) as specified in DESIGN.md §4.
 *   oracle_vsd_zbuf_batch  the spec's eye Z passed through a MODEL of vispy's
 *                       z-buffer (window depth with the per-render near / far of
 *                       renderer_vispy.py:447-456, stored as float32 or 24 / 16-bit
 *                       fixed point, read back and linearised as :526-536) before
 *                       the VSD of pose_error.py:47-93: a study of what the
 *                       spec's exact eye Z leaves unpinned.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_COST_STEP 0
#define ORACLE_COST_TLINEAR 1

/* ---------------------------------------------------------------- helpers */
static void rt_apply(const double* Rt, const double* p, double* o) {
  /* R.dot(p) + t, row-major R (misc.py:275). */
  for (int i = 0; i < 3; ++i)
    o[i] = ((Rt[3 * i + 0] * p[0] + Rt[3 * i + 1] * p[1]) + Rt[3 * i + 2] * p[2]) + Rt[9 + i];
}

static void compose_sym(const double* Rg_t /*12*/, const double* sym /*12*/, double* out) {
  /* R_gt_sym = R_gt.dot(sym['R']); t_gt_sym = R_gt.dot(sym['t']) + t_gt
     (pose_error.py:114-115). */
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) {
      out[3 * i + j] = (Rg_t[3 * i + 0] * sym[0 * 3 + j] + Rg_t[3 * i + 1] * sym[1 * 3 + j]) +
                       Rg_t[3 * i + 2] * sym[2 * 3 + j];
    }
    out[9 + i] = ((Rg_t[3 * i + 0] * sym[9] + Rg_t[3 * i + 1] * sym[10]) + Rg_t[3 * i + 2] * sym[11]) +
                 Rg_t[9 + i];
  }
}

static void proj_matrix(const double* K /*9*/, const double* Rt /*12*/, double* P /*12: 3x4 row-major*/) {
  /* P = K.dot(np.hstack((R, t))) (misc.py:103). */
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) {
      double m0 = (j < 3) ? Rt[0 * 3 + j] : Rt[9 + 0];
      double m1 = (j < 3) ? Rt[1 * 3 + j] : Rt[9 + 1];
      double m2 = (j < 3) ? Rt[2 * 3 + j] : Rt[9 + 2];
      P[4 * i + j] = (K[3 * i + 0] * m0 + K[3 * i + 1] * m1) + K[3 * i + 2] * m2;
    }
}

static void project(const double* P, const double* p, double* uv) {
  /* pts_im = P.dot(pts_h.T); pts_im /= pts_im[2, :] (misc.py:104-107). */
  double x = ((P[0] * p[0] + P[1] * p[1]) + P[2] * p[2]) + P[3];
  double y = ((P[4] * p[0] + P[5] * p[1]) + P[6] * p[2]) + P[7];
  double z = ((P[8] * p[0] + P[9] * p[1]) + P[10] * p[2]) + P[11];
  uv[0] = x / z;
  uv[1] = y / z;
}

/* ------------------------------------------------- point-based pose errors */
double oracle_mssd(const double* pts, int64_t nv, const double* syms, int64_t ns,
                   const double* pe, const double* pg) {
  double best = INFINITY;
  double* pts_est = (double*)malloc(sizeof(double) * 3 * (size_t)nv);
  for (int64_t v = 0; v < nv; ++v) rt_apply(pe, pts + 3 * v, pts_est + 3 * v);
  for (int64_t s = 0; s < ns; ++s) {
    double gs[12];
    compose_sym(pg, syms + 12 * s, gs);
    double emax = -INFINITY;
    for (int64_t v = 0; v < nv; ++v) {
      double q[3];
      rt_apply(gs, pts + 3 * v, q);
      double dx = pts_est[3 * v] - q[0], dy = pts_est[3 * v + 1] - q[1], dz = pts_est[3 * v + 2] - q[2];
      double d = sqrt((dx * dx + dy * dy) + dz * dz);
      if (d > emax || isnan(d)) emax = d;
    }
    if (emax < best || isnan(emax)) best = emax;
  }
  free(pts_est);
  return best;
}

double oracle_mspd(const double* pts, int64_t nv, const double* syms, int64_t ns,
                   const double* pe, const double* pg, const double* K) {
  double best = INFINITY, Pe[12];
  proj_matrix(K, pe, Pe);
  double* proj_est = (double*)malloc(sizeof(double) * 2 * (size_t)nv);
  for (int64_t v = 0; v < nv; ++v) project(Pe, pts + 3 * v, proj_est + 2 * v);
  for (int64_t s = 0; s < ns; ++s) {
    double gs[12], Pg[12];
    compose_sym(pg, syms + 12 * s, gs);
    proj_matrix(K, gs, Pg);
    double emax = -INFINITY;
    for (int64_t v = 0; v < nv; ++v) {
      double q[2];
      project(Pg, pts + 3 * v, q);
      double du = proj_est[2 * v] - q[0], dv = proj_est[2 * v + 1] - q[1];
      double d = sqrt(du * du + dv * dv);
      if (d > emax || isnan(d)) emax = d;
    }
    if (emax < best || isnan(emax)) best = emax;
  }
  free(proj_est);
  return best;
}

double oracle_add(const double* pts, int64_t nv, const double* pe, const double* pg) {
  double sum = 0.0;
  for (int64_t v = 0; v < nv; ++v) {
    double a[3], b[3];
    rt_apply(pe, pts + 3 * v, a);
    rt_apply(pg, pts + 3 * v, b);
    double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    sum += sqrt((dx * dx + dy * dy) + dz * dz);
  }
  return sum / (double)nv;
}

double oracle_adi(const double* pts, int64_t nv, const double* pe, const double* pg) {
  /* Exact NN distance from each GT-pose vertex to the est-pose vertex set
     (pose_error.py:175-183; cKDTree's answer is the exact NN distance). */
  double* e = (double*)malloc(sizeof(double) * 3 * (size_t)nv);
  for (int64_t v = 0; v < nv; ++v) rt_apply(pe, pts + 3 * v, e + 3 * v);
  double sum = 0.0;
  for (int64_t i = 0; i < nv; ++i) {
    double g[3];
    rt_apply(pg, pts + 3 * i, g);
    double best = INFINITY;
    for (int64_t j = 0; j < nv; ++j) {
      double dx = e[3 * j] - g[0], dy = e[3 * j + 1] - g[1], dz = e[3 * j + 2] - g[2];
      double d2 = (dx * dx + dy * dy) + dz * dz;
      if (d2 < best) best = d2;
    }
    sum += sqrt(best);
  }
  free(e);
  return sum / (double)nv;
}

double oracle_proj(const double* pts, int64_t nv, const double* pe, const double* pg,
                   const double* K) {
  double Pe[12], Pg[12], sum = 0.0;
  proj_matrix(K, pe, Pe);
  proj_matrix(K, pg, Pg);
  for (int64_t v = 0; v < nv; ++v) {
    double a[2], b[2];
    project(Pe, pts + 3 * v, a);
    project(Pg, pts + 3 * v, b);
    double du = a[0] - b[0], dv = a[1] - b[1];
    sum += sqrt(du * du + dv * dv);
  }
  return sum / (double)nv;
}

/* -------------------------------------------- depth -> distance, visibility */
void oracle_dist_im(const float* depth, int W, int H, double fx, double fy, double cx,
                    double cy, double* out) {
  /* pre_Xs = (xs - cx) / fx ; dist = sqrt((pX*d)**2 + (pY*d)**2 + d**2) in f64,
     summed left to right (misc.py:137-138, 158-161). */
  for (int r = 0; r < H; ++r) {
    double pY = ((double)r - cy) / fy;
    for (int c = 0; c < W; ++c) {
      double pX = ((double)c - cx) / fx;
      double d = (double)depth[(size_t)r * W + c];
      double a = pX * d, b = pY * d;
      out[(size_t)r * W + c] = sqrt((a * a + b * b) + d * d);
    }
  }
}

static int visib_px(double dt, double dm, float delta32, double delta64, int delta_f64, int mode) {
  float diff = (float)dm - (float)dt; /* visibility.py:31/35 */
  int le = delta_f64 ? ((double)diff <= delta64) : (diff <= delta32);
  if (mode == 0) return le && (dt > 0) && (dm > 0); /* bop18 :29-32 */
  return (le || dt == 0) && (dm > 0);               /* bop19 :34-37 */
}

void oracle_visib_mask(int64_t n, const double* d_test, const double* d_model,
                       const uint8_t* visib_gt, double delta, int delta_f64, int mode,
                       uint8_t* out) {
  float delta32 = (float)delta;
  for (int64_t i = 0; i < n; ++i) {
    int v = visib_px(d_test[i], d_model[i], delta32, delta, delta_f64, mode);
    if (visib_gt) v = v || (visib_gt[i] && d_model[i] > 0); /* visibility.py:74 */
    out[i] = (uint8_t)v;
  }
}

/* VSD given the three depth maps (pose_error.py:47-93). Returns 0, or -1 on a bad
   cost type with a non-empty union (the reference raises only then, :87-88). */
int oracle_vsd_depths(int W, int H, const float* depth_test, const float* depth_est,
                      const float* depth_gt, double fx, double fy, double cx, double cy,
                      double delta, int delta_f64, const double* taus, int n_tau,
                      int normalized, double diameter, int cost_type, double* out) {
  float delta32 = (float)delta;
  int64_t n_union = 0, n_inter = 0;
  int64_t cnt[64];
  double lin[64];
  for (int k = 0; k < n_tau; ++k) cnt[k] = 0, lin[k] = 0.0;
  for (int r = 0; r < H; ++r) {
    double pY = ((double)r - cy) / fy;
    for (int c = 0; c < W; ++c) {
      double pX = ((double)c - cx) / fx;
      size_t i = (size_t)r * W + c;
      double dist[3];
      float dep[3] = {depth_test[i], depth_gt[i], depth_est[i]};
      for (int k = 0; k < 3; ++k) {
        double d = (double)dep[k], a = pX * d, b = pY * d;
        dist[k] = sqrt((a * a + b * b) + d * d);
      }
      int vg = visib_px(dist[0], dist[1], delta32, delta, delta_f64, 1);
      int ve = visib_px(dist[0], dist[2], delta32, delta, delta_f64, 1);
      ve = ve || (vg && dist[2] > 0);
      if (vg || ve) ++n_union;
      if (vg && ve) {
        ++n_inter;
        double dd = fabs(dist[1] - dist[2]);
        if (normalized) dd /= diameter;
        for (int k = 0; k < n_tau; ++k) {
          if (dd >= taus[k]) ++cnt[k];
          double cst = dd / taus[k];
          lin[k] += cst > 1.0 ? 1.0 : cst;
        }
      }
    }
  }
  if (n_union == 0) {
    for (int k = 0; k < n_tau; ++k) out[k] = 1.0;
    return 0;
  }
  if (cost_type != ORACLE_COST_STEP && cost_type != ORACLE_COST_TLINEAR) return -1;
  int64_t comp = n_union - n_inter;
  for (int k = 0; k < n_tau; ++k) {
    if (cost_type == ORACLE_COST_STEP)
      out[k] = (double)(cnt[k] + comp) / (double)n_union;
    else
      out[k] = (lin[k] + (double)comp) / (double)n_union;
  }
  return 0;
}

/* ------------------------------------------------------------ depth raster */
/* Spec v5:
 *  - R, t, fx, fy, cx, cy rounded to float32 (GL uniforms, renderer_vispy.py:441-442);
 *    vertices float32 (renderer_vispy.py:373).
 *  - X = ((r0*x + r1*y) + r2*z) + t, float32, no FMA; valid iff Z > 0.
 *  - iz = 1.0f / Z, u = (fx*X)*iz + cx, v = (fy*Y)*iz + cy (float32);
 *    valid iff |u|,|v| <= 16384.
 *  - Snap to 1/256 px: U = rint(u*256), V = rint(v*256).
 *  - Pixel (c, r) samples (256c+128, 256r+128) (= pixel centre (c+0.5, r+0.5)).
 *  - Integer edge functions, top-left fill rule, both windings (no culling).
 *  - 1/Z is affine in screen space: per triangle (vertices a, b, c with area > 0),
 *    all float32: inv = 1.0f / (float)(double)area, dza = iz_a - iz_c, dzb = iz_b - iz_c,
 *      ga = ((float)(Vb - Vc)*dza + (float)(Vc - Va)*dzb) * inv
 *      gb = ((float)(Uc - Ub)*dza + (float)(Ua - Uc)*dzb) * inv
 *    and per fragment  q = fmaf(ga, (float)(px - Ua), fmaf(gb, (float)(py - Va), iz_a))
 *    (spec v5: fused, one rounding per step).
 *  - A triangle is regular iff |ga|, |gb| <= 2^64 and 2^10 * area >= bw^2 + bh^2
 *    (area = twice the fixed-point area, bw / bh = fixed-point bbox extents, exact
 *    integers); an irregular triangle's q is clamped: q = fminf(q, izmax), izmax the
 *    largest vertex iz (a NaN q becomes izmax). Every fragment is then <= izmax * (1 + 2^-8)
 *    (DESIGN.md §4), the bound k_vsd's occlusion test relies on.
 *    Fragments with q <= 0 are dropped.
 *  - z-test: keep the largest q per pixel; depth = 1.0f / q_max (float32), 0 = background.
 *    Since RN(1/x) is monotone, this equals min over fragments of RN(1/q).
 * The HIP rasteriser (bop_toolkit_amd/csrc/raster.h) must match this bit for bit. */
typedef struct {
  int32_t U, V;
  float iz;
  int ok;
} ovtx;

static ovtx oracle_vertex(const float* Rf, const float* tf, float fx, float fy, float cx,
                          float cy, const float* p) {
  ovtx o;
  float X = ((Rf[0] * p[0] + Rf[1] * p[1]) + Rf[2] * p[2]) + tf[0];
  float Y = ((Rf[3] * p[0] + Rf[4] * p[1]) + Rf[5] * p[2]) + tf[1];
  float Z = ((Rf[6] * p[0] + Rf[7] * p[1]) + Rf[8] * p[2]) + tf[2];
  o.ok = 0;
  o.U = o.V = 0;
  o.iz = 0.0f;
  if (!(Z > 0.0f)) return o;
  float iz = 1.0f / Z;
  float u = (fx * X) * iz + cx;
  float v = (fy * Y) * iz + cy;
  if (!(fabsf(u) <= 16384.0f) || !(fabsf(v) <= 16384.0f)) return o;
  o.U = (int32_t)rintf(u * 256.0f);
  o.V = (int32_t)rintf(v * 256.0f);
  o.iz = iz;
  o.ok = 1;
  return o;
}

static int64_t floor_div256(int64_t a) { return a >= 0 ? a / 256 : -((-a + 255) / 256); }

static int64_t edge(const ovtx* a, const ovtx* b, int64_t px, int64_t py) {
  return (int64_t)(b->U - a->U) * (py - a->V) - (int64_t)(b->V - a->V) * (px - a->U);
}

static int top_left(const ovtx* a, const ovtx* b) {
  int32_t dx = b->U - a->U, dy = b->V - a->V;
  return dy < 0 || (dy == 0 && dx > 0);
}

/* Rasterise into q-buffer `qbuf` (largest 1/Z per pixel, 0 = empty). */
static void raster_tri(ovtx a, ovtx b, ovtx c, int W, int H, float* qbuf) {
  if (!a.ok || !b.ok || !c.ok) return;
  int64_t area = edge(&a, &b, c.U, c.V);
  if (area == 0) return;
  if (area < 0) {
    ovtx tmp = b;
    b = c;
    c = tmp;
    area = -area;
  }
  float inv_area = 1.0f / (float)(double)area;
  float dza = a.iz - c.iz, dzb = b.iz - c.iz;
  float ga = ((float)(b.V - c.V) * dza + (float)(c.V - a.V) * dzb) * inv_area;
  float gb = ((float)(c.U - b.U) * dza + (float)(a.U - c.U) * dzb) * inv_area;
  int32_t minU = a.U < b.U ? (a.U < c.U ? a.U : c.U) : (b.U < c.U ? b.U : c.U);
  int32_t maxU = a.U > b.U ? (a.U > c.U ? a.U : c.U) : (b.U > c.U ? b.U : c.U);
  int32_t minV = a.V < b.V ? (a.V < c.V ? a.V : c.V) : (b.V < c.V ? b.V : c.V);
  int32_t maxV = a.V > b.V ? (a.V > c.V ? a.V : c.V) : (b.V > c.V ? b.V : c.V);
  /* pixel c covers centre 256c+128: c in [ceil((minU-128)/256), floor((maxU-128)/256)] */
  int64_t c0 = -floor_div256(-((int64_t)minU - 128)), c1 = floor_div256((int64_t)maxU - 128);
  int64_t r0 = -floor_div256(-((int64_t)minV - 128)), r1 = floor_div256((int64_t)maxV - 128);
  if (c0 < 0) c0 = 0;
  if (r0 < 0) r0 = 0;
  if (c1 > W - 1) c1 = W - 1;
  if (r1 > H - 1) r1 = H - 1;
  float izmax = a.iz > b.iz ? a.iz : b.iz;
  if (c.iz > izmax) izmax = c.iz;
  int64_t bw = (int64_t)maxU - minU, bh = (int64_t)maxV - minV;
  int regular = fabsf(ga) <= 0x1p64f && fabsf(gb) <= 0x1p64f && (area << 10) >= bw * bw + bh * bh;
  int tl0 = top_left(&b, &c), tl1 = top_left(&c, &a), tl2 = top_left(&a, &b);
  for (int64_t r = r0; r <= r1; ++r) {
    int64_t py = 256 * r + 128;
    for (int64_t col = c0; col <= c1; ++col) {
      int64_t px = 256 * col + 128;
      int64_t w0 = edge(&b, &c, px, py), w1 = edge(&c, &a, px, py), w2 = edge(&a, &b, px, py);
      if (!(w0 > 0 || (w0 == 0 && tl0))) continue;
      if (!(w1 > 0 || (w1 == 0 && tl1))) continue;
      if (!(w2 > 0 || (w2 == 0 && tl2))) continue;
      float q = fmaf(ga, (float)(px - a.U), fmaf(gb, (float)(py - a.V), a.iz));
      if (!regular) q = fminf(q, izmax);
      float* o = qbuf + (size_t)r * W + col;
      if (q > *o) *o = q;
    }
  }
}

void oracle_render_depth(const double* pts, int64_t nv, const uint32_t* faces, int64_t nf,
                         const double* R, const double* t, double fx, double fy, double cx,
                         double cy, int W, int H, float* out) {
  float Rf[9], tf[3];
  for (int i = 0; i < 9; ++i) Rf[i] = (float)R[i];
  for (int i = 0; i < 3; ++i) tf[i] = (float)t[i];
  float fxf = (float)fx, fyf = (float)fy, cxf = (float)cx, cyf = (float)cy;
  ovtx* vt = (ovtx*)malloc(sizeof(ovtx) * (size_t)(nv > 0 ? nv : 1));
  for (int64_t v = 0; v < nv; ++v) {
    float p[3] = {(float)pts[3 * v], (float)pts[3 * v + 1], (float)pts[3 * v + 2]};
    vt[v] = oracle_vertex(Rf, tf, fxf, fyf, cxf, cyf, p);
  }
  memset(out, 0, sizeof(float) * (size_t)W * H);
  for (int64_t f = 0; f < nf; ++f) {
    uint32_t i0 = faces[3 * f], i1 = faces[3 * f + 1], i2 = faces[3 * f + 2];
    if (i0 >= nv || i1 >= nv || i2 >= nv) continue;
    raster_tri(vt[i0], vt[i1], vt[i2], W, H, out);
  }
  for (size_t i = 0; i < (size_t)W * H; ++i)
    if (out[i] > 0.0f) out[i] = 1.0f / out[i];
  free(vt);
}

/* Coverage count raster (test helper for the fill-rule property tests). */
void oracle_coverage(const double* pts, int64_t nv, const uint32_t* faces, int64_t nf,
                     const double* R, const double* t, double fx, double fy, double cx,
                     double cy, int W, int H, int32_t* out) {
  float Rf[9], tf[3];
  for (int i = 0; i < 9; ++i) Rf[i] = (float)R[i];
  for (int i = 0; i < 3; ++i) tf[i] = (float)t[i];
  memset(out, 0, sizeof(int32_t) * (size_t)W * H);
  for (int64_t f = 0; f < nf; ++f) {
    ovtx v3[3];
    int ok = 1;
    for (int k = 0; k < 3; ++k) {
      uint32_t id = faces[3 * f + k];
      float p[3] = {(float)pts[3 * id], (float)pts[3 * id + 1], (float)pts[3 * id + 2]};
      v3[k] = oracle_vertex(Rf, tf, (float)fx, (float)fy, (float)cx, (float)cy, p);
      ok &= v3[k].ok;
    }
    if (!ok) continue;
    ovtx a = v3[0], b = v3[1], c = v3[2];
    int64_t area = edge(&a, &b, c.U, c.V);
    if (area == 0) continue;
    if (area < 0) {
      ovtx tmp = b;
      b = c;
      c = tmp;
    }
    int tl0 = top_left(&b, &c), tl1 = top_left(&c, &a), tl2 = top_left(&a, &b);
    for (int r = 0; r < H; ++r)
      for (int col = 0; col < W; ++col) {
        int64_t px = 256 * (int64_t)col + 128, py = 256 * (int64_t)r + 128;
        int64_t w0 = edge(&b, &c, px, py), w1 = edge(&c, &a, px, py), w2 = edge(&a, &b, px, py);
        if ((w0 > 0 || (w0 == 0 && tl0)) && (w1 > 0 || (w1 == 0 && tl1)) &&
            (w2 > 0 || (w2 == 0 && tl2)))
          out[(size_t)r * W + col] += 1;
      }
  }
}

/* ------------------------------------------------ z-buffer quantisation model */
/* The depth vispy returns is not the eye Z but its window depth, stored in the
   depth render buffer (gloo.RenderBuffer, renderer_vispy.py:294: the driver
   picks the format, typically 24-bit fixed point, 16 or 32F possible), read
   back as float32 (:526) and linearised in float64 (:532-535; NumPy 2 promotes
   the float32 buffer by the float64 scalars, NEP 50). Model, per render:
   - near / far = min / max over the model's 8 bbox corners (misc.calc_3d_bbox
     of the float64 PLY points, :313-324) of the float32 view row 2 (:440-452),
     evaluated in float64;
   - window depth of a pixel whose spec depth is Z (float32 eye Z):
     z_w = f (Z - n) / (Z (f - n)) (the y_down projection of _calc_calib_proj,
     :187-232, glDepthRange 0..1), exact (float64);
   - stored: bits 32 -> (float)z_w; bits 24 / 16 -> D = round(z_w (2^b - 1))
     as unorm, read back as (float)(D / (2^b - 1)); z_w < 0 (Z below the near
     plane by rounding; GL would clip) stored as 0;
   - background where the read value is 1 (cleared, :534-536), else
     depth = mult / (zr + addi), mult = n f / (n - f), addi = f / (n - f).
   bits 0 returns the spec depth itself (widened to float64). */
static void zbuf_depth(const float* spec, int W, int H, const double* bbmin, const double* bbsz,
                       const double* pose, int bits, double* out) {
  const float r6 = (float)pose[6], r7 = (float)pose[7], r8 = (float)pose[8], tz = (float)pose[11];
  double n = INFINITY, f = -INFINITY;
  for (int k = 0; k < 8; ++k) {
    double x = bbmin[0] + ((k >> 2) & 1 ? bbsz[0] : 0.0);
    double y = bbmin[1] + ((k >> 1) & 1 ? bbsz[1] : 0.0);
    double z = bbmin[2] + (k & 1 ? bbsz[2] : 0.0);
    double ez = (((double)r6 * x + (double)r7 * y) + (double)r8 * z) + (double)tz;
    if (ez < n) n = ez;
    if (ez > f) f = ez;
  }
  const double mult = (n * f) / (n - f), addi = f / (n - f);
  const double scale = bits == 24 ? 16777215.0 : 65535.0;
  for (size_t i = 0; i < (size_t)W * H; ++i) {
    const float Z = spec[i];
    if (bits == 0 || !(Z > 0.0f)) {
      out[i] = (double)Z;
      continue;
    }
    double zw = f * ((double)Z - n) / ((double)Z * (f - n));
    float zr;
    if (bits == 32) {
      zr = (float)zw;
    } else {
      double D = floor((zw < 0.0 ? 0.0 : zw) * scale + 0.5);
      if (D > scale) D = scale;
      zr = (float)(D / scale);
    }
    out[i] = zr == 1.0f ? 0.0 : mult / ((double)zr + addi);
  }
}

/* VSD of pose_error.py:47-93 (step cost) with float64 model depths. */
static void vsd_step64(int W, int H, const float* depth_test, const double* de, const double* dg,
                       double fx, double fy, double cx, double cy, double delta,
                       const double* taus, int n_tau, double diameter, double* out) {
  float delta32 = (float)delta;
  int64_t n_union = 0, n_inter = 0, cnt[64];
  for (int k = 0; k < n_tau; ++k) cnt[k] = 0;
  for (int r = 0; r < H; ++r) {
    double pY = ((double)r - cy) / fy;
    for (int c = 0; c < W; ++c) {
      double pX = ((double)c - cx) / fx;
      size_t i = (size_t)r * W + c;
      double dep[3] = {(double)depth_test[i], dg[i], de[i]}, dist[3];
      for (int k = 0; k < 3; ++k) {
        double d = dep[k], a = pX * d, b = pY * d;
        dist[k] = sqrt((a * a + b * b) + d * d);
      }
      int vg = visib_px(dist[0], dist[1], delta32, delta, 0, 1);
      int ve = visib_px(dist[0], dist[2], delta32, delta, 0, 1);
      ve = ve || (vg && dist[2] > 0);
      if (vg || ve) ++n_union;
      if (vg && ve) {
        ++n_inter;
        double dd = fabs(dist[1] - dist[2]) / diameter;
        for (int k = 0; k < n_tau; ++k)
          if (dd >= taus[k]) ++cnt[k];
      }
    }
  }
  for (int k = 0; k < n_tau; ++k)
    out[k] = n_union == 0 ? 1.0 : (double)(cnt[k] + (n_union - n_inter)) / (double)n_union;
}

/* Per tuple: both spec renders once, then the step-cost VSD (normalised by the
   diameter) under every z-buffer model of `bits` (n_modes entries of 0 / 32 /
   24 / 16): out[(i * n_modes + m) * n_tau + k]. OpenMP over tuples. */
void oracle_vsd_zbuf_batch(int64_t n, const int32_t* obj, const int64_t* pts_off,
                           const int64_t* nv, const double* pts_all, const int64_t* face_off,
                           const int64_t* nf, const uint32_t* faces_all, const double* pose_est,
                           const double* pose_gt, const int32_t* frame_idx, const float* frames,
                           int W, int H, const double* cam, double delta, const double* taus,
                           int n_tau, const double* diameters, int n_modes, const int32_t* bits,
                           double* out) {
#pragma omp parallel
  {
    float* se = (float*)malloc(sizeof(float) * (size_t)W * H);
    float* sg = (float*)malloc(sizeof(float) * (size_t)W * H);
    double* de = (double*)malloc(sizeof(double) * (size_t)W * H);
    double* dg = (double*)malloc(sizeof(double) * (size_t)W * H);
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = 0; i < n; ++i) {
      int o = obj[i];
      const double* pts = pts_all + 3 * pts_off[o];
      double bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int64_t v = 0; v < nv[o]; ++v)
        for (int a = 0; a < 3; ++a) {
          if (pts[3 * v + a] < bmin[a]) bmin[a] = pts[3 * v + a];
          if (pts[3 * v + a] > bmax[a]) bmax[a] = pts[3 * v + a];
        }
      double bsz[3] = {bmax[0] - bmin[0], bmax[1] - bmin[1], bmax[2] - bmin[2]};
      const uint32_t* fc = faces_all + 3 * face_off[o];
      const double* cm = cam + 4 * frame_idx[i];
      const double* pe = pose_est + 12 * i;
      const double* pg = pose_gt + 12 * i;
      oracle_render_depth(pts, nv[o], fc, nf[o], pe, pe + 9, cm[0], cm[1], cm[2], cm[3], W, H, se);
      oracle_render_depth(pts, nv[o], fc, nf[o], pg, pg + 9, cm[0], cm[1], cm[2], cm[3], W, H, sg);
      for (int m = 0; m < n_modes; ++m) {
        zbuf_depth(se, W, H, bmin, bsz, pe, bits[m], de);
        zbuf_depth(sg, W, H, bmin, bsz, pg, bits[m], dg);
        vsd_step64(W, H, frames + (size_t)frame_idx[i] * W * H, de, dg, cm[0], cm[1], cm[2],
                   cm[3], delta, taus, n_tau, diameters[i], out + ((size_t)i * n_modes + m) * n_tau);
      }
    }
    free(se);
    free(sg);
    free(de);
    free(dg);
  }
}

/* ------------------------------------------------ batched BOP19 CPU baseline */
/* One BOP19 tuple = VSD (n_tau) + MSSD + MSPD for an (est, gt) pair, computed
   as the reference does per tuple (two full-frame renders, three full-frame
   distance conversions, per-symmetry loops). OpenMP over tuples. Objects are
   passed as flat arrays with per-object offsets. */
void oracle_bop19_batch(int64_t n, const int32_t* obj, const int64_t* pts_off,
                        const int64_t* nv, const double* pts_all, const int64_t* face_off,
                        const int64_t* nf, const uint32_t* faces_all, const int64_t* sym_off,
                        const int64_t* ns, const double* syms_all, const double* pose_est,
                        const double* pose_gt, const int32_t* frame_idx, const float* frames,
                        int W, int H, const double* cam, double delta, const double* taus,
                        int n_tau, const double* diameters, double* out_vsd,
                        double* out_mssd, double* out_mspd) {
#pragma omp parallel
  {
    float* de = (float*)malloc(sizeof(float) * (size_t)W * H);
    float* dg = (float*)malloc(sizeof(float) * (size_t)W * H);
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = 0; i < n; ++i) {
      int o = obj[i];
      const double* pts = pts_all + 3 * pts_off[o];
      const uint32_t* fc = faces_all + 3 * face_off[o];
      const double* cm = cam + 4 * frame_idx[i];
      const double* pe = pose_est + 12 * i;
      const double* pg = pose_gt + 12 * i;
      double K[9] = {cm[0], 0.0, cm[2], 0.0, cm[1], cm[3], 0.0, 0.0, 1.0};
      oracle_render_depth(pts, nv[o], fc, nf[o], pe, pe + 9, cm[0], cm[1], cm[2], cm[3], W, H, de);
      oracle_render_depth(pts, nv[o], fc, nf[o], pg, pg + 9, cm[0], cm[1], cm[2], cm[3], W, H, dg);
      oracle_vsd_depths(W, H, frames + (size_t)frame_idx[i] * W * H, de, dg, cm[0], cm[1], cm[2],
                        cm[3], delta, 0, taus, n_tau, 1, diameters[i], ORACLE_COST_STEP,
                        out_vsd + (size_t)i * n_tau);
      out_mssd[i] = oracle_mssd(pts, nv[o], syms_all + 12 * sym_off[o], ns[o], pe, pg);
      out_mspd[i] = oracle_mspd(pts, nv[o], syms_all + 12 * sym_off[o], ns[o], pe, pg, K);
    }
    free(de);
    free(dg);
  }
}
