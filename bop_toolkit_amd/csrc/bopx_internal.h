// bopx_internal.h — device-side data layout shared by the gfx950 kernels and the
// runtime (runtime.hip). Not part of the public C-ABI (include/bopx.h).
//
// HBM layout of one registered object:
//   pts   : float64 SoA  x[nv] | y[nv] | z[nv]       (point errors, fp64 math)
//   vtx   : float32x4    (x, y, z, 0) per vertex     (rasteriser, GL-like fp32)
//   faces : uint32 x3 per triangle, re-ordered into meshlets of 64 triangles
//           sorted by the Morton code of the triangle centroid
//   mlet  : float32 x32 per meshlet: the 8 corners (xyz) of an oriented
//           bounding box of the meshlet's float32 vertices (conservative culling),
//           then the normal cone (axis xyz, cos alpha) and bounding sphere
//           (centre xyz, radius): back-facing classification (runtime.cpp meshlet_cone)
//   syms  : float64 x12 per symmetry [R row-major | t]
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bopx {

// Pointer into global memory (address space 1). Device code that reads a
// pointer out of memory (e.g. from ObjDesc) only knows it as a generic pointer
// and emits flat_load; casting to gptr gives global_load, which is tracked by
// vmcnt alone and can stay in flight across LDS waits.
template <class T>
using gptr = __attribute__((address_space(1))) T*;
typedef float f32x4 __attribute__((ext_vector_type(4)));  // native vector: works in any addrspace
typedef float f32x3 __attribute__((ext_vector_type(3)));

constexpr int kMeshletTris = 64;    // one wave lane per triangle
constexpr int kMeshletVerts = 64;   // unique vertices per meshlet (one per lane)
constexpr int kMletFloats = 32;     // per-meshlet culling record (ObjDesc::mlet)
#ifndef BOPX_MAX_MESHLETS
#define BOPX_MAX_MESHLETS 1024
#endif
#ifndef BOPX_TILE_W
#define BOPX_TILE_W 64
#define BOPX_TILE_H 64
#endif
constexpr int kMaxMeshlets = BOPX_MAX_MESHLETS;  // per object with rectangles in registers (VSD)
constexpr int kMaxTaus = 16;
constexpr int kVsdMaxTiles = 2048;  // k_vsd keeps 16-bit per-lane tau counters
constexpr int kCostCover = 2;  // k_vsd mode: silhouette union/inter + bboxes (cus, cou_bb_proj)
constexpr int kCoverCols = 10;  // union, inter, est bbox x0 y0 x1 y1, gt bbox x0 y0 x1 y1
constexpr int kCostGtInfo = 3;  // k_vsd mode: one (gt) pose, silhouette + visibility stats
constexpr int kGtInfoCols = 11;  // all, visib, obj bbox x0 y0 x1 y1, visib bbox, valid
// k_vsd mode: one pose rendered into an HBM q buffer over its ROI (VsdArgs::rois,
// qoff, qbuf), shared by every VSD tuple that uses the pose (k_vsd_pair)
constexpr int kCostRender = 4;
constexpr int kTileW = BOPX_TILE_W;  // VSD screen tile (LDS-resident q pair)
constexpr int kTileH = BOPX_TILE_H;
#ifndef BOPX_TILE_STRIDE
#define BOPX_TILE_STRIDE (BOPX_TILE_W + 1)
#endif
constexpr int kTileStride = BOPX_TILE_STRIDE;  // LDS row pitch of a q tile (dwords)
static_assert(kTileStride > kTileW, "the row walk may touch the column right of a tile");
constexpr float kGuardBand = 16384.0f;  // |u|,|v| limit of a rasterised vertex (px)

struct ObjDesc {
  const double* pts;         // 3*nv, SoA
  const float4* vtx;         // nv
  const uint32_t* faces;     // 3*nf (meshlet order)
  const float* mlet;         // kMletFloats*nm: OBB corners, normal cone, sphere per meshlet
  const int4* mlet_info;     // nm: {first triangle, #triangles, first vertex slot, #vertices}
  const float4* mlet_vtx;    // nm x 64: meshlet-local vertex blocks, fixed stride
                             // (vertices shared by neighbouring meshlets are duplicated)
  const uint32_t* mlet_tri;  // nm x 64: local indices a | b << 8 | c << 16, 0xFFFFFFFF = none
  const double* syms;        // 12*ns
  const double* seed;        // 3*nseed SoA: farthest-point-sampled vertices (MSSD/MSPD pruning)
  int nv, nf, nm, ns, nseed;
};
constexpr int kSymSeeds = 128;  // seed vertices per object (k_sym_error's symmetry bounds)

struct VsdArgs {
  const ObjDesc* objs;
  const int32_t* slots;
  const double* pose_est;
  const double* pose_gt;
  const int32_t* frame_idx;
  const float* frames;
  const double* cam;  // per frame: fx fy cx cy
  const double* diameters;
  double* out;
  int64_t n;
  int width, height;
  float delta32;
  int delta_f64;
  double delta64;
  // float32 threshold equivalent to the visibility compare (visib_thr32 in runtime.cpp)
  float dthr;
  int n_tau;
  int normalized;
  int max_nm;        // most meshlets of a registered object (sizes the rect registers)
  int img_w, img_h;  // test-depth frame size (= width/height except GT-info mode)
  int ox, oy;        // image origin inside the raster canvas (GT-info mode)
  uint8_t* masks;    // GT-info mode, optional: n x 2 x img_h x img_w (mask, mask_visib)
  const int32_t* order;  // optional launch order (launch_order_by_slot): block k takes tuple order[k]
  int ablate;  // BOPX_VSD_ABLATE, read only by -DBOPX_VSD_DIAG=1 builds (kern_vsd.hip)
  int cull;    // k_vsd occlusion test (BOPX_VSD_CULL; default -1 = back-face test for objects of
               // more than kCullAutoMeshlets meshlets)
  int qorder;  // k_vsd tile entry-queue order (BOPX_VSD_QORDER): 1 = large overlaps first
               // (default), 0 = near entries first; results are identical either way
  // Tile-parallel mode (every cost mode): `split` workgroups per tuple, workgroup
  // s walking ROI tiles s, s + split, ...; each writes one row of kVsdPartCols
  // doubles to `part` and k_vsd_combine reduces the rows in split order. Set by
  // launch_vsd (small batches, BOPX_VSD_SPLIT), 1 = one workgroup per tuple.
  // Tuples [0, split_from) of the launch order take one workgroup each, the
  // rest `split` each (0 for small batches; the tail of a large one otherwise).
  int split;
  int64_t split_from;
  double* part;
  double* unions;  // optional (BOPX_VSD_UNIONS): per tuple visibility-union pixel count
  // render mode (kCostRender): per render its ROI (x0, y0, x1, y1, from
  // launch_pose_roi) and the offset of its row-major q buffer in qbuf
  const int4* rois;
  const int64_t* qoff;
  uint32_t* qbuf;
  // ... and per ROI row the covered column span [smin, smax] (empty: INT_MAX, -1)
  const int64_t* rowoff;
  int32_t* smin;
  int32_t* smax;
  double taus[kMaxTaus];
};
constexpr int kVsdPartCols = 2 + 2 * kMaxTaus;  // union, inter, cnt[kMaxTaus], lin[kMaxTaus]
constexpr int kVsdMaxSplit = 16;

// Launchers (kernels in kern_pose.hip / kern_vsd.hip). All return hipError_t of
// the launch; inputs are device pointers.
hipError_t launch_sym_error(int mode, const ObjDesc* objs, int max_ns, int64_t n,
                            const int32_t* slots, const double* pe, const double* pg,
                            const double* K, double* out, const int32_t* order,
                            hipStream_t s);  // mode 0 = MSSD, 1 = MSPD; max_ns over objects
hipError_t launch_mean_error(int mode, const ObjDesc* objs, int64_t n, const int32_t* slots,
                             const double* pe, const double* pg, const double* K, double* out,
                             const int32_t* order, hipStream_t s);  // mode 0 = ADD, 1 = PROJ
hipError_t launch_adi(const ObjDesc* objs, int max_nv, int64_t n, const int32_t* slots,
                      const double* pe, const double* pg, double* out, const int32_t* order,
                      hipStream_t s);
// order: nullptr (block k takes tuple k) or a launch order from launch_order_by_slot
constexpr int kOrderMaxSlots = 16383;  // LDS buckets of k_order_by_slot
constexpr int kOrderCostClasses = 48;  // half-octave classes of the projected area (VSD order)
struct OrderCost {  // VSD inputs of the cost classes (pe == nullptr: order by slot only)
  const double* pe;
  const double* pg;
  const int32_t* frame_idx;
  const double* cam;
  const double* dia;
  const int32_t* slot_rank;  // pe == nullptr: key = slot_rank[slot] (slots by descending cost)
};
// keys: n int32 of scratch (the per-tuple sort keys)
hipError_t launch_order_by_slot(const int32_t* slots, int64_t n, int ns, int32_t* order,
                                int32_t* keys, hipStream_t s, const OrderCost* cost = nullptr);
hipError_t launch_vsd(const VsdArgs& a, int cost_type, hipStream_t s);  // or kCostCover

// Shared renders (GT-side / estimate reuse, multi-instance images): each
// distinct (object, pose, frame) is rasterised once (k_vsd, kCostRender) into an
// HBM q buffer over its ROI; every (est, gt) tuple then runs the VSD pixel pass
// on the two cached buffers (k_vsd_pair).
// ROI of each render: the union of its meshlet rectangles (k_vsd's own rule).
hipError_t launch_pose_roi(const ObjDesc* objs, int64_t n, const int32_t* slots,
                           const double* pose, const int32_t* frame_idx, const double* cam, int W,
                           int H, int4* rois, hipStream_t s);
struct PairArgs {
  const int4* rois;        // per render
  const int64_t* qoff;     // per render: offset of its q buffer in qbuf (dwords)
  const uint32_t* qbuf;    // q = 1/Z bits, 0 = background
  const int64_t* rowoff;   // per render: offset of its row spans in smin / smax
  const int32_t* smin;     // per ROI row: first / last covered column (INT_MAX / -1: none)
  const int32_t* smax;
  const int32_t* rframe;   // per render: frame index
  const int32_t* est_r;    // per tuple: render of the estimate
  const int32_t* gt_r;     // per tuple: render of the GT
  int64_t n_renders;       // render indices outside [0, n_renders) give NaN errors
  const float* frames;     // n_frames x H x W test depth
  const double* cam;       // per frame fx fy cx cy
  const double* diameters; // per tuple
  double* out;             // n x n_tau
  double* unions;          // optional: per tuple visibility-union count
  int64_t n;
  int width, height;
  float dthr;
  int n_tau, normalized;
  double taus[kMaxTaus];
};
hipError_t launch_vsd_pair(const PairArgs& a, int cost_type, hipStream_t s);
hipError_t launch_cover_depths(int W, int H, const float* de, const float* dg,
                               long long* acc /* kCoverCols, device */, hipStream_t s);
hipError_t read_vsd_stats(unsigned long long* out, int reset);  // diagnostics
// Load each translation unit's code object on the current device now (the
// runtime otherwise loads it at the first launch of one of its kernels):
// hipFuncGetAttributes on one kernel per unit.
hipError_t preload_pose_kernels();
hipError_t preload_vsd_kernels();
hipError_t preload_png_kernels();
hipError_t launch_vsd_depths(int W, int H, const float* dt, const float* de, const float* dg,
                             double fx, double fy, double cx, double cy, float delta32,
                             int delta_f64, double delta64, const double* taus_host, int n_tau,
                             int normalized, double diameter, double* partials, int n_blocks,
                             hipStream_t s);
int vsd_depths_blocks(int W, int H);
hipError_t launch_dist_im(int W, int H, const float* depth, double fx, double fy, double cx,
                          double cy, double* out, hipStream_t s);
hipError_t launch_visib(int64_t n, const double* dt, const double* dm, const uint8_t* vg,
                        float delta32, int delta_f64, double delta64, int mode, uint8_t* out,
                        hipStream_t s);
hipError_t launch_depth_fill(float* frames, int64_t n_pixels, int to_background,
                             hipStream_t s);
hipError_t launch_render_batch(const ObjDesc* objs, int max_nf, int64_t n, const int32_t* slots,
                               const double* pose, const int32_t* frame_idx, const double* cam,
                               float* frames, int W, int H, hipStream_t s);

// kern_png.hip: 16-bit grayscale PNG decode (bopx_png_decode_dev).
constexpr int kPngMaxWidth = 4096;  // k_png_unfilter's carry row (LDS)
constexpr int kPngMaxRaw = 1 << 28; // inflated bytes per frame, H * (2W + 1); the Adler-32
                                     // B sum (<= 255 N^2 / 2) fits in 64 bits up to here
hipError_t launch_png_decode(int64_t n, const uint8_t* zdata, const int64_t* z_off,
                             const int32_t* z_len, int H, int W, const float* scales, uint8_t* raw,
                             int64_t raw_stride, float* frames, int32_t* status, hipStream_t s);

}  // namespace bopx
