/*
 * bopx.h — C-ABI of the MI355X-native BOP pose-error evaluator (libbopx.so).
 *
 * This is the drop-in boundary for the reference's hot path:
 *   bop_toolkit_lib/pose_error.py   vsd :17-93, mssd :96-118, mspd :121-144,
 *                                   add :147-161, adi :164-184, proj :217-232
 *   bop_toolkit_lib/visibility.py   _estimate_visib_mask :9-42 (+ _gt :45, _est :58)
 *   bop_toolkit_lib/misc.py         depth_im_to_dist_im_fast :143-163
 *   bop_toolkit_lib/renderer.py     Renderer.add_object/remove_object/render_object :47-74
 *                                   (the vispy/glumpy/cpp depth rasterisers behind it:
 *                                    renderer_vispy.py:433-538, renderer_py.py:422-555,
 *                                    renderer_cpp.py:17-62)
 * The reference is pure Python; its "FFI" is the Python call surface above. The
 * ctypes binding lives in bop_toolkit_amd/_lib.py and is shown in INTEGRATION.md.
 *
 * Conventions
 *  - Every entry point returns an int status (BOPX_OK == 0). On failure the
 *    message is available from bopx_last_error(ctx) until the next call.
 *  - Poses are 12 doubles: R row-major (9) then t (3), i.e. [R | t] of
 *    x_cam = R x_model + t (reference: inout.py:250-253, misc.py:266-276).
 *  - Intrinsics are either a full row-major 3x3 K (9 doubles) or the 4-tuple
 *    (fx, fy, cx, cy) = (K[0,0], K[1,1], K[0,2], K[1,2]) exactly as the reference
 *    extracts them (pose_error.py:41, misc.py:137-138).
 *  - *_batch functions take caller-owned HOST buffers that are borrowed for the
 *    duration of the call (copied to HBM, computed, copied back, synchronised).
 *  - *_dev functions take DEVICE pointers, enqueue on `stream` (a hipStream_t;
 *    NULL = the null/default stream) and return without synchronising. Object
 *    references in *_dev calls are slots from bopx_object_slot(), not obj_ids.
 *  - One context per device per host thread; a context is not thread-safe
 *    (like the reference's singleton GL context, renderer_vispy.py:235-246).
 *  - Results are deterministic: integer LDS atomics only, fixed reduction order.
 */
#ifndef BOPX_H
#define BOPX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BOPX_OK 0
#define BOPX_E_INVALID 1     /* bad argument (shape, size, unknown mode)       */
#define BOPX_E_NOT_FOUND 2   /* unknown obj_id / slot                          */
#define BOPX_E_HIP 3         /* HIP runtime error                              */
#define BOPX_E_OOM 4         /* device allocation failed                       */
#define BOPX_E_UNSUPPORTED 5 /* input outside the kernels' supported envelope  */
#define BOPX_E_INTERNAL 6    /* object registry inconsistent (a registry update
                                failed part-way): no kernel is launched        */

/* VSD pixel matching cost (pose_error.py:82-88). */
#define BOPX_COST_STEP 0
#define BOPX_COST_TLINEAR 1

/* Visibility mode (visibility.py:29-40). */
#define BOPX_VISIB_BOP18 0
#define BOPX_VISIB_BOP19 1

/* Flags for delta handling (visibility.py:31,35-37). The reference compares the
 * float32 difference with `delta`; a Python float/int delta is weakly typed
 * under NumPy >= 2 and the comparison happens in float32 (the default here).
 * A numpy.float64 delta promotes the comparison to float64: set this flag. */
#define BOPX_DELTA_F64 1
/* Flag for the VSD entry points: also report each tuple's visibility-union
 * pixel count (pose_error.py:64), appended after the n x n_tau errors (out
 * then holds n x n_tau + n doubles). A union of 0 is the reference's
 * `[1.0] * len(taus)` branch (pose_error.py:75-76), whose elements are Python
 * floats rather than numpy.float64: the drop-in needs it to return the same
 * element types. */
#define BOPX_VSD_UNIONS 2

/* Maximum number of VSD misalignment tolerances per call (the Python layer,
 * bop_toolkit_amd.pose_error.vsd / batch.vsd, splits longer tau lists into
 * calls of at most this many, so callers see no limit). */
#define BOPX_MAX_TAUS 16

typedef struct bopx_ctx bopx_ctx;

/* ---- library / context --------------------------------------------------- */
int bopx_version(void); /* (major << 16) | minor */
int bopx_device_count(int* n);
int bopx_create(int device, bopx_ctx** out);
void bopx_destroy(bopx_ctx* ctx);
const char* bopx_last_error(const bopx_ctx* ctx);
int bopx_synchronize(bopx_ctx* ctx);
/* The context's HIP stream (hipStream_t) as an opaque pointer. */
void* bopx_stream(bopx_ctx* ctx);

/* ---- object registry (renderer.py:47-60; eval_calc_errors.py:162-191) ---- */
/* pts: nv x 3 float64 model vertices (inout.load_ply 'pts', models_eval).
 * faces: nf x 3 uint32 triangle indices (may be NULL with nf == 0; such an
 * object supports the point-based errors but not rendering / VSD). */
int bopx_add_object(bopx_ctx* ctx, int obj_id, const double* pts, int64_t nv,
                    const uint32_t* faces, int64_t nf);
int bopx_remove_object(bopx_ctx* ctx, int obj_id);
/* syms: ns x 12 (R row-major, t) from misc.get_symmetry_transformations
 * (misc.py:43-90); ns >= 1. */
int bopx_set_symmetries(bopx_ctx* ctx, int obj_id, const double* syms, int64_t ns);
/* bopx_set_symmetries for n objects in one call (one stream synchronisation and
 * one descriptor upload instead of n): object obj_ids[i] gets the ns[i] rows
 * starting at row sum(ns[0..i-1]) of syms. Nothing changes when an obj_id is
 * unknown or an ns[i] < 1 (checked before any upload), nor when an allocation
 * or copy fails (the new sets are uploaded first and swapped in only when all
 * are resident; the same holds for bopx_set_symmetries). */
int bopx_set_symmetries_many(bopx_ctx* ctx, int n, const int* obj_ids, const int64_t* ns,
                             const double* syms);
int bopx_object_slot(const bopx_ctx* ctx, int obj_id, int* slot);
/* Load the library's GPU code objects on the context's device now instead of
 * at the first launch of each (the first MSSD / VSD / PNG launch of a process
 * otherwise waits for it). Touches no other context state, so it may run on a
 * thread of its own while the caller registers objects. */
int bopx_preload(bopx_ctx* ctx);

/* ---- point-based pose errors, one output per tuple ----------------------- */
/* mssd: pose_error.py:96-118. */
int bopx_mssd_batch(bopx_ctx* ctx, int64_t n, const int32_t* obj_ids,
                    const double* pose_est, const double* pose_gt, double* out);
/* mspd: pose_error.py:121-144 (+ misc.project_pts :93-107); K: n x 9. */
int bopx_mspd_batch(bopx_ctx* ctx, int64_t n, const int32_t* obj_ids,
                    const double* pose_est, const double* pose_gt,
                    const double* K, double* out);
/* add: pose_error.py:147-161. */
int bopx_add_batch(bopx_ctx* ctx, int64_t n, const int32_t* obj_ids,
                   const double* pose_est, const double* pose_gt, double* out);
/* adi: pose_error.py:164-184 (cKDTree NN replaced by exact brute force). */
int bopx_adi_batch(bopx_ctx* ctx, int64_t n, const int32_t* obj_ids,
                   const double* pose_est, const double* pose_gt, double* out);
/* proj: pose_error.py:217-232; K: n x 9. */
int bopx_proj_batch(bopx_ctx* ctx, int64_t n, const int32_t* obj_ids,
                    const double* pose_est, const double* pose_gt,
                    const double* K, double* out);

/* ---- VSD with the on-device depth rasteriser ----------------------------- */
/* vsd: pose_error.py:17-93, both renders done by the HIP rasteriser.
 * frames: n_frames x height x width float32 test depth in mm (inout.load_depth
 * * depth_scale, eval_calc_errors.py:239-243); frame_idx: n (which frame each
 * tuple uses); cam: n_frames x 4 (fx, fy, cx, cy); diameters: n;
 * out: n x n_tau. Objects of any size (beyond 1024 meshlets the kernel
 * recomputes the meshlet rectangles per tile). */
int bopx_vsd_batch(bopx_ctx* ctx, int64_t n, const int32_t* obj_ids,
                   const double* pose_est, const double* pose_gt,
                   const int32_t* frame_idx, const float* frames, int64_t n_frames,
                   int width, int height, const double* cam, double delta, int flags,
                   const double* taus, int n_tau, int normalized_by_diameter,
                   const double* diameters, int cost_type, double* out);

/* vsd with shared renders: pose_error.py:17-93 for n (est, gt) tuples whose
 * poses come from a list of distinct renders (obj_id, pose 12, frame). The
 * reference renders both poses of every tuple (pose_error.py:42-45), and
 * eval_calc_errors.py:281-290 pairs every estimate with every GT instance of
 * its object, so an image with k instances and k estimates costs 2k^2 renders
 * there; here each render is rasterised once (2k) into an HBM depth buffer over
 * its ROI and every tuple runs the VSD pixel pass on its two buffers.
 * est_render / gt_render: n indices into the render list (both renders of a
 * tuple must use the same frame); everything else as bopx_vsd_batch. Step-cost
 * results are bit-identical to bopx_vsd_batch on the same tuples (tlinear:
 * float64 sums in another order, ~1e-13). */
int bopx_vsd_shared_batch(bopx_ctx* ctx, int64_t n_renders, const int32_t* render_obj_ids,
                          const double* render_poses, const int32_t* render_frame_idx,
                          int64_t n, const int32_t* est_render, const int32_t* gt_render,
                          const float* frames, int64_t n_frames, int width, int height,
                          const double* cam, double delta, int flags, const double* taus,
                          int n_tau, int normalized_by_diameter, const double* diameters,
                          int cost_type, double* out);

/* vsd given already-rendered depth maps (for foreign renderers, e.g. a
 * reference vispy/cpp renderer passed to pose_error.vsd). All maps h x w f32. */
int bopx_vsd_from_depths(bopx_ctx* ctx, int width, int height, const float* depth_test,
                         const float* depth_est, const float* depth_gt, double fx,
                         double fy, double cx, double cy, double delta, int flags,
                         const double* taus, int n_tau, int normalized_by_diameter,
                         double diameter, int cost_type, double* out);

/* ---- silhouette overlap: cus / cou_bb_proj (pose_error.py:256-330) -------- */
/* Both poses rasterised by the HIP rasteriser (the VSD raster spec). Per tuple
 * out[10] float64: pixel counts of the union and the intersection of the two
 * masks (depth > 0), then the est and the gt mask bbox (x0, y0, x1, y1,
 * inclusive pixel coordinates; an empty mask has x1 = y1 = -1). frame_idx
 * selects each tuple's camera row in cam (n_frames x 4: fx, fy, cx, cy). */
int bopx_cover_batch(bopx_ctx* ctx, int64_t n, const int32_t* obj_ids,
                     const double* pose_est, const double* pose_gt,
                     const int32_t* frame_idx, int64_t n_frames, int width, int height,
                     const double* cam, double* out);
/* The same from two already-rendered h x w float32 depth maps (foreign
 * renderers); out[10]. */
int bopx_cover_from_depths(bopx_ctx* ctx, int width, int height, const float* depth_est,
                           const float* depth_gt, double* out);

/* ---- GT-side statistics: calc_gt_info.py:95-160, calc_gt_masks.py:95-125 -- */
/* For n GT instances (obj_ids, pose n x 12 [R | t]) in test frames
 * (frames n_frames x height x width float32 depth in mm, cam n_frames x 4):
 * the instance is rasterised on a canvas canvas_scale (1 or 3) times the image
 * (3 = calc_gt_info's enlarged canvas, the image in its centre; 1 =
 * calc_gt_masks), compared with the test depth (bop19 visibility, tolerance
 * delta). out n x 11 float64: px_count_all (whole canvas silhouette),
 * px_count_visib, silhouette bbox (x0, y0, x1, y1 in image coordinates),
 * visible-part bbox (x0, y0, x1, y1; x1 = -1 when empty), px_count_valid.
 * masks (optional, NULL = none): n x 2 x height x width uint8, 255 inside the
 * silhouette (plane 0) and the visible part (plane 1), 0 elsewhere. */
int bopx_gt_info_batch(bopx_ctx* ctx, int64_t n, const int32_t* obj_ids, const double* pose,
                       const int32_t* frame_idx, const float* frames, int64_t n_frames,
                       int width, int height, const double* cam, double delta, int flags,
                       int canvas_scale, double* out, uint8_t* masks);

/* ---- renderer plugin (renderer.py:62-74) ---------------------------------- */
/* Depth (eye Z in model units, 0 = background) of one object in one pose;
 * out: height x width float32. */
int bopx_render_depth(bopx_ctx* ctx, int obj_id, const double* R, const double* t,
                      double fx, double fy, double cx, double cy, int width, int height,
                      float* out);

/* ---- geometry / visibility primitives ------------------------------------ */
/* misc.depth_im_to_dist_im_fast (misc.py:143-163): out h x w float64. */
int bopx_dist_im(bopx_ctx* ctx, int width, int height, const float* depth, double fx,
                 double fy, double cx, double cy, double* out);
/* visibility._estimate_visib_mask (+ the est-side OR of visibility.py:74 when
 * visib_gt != NULL): d_test, d_model n float64; out n uint8 (0/1). */
int bopx_visib_mask(bopx_ctx* ctx, int64_t n, const double* d_test, const double* d_model,
                    const uint8_t* visib_gt, double delta, int flags, int visib_mode,
                    uint8_t* out);

/* ---- device-pointer variants (all pointers in HBM; async on `stream`) ----- */
int bopx_mssd_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots,
                        const double* pose_est, const double* pose_gt, double* out,
                        void* stream);
int bopx_mspd_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots,
                        const double* pose_est, const double* pose_gt, const double* K,
                        double* out, void* stream);
int bopx_add_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots,
                       const double* pose_est, const double* pose_gt, double* out,
                       void* stream);
int bopx_adi_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots,
                       const double* pose_est, const double* pose_gt, double* out,
                       void* stream);
/* PROJ (pose_error.py:217-232); K n x 9 row-major. */
int bopx_proj_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots,
                        const double* pose_est, const double* pose_gt, const double* K,
                        double* out, void* stream);
int bopx_vsd_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots,
                       const double* pose_est, const double* pose_gt,
                       const int32_t* frame_idx, const float* frames, int width,
                       int height, const double* cam, double delta, int flags,
                       const double* taus, int n_tau, int normalized_by_diameter,
                       const double* diameters, int cost_type, double* out,
                       void* stream);
/* bopx_vsd_shared_batch on device pointers (render_slots: object slots). It
 * synchronises `stream` once (the renders' ROI sizes lay out the depth
 * buffers, stream-ordered scratch); render indices outside [0, n_renders) give
 * NaN errors for that tuple. */
int bopx_vsd_shared_batch_dev(bopx_ctx* ctx, int64_t n_renders, const int32_t* render_slots,
                              const double* render_poses, const int32_t* render_frame_idx,
                              int64_t n, const int32_t* est_render, const int32_t* gt_render,
                              const float* frames, int width, int height, const double* cam,
                              double delta, int flags, const double* taus, int n_tau,
                              int normalized_by_diameter, const double* diameters,
                              int cost_type, double* out, void* stream);
int bopx_cover_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots,
                         const double* pose_est, const double* pose_gt,
                         const int32_t* frame_idx, int width, int height, const double* cam,
                         double* out, void* stream);
int bopx_gt_info_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots, const double* pose,
                           const int32_t* frame_idx, const float* frames, int width,
                           int height, const double* cam, double delta, int flags,
                           int canvas_scale, double* out, uint8_t* masks, void* stream);
/* Composite render of many (object, pose) instances into frames:
 * frames (n_frames x h x w f32, device) must be pre-filled with +inf bit
 * patterns by bopx_depth_clear_dev; instances are min-composited (z-buffer);
 * bopx_depth_finish_dev maps +inf to 0 (background). Used to synthesise test
 * depth and by the batched renderer. */
int bopx_depth_clear_dev(bopx_ctx* ctx, float* frames, int64_t n_pixels, void* stream);
int bopx_render_depth_batch_dev(bopx_ctx* ctx, int64_t n, const int32_t* slots,
                                const double* pose, const int32_t* frame_idx,
                                const double* cam, float* frames, int width, int height,
                                void* stream);
int bopx_depth_finish_dev(bopx_ctx* ctx, float* frames, int64_t n_pixels, void* stream);

/* Depth PNG decode on the device (kern_png.hip), the GPU side of
 * inout.load_depth (bop_toolkit_lib/inout.py:39-46) + the float32
 * `depth *= depth_scale` (scripts/eval_calc_errors.py:242-243): n zlib
 * streams — the concatenated IDAT payloads of n 16-bit grayscale,
 * non-interlaced PNGs of height x width, as bopx_pack_depth_pngs
 * (include/bopx_io.h) lays them out — are inflated, unfiltered and scaled
 * into frames (n x height x width float32, dst = sample * scales[k], scales
 * NULL = 1). Device pointers:
 *   zdata   stream k at zdata + z_off[k] (a multiple of 256), z_len[k] bytes;
 *           readable for 2048 bytes past every stream's end;
 *   raw     scratch, n x raw_stride bytes, raw_stride >= round_up(height *
 *           (2 width + 1) + 64, 1024);
 *   status  2n int32: status[2k] = BOPX_PNG_OK or BOPX_PNG_CORRUPT (any
 *           defect: zlib header, Huffman code, distance, size, Adler-32, filter
 *           type); status[2k + 1] is scratch. A corrupt frame's pixels are
 *           undefined; decode that file on the host (bopx_load_depth_pngs),
 *           which reports the host path's own result or error.
 * width <= 4096, height * (2 width + 1) <= 2^28
 * (the Adler-32 sums of k_png_unfilter stay inside 64 bits). */
enum { BOPX_PNG_OK = 0, BOPX_PNG_CORRUPT = 2 };
int bopx_png_decode_dev(bopx_ctx* ctx, int64_t n, const uint8_t* zdata, const int64_t* z_off,
                        const int32_t* z_len, int height, int width, const float* scales,
                        uint8_t* raw, int64_t raw_stride, float* frames, int32_t* status,
                        void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BOPX_H */
