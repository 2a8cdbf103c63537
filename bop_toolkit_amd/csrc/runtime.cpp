// runtime.cpp — libbopx host runtime: contexts, the on-device object registry
// (meshes, meshlets, symmetry tables) and the C-ABI of include/bopx.h.
//
// The registry is what renderer.add_object (renderer_vispy.py:291-418) and the
// per-dataset precompute of eval_calc_errors.py:162-191 (models, symmetries)
// amount to: every object is uploaded once and stays resident in HBM, so a
// batch of tuples touches only its poses, its test depth and its outputs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/bopx.h"
#include "bopx_internal.h"

using bopx::ObjDesc;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
};

struct Object {
  int obj_id = -1;
  bool live = false;
  int64_t nv = 0, nf = 0, nm = 0, ns = 0;
  double* d_pts = nullptr;
  float4* d_vtx = nullptr;
  uint32_t* d_faces = nullptr;
  float* d_mlet = nullptr;
  int4* d_minfo = nullptr;
  float4* d_mvtx = nullptr;
  uint32_t* d_mtri = nullptr;
  double* d_syms = nullptr;
  double* d_seed = nullptr;
  int64_t nseed = 0;
};

}  // namespace

struct bopx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::unordered_map<int, int> slot_of;
  std::vector<Object> objs;
  ObjDesc* d_desc = nullptr;
  int32_t* d_rank = nullptr;  // slot -> rank by descending symmetry-error cost (nv * ns)
  size_t desc_cap = 0;
  int max_nf = 0;
  int max_nv = 0;  // most vertices of a live object (ADI scratch stride)
  int max_ns = 0;  // most symmetries of a live object (MSSD/MSPD grid)
  int max_nm = 0;  // most meshlets of a live object (k_vsd rect registers)
  DevBuf ws;  // scratch for host-buffer calls
};

namespace {

int fail(bopx_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIPCHK(c, expr)                                                              \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      return fail((c), BOPX_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                  __FILE__, __LINE__);                                              \
  } while (0)

int set_dev(bopx_ctx* c) {
  HIPCHK(c, hipSetDevice(c->device));
  return BOPX_OK;
}

// Launch prologue: the device, then the registry invariant every kernel shape
// relies on. The launchers size their per-workgroup state from the context's
// maxima, not from the objects of the batch: k_vsd's instantiation (rectangle
// registers and the LDS entry queue, RPT = ceil((1 or 2) x max_nm / 512)),
// k_sym_error's unit layout (max_ns), k_adi's scratch stride (max_nv on the
// device entry) and k_render_batch's (max_nf); the kernels read each object's
// own counts from the device descriptor table. Both come from sync_desc, which
// ends every registry change; if that failed part-way the maxima could lag a
// live object, and a kernel sized from them would index past its LDS / scratch
// (the class of the round-5 vertex-cache fault). So every launch
// entry recomputes the maxima from the live objects and refuses to launch on a
// mismatch (BOPX_E_INTERNAL), instead of launching out of range.
int launch_dev(bopx_ctx* c) {
  if (int r = set_dev(c)) return r;
  int nf = 0, nv = 0, ns = 0, nm = 0;
  for (const Object& o : c->objs)
    if (o.live) {
      nf = std::max(nf, (int)o.nf);
      nv = std::max(nv, (int)o.nv);
      ns = std::max(ns, (int)o.ns);
      nm = std::max(nm, (int)o.nm);
    }
  if (nf != c->max_nf || nv != c->max_nv || ns != c->max_ns || nm != c->max_nm)
    return fail(c, BOPX_E_INTERNAL,
                "object registry maxima are stale (nf %d/%d nv %d/%d ns %d/%d nm %d/%d): a "
                "registry update did not complete; re-register the objects",
                nf, c->max_nf, nv, c->max_nv, ns, c->max_ns, nm, c->max_nm);
  return BOPX_OK;
}

// *_dev calls run on exactly the stream they are given; NULL is the null
// (default) stream, as for any HIP API -- never the context's private stream.
hipStream_t pick_stream(bopx_ctx*, void* s) { return (hipStream_t)s; }

// Grow-only scratch; one allocation serves a whole host-buffer call.
int ws_reserve(bopx_ctx* c, size_t bytes) {
  if (c->ws.n >= bytes) return BOPX_OK;
  if (c->ws.p) HIPCHK(c, hipFree(c->ws.p));
  c->ws.p = nullptr;
  c->ws.n = 0;
  size_t want = std::max(bytes, (size_t)1 << 20);
  if (hipMalloc(&c->ws.p, want) != hipSuccess) {
    (void)hipGetLastError();
    return fail(c, BOPX_E_OOM, "workspace allocation of %zu bytes failed", want);
  }
  c->ws.n = want;
  return BOPX_OK;
}

// Bump allocator over the scratch (256-B aligned pieces).
struct Carve {
  char* base;
  size_t off = 0;
  template <class T>
  T* take(size_t count) {
    off = (off + 255) & ~(size_t)255;
    T* p = (T*)(base + off);
    off += count * sizeof(T);
    return p;
  }
};
static size_t carve_size(std::initializer_list<size_t> bytes) {
  size_t s = 0;
  for (size_t b : bytes) s += ((b + 255) & ~(size_t)255);
  return s + 256;
}

// Object-grouped launch order of a batch (bopx::launch_order_by_slot) in
// stream-ordered memory, freed behind the launches that read it. Batches below
// kOrderMinTuples and BOPX_LAUNCH_ORDER=0 keep the identity order (nullptr).
struct LaunchOrder {
  int32_t* p = nullptr;
  hipStream_t s = nullptr;
  LaunchOrder() = default;
  LaunchOrder(const LaunchOrder&) = delete;
  LaunchOrder& operator=(const LaunchOrder&) = delete;
  ~LaunchOrder() {
    if (p) (void)hipFreeAsync(p, s);
  }
};
constexpr int64_t kOrderMinTuples = 1024;

int make_order(bopx_ctx* c, int64_t n, const int32_t* slots, hipStream_t s, LaunchOrder& o,
               const bopx::OrderCost* cost = nullptr) {
  static const bool on = [] {
    const char* e = getenv("BOPX_LAUNCH_ORDER");
    return !(e && e[0] == '0');
  }();
  if (!on || n < kOrderMinTuples || n > INT32_MAX ||
      (int64_t)c->objs.size() > bopx::kOrderMaxSlots)
    return BOPX_OK;
  // order (n) + sort-key scratch (n), one stream-ordered allocation
  HIPCHK(c, hipMallocAsync((void**)&o.p, 2 * (size_t)n * sizeof(int32_t), s));
  o.s = s;
  HIPCHK(c, bopx::launch_order_by_slot(slots, n, (int)c->objs.size(), o.p, o.p + n, s, cost));
  return BOPX_OK;
}

bopx::OrderCost sym_order_cost(const bopx_ctx* c) {
  bopx::OrderCost oc{};
  oc.slot_rank = c->d_rank;
  return oc;
}

int sync_desc(bopx_ctx* c) {
  std::vector<ObjDesc> h(c->objs.size());
  int max_nf = 0, max_nv = 0, max_ns = 0, max_nm = 0;
  for (size_t i = 0; i < c->objs.size(); ++i) {
    const Object& o = c->objs[i];
    ObjDesc d{};
    if (o.live) {
      d.pts = o.d_pts;
      d.vtx = o.d_vtx;
      d.faces = o.d_faces;
      d.mlet = o.d_mlet;
      d.mlet_info = o.d_minfo;
      d.mlet_vtx = o.d_mvtx;
      d.mlet_tri = o.d_mtri;
      d.syms = o.d_syms;
      d.seed = o.d_seed;
      d.nseed = (int)o.nseed;
      d.nv = (int)o.nv;
      d.nf = (int)o.nf;
      d.nm = (int)o.nm;
      d.ns = (int)o.ns;
      max_nf = std::max(max_nf, (int)o.nf);
      max_nv = std::max(max_nv, (int)o.nv);
      max_ns = std::max(max_ns, (int)o.ns);
      max_nm = std::max(max_nm, (int)o.nm);
    }
    h[i] = d;
  }
  c->max_nf = max_nf;
  c->max_nv = max_nv;
  c->max_ns = max_ns;
  c->max_nm = max_nm;
  if (h.size() > c->desc_cap) {
    if (c->d_desc) HIPCHK(c, hipFree(c->d_desc));
    if (c->d_rank) HIPCHK(c, hipFree(c->d_rank));
    c->d_rank = nullptr;
    size_t cap = std::max<size_t>(64, h.size() * 2);
    HIPCHK(c, hipMalloc(&c->d_desc, cap * sizeof(ObjDesc)));
    HIPCHK(c, hipMalloc(&c->d_rank, cap * sizeof(int32_t)));
    c->desc_cap = cap;
  }
  // MSSD / MSPD launch order: the slots by descending work (nv * ns; free slots
  // last), so the heavy objects' tuples start first (LPT; a heavy tail of
  // continuous-symmetry tuples otherwise sets the end of the launch)
  std::vector<int32_t> by_cost(h.size()), rank(h.size());
  for (size_t i = 0; i < h.size(); ++i) by_cost[i] = (int32_t)i;
  std::stable_sort(by_cost.begin(), by_cost.end(), [&](int32_t x, int32_t y) {
    return (int64_t)h[x].nv * std::max(h[x].ns, 1) > (int64_t)h[y].nv * std::max(h[y].ns, 1);
  });
  for (size_t i = 0; i < h.size(); ++i) rank[by_cost[i]] = (int32_t)i;
  if (!h.empty()) {
    HIPCHK(c, hipMemcpyAsync(c->d_desc, h.data(), h.size() * sizeof(ObjDesc),
                             hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_rank, rank.data(), rank.size() * sizeof(int32_t),
                             hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BOPX_OK;
}

void free_object(Object& o) {
  if (o.d_pts) (void)hipFree(o.d_pts);
  if (o.d_vtx) (void)hipFree(o.d_vtx);
  if (o.d_faces) (void)hipFree(o.d_faces);
  if (o.d_mlet) (void)hipFree(o.d_mlet);
  if (o.d_minfo) (void)hipFree(o.d_minfo);
  if (o.d_mvtx) (void)hipFree(o.d_mvtx);
  if (o.d_mtri) (void)hipFree(o.d_mtri);
  if (o.d_syms) (void)hipFree(o.d_syms);
  if (o.d_seed) (void)hipFree(o.d_seed);
  o = Object();
}

uint32_t spread10(uint32_t x) {
  x &= 0x3FF;
  x = (x | (x << 16)) & 0x30000FF;
  x = (x | (x << 8)) & 0x300F00F;
  x = (x | (x << 4)) & 0x30C30C3;
  x = (x | (x << 2)) & 0x9249249;
  return x;
}

// 3D Hilbert index of 10-bit coordinates (Skilling, "Programming the Hilbert
// curve", AIP Conf. Proc. 707, 2004: axes to transposed form, then bits
// interleaved most significant first).
uint32_t hilbert3(const uint32_t q[3]) {
  uint32_t x[3] = {q[0], q[1], q[2]};
  for (uint32_t Q = 1u << 9; Q > 1; Q >>= 1) {
    const uint32_t P = Q - 1;
    for (int i = 0; i < 3; ++i) {
      if (x[i] & Q) {
        x[0] ^= P;
      } else {
        const uint32_t t = (x[0] ^ x[i]) & P;
        x[0] ^= t;
        x[i] ^= t;
      }
    }
  }
  for (int i = 1; i < 3; ++i) x[i] ^= x[i - 1];
  uint32_t t = 0;
  for (uint32_t Q = 1u << 9; Q > 1; Q >>= 1)
    if (x[2] & Q) t ^= Q - 1;
  for (int i = 0; i < 3; ++i) x[i] ^= t;
  uint32_t key = 0;
  for (int b = 9; b >= 0; --b)
    for (int i = 0; i < 3; ++i) key = (key << 1) | ((x[i] >> b) & 1u);
  return key;
}

template <class T>
int upload(bopx_ctx* c, T** dst, const T* src, size_t count) {
  if (count == 0) return BOPX_OK;
  if (hipMalloc((void**)dst, count * sizeof(T)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(c, BOPX_E_OOM, "object allocation failed");
  }
  HIPCHK(c, hipMemcpy(*dst, src, count * sizeof(T), hipMemcpyHostToDevice));
  return BOPX_OK;
}

int slot_checked(const bopx_ctx* c, int obj_id, int* slot) {
  auto it = c->slot_of.find(obj_id);
  if (it == c->slot_of.end()) return BOPX_E_NOT_FOUND;
  *slot = it->second;
  return BOPX_OK;
}

// Map obj_ids to slots on the host and validate the per-call requirements.
int map_slots(bopx_ctx* c, int64_t n, const int32_t* obj_ids, std::vector<int32_t>& slots,
              bool need_syms, bool need_faces) {
  slots.resize((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    int s;
    if (slot_checked(c, obj_ids[i], &s) != BOPX_OK)
      return fail(c, BOPX_E_NOT_FOUND, "unknown obj_id %d", obj_ids[i]);
    const Object& o = c->objs[s];
    if (o.nv <= 0) return fail(c, BOPX_E_INVALID, "obj_id %d has no vertices", obj_ids[i]);
    if (need_syms && o.ns <= 0)
      return fail(c, BOPX_E_INVALID, "obj_id %d has no symmetry set", obj_ids[i]);
    if (need_faces && o.nf <= 0)
      return fail(c, BOPX_E_INVALID, "obj_id %d has no faces", obj_ids[i]);
    slots[i] = s;
  }
  return BOPX_OK;
}

int check_taus(bopx_ctx* c, const double* taus, int n_tau) {
  if (n_tau < 1 || n_tau > BOPX_MAX_TAUS)
    return fail(c, BOPX_E_INVALID, "n_tau = %d outside [1, %d]", n_tau, BOPX_MAX_TAUS);
  if (!taus) return fail(c, BOPX_E_INVALID, "taus is NULL");
  return BOPX_OK;
}

}  // namespace

extern "C" {

int bopx_version(void) { return (0 << 16) | 1; }

int bopx_device_count(int* n) {
  int k = 0;
  if (hipGetDeviceCount(&k) != hipSuccess) {
    (void)hipGetLastError();
    k = 0;
  }
  if (n) *n = k;
  return BOPX_OK;
}

int bopx_create(int device, bopx_ctx** out) {
  if (!out) return BOPX_E_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    (void)hipGetLastError();
    return BOPX_E_INVALID;
  }
  bopx_ctx* c = new bopx_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return BOPX_E_HIP;
  }
  *out = c;
  return BOPX_OK;
}

void bopx_destroy(bopx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (Object& o : c->objs) free_object(o);
  if (c->d_desc) (void)hipFree(c->d_desc);
  if (c->d_rank) (void)hipFree(c->d_rank);
  if (c->ws.p) (void)hipFree(c->ws.p);
  (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* bopx_last_error(const bopx_ctx* c) { return c ? c->err.c_str() : "null context"; }

int bopx_synchronize(bopx_ctx* c) {
  if (!c) return BOPX_E_INVALID;
  if (int r = set_dev(c)) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BOPX_OK;
}

void* bopx_stream(bopx_ctx* c) { return c ? (void*)c->stream : nullptr; }

// Oriented bounding box of a meshlet's vertices (principal axes of their
// covariance, Jacobi rotations), appended as 8 float32 corners (x, y, z each).
// A surface patch is thin along its normal, so its projected OBB is much
// tighter than that of an object-space AABB: fewer (meshlet, tile) entries in
// k_vsd. The box is inflated by 1e-4 of its extent (+1e-3) so float32 rounding
// of the corners cannot make it non-conservative.
static void jacobi3(double a[3][3], double v[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) v[i][j] = i == j;
  for (int sweep = 0; sweep < 32; ++sweep) {
    const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    if (off < 1e-30) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        if (std::fabs(a[p][q]) < 1e-300) continue;
        const double th = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
        const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), sn = t * c;
        for (int k = 0; k < 3; ++k) {  // A <- A J
          const double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - sn * akq;
          a[k][q] = sn * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {  // A <- J^T A
          const double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - sn * aqk;
          a[q][k] = sn * apk + c * aqk;
        }
        for (int k = 0; k < 3; ++k) {  // V <- V J
          const double vkp = v[k][p], vkq = v[k][q];
          v[k][p] = c * vkp - sn * vkq;
          v[k][q] = sn * vkp + c * vkq;
        }
      }
  }
}

static void obb_corners(const std::vector<float4>& vtx, const std::vector<uint32_t>& ids,
                        std::vector<float>& out) {
  const size_t n = ids.size();
  double mean[3] = {0, 0, 0};
  for (uint32_t v : ids) {
    mean[0] += vtx[v].x;
    mean[1] += vtx[v].y;
    mean[2] += vtx[v].z;
  }
  for (int k = 0; k < 3; ++k) mean[k] /= (double)std::max<size_t>(n, 1);
  double cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, ax[3][3];
  for (uint32_t v : ids) {
    const double d[3] = {vtx[v].x - mean[0], vtx[v].y - mean[1], vtx[v].z - mean[2]};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) cov[i][j] += d[i] * d[j];
  }
  jacobi3(cov, ax);  // columns of ax: orthonormal principal axes
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (uint32_t v : ids) {
    const double d[3] = {vtx[v].x - mean[0], vtx[v].y - mean[1], vtx[v].z - mean[2]};
    for (int k = 0; k < 3; ++k) {
      const double t = d[0] * ax[0][k] + d[1] * ax[1][k] + d[2] * ax[2][k];
      lo[k] = std::min(lo[k], t);
      hi[k] = std::max(hi[k], t);
    }
  }
  double ext = 0;
  for (int k = 0; k < 3; ++k) ext = std::max(ext, hi[k] - lo[k]);
  const double pad = 1e-4 * ext + 1e-3;
  for (int k = 0; k < 3; ++k) lo[k] -= pad, hi[k] += pad;
  for (int c = 0; c < 8; ++c) {
    const double t[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
    for (int i = 0; i < 3; ++i)
      out.push_back((float)(mean[i] + t[0] * ax[i][0] + t[1] * ax[i][1] + t[2] * ax[i][2]));
  }
}

// Normal cone + bounding sphere of one meshlet (8 floats appended to its 24
// corner floats, kMletFloats per meshlet): unit axis a, cos(alpha), centre c,
// radius r. Every triangle normal (outward: `sign` = orientation of the whole
// mesh from its signed volume) lies within alpha of a, and every vertex within
// r of c. k_vsd uses it only to classify (pose, meshlet) entries as back-facing
// (tested for occlusion, queued last): a wrong class costs time, never a bit.
// cos(alpha) = -2 marks a meshlet that is never back-facing (alpha >= 90 deg).
static void meshlet_cone(const std::vector<float4>& vtx, const uint32_t* tri, int32_t ntri,
                         double sign, std::vector<float>& out) {
  const float* cr = out.data() + out.size() - 24;  // this meshlet's OBB corners
  double c[3] = {0, 0, 0}, r = 0;
  for (int k = 0; k < 8; ++k)
    for (int i = 0; i < 3; ++i) c[i] += cr[3 * k + i] / 8.0;
  for (int k = 0; k < 8; ++k) {
    const double d[3] = {cr[3 * k] - c[0], cr[3 * k + 1] - c[1], cr[3 * k + 2] - c[2]};
    r = std::max(r, std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]));
  }
  std::vector<double> nrm;
  double ax[3] = {0, 0, 0};
  for (int32_t t = 0; t < ntri; ++t) {
    const float4 p0 = vtx[tri[3 * t]], p1 = vtx[tri[3 * t + 1]], p2 = vtx[tri[3 * t + 2]];
    const double e1[3] = {(double)p1.x - p0.x, (double)p1.y - p0.y, (double)p1.z - p0.z};
    const double e2[3] = {(double)p2.x - p0.x, (double)p2.y - p0.y, (double)p2.z - p0.z};
    double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                   e1[0] * e2[1] - e1[1] * e2[0]};
    const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    if (!(len > 0)) continue;  // degenerate: no fragments, no constraint
    for (int i = 0; i < 3; ++i) {
      n[i] *= sign / len;
      ax[i] += n[i];
      nrm.push_back(n[i]);
    }
  }
  const double alen = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
  double cosa = -2.0;
  if (alen > 0 && !nrm.empty()) {
    for (int i = 0; i < 3; ++i) ax[i] /= alen;
    cosa = 1.0;
    for (size_t k = 0; k < nrm.size(); k += 3)
      cosa = std::min(cosa, nrm[k] * ax[0] + nrm[k + 1] * ax[1] + nrm[k + 2] * ax[2]);
    cosa -= 1e-6;  // rounding slack (a heuristic either way)
    if (!(cosa > 0.0)) cosa = -2.0;
  }
  for (int i = 0; i < 3; ++i) out.push_back((float)ax[i]);
  out.push_back((float)cosa);
  for (int i = 0; i < 3; ++i) out.push_back((float)c[i]);
  out.push_back((float)(r * (1.0 + 1e-6) + 1e-3));
}

// Meshlet partitions of the faces (host, once per object; the raster result
// does not depend on them, only k_vsd's culling work does).
// greedy: consecutive runs of the Morton order of the face centroids.
static void greedy_meshlets(const uint32_t* faces, int64_t nv, int64_t nf,
                            const std::vector<std::pair<uint32_t, uint32_t>>& key,
                            std::vector<uint32_t>& forder, std::vector<int32_t>& msize) {
  std::vector<char> used(nv, 0);
  std::vector<uint32_t> touched;
  int64_t f = 0;
  while (f < nf) {
    const int64_t f0 = f;
    touched.clear();
    while (f < nf && f - f0 < bopx::kMeshletTris) {
      const uint32_t* t = faces + 3 * (size_t)key[f].second;
      int fresh = 0;
      for (int j = 0; j < 3; ++j) fresh += !used[t[j]];  // (repeats counted twice: safe)
      if ((int)touched.size() + fresh > bopx::kMeshletVerts) break;
      for (int j = 0; j < 3; ++j)
        if (!used[t[j]]) used[t[j]] = 1, touched.push_back(t[j]);
      forder.push_back(key[f].second);
      ++f;
    }
    for (uint32_t v : touched) used[v] = 0;
    msize.push_back((int32_t)(f - f0));
  }
}

// Seed vertices of the MSSD / MSPD symmetry bounds (kern_pose.hip): up to
// kSymSeeds vertices by farthest-point sampling from the one farthest from the
// centroid, SoA x | y | z. The max of a pose error over a spread-out subset is
// a tight lower bound of its max over all vertices, which lets k_sym_error skip
// symmetries that cannot be the minimum. Only the speed depends on the choice.
static std::vector<double> seed_vertices(const double* pts, int64_t nv) {
  const int64_t np = std::min<int64_t>(nv, bopx::kSymSeeds);
  std::vector<double> seed(3 * (size_t)np);
  double cx = 0.0, cy = 0.0, cz = 0.0;
  for (int64_t v = 0; v < nv; ++v) {
    cx += pts[3 * v];
    cy += pts[3 * v + 1];
    cz += pts[3 * v + 2];
  }
  cx /= (double)nv;
  cy /= (double)nv;
  cz /= (double)nv;
  auto d2 = [&](int64_t v, double x, double y, double z) {
    const double dx = pts[3 * v] - x, dy = pts[3 * v + 1] - y, dz = pts[3 * v + 2] - z;
    return dx * dx + dy * dy + dz * dz;
  };
  std::vector<double> near((size_t)nv);
  int64_t pick = 0;
  for (int64_t v = 0; v < nv; ++v) {
    near[v] = d2(v, cx, cy, cz);
    if (near[v] > near[pick]) pick = v;
  }
  for (int64_t i = 0; i < np; ++i) {
    const double x = pts[3 * pick], y = pts[3 * pick + 1], z = pts[3 * pick + 2];
    seed[i] = x;
    seed[np + i] = y;
    seed[2 * np + i] = z;
    int64_t next = pick;
    double far = -1.0;
    for (int64_t v = 0; v < nv; ++v) {
      const double e = d2(v, x, y, z);
      if (i == 0 || e < near[v]) near[v] = e;
      if (near[v] > far) {
        far = near[v];
        next = v;
      }
    }
    pick = next;
  }
  return seed;
}

int bopx_add_object(bopx_ctx* c, int obj_id, const double* pts, int64_t nv,
                    const uint32_t* faces, int64_t nf) {
  if (!c) return BOPX_E_INVALID;
  if (nv <= 0 || !pts) return fail(c, BOPX_E_INVALID, "object %d: no vertices", obj_id);
  if (nv > (1LL << 30) || nf > (1LL << 30))
    return fail(c, BOPX_E_UNSUPPORTED, "object %d too large", obj_id);
  if (nf > 0 && !faces) return fail(c, BOPX_E_INVALID, "object %d: faces is NULL", obj_id);
  for (int64_t i = 0; i < 3 * nf; ++i)
    if (faces[i] >= (uint64_t)nv)
      return fail(c, BOPX_E_INVALID, "object %d: face index %u >= nv", obj_id, faces[i]);
  if (int r = set_dev(c)) return r;
  if (c->slot_of.count(obj_id)) bopx_remove_object(c, obj_id);

  Object o;
  o.obj_id = obj_id;
  o.nv = nv;
  o.nf = nf;
  // float64 SoA points.
  std::vector<double> soa(3 * (size_t)nv);
  for (int64_t v = 0; v < nv; ++v)
    for (int k = 0; k < 3; ++k) soa[k * (size_t)nv + v] = pts[3 * v + k];
  // float32 raster vertices (GL vertex buffers are float32, renderer_vispy.py:373).
  std::vector<float4> vtx((size_t)nv);
  for (int64_t v = 0; v < nv; ++v)
    vtx[v] = make_float4((float)pts[3 * v], (float)pts[3 * v + 1], (float)pts[3 * v + 2], 0.f);
  // Meshlets: triangles sorted by the Morton code of their centroid, 64 per meshlet.
  std::vector<uint32_t> fsorted, mtri;
  std::vector<float> mlet;
  std::vector<int4> minfo;
  std::vector<float4> mvtx;
  if (nf > 0) {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t v = 0; v < nv; ++v) {
      const float p[3] = {vtx[v].x, vtx[v].y, vtx[v].z};
      for (int k = 0; k < 3; ++k) lo[k] = std::min(lo[k], p[k]), hi[k] = std::max(hi[k], p[k]);
    }
    // Space-filling curve over the face centroids (10 bits per axis): Hilbert
    // (default; no long jumps, so runs of 64 faces are compact patches: ~10 %
    // fewer (meshlet, tile) entries in k_vsd than Morton) or Morton
    // (BOPX_MESHLET_CURVE=morton).
    static const int curve = [] {
      const char* e = getenv("BOPX_MESHLET_CURVE");
      return (e && std::string(e) == "morton") ? 0 : 1;
    }();
    std::vector<std::pair<uint32_t, uint32_t>> key((size_t)nf);
    for (int64_t f = 0; f < nf; ++f) {
      uint32_t q[3];
      for (int k = 0; k < 3; ++k) {
        const float* p0 = &vtx[faces[3 * f]].x;
        const float* p1 = &vtx[faces[3 * f + 1]].x;
        const float* p2 = &vtx[faces[3 * f + 2]].x;
        float cen = (p0[k] + p1[k] + p2[k]) / 3.0f;
        float ext = hi[k] - lo[k];
        float u = ext > 0 ? (cen - lo[k]) / ext : 0.f;
        q[k] = (uint32_t)std::min(1023.0f, std::max(0.0f, u * 1023.0f));
      }
      key[f] = {curve == 1 ? hilbert3(q) : spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2),
                (uint32_t)f};
    }
    std::stable_sort(key.begin(), key.end());
    // Meshlet partition (face order + sizes); both builders keep <= 64
    // triangles and <= 64 unique vertices per meshlet.
    std::vector<uint32_t> forder;
    std::vector<int32_t> msize;
    greedy_meshlets(faces, nv, nf, key, forder, msize);
    fsorted.resize(3 * (size_t)nf);
    for (int64_t i = 0; i < nf; ++i)
      for (int k = 0; k < 3; ++k) fsorted[3 * i + k] = faces[3 * (size_t)forder[i] + k];
    // Pack each meshlet into fixed-stride slots (64 float32x4 vertices, 64
    // triangle words; padding vertices repeat vertex 0, padding triangles are
    // 0xFFFFFFFF) so a wave addresses meshlet m's data from m alone. Triangle
    // words hold 8-bit local vertex indices a | b << 8 | c << 16.
    std::vector<int32_t> local(nv, -1);
    std::vector<uint32_t> touched;
    // orientation of the mesh (signed volume): outward normals for the cones
    double vol = 0.0;
    for (int64_t t = 0; t < nf; ++t) {
      const float4 p0 = vtx[faces[3 * t]], p1 = vtx[faces[3 * t + 1]], p2 = vtx[faces[3 * t + 2]];
      vol += (double)p0.x * ((double)p1.y * p2.z - (double)p1.z * p2.y) +
             (double)p0.y * ((double)p1.z * p2.x - (double)p1.x * p2.z) +
             (double)p0.z * ((double)p1.x * p2.y - (double)p1.y * p2.x);
    }
    const double sign = vol < 0.0 ? -1.0 : 1.0;
    int64_t f = 0;
    for (const int32_t sz : msize) {
      const int32_t tri0 = (int32_t)f, vtx0 = (int32_t)mvtx.size();
      const size_t tslot0 = mtri.size();
      touched.clear();
      for (; f < tri0 + sz; ++f) {
        uint32_t pk = 0;
        for (int j = 0; j < 3; ++j) {
          const uint32_t v = fsorted[3 * f + j];
          if (local[v] < 0) {
            local[v] = (int32_t)touched.size();
            touched.push_back(v);
            mvtx.push_back(vtx[v]);
          }
          pk |= (uint32_t)local[v] << (8 * j);
        }
        mtri.push_back(pk);
      }
      obb_corners(vtx, touched, mlet);
      meshlet_cone(vtx, fsorted.data() + 3 * (size_t)tri0, sz, sign, mlet);
      for (uint32_t v : touched) local[v] = -1;
      const float4 pad = mvtx[vtx0];
      while (mvtx.size() - vtx0 < (size_t)bopx::kMeshletVerts) mvtx.push_back(pad);
      while (mtri.size() - tslot0 < (size_t)bopx::kMeshletTris) mtri.push_back(0xFFFFFFFFu);
      minfo.push_back(make_int4(tri0, (int32_t)(f - tri0), vtx0, (int32_t)touched.size()));
    }
    o.nm = (int64_t)minfo.size();
  }
  const std::vector<double> seed = seed_vertices(pts, nv);
  o.nseed = (int64_t)seed.size() / 3;
  int r;
  if ((r = upload(c, &o.d_pts, soa.data(), soa.size())) ||
      (r = upload(c, &o.d_seed, seed.data(), seed.size())) ||
      (r = upload(c, &o.d_vtx, vtx.data(), vtx.size())) ||
      (r = upload(c, &o.d_faces, fsorted.data(), fsorted.size())) ||
      (r = upload(c, &o.d_mlet, mlet.data(), mlet.size())) ||
      (r = upload(c, &o.d_minfo, minfo.data(), minfo.size())) ||
      (r = upload(c, &o.d_mvtx, mvtx.data(), mvtx.size())) ||
      (r = upload(c, &o.d_mtri, mtri.data(), mtri.size()))) {
    free_object(o);
    return r;
  }
  o.live = true;
  int slot = -1;
  for (size_t i = 0; i < c->objs.size(); ++i)
    if (!c->objs[i].live) {
      slot = (int)i;
      break;
    }
  if (slot < 0) {
    slot = (int)c->objs.size();
    c->objs.push_back(Object());
  }
  c->objs[slot] = o;
  c->slot_of[obj_id] = slot;
  return sync_desc(c);
}

int bopx_remove_object(bopx_ctx* c, int obj_id) {
  if (!c) return BOPX_E_INVALID;
  int s;
  if (slot_checked(c, obj_id, &s) != BOPX_OK)
    return fail(c, BOPX_E_NOT_FOUND, "unknown obj_id %d", obj_id);
  if (int r = set_dev(c)) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  free_object(c->objs[s]);
  c->slot_of.erase(obj_id);
  return sync_desc(c);
}

// The new sets are allocated and uploaded first and swapped in only when every
// one of them is resident: a failure part-way (OOM, a copy error) frees the new
// buffers and leaves every object's old set and the device descriptor table as
// they were, so no later launch reads a freed buffer.
static int replace_symmetries(bopx_ctx* c, int n, const int* slots, const int64_t* ns,
                              const double* syms) {
  std::vector<double*> fresh((size_t)n, nullptr);
  auto drop = [&]() {
    for (double* p : fresh)
      if (p) (void)hipFree(p);
  };
  const double* src = syms;
  for (int i = 0; i < n; ++i) {
    const size_t count = 12 * (size_t)ns[i];
    if (hipMalloc((void**)&fresh[(size_t)i], count * sizeof(double)) != hipSuccess) {
      (void)hipGetLastError();
      fresh[(size_t)i] = nullptr;
      (void)hipStreamSynchronize(c->stream);  // earlier copies into `fresh` have landed
      drop();
      return fail(c, BOPX_E_OOM, "symmetry set allocation failed");
    }
    hipError_t e = hipMemcpyAsync(fresh[(size_t)i], src, count * sizeof(double),
                                  hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      (void)hipStreamSynchronize(c->stream);
      drop();
      return fail(c, BOPX_E_HIP, "symmetry upload: %s", hipGetErrorString(e));
    }
    src += count;
  }
  for (int i = 0; i < n; ++i) {  // every new set is resident: swap them in
    Object& o = c->objs[(size_t)slots[i]];
    if (o.d_syms) (void)hipFree(o.d_syms);  // no launch reads it (the stream was drained)
    o.d_syms = fresh[(size_t)i];
    o.ns = ns[i];
  }
  return sync_desc(c);  // one descriptor upload, then the stream is drained
}

int bopx_set_symmetries(bopx_ctx* c, int obj_id, const double* syms, int64_t ns) {
  if (!c) return BOPX_E_INVALID;
  int s;
  if (slot_checked(c, obj_id, &s) != BOPX_OK)
    return fail(c, BOPX_E_NOT_FOUND, "unknown obj_id %d", obj_id);
  if (ns < 1 || !syms) return fail(c, BOPX_E_INVALID, "empty symmetry set");
  if (int r = set_dev(c)) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // no launch still reads the old set
  return replace_symmetries(c, 1, &s, &ns, syms);
}

int bopx_set_symmetries_many(bopx_ctx* c, int n, const int* obj_ids, const int64_t* ns,
                             const double* syms) {
  if (!c) return BOPX_E_INVALID;
  if (n < 0 || (n > 0 && (!obj_ids || !ns || !syms))) return fail(c, BOPX_E_INVALID, "NULL buffer");
  std::vector<int> slots((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (slot_checked(c, obj_ids[i], &slots[(size_t)i]) != BOPX_OK)
      return fail(c, BOPX_E_NOT_FOUND, "unknown obj_id %d", obj_ids[i]);
    if (ns[i] < 1) return fail(c, BOPX_E_INVALID, "empty symmetry set");
  }
  if (n == 0) return BOPX_OK;
  if (int r = set_dev(c)) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // no launch still reads the old sets
  return replace_symmetries(c, n, slots.data(), ns, syms);
}

int bopx_preload(bopx_ctx* c) {
  if (!c) return BOPX_E_INVALID;
  // no context state is touched (a caller may run this on a thread of its own
  // while it registers objects): the device, then the three code objects
  if (hipSetDevice(c->device) != hipSuccess) {
    (void)hipGetLastError();
    return BOPX_E_HIP;
  }
  hipError_t e = bopx::preload_pose_kernels();
  if (e == hipSuccess) e = bopx::preload_vsd_kernels();
  if (e == hipSuccess) e = bopx::preload_png_kernels();
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return BOPX_E_HIP;
  }
  return BOPX_OK;
}

int bopx_object_slot(const bopx_ctx* c, int obj_id, int* slot) {
  if (!c || !slot) return BOPX_E_INVALID;
  return slot_checked(c, obj_id, slot);
}

// ---------------------------------------------------------------- point errors
static int point_batch(bopx_ctx* c, int kind, int64_t n, const int32_t* obj_ids,
                       const double* pe, const double* pg, const double* K, double* out) {
  // kind: 0 mssd, 1 mspd, 2 add, 3 adi, 4 proj
  if (!c) return BOPX_E_INVALID;
  if (n < 0) return fail(c, BOPX_E_INVALID, "n < 0");
  if (n == 0) return BOPX_OK;
  if (!obj_ids || !pe || !pg || !out) return fail(c, BOPX_E_INVALID, "NULL buffer");
  const bool needK = kind == 1 || kind == 4;
  if (needK && !K) return fail(c, BOPX_E_INVALID, "K is NULL");
  if (int r = launch_dev(c)) return r;
  std::vector<int32_t> slots;
  if (int r = map_slots(c, n, obj_ids, slots, kind <= 1, false)) return r;
  const size_t bytes = carve_size({4 * (size_t)n, 96 * (size_t)n, 96 * (size_t)n,
                                   needK ? 72 * (size_t)n : 0, 8 * (size_t)n});
  if (int r = ws_reserve(c, bytes)) return r;
  Carve cv{(char*)c->ws.p};
  int32_t* d_s = cv.take<int32_t>(n);
  double* d_pe = cv.take<double>(12 * n);
  double* d_pg = cv.take<double>(12 * n);
  double* d_K = needK ? cv.take<double>(9 * n) : nullptr;
  const size_t small = cv.off;
  double* d_out = cv.take<double>(n);
  hipStream_t s = c->stream;
  // small batches (per-call latency): inputs staged in one host block, one
  // upload; large ones copy each array directly (no extra host pass)
  std::vector<char> h(n <= 4096 ? small : 0);
  const auto stage = [&](void* d, const void* src, size_t nb) -> hipError_t {
    if (h.empty()) return hipMemcpyAsync(d, src, nb, hipMemcpyHostToDevice, s);
    std::memcpy(h.data() + ((const char*)d - (const char*)c->ws.p), src, nb);
    return hipSuccess;
  };
  HIPCHK(c, stage(d_s, slots.data(), 4 * n));
  HIPCHK(c, stage(d_pe, pe, 96 * n));
  HIPCHK(c, stage(d_pg, pg, 96 * n));
  if (needK) HIPCHK(c, stage(d_K, K, 72 * n));
  if (!h.empty()) HIPCHK(c, hipMemcpyAsync(c->ws.p, h.data(), small, hipMemcpyHostToDevice, s));
  LaunchOrder ord;
  const bopx::OrderCost sc = sym_order_cost(c);
  if (int r = make_order(c, n, d_s, s, ord, kind <= 1 ? &sc : nullptr)) return r;
  hipError_t e;
  if (kind <= 1)
    e = bopx::launch_sym_error(kind, c->d_desc, c->max_ns, n, d_s, d_pe, d_pg, d_K, d_out, ord.p,
                               s);
  else if (kind == 3) {
    // ADI scratch stride: the largest object of THIS batch (the host knows the
    // slots), not of the context, so small-object calls do not pay for a large
    // resident model
    int batch_nv = 1;
    for (int32_t sl : slots) batch_nv = std::max(batch_nv, (int)c->objs[sl].nv);
    e = bopx::launch_adi(c->d_desc, batch_nv, n, d_s, d_pe, d_pg, d_out, ord.p, s);
  }
  else
    e = bopx::launch_mean_error(kind == 2 ? 0 : 1, c->d_desc, n, d_s, d_pe, d_pg, d_K, d_out,
                                ord.p, s);
  HIPCHK(c, e);
  HIPCHK(c, hipMemcpyAsync(out, d_out, 8 * n, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return BOPX_OK;
}

int bopx_mssd_batch(bopx_ctx* c, int64_t n, const int32_t* ids, const double* pe,
                    const double* pg, double* out) {
  return point_batch(c, 0, n, ids, pe, pg, nullptr, out);
}
int bopx_mspd_batch(bopx_ctx* c, int64_t n, const int32_t* ids, const double* pe,
                    const double* pg, const double* K, double* out) {
  return point_batch(c, 1, n, ids, pe, pg, K, out);
}
int bopx_add_batch(bopx_ctx* c, int64_t n, const int32_t* ids, const double* pe,
                   const double* pg, double* out) {
  return point_batch(c, 2, n, ids, pe, pg, nullptr, out);
}
int bopx_adi_batch(bopx_ctx* c, int64_t n, const int32_t* ids, const double* pe,
                   const double* pg, double* out) {
  return point_batch(c, 3, n, ids, pe, pg, nullptr, out);
}
int bopx_proj_batch(bopx_ctx* c, int64_t n, const int32_t* ids, const double* pe,
                    const double* pg, const double* K, double* out) {
  return point_batch(c, 4, n, ids, pe, pg, K, out);
}

int bopx_mssd_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pe,
                        const double* pg, double* out, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = launch_dev(c)) return r;
  hipStream_t s = pick_stream(c, stream);
  LaunchOrder ord;
  const bopx::OrderCost sc = sym_order_cost(c);
  if (int r = make_order(c, n, slots, s, ord, &sc)) return r;
  HIPCHK(c, bopx::launch_sym_error(0, c->d_desc, c->max_ns, n, slots, pe, pg, nullptr, out, ord.p,
                                   s));
  return BOPX_OK;
}
int bopx_mspd_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pe,
                        const double* pg, const double* K, double* out, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = launch_dev(c)) return r;
  hipStream_t s = pick_stream(c, stream);
  LaunchOrder ord;
  const bopx::OrderCost sc = sym_order_cost(c);
  if (int r = make_order(c, n, slots, s, ord, &sc)) return r;
  HIPCHK(c, bopx::launch_sym_error(1, c->d_desc, c->max_ns, n, slots, pe, pg, K, out, ord.p, s));
  return BOPX_OK;
}
int bopx_add_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pe,
                       const double* pg, double* out, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = launch_dev(c)) return r;
  hipStream_t s = pick_stream(c, stream);
  LaunchOrder ord;
  if (int r = make_order(c, n, slots, s, ord)) return r;
  HIPCHK(c, bopx::launch_mean_error(0, c->d_desc, n, slots, pe, pg, nullptr, out, ord.p, s));
  return BOPX_OK;
}
int bopx_adi_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pe,
                       const double* pg, double* out, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = launch_dev(c)) return r;
  hipStream_t s = pick_stream(c, stream);
  LaunchOrder ord;
  if (int r = make_order(c, n, slots, s, ord)) return r;
  HIPCHK(c, bopx::launch_adi(c->d_desc, c->max_nv, n, slots, pe, pg, out, ord.p, s));
  return BOPX_OK;
}

int bopx_proj_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pe,
                        const double* pg, const double* K, double* out, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = launch_dev(c)) return r;
  hipStream_t s = pick_stream(c, stream);
  LaunchOrder ord;
  if (int r = make_order(c, n, slots, s, ord)) return r;
  HIPCHK(c, bopx::launch_mean_error(1, c->d_desc, n, slots, pe, pg, K, out, ord.p, s));
  return BOPX_OK;
}

// ------------------------------------------------------------------------ VSD
// The float32 threshold t with (diff <= t) == the visibility test of
// visibility.py:35-37 for every float32 diff: delta itself (cast to float32,
// NumPy's weak Python-float scalar) or, for a float64 delta (BOPX_DELTA_F64,
// the comparison promoted to float64), the largest float32 <= delta.
static float visib_thr32(double delta, int flags) {
  float f = (float)delta;
  if ((flags & BOPX_DELTA_F64) && (double)f > delta) f = std::nextafter(f, -INFINITY);
  return f;
}

// k_vsd's occlusion test of far meshlet entries (bit-identical results either
// way). Read per call, so a test can compare the modes: BOPX_VSD_CULL=1 on,
// 0 off, 2 test only (timing), 3 back-face occlusion test (meshlet normal
// cones: back-facing entries queued last and tested against their corner bound
// before any of their data is fetched), unset = -1: the back-face test for the
// tuples whose object has more than kCullAutoMeshlets meshlets (kern_vsd.hip;
// it costs +3.2 % on 10k-triangle meshes and saves 3 % on 30k-triangle ones).
static int vsd_cull_enabled() {
  const char* e = getenv("BOPX_VSD_CULL");
  return e ? atoi(e) : -1;
}

// k_vsd tile entry-queue order (kern_vsd.hip kLptOverlap): 1 = large overlaps
// first (default), 0 = near entries first. Read per call like BOPX_VSD_CULL.
static int vsd_queue_order() {
  const char* e = getenv("BOPX_VSD_QORDER");
  return e ? (atoi(e) != 0) : 1;
}

// k_vsd launch order: cost classes (projected bounding-sphere area, expensive
// tuples first) then object slot. Measured on the bench workload (round 2,
// same box): 10.76 -> 10.0 ms against the slot-only order; the slot grouping
// within a class keeps MSSD / MSPD-style L2 reuse of the meshlet data.
static bopx::OrderCost vsd_order_cost(const bopx::VsdArgs& a) {
  bopx::OrderCost oc{};
  if (a.diameters && a.pose_est && a.pose_gt && a.frame_idx && a.cam) {
    oc.pe = a.pose_est;
    oc.pg = a.pose_gt;
    oc.frame_idx = a.frame_idx;
    oc.cam = a.cam;
    oc.dia = a.diameters;
  }
  return oc;
}

static int fill_vsd_args(bopx_ctx* c, bopx::VsdArgs& a, int width, int height, double delta,
                         int flags, const double* taus, int n_tau, int normalized,
                         int cost_type) {
  if (width <= 0 || height <= 0 || width > 32767 || height > 32767)
    return fail(c, BOPX_E_INVALID, "bad image size %dx%d", width, height);
  if ((int64_t)((width + bopx::kTileW - 1) / bopx::kTileW) *
          ((height + bopx::kTileH - 1) / bopx::kTileH) > bopx::kVsdMaxTiles)
    return fail(c, BOPX_E_UNSUPPORTED, "image %dx%d exceeds the fused VSD kernel's %d tiles",
                width, height, bopx::kVsdMaxTiles);
  if (cost_type != BOPX_COST_STEP && cost_type != BOPX_COST_TLINEAR)
    return fail(c, BOPX_E_INVALID, "Unknown pixel matching cost.");
  if (int r = check_taus(c, taus, n_tau)) return r;
  a.width = a.img_w = width;
  a.height = a.img_h = height;
  a.delta32 = (float)delta;
  a.delta64 = delta;
  a.delta_f64 = (flags & BOPX_DELTA_F64) ? 1 : 0;
  a.dthr = visib_thr32(delta, flags);
  a.n_tau = n_tau;
  a.normalized = normalized ? 1 : 0;
  static const int ablate = [] {
    const char* e = getenv("BOPX_VSD_ABLATE");  // timing diagnostics only
    return e ? atoi(e) : 0;
  }();
  a.ablate = ablate;
  for (int k = 0; k < bopx::kMaxTaus; ++k) a.taus[k] = k < n_tau ? taus[k] : 1.0;
  return BOPX_OK;
}

int bopx_vsd_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pe,
                       const double* pg, const int32_t* frame_idx, const float* frames,
                       int width, int height, const double* cam, double delta, int flags,
                       const double* taus, int n_tau, int normalized, const double* diameters,
                       int cost_type, double* out, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = launch_dev(c)) return r;
  bopx::VsdArgs a{};
  a.cull = vsd_cull_enabled();
  a.qorder = vsd_queue_order();
  if (int r = fill_vsd_args(c, a, width, height, delta, flags, taus, n_tau, normalized,
                            cost_type))
    return r;
  a.objs = c->d_desc;
  a.max_nm = c->max_nm;
  a.slots = slots;
  a.pose_est = pe;
  a.pose_gt = pg;
  a.frame_idx = frame_idx;
  a.frames = frames;
  a.cam = cam;
  a.diameters = diameters;
  a.out = out;
  a.unions = (flags & BOPX_VSD_UNIONS) ? out + n * n_tau : nullptr;
  a.n = n;
  {
    const hipStream_t so = pick_stream(c, stream);
    LaunchOrder ord;
    const bopx::OrderCost oc = vsd_order_cost(a);
    if (int r = make_order(c, a.n, a.slots, so, ord, oc.pe ? &oc : nullptr)) return r;
    a.order = ord.p;
    HIPCHK(c, bopx::launch_vsd(a, cost_type, so));
  }
  return BOPX_OK;
}

int bopx_vsd_batch(bopx_ctx* c, int64_t n, const int32_t* obj_ids, const double* pe,
                   const double* pg, const int32_t* frame_idx, const float* frames,
                   int64_t n_frames, int width, int height, const double* cam, double delta,
                   int flags, const double* taus, int n_tau, int normalized,
                   const double* diameters, int cost_type, double* out) {
  if (!c) return BOPX_E_INVALID;
  if (n < 0 || n_frames < 0) return fail(c, BOPX_E_INVALID, "negative size");
  if (n == 0) return BOPX_OK;
  if (!obj_ids || !pe || !pg || !frame_idx || !frames || !cam || !diameters || !out)
    return fail(c, BOPX_E_INVALID, "NULL buffer");
  for (int64_t i = 0; i < n; ++i)
    if (frame_idx[i] < 0 || frame_idx[i] >= n_frames)
      return fail(c, BOPX_E_INVALID, "frame_idx[%lld] = %d out of range", (long long)i,
                  frame_idx[i]);
  if (int r = launch_dev(c)) return r;
  bopx::VsdArgs a{};
  a.cull = vsd_cull_enabled();
  a.qorder = vsd_queue_order();
  if (int r = fill_vsd_args(c, a, width, height, delta, flags, taus, n_tau, normalized,
                            cost_type))
    return r;
  std::vector<int32_t> slots;
  if (int r = map_slots(c, n, obj_ids, slots, false, true)) return r;
  const size_t fbytes = (size_t)n_frames * width * height * sizeof(float);
  const size_t n_out = (size_t)n * n_tau + ((flags & BOPX_VSD_UNIONS) ? (size_t)n : 0);
  const size_t bytes = carve_size({4 * (size_t)n, 96 * (size_t)n, 96 * (size_t)n,
                                   4 * (size_t)n, 32 * (size_t)n_frames, 8 * (size_t)n,
                                   fbytes, 8 * n_out});
  if (int r = ws_reserve(c, bytes)) return r;
  // The per-tuple arrays are carved first and staged in one host block with the
  // same offsets: one small upload instead of six (per-call latency), then the
  // frames.
  Carve cv{(char*)c->ws.p};
  int32_t* d_s = cv.take<int32_t>(n);
  double* d_pe = cv.take<double>(12 * n);
  double* d_pg = cv.take<double>(12 * n);
  int32_t* d_fi = cv.take<int32_t>(n);
  double* d_cam = cv.take<double>(4 * n_frames);
  double* d_dia = cv.take<double>(n);
  const size_t small = cv.off;
  float* d_fr = cv.take<float>((size_t)n_frames * width * height);
  double* d_out = cv.take<double>(n_out);
  std::vector<char> h(small);
  const auto stage = [&](const void* d, const void* src, size_t nb) {
    std::memcpy(h.data() + ((const char*)d - (const char*)c->ws.p), src, nb);
  };
  stage(d_s, slots.data(), 4 * n);
  stage(d_pe, pe, 96 * n);
  stage(d_pg, pg, 96 * n);
  stage(d_fi, frame_idx, 4 * n);
  stage(d_cam, cam, 32 * n_frames);
  stage(d_dia, diameters, 8 * n);
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(c->ws.p, h.data(), small, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_fr, frames, fbytes, hipMemcpyHostToDevice, s));
  a.objs = c->d_desc;
  a.max_nm = c->max_nm;
  a.slots = d_s;
  a.pose_est = d_pe;
  a.pose_gt = d_pg;
  a.frame_idx = d_fi;
  a.frames = d_fr;
  a.cam = d_cam;
  a.diameters = d_dia;
  a.out = d_out;
  a.unions = (flags & BOPX_VSD_UNIONS) ? d_out + (size_t)n * n_tau : nullptr;
  a.n = n;
  {
    const hipStream_t so = s;
    LaunchOrder ord;
    const bopx::OrderCost oc = vsd_order_cost(a);
    if (int r = make_order(c, a.n, a.slots, so, ord, oc.pe ? &oc : nullptr)) return r;
    a.order = ord.p;
    HIPCHK(c, bopx::launch_vsd(a, cost_type, so));
  }
  HIPCHK(c, hipMemcpyAsync(out, d_out, 8 * n_out, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return BOPX_OK;
}

// -------------------------------------------------------------- shared renders
// VSD of many (est, gt) tuples over a set of distinct renders (multi-instance
// images: k estimates x k GT instances of an object share 2k renders instead of
// 2k^2). Device pointers, stream s; one host synchronisation (the ROI sizes
// decide the q buffer layout).
static int vsd_shared_core(bopx_ctx* c, int64_t nr, const int32_t* rslots, const double* rpose,
                           const int32_t* rframe, int64_t n, const int32_t* est_r,
                           const int32_t* gt_r, const float* frames, int width, int height,
                           const double* cam, double delta, int flags, const double* taus,
                           int n_tau, int normalized, const double* dia, int cost_type,
                           double* out, hipStream_t s) {
  bopx::VsdArgs a{};
  a.cull = vsd_cull_enabled();
  a.qorder = vsd_queue_order();
  if (int r = fill_vsd_args(c, a, width, height, delta, flags, taus, n_tau, normalized,
                            cost_type))
    return r;
  if (n <= 0) return BOPX_OK;
  // tuples without renders: every render index is out of range, and nothing
  // would write the caller's output
  if (nr <= 0) return fail(c, BOPX_E_INVALID, "%lld tuples but no renders", (long long)n);
  int4* d_roi = nullptr;
  int64_t* d_off = nullptr;
  uint32_t* d_q = nullptr;
  HIPCHK(c, hipMallocAsync((void**)&d_roi, (size_t)nr * (sizeof(int4) + 2 * sizeof(int64_t)), s));
  d_off = reinterpret_cast<int64_t*>(d_roi + nr);
  int64_t* d_roff = d_off + nr;
  int rc = BOPX_OK;
  std::vector<int4> roi((size_t)nr);
  std::vector<int64_t> off(2 * (size_t)nr);  // q offsets, then row-span offsets
  int64_t total = 0, rows = 0;
  hipError_t e = bopx::launch_pose_roi(c->d_desc, nr, rslots, rpose, rframe, cam, width, height,
                                       d_roi, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(roi.data(), d_roi, (size_t)nr * sizeof(int4), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess) {
    for (int64_t i = 0; i < nr; ++i) {
      off[i] = total;
      off[nr + i] = rows;
      const int4 r = roi[i];
      if (r.x <= r.z && r.y <= r.w) {
        total += (int64_t)(r.z - r.x + 1) * (r.w - r.y + 1);
        rows += r.w - r.y + 1;
      }
    }
    e = hipMemcpyAsync(d_off, off.data(), 2 * (size_t)nr * sizeof(int64_t),
                       hipMemcpyHostToDevice, s);
  }
  // q buffers (0 = background), then the row spans: min 0x7F7F7F7F, max -1
  const size_t qn = (size_t)std::max<int64_t>(total, 1), sn = (size_t)std::max<int64_t>(rows, 1);
  // BOPX_SHARED_MAX_BYTES caps this scratch (read per call; unset = no cap
  // beyond the device's free memory): past it the call fails like an OOM
  const char* cap_env = getenv("BOPX_SHARED_MAX_BYTES");
  const bool over_cap = cap_env && 4 * (qn + 2 * sn) > (size_t)strtoull(cap_env, nullptr, 10);
  if (e == hipSuccess &&
      (over_cap || hipMallocAsync((void**)&d_q, 4 * (qn + 2 * sn), s) != hipSuccess)) {
    (void)hipGetLastError();
    d_q = nullptr;
    (void)hipFreeAsync(d_roi, s);
    return fail(c, BOPX_E_OOM, "shared-render depth buffers of %zu bytes do not fit; split the "
                "batch or use bopx_vsd_batch", 4 * (qn + 2 * sn));
  }
  if (e == hipSuccess) e = hipMemsetAsync(d_q, 0, 4 * qn, s);
  int32_t* d_smin = reinterpret_cast<int32_t*>(d_q + qn);
  int32_t* d_smax = d_smin + sn;
  if (e == hipSuccess) e = hipMemsetAsync(d_smin, 0x7F, 4 * sn, s);
  if (e == hipSuccess) e = hipMemsetAsync(d_smax, 0xFF, 4 * sn, s);
  if (e == hipSuccess) {
    a.objs = c->d_desc;
    a.max_nm = c->max_nm;
    a.slots = rslots;
    a.pose_est = rpose;
    a.pose_gt = rpose;
    a.frame_idx = rframe;
    a.frames = frames;
    a.cam = cam;
    a.rois = d_roi;
    a.qoff = d_off;
    a.qbuf = d_q;
    a.rowoff = d_roff;
    a.smin = d_smin;
    a.smax = d_smax;
    a.n = nr;
    LaunchOrder ord;
    rc = make_order(c, nr, rslots, s, ord);
    if (rc == BOPX_OK) {
      a.order = ord.p;
      e = bopx::launch_vsd(a, bopx::kCostRender, s);
    }
  }
  if (rc == BOPX_OK && e == hipSuccess) {
    bopx::PairArgs p{};
    p.rois = d_roi;
    p.qoff = d_off;
    p.qbuf = d_q;
    p.rowoff = d_roff;
    p.smin = d_smin;
    p.smax = d_smax;
    p.rframe = rframe;
    p.est_r = est_r;
    p.gt_r = gt_r;
    p.n_renders = nr;
    p.frames = frames;
    p.cam = cam;
    p.diameters = dia;
    p.out = out;
    p.unions = (flags & BOPX_VSD_UNIONS) ? out + n * n_tau : nullptr;
    p.n = n;
    p.width = width;
    p.height = height;
    p.dthr = a.dthr;
    p.n_tau = n_tau;
    p.normalized = a.normalized;
    for (int k = 0; k < bopx::kMaxTaus; ++k) p.taus[k] = a.taus[k];
    e = bopx::launch_vsd_pair(p, cost_type, s);
  }
  // scratch freed on every path, behind the launches that read it
  const hipError_t f1 = d_q ? hipFreeAsync(d_q, s) : hipSuccess;
  const hipError_t f2 = hipFreeAsync(d_roi, s);
  if (rc != BOPX_OK) return rc;
  HIPCHK(c, e);
  HIPCHK(c, f1);
  HIPCHK(c, f2);
  return BOPX_OK;
}

int bopx_vsd_shared_batch_dev(bopx_ctx* c, int64_t n_renders, const int32_t* render_slots,
                              const double* render_poses, const int32_t* render_frame_idx,
                              int64_t n, const int32_t* est_render, const int32_t* gt_render,
                              const float* frames, int width, int height, const double* cam,
                              double delta, int flags, const double* taus, int n_tau,
                              int normalized, const double* diameters, int cost_type,
                              double* out, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (n < 0 || n_renders < 0) return fail(c, BOPX_E_INVALID, "negative size");
  if (int r = launch_dev(c)) return r;
  return vsd_shared_core(c, n_renders, render_slots, render_poses, render_frame_idx, n,
                         est_render, gt_render, frames, width, height, cam, delta, flags, taus,
                         n_tau, normalized, diameters, cost_type, out, pick_stream(c, stream));
}

int bopx_vsd_shared_batch(bopx_ctx* c, int64_t n_renders, const int32_t* render_obj_ids,
                          const double* render_poses, const int32_t* render_frame_idx, int64_t n,
                          const int32_t* est_render, const int32_t* gt_render,
                          const float* frames, int64_t n_frames, int width, int height,
                          const double* cam, double delta, int flags, const double* taus,
                          int n_tau, int normalized, const double* diameters, int cost_type,
                          double* out) {
  if (!c) return BOPX_E_INVALID;
  if (n < 0 || n_renders < 0 || n_frames < 0) return fail(c, BOPX_E_INVALID, "negative size");
  if (n == 0) return BOPX_OK;
  if (!render_obj_ids || !render_poses || !render_frame_idx || !est_render || !gt_render ||
      !frames || !cam || !diameters || !out)
    return fail(c, BOPX_E_INVALID, "NULL buffer");
  for (int64_t i = 0; i < n_renders; ++i)
    if (render_frame_idx[i] < 0 || render_frame_idx[i] >= n_frames)
      return fail(c, BOPX_E_INVALID, "render_frame_idx[%lld] = %d out of range", (long long)i,
                  render_frame_idx[i]);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t e = est_render[i], g = gt_render[i];
    if (e < 0 || e >= n_renders || g < 0 || g >= n_renders)
      return fail(c, BOPX_E_INVALID, "tuple %lld: render index out of range", (long long)i);
    if (render_frame_idx[e] != render_frame_idx[g])
      return fail(c, BOPX_E_INVALID, "tuple %lld: est and gt renders of different frames",
                  (long long)i);
  }
  if (int r = launch_dev(c)) return r;
  std::vector<int32_t> slots;
  if (int r = map_slots(c, n_renders, render_obj_ids, slots, false, true)) return r;
  const size_t fbytes = (size_t)n_frames * width * height * sizeof(float);
  const size_t n_out = (size_t)n * n_tau + ((flags & BOPX_VSD_UNIONS) ? (size_t)n : 0);
  const size_t nr = (size_t)n_renders;
  if (int r = ws_reserve(c, carve_size({4 * nr, 96 * nr, 4 * nr, 4 * (size_t)n, 4 * (size_t)n,
                                        32 * (size_t)n_frames, 8 * (size_t)n, fbytes,
                                        8 * n_out})))
    return r;
  Carve cv{(char*)c->ws.p};
  int32_t* d_rs = cv.take<int32_t>(nr);
  double* d_rp = cv.take<double>(12 * nr);
  int32_t* d_rf = cv.take<int32_t>(nr);
  int32_t* d_e = cv.take<int32_t>(n);
  int32_t* d_g = cv.take<int32_t>(n);
  double* d_cam = cv.take<double>(4 * n_frames);
  double* d_dia = cv.take<double>(n);
  float* d_fr = cv.take<float>((size_t)n_frames * width * height);
  double* d_out = cv.take<double>(n_out);
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_rs, slots.data(), 4 * nr, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_rp, render_poses, 96 * nr, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_rf, render_frame_idx, 4 * nr, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_e, est_render, 4 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_g, gt_render, 4 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_cam, cam, 32 * n_frames, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_dia, diameters, 8 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_fr, frames, fbytes, hipMemcpyHostToDevice, s));
  if (int r = vsd_shared_core(c, n_renders, d_rs, d_rp, d_rf, n, d_e, d_g, d_fr, width, height,
                              d_cam, delta, flags, taus, n_tau, normalized, d_dia, cost_type,
                              d_out, s))
    return r;
  HIPCHK(c, hipMemcpyAsync(out, d_out, 8 * n_out, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return BOPX_OK;
}

// ----------------------------------------------------------- silhouette cover
static int cover_args(bopx_ctx* c, bopx::VsdArgs& a, int width, int height) {
  if (width <= 0 || height <= 0 || width > 32767 || height > 32767)
    return fail(c, BOPX_E_INVALID, "bad image size %dx%d", width, height);
  // no tile limit: the 16-bit per-tau counters behind kVsdMaxTiles are VSD-only
  a.width = a.img_w = width;
  a.height = a.img_h = height;
  a.n_tau = 0;
  return BOPX_OK;
}

// ------------------------------------------------------------------- GT info
static int gt_info_args(bopx_ctx* c, bopx::VsdArgs& a, int width, int height, double delta,
                        int flags, int canvas_scale) {
  if (canvas_scale != 1 && canvas_scale != 3)
    return fail(c, BOPX_E_INVALID, "canvas_scale must be 1 or 3");
  if (width <= 0 || height <= 0 || (int64_t)width * canvas_scale > 32767 ||
      (int64_t)height * canvas_scale > 32767)
    return fail(c, BOPX_E_INVALID, "bad image size %dx%d", width, height);
  a.img_w = width;
  a.img_h = height;
  a.width = width * canvas_scale;
  a.height = height * canvas_scale;
  a.ox = canvas_scale == 3 ? width : 0;
  a.oy = canvas_scale == 3 ? height : 0;
  a.delta32 = (float)delta;
  a.delta64 = delta;
  a.delta_f64 = (flags & BOPX_DELTA_F64) ? 1 : 0;
  a.dthr = visib_thr32(delta, flags);
  a.n_tau = 0;
  return BOPX_OK;
}

int bopx_gt_info_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pose,
                           const int32_t* frame_idx, const float* frames, int width, int height,
                           const double* cam, double delta, int flags, int canvas_scale,
                           double* out, uint8_t* masks, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = launch_dev(c)) return r;
  bopx::VsdArgs a{};
  a.cull = vsd_cull_enabled();
  a.qorder = vsd_queue_order();
  if (int r = gt_info_args(c, a, width, height, delta, flags, canvas_scale)) return r;
  hipStream_t s = pick_stream(c, stream);
  if (masks && n > 0)
    HIPCHK(c, hipMemsetAsync(masks, 0, (size_t)n * 2 * width * height, s));
  a.objs = c->d_desc;
  a.max_nm = c->max_nm;
  a.slots = slots;
  a.pose_est = pose;
  a.pose_gt = pose;
  a.frame_idx = frame_idx;
  a.frames = frames;
  a.cam = cam;
  a.out = out;
  a.masks = masks;
  a.n = n;
  {
    const hipStream_t so = s;
    LaunchOrder ord;
    if (int r = make_order(c, a.n, a.slots, so, ord)) return r;
    a.order = ord.p;
    HIPCHK(c, bopx::launch_vsd(a, bopx::kCostGtInfo, so));
  }
  return BOPX_OK;
}

int bopx_gt_info_batch(bopx_ctx* c, int64_t n, const int32_t* obj_ids, const double* pose,
                       const int32_t* frame_idx, const float* frames, int64_t n_frames,
                       int width, int height, const double* cam, double delta, int flags,
                       int canvas_scale, double* out, uint8_t* masks) {
  if (!c) return BOPX_E_INVALID;
  if (n < 0 || n_frames < 0) return fail(c, BOPX_E_INVALID, "negative size");
  if (n == 0) return BOPX_OK;
  if (!obj_ids || !pose || !frame_idx || !frames || !cam || !out)
    return fail(c, BOPX_E_INVALID, "NULL buffer");
  for (int64_t i = 0; i < n; ++i)
    if (frame_idx[i] < 0 || frame_idx[i] >= n_frames)
      return fail(c, BOPX_E_INVALID, "frame_idx[%lld] = %d out of range", (long long)i,
                  frame_idx[i]);
  if (int r = launch_dev(c)) return r;
  bopx::VsdArgs a{};
  a.cull = vsd_cull_enabled();
  a.qorder = vsd_queue_order();
  if (int r = gt_info_args(c, a, width, height, delta, flags, canvas_scale)) return r;
  std::vector<int32_t> slots;
  if (int r = map_slots(c, n, obj_ids, slots, false, true)) return r;
  const size_t fpx = (size_t)width * height, cols = bopx::kGtInfoCols;
  const size_t mbytes = masks ? 2 * fpx * (size_t)n : 0;
  if (int r = ws_reserve(c, carve_size({4 * (size_t)n, 96 * (size_t)n, 4 * (size_t)n,
                                        4 * fpx * (size_t)n_frames, 32 * (size_t)n_frames,
                                        8 * cols * (size_t)n, mbytes})))
    return r;
  Carve cv{(char*)c->ws.p};
  int32_t* d_s = cv.take<int32_t>(n);
  double* d_p = cv.take<double>(12 * n);
  int32_t* d_fi = cv.take<int32_t>(n);
  float* d_fr = cv.take<float>(fpx * n_frames);
  double* d_cam = cv.take<double>(4 * n_frames);
  double* d_out = cv.take<double>(cols * n);
  uint8_t* d_m = masks ? cv.take<uint8_t>(mbytes) : nullptr;
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_s, slots.data(), 4 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_p, pose, 96 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_fi, frame_idx, 4 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_fr, frames, 4 * fpx * n_frames, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_cam, cam, 32 * n_frames, hipMemcpyHostToDevice, s));
  if (d_m) HIPCHK(c, hipMemsetAsync(d_m, 0, mbytes, s));
  a.objs = c->d_desc;
  a.max_nm = c->max_nm;
  a.slots = d_s;
  a.pose_est = d_p;
  a.pose_gt = d_p;
  a.frame_idx = d_fi;
  a.frames = d_fr;
  a.cam = d_cam;
  a.out = d_out;
  a.masks = d_m;
  a.n = n;
  {
    const hipStream_t so = s;
    LaunchOrder ord;
    if (int r = make_order(c, a.n, a.slots, so, ord)) return r;
    a.order = ord.p;
    HIPCHK(c, bopx::launch_vsd(a, bopx::kCostGtInfo, so));
  }
  HIPCHK(c, hipMemcpyAsync(out, d_out, 8 * cols * n, hipMemcpyDeviceToHost, s));
  if (d_m) HIPCHK(c, hipMemcpyAsync(masks, d_m, mbytes, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return BOPX_OK;
}

int bopx_cover_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pe,
                         const double* pg, const int32_t* frame_idx, int width, int height,
                         const double* cam, double* out, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = launch_dev(c)) return r;
  bopx::VsdArgs a{};
  a.cull = vsd_cull_enabled();
  a.qorder = vsd_queue_order();
  if (int r = cover_args(c, a, width, height)) return r;
  a.objs = c->d_desc;
  a.max_nm = c->max_nm;
  a.slots = slots;
  a.pose_est = pe;
  a.pose_gt = pg;
  a.frame_idx = frame_idx;
  a.cam = cam;
  a.out = out;
  a.n = n;
  {
    const hipStream_t so = pick_stream(c, stream);
    LaunchOrder ord;
    if (int r = make_order(c, a.n, a.slots, so, ord)) return r;
    a.order = ord.p;
    HIPCHK(c, bopx::launch_vsd(a, bopx::kCostCover, so));
  }
  return BOPX_OK;
}

int bopx_cover_batch(bopx_ctx* c, int64_t n, const int32_t* obj_ids, const double* pe,
                     const double* pg, const int32_t* frame_idx, int64_t n_frames, int width,
                     int height, const double* cam, double* out) {
  if (!c) return BOPX_E_INVALID;
  if (n < 0 || n_frames < 0) return fail(c, BOPX_E_INVALID, "negative size");
  if (n == 0) return BOPX_OK;
  if (!obj_ids || !pe || !pg || !frame_idx || !cam || !out)
    return fail(c, BOPX_E_INVALID, "NULL buffer");
  for (int64_t i = 0; i < n; ++i)
    if (frame_idx[i] < 0 || frame_idx[i] >= n_frames)
      return fail(c, BOPX_E_INVALID, "frame_idx[%lld] = %d out of range", (long long)i,
                  frame_idx[i]);
  if (int r = launch_dev(c)) return r;
  bopx::VsdArgs a{};
  a.cull = vsd_cull_enabled();
  a.qorder = vsd_queue_order();
  if (int r = cover_args(c, a, width, height)) return r;
  std::vector<int32_t> slots;
  if (int r = map_slots(c, n, obj_ids, slots, false, true)) return r;
  const size_t cols = bopx::kCoverCols;
  if (int r = ws_reserve(c, carve_size({4 * (size_t)n, 96 * (size_t)n, 96 * (size_t)n,
                                        4 * (size_t)n, 32 * (size_t)n_frames,
                                        8 * cols * (size_t)n})))
    return r;
  Carve cv{(char*)c->ws.p};
  int32_t* d_s = cv.take<int32_t>(n);
  double* d_pe = cv.take<double>(12 * n);
  double* d_pg = cv.take<double>(12 * n);
  int32_t* d_fi = cv.take<int32_t>(n);
  double* d_cam = cv.take<double>(4 * n_frames);
  double* d_out = cv.take<double>(cols * n);
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_s, slots.data(), 4 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_pe, pe, 96 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_pg, pg, 96 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_fi, frame_idx, 4 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_cam, cam, 32 * n_frames, hipMemcpyHostToDevice, s));
  a.objs = c->d_desc;
  a.max_nm = c->max_nm;
  a.slots = d_s;
  a.pose_est = d_pe;
  a.pose_gt = d_pg;
  a.frame_idx = d_fi;
  a.cam = d_cam;
  a.out = d_out;
  a.n = n;
  {
    const hipStream_t so = s;
    LaunchOrder ord;
    if (int r = make_order(c, a.n, a.slots, so, ord)) return r;
    a.order = ord.p;
    HIPCHK(c, bopx::launch_vsd(a, bopx::kCostCover, so));
  }
  HIPCHK(c, hipMemcpyAsync(out, d_out, 8 * cols * n, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return BOPX_OK;
}

int bopx_cover_from_depths(bopx_ctx* c, int width, int height, const float* depth_est,
                           const float* depth_gt, double* out) {
  if (!c) return BOPX_E_INVALID;
  if (width <= 0 || height <= 0) return fail(c, BOPX_E_INVALID, "bad image size");
  if (!depth_est || !depth_gt || !out) return fail(c, BOPX_E_INVALID, "NULL buffer");
  if (int r = set_dev(c)) return r;
  const size_t npx = (size_t)width * height;
  if (int r = ws_reserve(c, carve_size({4 * npx, 4 * npx, 8 * bopx::kCoverCols}))) return r;
  Carve cv{(char*)c->ws.p};
  float* d_e = cv.take<float>(npx);
  float* d_g = cv.take<float>(npx);
  long long* d_acc = cv.take<long long>(bopx::kCoverCols);
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_e, depth_est, 4 * npx, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_g, depth_gt, 4 * npx, hipMemcpyHostToDevice, s));
  HIPCHK(c, bopx::launch_cover_depths(width, height, d_e, d_g, d_acc, s));
  long long acc[bopx::kCoverCols];
  HIPCHK(c, hipMemcpyAsync(acc, d_acc, sizeof(acc), hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  for (int k = 0; k < bopx::kCoverCols; ++k) out[k] = (double)acc[k];
  return BOPX_OK;
}

int bopx_vsd_from_depths(bopx_ctx* c, int width, int height, const float* depth_test,
                         const float* depth_est, const float* depth_gt, double fx, double fy,
                         double cx, double cy, double delta, int flags, const double* taus,
                         int n_tau, int normalized, double diameter, int cost_type,
                         double* out) {
  if (!c) return BOPX_E_INVALID;
  if (width <= 0 || height <= 0) return fail(c, BOPX_E_INVALID, "bad image size");
  if (!depth_test || !depth_est || !depth_gt || !out)
    return fail(c, BOPX_E_INVALID, "NULL buffer");
  if (int r = check_taus(c, taus, n_tau)) return r;
  if (int r = set_dev(c)) return r;
  const size_t npx = (size_t)width * height;
  const int nb = bopx::vsd_depths_blocks(width, height);
  const int stride = 2 + 2 * bopx::kMaxTaus;
  if (int r = ws_reserve(c, carve_size({4 * npx, 4 * npx, 4 * npx, 8 * (size_t)nb * stride})))
    return r;
  Carve cv{(char*)c->ws.p};
  float* d_t = cv.take<float>(npx);
  float* d_e = cv.take<float>(npx);
  float* d_g = cv.take<float>(npx);
  double* d_p = cv.take<double>((size_t)nb * stride);
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_t, depth_test, 4 * npx, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_e, depth_est, 4 * npx, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_g, depth_gt, 4 * npx, hipMemcpyHostToDevice, s));
  HIPCHK(c, bopx::launch_vsd_depths(width, height, d_t, d_e, d_g, fx, fy, cx, cy, (float)delta,
                                    (flags & BOPX_DELTA_F64) ? 1 : 0, delta, taus, n_tau,
                                    normalized ? 1 : 0, diameter, d_p, nb, s));
  std::vector<double> part((size_t)nb * stride);
  HIPCHK(c, hipMemcpyAsync(part.data(), d_p, 8 * part.size(), hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  std::vector<double> tot(stride, 0.0);
  for (int b = 0; b < nb; ++b)
    for (int k = 0; k < stride; ++k) tot[k] += part[(size_t)b * stride + k];
  const double un = tot[0], comp = tot[0] - tot[1];
  if (flags & BOPX_VSD_UNIONS) out[n_tau] = un;
  if (un == 0.0) {
    for (int k = 0; k < n_tau; ++k) out[k] = 1.0;
    return BOPX_OK;
  }
  // The reference raises on an unknown cost type only when the union is non-empty
  // (pose_error.py:75-88).
  if (cost_type != BOPX_COST_STEP && cost_type != BOPX_COST_TLINEAR)
    return fail(c, BOPX_E_INVALID, "Unknown pixel matching cost.");
  for (int k = 0; k < n_tau; ++k) {
    if (cost_type == BOPX_COST_STEP)
      out[k] = (double)((int64_t)tot[2 + k] + (int64_t)comp) / un;
    else
      out[k] = (tot[2 + bopx::kMaxTaus + k] + comp) / un;
  }
  return BOPX_OK;
}

// -------------------------------------------------------------------- renderer
int bopx_depth_clear_dev(bopx_ctx* c, float* frames, int64_t n_pixels, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = set_dev(c)) return r;
  HIPCHK(c, bopx::launch_depth_fill(frames, n_pixels, 0, pick_stream(c, stream)));
  return BOPX_OK;
}

int bopx_depth_finish_dev(bopx_ctx* c, float* frames, int64_t n_pixels, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (int r = set_dev(c)) return r;
  HIPCHK(c, bopx::launch_depth_fill(frames, n_pixels, 1, pick_stream(c, stream)));
  return BOPX_OK;
}

int bopx_png_decode_dev(bopx_ctx* c, int64_t n, const uint8_t* zdata, const int64_t* z_off,
                        const int32_t* z_len, int height, int width, const float* scales,
                        uint8_t* raw, int64_t raw_stride, float* frames, int32_t* status,
                        void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (n < 0) return fail(c, BOPX_E_INVALID, "n = %lld", (long long)n);
  if (width <= 0 || height <= 0 || width > bopx::kPngMaxWidth ||
      (int64_t)height * (2 * (int64_t)width + 1) > bopx::kPngMaxRaw)
    return fail(c, BOPX_E_INVALID, "png size %d x %d outside the device decoder's range", width,
                height);
  const int64_t need = ((int64_t)height * (2 * width + 1) + 64 + 1023) / 1024 * 1024;
  if (raw_stride < need)
    return fail(c, BOPX_E_INVALID, "raw_stride %lld < %lld", (long long)raw_stride,
                (long long)need);
  if (n == 0) return BOPX_OK;
  if (!zdata || !z_off || !z_len || !raw || !frames || !status)
    return fail(c, BOPX_E_INVALID, "null device pointer");
  if (int r = set_dev(c)) return r;
  HIPCHK(c, bopx::launch_png_decode(n, zdata, z_off, z_len, height, width, scales, raw, raw_stride,
                                    frames, status, pick_stream(c, stream)));
  return BOPX_OK;
}

int bopx_render_depth_batch_dev(bopx_ctx* c, int64_t n, const int32_t* slots, const double* pose,
                                const int32_t* frame_idx, const double* cam, float* frames,
                                int width, int height, void* stream) {
  if (!c) return BOPX_E_INVALID;
  if (width <= 0 || height <= 0) return fail(c, BOPX_E_INVALID, "bad image size");
  if (int r = launch_dev(c)) return r;
  if (n <= 0 || c->max_nf <= 0) return BOPX_OK;
  HIPCHK(c, bopx::launch_render_batch(c->d_desc, c->max_nf, n, slots, pose, frame_idx, cam,
                                      frames, width, height, pick_stream(c, stream)));
  return BOPX_OK;
}

int bopx_render_depth(bopx_ctx* c, int obj_id, const double* R, const double* t, double fx,
                      double fy, double cx, double cy, int width, int height, float* out) {
  if (!c) return BOPX_E_INVALID;
  if (!R || !t || !out) return fail(c, BOPX_E_INVALID, "NULL buffer");
  if (width <= 0 || height <= 0) return fail(c, BOPX_E_INVALID, "bad image size");
  if (int r = launch_dev(c)) return r;
  std::vector<int32_t> slots;
  int32_t id = obj_id;
  if (int r = map_slots(c, 1, &id, slots, false, true)) return r;
  const size_t npx = (size_t)width * height;
  if (int r = ws_reserve(c, carve_size({4 * npx, 4, 96, 4, 32}))) return r;
  Carve cv{(char*)c->ws.p};
  float* d_f = cv.take<float>(npx);
  int32_t* d_s = cv.take<int32_t>(1);
  double* d_pose = cv.take<double>(12);
  int32_t* d_fi = cv.take<int32_t>(1);
  double* d_cam = cv.take<double>(4);
  double pose[12], cam[4] = {fx, fy, cx, cy};
  for (int i = 0; i < 9; ++i) pose[i] = R[i];
  for (int i = 0; i < 3; ++i) pose[9 + i] = t[i];
  const int32_t zero = 0;
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_s, slots.data(), 4, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_pose, pose, 96, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_fi, &zero, 4, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_cam, cam, 32, hipMemcpyHostToDevice, s));
  HIPCHK(c, bopx::launch_depth_fill(d_f, (int64_t)npx, 0, s));
  HIPCHK(c, bopx::launch_render_batch(c->d_desc, (int)c->objs[slots[0]].nf, 1, d_s, d_pose, d_fi,
                                      d_cam, d_f, width, height, s));
  HIPCHK(c, bopx::launch_depth_fill(d_f, (int64_t)npx, 1, s));
  HIPCHK(c, hipMemcpyAsync(out, d_f, 4 * npx, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return BOPX_OK;
}

// ------------------------------------------------------- geometry/visibility
int bopx_dist_im(bopx_ctx* c, int width, int height, const float* depth, double fx, double fy,
                 double cx, double cy, double* out) {
  if (!c) return BOPX_E_INVALID;
  if (width <= 0 || height <= 0 || !depth || !out)
    return fail(c, BOPX_E_INVALID, "bad arguments");
  if (int r = set_dev(c)) return r;
  const size_t npx = (size_t)width * height;
  if (int r = ws_reserve(c, carve_size({4 * npx, 8 * npx}))) return r;
  Carve cv{(char*)c->ws.p};
  float* d_in = cv.take<float>(npx);
  double* d_out = cv.take<double>(npx);
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_in, depth, 4 * npx, hipMemcpyHostToDevice, s));
  HIPCHK(c, bopx::launch_dist_im(width, height, d_in, fx, fy, cx, cy, d_out, s));
  HIPCHK(c, hipMemcpyAsync(out, d_out, 8 * npx, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return BOPX_OK;
}

int bopx_visib_mask(bopx_ctx* c, int64_t n, const double* d_test, const double* d_model,
                    const uint8_t* visib_gt, double delta, int flags, int visib_mode,
                    uint8_t* out) {
  if (!c) return BOPX_E_INVALID;
  if (visib_mode != BOPX_VISIB_BOP18 && visib_mode != BOPX_VISIB_BOP19)
    return fail(c, BOPX_E_INVALID, "Unknown visibility mode.");
  if (n < 0 || (n > 0 && (!d_test || !d_model || !out)))
    return fail(c, BOPX_E_INVALID, "bad arguments");
  if (n == 0) return BOPX_OK;
  if (int r = set_dev(c)) return r;
  if (int r = ws_reserve(c, carve_size({8 * (size_t)n, 8 * (size_t)n, (size_t)n, (size_t)n})))
    return r;
  Carve cv{(char*)c->ws.p};
  double* d_t = cv.take<double>(n);
  double* d_m = cv.take<double>(n);
  uint8_t* d_vg = cv.take<uint8_t>(n);
  uint8_t* d_o = cv.take<uint8_t>(n);
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_t, d_test, 8 * n, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_m, d_model, 8 * n, hipMemcpyHostToDevice, s));
  if (visib_gt) HIPCHK(c, hipMemcpyAsync(d_vg, visib_gt, n, hipMemcpyHostToDevice, s));
  HIPCHK(c, bopx::launch_visib(n, d_t, d_m, visib_gt ? d_vg : nullptr, (float)delta,
                               (flags & BOPX_DELTA_F64) ? 1 : 0, delta, visib_mode, d_o, s));
  HIPCHK(c, hipMemcpyAsync(out, d_o, n, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return BOPX_OK;
}

// Diagnostics (not in include/bopx.h): out[0..15] = k_vsd workload counters
// (BOPX_VSD_ABLATE bit 2: tiles, meshlet entries, triangle set-ups, bbox
// pixels, row items, fragments, covered pixels, row passes, sum of per-pass
// widest rows), out[16..31] = phase clocks (bit 3), out[32..47] = wave-level
// loop trip counts (bit 2, tools/isa_census.py). out holds 48 values.
int bopx_debug_vsd_stats(bopx_ctx* c, unsigned long long* out, int reset) {
  if (!c || !out) return BOPX_E_INVALID;
  if (int r = set_dev(c)) return r;
  HIPCHK(c, hipDeviceSynchronize());
  HIPCHK(c, bopx::read_vsd_stats(out, reset));
  return BOPX_OK;
}

}  // extern "C"
