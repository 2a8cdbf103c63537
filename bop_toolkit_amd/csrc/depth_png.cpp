// Host-side 16-bit depth PNG decoder behind include/bopx_io.h.
//
// The evaluation scripts spend most of their host time reading test depth:
// inout.load_depth (bop_toolkit_lib/inout.py:39-46) decodes one PNG per image
// through imageio, then eval_calc_errors.py:242-243 scales it in float32. Here
// one call reads and decodes a whole scene's files on worker threads, straight
// into the caller's (page-locked) float32 frames: chunk walk with CRC check,
// one inflate of the concatenated IDAT stream (libdeflate when the image has
// it, zlib otherwise; both are exact), row unfiltering fused with the
// big-endian sample -> float32 conversion and the depth_scale multiply.
//
// Only the layout BOP depth maps use is decoded (bit depth 16, colour type 0,
// no interlace); anything else reports BOPX_IO_UNSUPPORTED and the Python
// caller hands that file to Pillow.
#include "../../include/bopx_io.h"

#include <dlfcn.h>
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace {

// ---- inflate back-ends ------------------------------------------------------

// libdeflate ABI (libdeflate.h; the image ships the runtime library only).
using ld_alloc_t = void* (*)();
using ld_free_t = void (*)(void*);
using ld_zlib_t = int (*)(void*, const void*, size_t, void*, size_t, size_t*);
using ld_crc_t = uint32_t (*)(uint32_t, const void*, size_t);

struct Deflate {
  ld_alloc_t alloc = nullptr;
  ld_free_t free = nullptr;
  ld_zlib_t zlib = nullptr;
  ld_crc_t crc = nullptr;
  bool ok = false;
};

const Deflate& deflate_lib() {
  static Deflate d;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* force = std::getenv("BOPX_IO_ZLIB");
    if (force && force[0] == '1') return;
    void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    d.alloc = (ld_alloc_t)dlsym(h, "libdeflate_alloc_decompressor");
    d.free = (ld_free_t)dlsym(h, "libdeflate_free_decompressor");
    d.zlib = (ld_zlib_t)dlsym(h, "libdeflate_zlib_decompress");
    d.crc = (ld_crc_t)dlsym(h, "libdeflate_crc32");
    d.ok = d.alloc && d.free && d.zlib && d.crc;
  });
  return d;
}

// Per-thread decoder state: buffers are reused across the files of one call.
struct Worker {
  void* ld = nullptr;  // libdeflate decompressor
  std::vector<uint8_t> file, idat, raw;

  Worker() {
    const Deflate& d = deflate_lib();
    if (d.ok) ld = d.alloc();
  }
  ~Worker() {
    if (ld) deflate_lib().free(ld);
  }
  Worker(const Worker&) = delete;
  Worker& operator=(const Worker&) = delete;

  uint32_t crc(const uint8_t* p, size_t n) const {
    if (ld) return deflate_lib().crc(0, p, n);
    uint32_t c = (uint32_t)crc32(0L, Z_NULL, 0);
    while (n) {  // zlib's length argument is 32-bit
      const uInt k = n > (1u << 30) ? (1u << 30) : (uInt)n;
      c = (uint32_t)crc32(c, p, k);
      p += k;
      n -= k;
    }
    return c;
  }

  // Inflate a zlib stream into exactly `out_n` bytes (the stream must end there).
  bool inflate_exact(const uint8_t* in, size_t in_n, uint8_t* out, size_t out_n) {
    if (ld) return deflate_lib().zlib(ld, in, in_n, out, out_n, nullptr) == 0;
    if (in_n > 0xFFFFFFFFu || out_n > 0xFFFFFFFFu) return false;  // zlib's 32-bit counters
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (inflateInit(&zs) != Z_OK) return false;
    zs.next_in = const_cast<uint8_t*>(in);
    zs.avail_in = (uInt)in_n;
    zs.next_out = out;
    zs.avail_out = (uInt)out_n;
    const int rc = inflate(&zs, Z_FINISH);
    const bool ok = rc == Z_STREAM_END && zs.total_out == out_n;
    inflateEnd(&zs);
    return ok;
  }

  int decode(const uint8_t* data, size_t n, int h, int w, float scale, float* dst);
  int pack(const char* path, int64_t size, int h, int w, uint8_t* dst, int64_t* z_n);
};

inline uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

inline uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c;
  const int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  return (uint8_t)(pa <= pb && pa <= pc ? a : (pb <= pc ? b : c));
}

// Undo one row's filter in place (PNG spec 9.2-9.4, 2 bytes per pixel).
// prev = the previous unfiltered row, or nullptr for the first row.
inline bool unfilter_row(int f, uint8_t* cur, const uint8_t* prev, int rb) {
  constexpr int bpp = 2;
  switch (f) {
    case 0:
      return true;
    case 1:  // Sub
      for (int i = bpp; i < rb; ++i) cur[i] = (uint8_t)(cur[i] + cur[i - bpp]);
      return true;
    case 2:  // Up
      if (prev)
        for (int i = 0; i < rb; ++i) cur[i] = (uint8_t)(cur[i] + prev[i]);
      return true;
    case 3:  // Average
      if (prev) {
        for (int i = 0; i < bpp; ++i) cur[i] = (uint8_t)(cur[i] + (prev[i] >> 1));
        for (int i = bpp; i < rb; ++i)
          cur[i] = (uint8_t)(cur[i] + ((cur[i - bpp] + prev[i]) >> 1));
      } else {
        for (int i = bpp; i < rb; ++i) cur[i] = (uint8_t)(cur[i] + (cur[i - bpp] >> 1));
      }
      return true;
    case 4:  // Paeth (with no previous row it reduces to Sub)
      if (prev) {
        for (int i = 0; i < bpp; ++i) cur[i] = (uint8_t)(cur[i] + prev[i]);
        for (int i = bpp; i < rb; ++i)
          cur[i] = (uint8_t)(cur[i] + paeth(cur[i - bpp], prev[i], prev[i - bpp]));
      } else {
        for (int i = bpp; i < rb; ++i) cur[i] = (uint8_t)(cur[i] + cur[i - bpp]);
      }
      return true;
    default:
      return false;
  }
}

// Chunk walk (PNG spec 5.3-5.6, 11.2): signature, chunk lengths, CRCs, IHDR
// (16-bit gray, no interlace, h x w), critical chunks, IEND. Calls
// on_idat(body, len) for every IDAT payload, in order.
template <class F>
int walk_chunks(const Worker& wk, const uint8_t* data, size_t n, int h, int w, F&& on_idat) {
  static const uint8_t kSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  if (n < 8 || std::memcmp(data, kSig, 8) != 0) return BOPX_IO_CORRUPT;
  size_t pos = 8;
  bool have_hdr = false, have_end = false;
  uint32_t pw = 0, ph = 0;
  int n_idat = 0;
  while (pos + 12 <= n) {
    const uint32_t len = be32(data + pos);
    if (len > n - pos - 12) return BOPX_IO_CORRUPT;
    const uint8_t* type = data + pos + 4;
    const uint8_t* body = data + pos + 8;
    if (wk.crc(type, (size_t)len + 4) != be32(body + len)) return BOPX_IO_CORRUPT;
    if (!have_hdr) {
      if (std::memcmp(type, "IHDR", 4) != 0 || len != 13) return BOPX_IO_CORRUPT;
      pw = be32(body);
      ph = be32(body + 4);
      // bit depth, colour type, compression, filter method, interlace
      if (body[8] != 16 || body[9] != 0 || body[10] != 0 || body[11] != 0 || body[12] != 0)
        return BOPX_IO_UNSUPPORTED;
      if (pw == 0 || ph == 0) return BOPX_IO_CORRUPT;
      have_hdr = true;
    } else if (std::memcmp(type, "IDAT", 4) == 0) {
      on_idat(body, (size_t)len);
      ++n_idat;
    } else if (std::memcmp(type, "IEND", 4) == 0) {
      have_end = true;
      break;
    } else if (!(type[0] & 0x20)) {
      return BOPX_IO_UNSUPPORTED;  // unknown critical chunk (e.g. PLTE on gray)
    }
    pos += (size_t)len + 12;
  }
  if (!have_hdr || !have_end || n_idat == 0) return BOPX_IO_CORRUPT;
  if ((int64_t)pw != w || (int64_t)ph != h) return BOPX_IO_SIZE;
  return BOPX_IO_OK;
}

int Worker::decode(const uint8_t* data, size_t n, int h, int w, float scale, float* dst) {
  const uint8_t* single = nullptr;  // the IDAT payload when there is one chunk
  size_t single_n = 0;
  int n_idat = 0;
  idat.clear();
  const int st = walk_chunks(*this, data, n, h, w, [&](const uint8_t* body, size_t len) {
    if (n_idat == 1) idat.assign(single, single + single_n);
    if (n_idat >= 1) idat.insert(idat.end(), body, body + len);
    single = body;
    single_n = len;
    ++n_idat;
  });
  if (st != BOPX_IO_OK) return st;

  const size_t rb = 2 * (size_t)w;
  const size_t raw_n = (size_t)h * (rb + 1);
  raw.resize(raw_n);
  const uint8_t* in = n_idat == 1 ? single : idat.data();
  const size_t in_n = n_idat == 1 ? single_n : idat.size();
  if (!inflate_exact(in, in_n, raw.data(), raw_n)) return BOPX_IO_CORRUPT;

  const uint8_t* prev = nullptr;
  for (int r = 0; r < h; ++r) {
    uint8_t* row = raw.data() + (size_t)r * (rb + 1);
    uint8_t* cur = row + 1;
    if (!unfilter_row(row[0], cur, prev, (int)rb)) return BOPX_IO_CORRUPT;
    float* o = dst + (size_t)r * w;
    for (int c = 0; c < w; ++c) o[c] = (float)(uint32_t)(cur[2 * c] << 8 | cur[2 * c + 1]) * scale;
    prev = cur;
  }
  return BOPX_IO_OK;
}

// Read a file of `size` bytes into dst, check its chunks as decode() does and
// move the concatenated IDAT payload to dst[0, *z_n) (payloads only move
// towards the start, over chunks already checked).
int Worker::pack(const char* path, int64_t size, int h, int w, uint8_t* dst, int64_t* z_n) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return BOPX_IO_READ;
  const bool ok = size >= 0 && std::fread(dst, 1, (size_t)size, f) == (size_t)size &&
                  std::fgetc(f) == EOF;
  std::fclose(f);
  if (!ok) return BOPX_IO_READ;
  size_t wp = 0;
  const int st = walk_chunks(*this, dst, (size_t)size, h, w, [&](const uint8_t* body, size_t len) {
    std::memmove(dst + wp, body, len);
    wp += len;
  });
  *z_n = (int64_t)wp;
  if (st == BOPX_IO_OK && wp > 0x7FFFFFFF) return BOPX_IO_UNSUPPORTED;
  return st;
}

bool read_file(const char* path, std::vector<uint8_t>& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  bool ok = std::fseek(f, 0, SEEK_END) == 0;
  const long sz = ok ? std::ftell(f) : -1;
  ok = ok && sz >= 0 && std::fseek(f, 0, SEEK_SET) == 0;
  if (ok) {
    buf.resize((size_t)sz);
    ok = std::fread(buf.data(), 1, buf.size(), f) == buf.size();
  }
  std::fclose(f);
  return ok;
}

}  // namespace

extern "C" int bopx_decode_depth_png(const uint8_t* data, size_t n, int h, int w, float scale,
                                     float* dst) {
  if (!data || !dst || h <= 0 || w <= 0) return BOPX_IO_SIZE;
  Worker wk;
  return wk.decode(data, n, h, w, scale, dst);
}

extern "C" int bopx_load_depth_pngs(const char* const* paths, int n, const int* h, const int* w,
                                    const float* scales, float* const* dst, int threads,
                                    int* status) {
  if (n <= 0) return 0;
  int nt = threads > 0 ? threads : 16;
  if (nt > n) nt = n;
  std::atomic<int> next{0}, failed{0};
  auto run = [&] {
    Worker wk;
    for (int k; (k = next.fetch_add(1)) < n;) {
      int st;
      if (!read_file(paths[k], wk.file))
        st = BOPX_IO_READ;
      else if (h[k] <= 0 || w[k] <= 0 || !dst[k])
        st = BOPX_IO_SIZE;
      else
        st = wk.decode(wk.file.data(), wk.file.size(), h[k], w[k], scales ? scales[k] : 1.0f,
                       dst[k]);
      status[k] = st;
      if (st) failed.fetch_add(1);
    }
  };
  if (nt == 1) {
    run();
  } else {
    std::vector<std::thread> pool;
    pool.reserve(nt - 1);
    for (int i = 1; i < nt; ++i) pool.emplace_back(run);
    run();
    for (auto& t : pool) t.join();
  }
  return failed.load();
}

extern "C" int bopx_pack_depth_pngs(const char* const* paths, int n, const int* h, const int* w,
                                    uint8_t* dst, int64_t cap, int64_t* z_off, int32_t* z_len,
                                    int threads, int* status, int64_t* need) {
  if (n <= 0 || !paths || !h || !w || !z_off || !z_len || !status) {
    if (need) *need = 2048;
    return n <= 0 ? 0 : -1;
  }
  std::vector<int64_t> size(n);
  int64_t off = 0;
  for (int k = 0; k < n; ++k) {
    struct stat sb;
    size[k] = stat(paths[k], &sb) == 0 ? (int64_t)sb.st_size : -1;
    z_off[k] = off;
    off += (std::max<int64_t>(size[k], 0) + 255) / 256 * 256;
  }
  if (need) *need = off + 2048;
  if (!dst || cap < off + 2048) return -1;
  int nt = threads > 0 ? threads : 16;
  if (nt > n) nt = n;
  std::atomic<int> next{0}, failed{0};
  auto run = [&] {
    Worker wk;
    for (int k; (k = next.fetch_add(1)) < n;) {
      int64_t zn = 0;
      int st = BOPX_IO_SIZE;
      if (size[k] < 0)
        st = BOPX_IO_READ;
      else if (h[k] > 0 && w[k] > 0)
        st = wk.pack(paths[k], size[k], h[k], w[k], dst + z_off[k], &zn);
      z_len[k] = st == BOPX_IO_OK ? (int32_t)zn : 0;
      status[k] = st;
      if (st) failed.fetch_add(1);
    }
  };
  if (nt == 1) {
    run();
  } else {
    std::vector<std::thread> pool;
    pool.reserve(nt - 1);
    for (int i = 1; i < nt; ++i) pool.emplace_back(run);
    run();
    for (auto& t : pool) t.join();
  }
  return failed.load();
}

extern "C" int bopx_io_backend(void) { return deflate_lib().ok ? 1 : 0; }
