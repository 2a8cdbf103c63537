// kern_png.hip — 16-bit depth PNG decode on the GPU: inflate (RFC 1950/1951)
// and row unfiltering (PNG spec 9.2-9.4) fused with the float32 depth_scale
// multiply. The input side of the VSD pass: the reference reads every test
// depth image with inout.load_depth (bop_toolkit_lib/inout.py:39-46, imageio)
// and scales it in float32 (scripts/eval_calc_errors.py:242-243); the host
// decoder (depth_png.cpp) does that in ~4 ms per 640x480 frame and core, most
// of it in the inflate. Here the host only parses chunks (CRC, IHDR) and packs
// the IDAT payloads; the frames are produced in HBM where k_vsd reads them.
//
// k_png_inflate: one wave per zlib stream. A deflate stream is sequential, so
// the wave decodes it with wave-uniform control (bit buffer, positions and
// table entries in SGPRs via readfirstlane) and uses its lanes where the work
// is parallel: building the Huffman tables, back-reference copies (64 bytes a
// round), flushing the output ring, and literal runs a 64-bit window at a time
// (lane l looks the table up at bit offset l; the chain of steps through the
// window is followed with v_readlane, long codes in the window are decoded
// lane-parallel). Per wave LDS: a 1024-entry literal/length table (32-bit
// entries: symbol << 4 | length, and the entry's chain step with a second
// literal), a 256-entry distance table (16-bit; longer codes take a canonical
// path from the per-length limits), the symbols sorted by code, the code
// lengths, and a 4 KB ring of the latest output. The input is read 1 KB at a
// time into four VGPRs per lane (v_readlane per 32 bits), so one load latency
// per KB of input is on the chain. The ring is flushed to HBM every 1 KB;
// distances beyond the ring read the flushed bytes back from L2. At the
// callers' batch sizes a launch lasts one stream's instruction stream, so the
// window's instruction count is what the kernel is tuned on.
//
// k_png_unfilter: one wave per frame, 64 rows in flight (lane = row), lane k
// working on pixel t - 2k at step t: the pixels a filter needs from the row
// above (up, up-left) were produced by lane k - 1 two and three steps earlier
// (a 4-pixel LDS ring per lane; the first row of a pass reads the last row of
// the previous pass from a carry row). Every filter type (None, Sub, Up,
// Average, Paeth) then runs at the same rate. The same pass computes the
// zlib Adler-32 of the inflated bytes.
//
// Acceptance matches the host decoder's strictest back end: a stream is
// accepted only if it is a valid zlib stream (header, complete Huffman codes
// or a single length-1 code, distances inside the output, exact output size,
// input not overrun, Adler-32), every filter byte is <= 4. Anything else gets
// status BOPX_PNG_CORRUPT and the caller decodes that file on the host, which
// reproduces the host path's own result or error.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bopx_internal.h"

namespace bopx {
namespace {

constexpr int kInfWaves = 4;  // streams per workgroup, one wave each
constexpr int kLitRoot = 10, kDistRoot = 8, kPreRoot = 7;
constexpr int kRing = 4096, kRingMask = kRing - 1;
constexpr int kFlush = 1024;       // bytes per ring flush (16 B per lane)
constexpr int kVmcnt0 = 0x0F70;    // s_waitcnt vmcnt(0) (expcnt / lgkmcnt not waited)
constexpr int kErr = 2;            // BOPX_PNG_CORRUPT
constexpr uint16_t kNoCode = 0xFFFF;  // table entry: code longer than the root, or none

__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct InfLds {
  // literal/length root table; high half: the entry's chain step (its bit
  // count, or kStop) and a second literal whose code fits in the same kLitRoot
  // bits (add_literal_steps). Also the code-length code's table (128 entries,
  // low halves only).
  uint32_t lit[1 << kLitRoot];
  uint16_t dist[1 << kDistRoot];
  uint16_t sorted[288 + 32];      // symbols by code: literal/length, then distance
  uint8_t lens[288 + 32];         // code lengths: literal/length, then distance
  alignas(16) uint8_t ring[kRing + 64];  // the latest kRing output bytes; a spare byte per lane
};

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int popc_lt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Huffman table of the n code lengths lens[0..n) (LDS), with the per-length
// quantities held lane-parallel (lane L = code length L, 1..15):
//   lim  = (first code + count) << (15 - L): left-justified end of the length's
//          codes (canonical codes of one length are consecutive, and the
//          lengths' ranges follow each other), so a code's length is the
//          smallest L with left-justified bits < lim[L];
//   base = index in `sorted` of the length's first symbol minus its first code.
// Writes tab (1 << ROOT entries: symbol << 4 | length, kNoCode = longer than
// ROOT or no code; so a literal with a short code is an entry < 256 << 4) and sorted (symbols in code order). Returns 0, 1 for an empty code
// (all lengths 0), or -1 for an over-subscribed code or an incomplete one
// other than a single length-1 code (zlib inftrees.c; libdeflate accepts the
// same codes).
template <int ROOT, class Tab>
__device__ int build_code(const uint8_t* lens, int n, Tab* tab, uint16_t* sorted, int& lim,
                          int& base, int lane) {
  const bool len_lane = lane >= 1 && lane <= 15;
  const int nch = (n + 63) >> 6;
  int cnt = 0;
  for (int ch = 0; ch < nch; ++ch) {
    const int s = ch * 64 + lane;
    const int l = s < n ? lens[s] : 0;
#pragma unroll 1
    for (int L = 1; L < 16; ++L) {
      const int c = __popcll(__ballot(l == L));
      if (lane == L) cnt += c;
    }
  }
  // Kraft sum in units of 2^-15 and symbol offsets: inclusive scans over lanes
  const int w = len_lane ? cnt << (15 - lane) : 0;
  int ws = w, cs = len_lane ? cnt : 0;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    const int tw = __shfl_up(ws, o, 64), tc = __shfl_up(cs, o, 64);
    if (lane >= o) {
      ws += tw;
      cs += tc;
    }
  }
  const int kraft = __builtin_amdgcn_readlane(ws, 15), total = __builtin_amdgcn_readlane(cs, 15);
  if (kraft > 32768) return -1;  // over-subscribed (every prefix then is too)
  if (total == 0) return 1;
  const uint64_t used = __ballot(len_lane && cnt > 0);
  if (kraft < 32768 && used != 2) return -1;  // incomplete, not a single length-1 code
  lim = ws;
  const int first = len_lane ? (ws - w) >> (15 - lane) : 0;
  const int offs = cs - cnt;
  base = offs - first;
  int run = offs;
  for (int ch = 0; ch < nch; ++ch) {
    const int s = ch * 64 + lane;
    const int l = s < n ? lens[s] : 0;
    int my = 0;
#pragma unroll 1
    for (int L = 1; L < 16; ++L) {
      const uint64_t m = __ballot(l == L);
      const int r = __builtin_amdgcn_readlane(run, L);
      if (l == L) my = r + popc_lt(m);
      if (lane == L) run += __popcll(m);
    }
    if (l) sorted[my] = (uint16_t)s;
  }
  wave_sync();
#pragma unroll 1
  for (int j = 0; j < (1 << ROOT) / 64; ++j) {
    const int e = j * 64 + lane;
    const int r15 = (int)(__builtin_bitreverse32((uint32_t)e) >> (32 - ROOT)) << (15 - ROOT);
    int idx = -1, len = 0;
#pragma unroll 1
    for (int L = ROOT; L >= 1; --L) {  // the smallest length whose range holds the bits
      const int lim_l = __builtin_amdgcn_readlane(lim, L);
      const int base_l = __builtin_amdgcn_readlane(base, L);
      if (r15 < lim_l) {
        idx = base_l + (r15 >> (15 - L));
        len = L;
      }
    }
    tab[e] = (Tab)(idx >= 0 ? (uint16_t)(sorted[idx] << 4 | len) : kNoCode);
  }
  wave_sync();
  return 0;
}

// A code longer than ROOT: the smallest length L > ROOT with the 15 bits
// (first bit most significant) below lim[L]; -1 if none (no such code).
// High half of the literal/length root table entries, for the window loop:
// bits 24-30 = the bits a chain step consumes (kStop: the entry is not a
// literal with a code of <= ROOT bits, the chain stops there), bit 31 = the
// step emits a second literal, bits 16-23 = that literal. Entry e (bits of
// the window, first bit lowest) whose code is a literal of length L1 leaves
// ROOT - L1 known bits; if they hold a whole literal code of length L2 (the
// table entry of those bits with the unknown high bits zero has L2 <= ROOT -
// L1: a code shorter than ROOT is replicated over every suffix), the step
// takes both (L1 + L2 bits). Depth rows are ~40 % 1-bit codes.
constexpr uint32_t kStop = 127;
template <int ROOT>
__device__ void add_literal_steps(uint32_t* tab, int lane) {
#pragma unroll 1
  for (int j = 0; j < (1 << ROOT) / 64; ++j) {
    const int e = j * 64 + lane;
    const uint32_t t = tab[e] & 0xFFFFu;
    uint32_t hi = kStop << 24;
    if (t < (256u << 4)) {  // a literal with a code of <= ROOT bits
      const int L1 = (int)(t & 15u);
      const uint32_t t2 = tab[e >> L1] & 0xFFFFu;
      hi = (uint32_t)L1 << 24;
      if (t2 < (256u << 4) && (int)(t2 & 15u) <= ROOT - L1)
        hi = 1u << 31 | (uint32_t)(L1 + (int)(t2 & 15u)) << 24 | (t2 >> 4) << 16;
    }
    wave_sync();  // every lane has read before any high half is written
    tab[e] = t | hi;
  }
  wave_sync();
}

template <int ROOT>
__device__ __forceinline__ int slow_index(uint64_t bb, int lim, int base, int lane, int& L) {
  const int r15 = (int)(__builtin_bitreverse32((uint32_t)bb) >> 17);
  const uint64_t m = __ballot(lane > ROOT && lane <= 15 && r15 < lim);
  if (m == 0) return -1;
  L = __builtin_ctzll(m);
  return __builtin_amdgcn_readlane(base, L) + (r15 >> (15 - L));
}

// Inflate one zlib stream (in, in_n bytes, 16-byte aligned, readable up to
// in_n + 2048) into out (out_n bytes exactly; writable up to round_up(out_n,
// 1024)). Returns 0 or kErr; *adler = the stream's Adler-32 field.
__device__ __forceinline__ int inflate_stream(const uint8_t* __restrict__ in, int in_n, uint8_t* __restrict__ out,
                              int out_n, InfLds& S, int lane, uint32_t* adler) {
  // input: 1 KB chunks, words [256 (seg >> 2), + 256) in four VGPRs, lane l
  // holding word 64 k + l of the chunk in component k (four coalesced dword
  // loads), read with v_readlane from `cw`, the component of the current 64
  // words (segment seg; a copy every 64 words instead of a four-way branch per
  // word). The next chunk is loaded when the current one is used up (one load
  // latency per KB of input; a prefetch into a loop-carried register makes the
  // compiler copy it, and the copy waits for the load anyway). The next word
  // is 64 seg + li. Reads past the stream are caught once per segment (the
  // readable padding is 2048 bytes) and exactly by the final check: a stream
  // whose bits end inside its bytes never loads a word past in_n + 8 (the bit
  // buffer holds <= 64 bits).
  const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
  const int in_chunks = (in_n + 2048) >> 10;  // 1 KB chunks inside the readable bytes
  uint32_t c0 = in32[lane], c1 = in32[64 + lane], c2 = in32[128 + lane], c3 = in32[192 + lane];
  uint32_t cw = c0;
  int seg = 0, li = 0;
  uint64_t bb = 0;
  int nb = 0;
  int p = 0, flushed = 0;
  int nfe = min(kFlush, out_n + 1);  // next flush point, or the first position past the frame

  // over: a segment past the stream was entered. Sticky, and checked where a
  // loop iteration makes no output (block headers, the slow symbol path) and
  // at the end, so the literal windows carry no exit for it.
  bool over = false;
  auto refill_word = [&]() __attribute__((always_inline)) -> bool {
    if (__builtin_expect(li == 64, 0)) {  // the next 64 words
      ++seg;
      li = 0;
      over |= seg * 256 > in_n + 8;  // past the stream
      const int sc = seg & 3;
      if (sc == 0) {
        const int ch = min(seg >> 2, max(in_chunks - 1, 0));
        const uint32_t* w32 = in32 + ch * 256;
        c0 = w32[lane];
        c1 = w32[64 + lane];
        c2 = w32[128 + lane];
        c3 = w32[192 + lane];
        cw = c0;
      } else {
        // values, not lvalues: a conditional over the captured variables would
        // select their addresses and put them in scratch
        const uint32_t v1 = c1, v2 = c2, v3 = c3;
        cw = sc == 1 ? v1 : (sc == 2 ? v2 : v3);
      }
    }
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)cw, li);
    bb |= (uint64_t)w << nb;
    nb += 32;
    ++li;
    return !over;
  };
  auto refill = [&]() __attribute__((always_inline)) -> bool {
    if (nb <= 32) refill_word();
    return !over;
  };
  auto flush_block = [&](int f) __attribute__((always_inline)) {
    wave_sync();
    const uint4 v = reinterpret_cast<const uint4*>(S.ring)[((f & kRingMask) >> 4) + lane];
    __builtin_amdgcn_s_waitcnt(kVmcnt0);  // earlier flushes have landed: far reads below see them
    reinterpret_cast<uint4*>(out)[(f >> 4) + lane] = v;
  };
  // one output byte (p - flushed < kFlush before and after)
  auto put = [&](int byte) __attribute__((always_inline)) {
    if (lane == 0) S.ring[p & kRingMask] = (uint8_t)byte;
    ++p;
    if ((p & (kFlush - 1)) == 0) {
      flush_block(flushed);
      flushed += kFlush;
      nfe = min(flushed + kFlush, out_n + 1);
    }
  };

  refill_word();
  {  // zlib header (RFC 1950 2.2): CM 8, CINFO <= 7, FCHECK, no preset dictionary
    const int cmf = (int)(bb & 255), flg = (int)((bb >> 8) & 255);
    if ((cmf & 15) != 8 || (cmf >> 4) > 7 || (cmf * 256 + flg) % 31 != 0 || (flg & 32)) return kErr;
    bb >>= 16;
    nb -= 16;
  }
  int lit_lim = 0, lit_base = 0, dist_lim = 0, dist_base = 0;  // lane L: length L (build_code)
  bool final = false;
  while (!final) {
    if (!refill()) return kErr;
    final = bb & 1;
    const int type = (int)((bb >> 1) & 3);
    bb >>= 3;
    nb -= 3;
    if (type == 0) {  // stored
      const int drop = nb & 7;
      bb >>= drop;
      nb -= drop;
      if (!refill()) return kErr;
      const int len = (int)(bb & 0xFFFF), nlen = (int)((bb >> 16) & 0xFFFF);
      bb >>= 32;
      nb -= 32;
      if (len != (~nlen & 0xFFFF) || len > out_n - p) return kErr;
      for (int k = 0; k < len; ++k) {
            if (nb < 8 && !refill_word()) return kErr;
        put((int)(bb & 255));
        bb >>= 8;
        nb -= 8;
      }
      continue;
    }
    if (type == 3) return kErr;
    int hlit = 288, hdist = 32;
    if (type == 1) {  // fixed codes (RFC 1951 3.2.6)
      for (int s = lane; s < 320; s += 64)
        S.lens[s] = s >= 288 ? 5 : s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
      wave_sync();
    } else {  // dynamic: the code-length code, then the two codes' lengths
      if (!refill()) return kErr;
      hlit = (int)(bb & 31) + 257;
      hdist = (int)((bb >> 5) & 31) + 1;
      const int hclen = (int)((bb >> 10) & 15) + 4;
      bb >>= 14;
      nb -= 14;
      if (hlit > 286 || hdist > 30) return kErr;
      if (lane < 19) S.lens[288 + lane] = 0;  // code-length code lengths live past the table
      wave_sync();
      for (int i = 0; i < hclen; ++i) {
            if (!refill()) return kErr;
        const int v = (int)(bb & 7);
        bb >>= 3;
        nb -= 3;
        if (lane == 0) S.lens[288 + c_clorder[i]] = (uint8_t)v;
      }
      wave_sync();
      int pre_lim, pre_base;
      if (build_code<kPreRoot>(S.lens + 288, 19, S.lit, S.sorted, pre_lim, pre_base, lane) != 0)
        return kErr;
      const int ntot = hlit + hdist;
      int k = 0, prev = -1;
      while (k < ntot) {
            if (!refill()) return kErr;
        const int e = uni((int)(S.lit[bb & ((1 << kPreRoot) - 1)] & 0xFFFFu));
        if (e == kNoCode) return kErr;  // every code-length code is <= 7 bits: no code
        const int sym = e >> 4;
        bb >>= e & 15;
        nb -= e & 15;
        int val, rep;
        if (sym < 16) {
          val = sym;
          rep = 1;
        } else if (sym == 16) {
          if (prev < 0) return kErr;
          val = prev;
          rep = 3 + (int)(bb & 3);
          bb >>= 2;
          nb -= 2;
        } else if (sym == 17) {
          val = 0;
          rep = 3 + (int)(bb & 7);
          bb >>= 3;
          nb -= 3;
        } else {
          val = 0;
          rep = 11 + (int)(bb & 127);
          bb >>= 7;
          nb -= 7;
        }
        if (rep > ntot - k) return kErr;
        // lengths k.. (literal/length codes at [0, hlit), distance codes at 288 +)
        for (int j = lane; j < rep; j += 64) {
          const int idx = k + j;
          S.lens[idx < hlit ? idx : 288 + idx - hlit] = (uint8_t)val;
        }
        k += rep;
        prev = val;
      }
      wave_sync();
      if (uni(S.lens[256]) == 0) return kErr;  // no end-of-block code
    }
    if (build_code<kLitRoot>(S.lens, hlit, S.lit, S.sorted, lit_lim, lit_base, lane) != 0)
      return kErr;
    add_literal_steps<kLitRoot>(S.lit, lane);
    const int dst =
        build_code<kDistRoot>(S.lens + 288, hdist, S.dist, S.sorted + 288, dist_lim, dist_base, lane);
    if (dst < 0) return kErr;
    const bool no_dist = dst == 1;

    // errors leave the symbol loop by the same exit as the end-of-block code
    // (one exit besides the back edges: no per-window exit dispatch)
    bool err = false;
    for (;;) {  // symbols of this block
      // Literal runs, a bit-buffer window at a time: lane l looks the table up
      // at bit offset l (one LDS gather), the chain of short literal codes
      // through the window is followed with v_readlane (no LDS round trip per
      // symbol), and the lanes on the chain store their bytes at once. A step
      // is taken while its code(s) end inside the buffer's nb valid bits: the
      // bits above nb are zero, and a code that reaches past them cannot match
      // a shorter entry (prefix-free), so its entry's step ends past nb too.
      if (nb <= 32) {  // to nb in (32, 64]; a read past the stream is caught below
        refill_word();
        if (nb <= 32) refill_word();
      }
      const int lim = min(nb, 63);  // chain offsets stay lane indices
      const uint32_t bits = (uint32_t)(bb >> lane);
      uint32_t ev = S.lit[bits & ((1 << kLitRoot) - 1)];
      int off = 0;
      uint64_t run = 0;  // bit l: a chain step (one or two literals) starts at offset l
      // lane l: the offset after the step that starts at l (> 63 at a stop),
      // so a chain step is one v_readlane and one compare
      int jv = lane + (int)((ev >> 24) & kStop);
      for (int nxt = __builtin_amdgcn_readlane(jv, 0); nxt <= lim;
           nxt = __builtin_amdgcn_readlane(jv, off)) {
        asm("s_bitset1_b64 %0, %1" : "+s"(run) : "s"(off));  // run |= 1 << off, one instruction
        off = nxt;
      }
      int e = __builtin_amdgcn_readlane((int)ev, off);
      if (__builtin_expect((e & 0xFFFF) == (int)kNoCode, 0) && off + 15 <= nb) {
        // The chain stopped at a code longer than the root: decode the long
        // codes at every offset with 15 valid bits lane-parallel (canonical,
        // from the per-length limits of lanes 11-15, then `sorted`), make the
        // literals among them chain steps, and follow the chain on.
        const int m11 = __builtin_amdgcn_readlane(lit_lim, 11), m12 = __builtin_amdgcn_readlane(lit_lim, 12),
                  m13 = __builtin_amdgcn_readlane(lit_lim, 13), m14 = __builtin_amdgcn_readlane(lit_lim, 14),
                  m15 = __builtin_amdgcn_readlane(lit_lim, 15);
        const int b11 = __builtin_amdgcn_readlane(lit_base, 11), b12 = __builtin_amdgcn_readlane(lit_base, 12),
                  b13 = __builtin_amdgcn_readlane(lit_base, 13), b14 = __builtin_amdgcn_readlane(lit_base, 14),
                  b15 = __builtin_amdgcn_readlane(lit_base, 15);
        const int r15 = (int)(__builtin_bitreverse32(bits) >> 17);
        const int L = 11 + (r15 >= m11) + (r15 >= m12) + (r15 >= m13) + (r15 >= m14) + (r15 >= m15);
        const int bs = L <= 12 ? (L == 11 ? b11 : b12) : L <= 14 ? (L == 13 ? b13 : b14) : b15;
        const bool cand = (ev & 0xFFFFu) == kNoCode && lane + 15 <= nb && L <= 15;
        const int sym = S.sorted[cand ? bs + (r15 >> (15 - L)) : 0];
        if (cand && sym < 256) {
          ev = (uint32_t)L << 24 | (uint32_t)sym << 4 | (uint32_t)L;
          jv = lane + L;
        }
        for (int nxt = __builtin_amdgcn_readlane(jv, off); nxt <= lim;
             nxt = __builtin_amdgcn_readlane(jv, off)) {
          asm("s_bitset1_b64 %0, %1" : "+s"(run) : "s"(off));
          off = nxt;
        }
        e = __builtin_amdgcn_readlane((int)ev, off);
      }
      if (run) {
        // chain steps with two literals (entries with bit 31 set, on the chain)
        const uint64_t run2 = run & __builtin_amdgcn_ballot_w64((int)ev < 0);
        const int nlit = __popcll(run) + __popcll(run2);
        bb >>= off;  // off <= 63
        nb -= off;
        // every lane stores (no exec mask to set up): the lanes off the chain,
        // and the second byte of one-literal steps, into the lane's spare byte;
        // the step masks pick the address per lane as v_cndmask conditions
        const int q = p + popc_lt(run) + popc_lt(run2);
        const uint32_t spare = (uint32_t)(kRing + lane);
        uint32_t a1, a2;
        asm("v_cndmask_b32_e64 %0, %1, %2, %3"
            : "=v"(a1) : "v"(spare), "v"((uint32_t)(q & kRingMask)), "s"(run));
        asm("v_cndmask_b32_e64 %0, %1, %2, %3"
            : "=v"(a2) : "v"(spare), "v"((uint32_t)((q + 1) & kRingMask)), "s"(run2));
        S.ring[a1] = (uint8_t)(ev >> 4);
        S.ring[a2] = (uint8_t)(ev >> 16);
        p += nlit;
        if (p >= nfe) {  // a flush is due, or the output ran past the frame (one compare)
          if (p > out_n) { err = true; break; }
          do {
            flush_block(flushed);
            flushed += kFlush;
          } while (p - flushed >= kFlush);
          nfe = min(flushed + kFlush, out_n + 1);
        }
      }
      if (((e >> 24) & (int)kStop) != (int)kStop) continue;  // a literal past the window
      // a long code too close to the window's end: the next window starts at it
      // (one with 15 valid bits is a length / end-of-block code or none)
      if ((e & 0xFFFF) == (int)kNoCode && off + 15 > nb) continue;
      // not a literal with a short code: its entry again, from valid bits (a
      // long code plus length extra bits need up to 20)
      if (nb <= 32) refill_word();
      if (over) { err = true; break; }
      e = uni((int)(S.lit[(uint32_t)bb & ((1 << kLitRoot) - 1)] & 0xFFFFu));
      int L = e & 15, sym = e >> 4;
      if (e == kNoCode) {
        const int idx = slow_index<kLitRoot>(bb, lit_lim, lit_base, lane, L);
        if (idx < 0) { err = true; break; }
        sym = uni(S.sorted[idx]);
      }
      bb >>= L;
      nb -= L;
      if (sym < 256) {
        if (p >= out_n) { err = true; break; }
        put(sym);
        continue;
      }
      if (sym == 256) break;
      if (sym > 285 || no_dist) { err = true; break; }
      // length: base and extra bits of RFC 1951 3.2.5 in closed form
      const int ls = sym - 257;
      const int lx = ls < 8 || ls == 28 ? 0 : (ls >> 2) - 1;
      const int lbase = ls < 8 ? ls + 3 : ls == 28 ? 258 : ((4 + (ls & 3)) << lx) + 3;
      const int len = lbase + (int)(bb & ((1u << lx) - 1));
      bb >>= lx;
      nb -= lx;
      if (!refill()) { err = true; break; }
      e = uni(S.dist[bb & ((1 << kDistRoot) - 1)]);
      L = e & 15;
      int ds = e >> 4;
      if (e == kNoCode) {
        const int idx = slow_index<kDistRoot>(bb, dist_lim, dist_base, lane, L);
        if (idx < 0) { err = true; break; }
        ds = uni(S.sorted[288 + idx]);
      }
      bb >>= L;
      nb -= L;
      if (ds >= 30) { err = true; break; }
      const int dx = ds < 4 ? 0 : (ds >> 1) - 1;
      const int dbase = ds < 4 ? ds + 1 : ((2 + (ds & 1)) << dx) + 1;
      const int dist = dbase + (int)(bb & ((1u << dx) - 1));
      bb >>= dx;
      nb -= dx;
      if (dist > p || len > out_n - p) { err = true; break; }
      // copy: byte i of the match = out[p - dist + i % dist]; sources all lie
      // before p, so each 64-byte round reads, then writes. Rounds before r0
      // wrote ring slots p .. p + r0 - 1, which hold the sources q with
      // kRing - r0 < p - q <= kRing: those are read from the flushed output
      // (p - q > kRing - 256 lies more than two flushes back).
      const bool overlap = dist < len;
      // i / dist for the overlapping case, from the hardware reciprocal: the
      // quotient estimate below is then within one of floor(i / dist) (i < 322,
      // relative error < 2^-22), which the two fix-ups correct
      const float rd = __builtin_amdgcn_rcpf((float)dist);
      for (int r0 = 0; r0 < len; r0 += 64) {
        const int i = r0 + lane;
        int j = i;
        if (overlap) {
          j = i - (int)((float)i * rd) * dist;
          if (j >= dist) j -= dist;
          if (j < 0) j += dist;
        }
        const int q = p - dist + j;
        int b = 0;
        if (i < len) {
          if (dist - j <= kRing - r0) {
            b = S.ring[q & kRingMask];
          } else {  // flushed at least one flush before the last (see flush_block)
            const uint32_t w = __hip_atomic_load(
                reinterpret_cast<uint32_t*>(out + (q & ~3)), __ATOMIC_RELAXED,
                __HIP_MEMORY_SCOPE_AGENT);
            b = (int)((w >> ((q & 3) * 8)) & 255);
          }
        }
        wave_sync();
        if (i < len) S.ring[(p + i) & kRingMask] = (uint8_t)b;
      }
      p += len;
      while (p - flushed >= kFlush) {
        flush_block(flushed);
        flushed += kFlush;
      }
      nfe = min(flushed + kFlush, out_n + 1);
    }
    if (err) return kErr;
  }
  if (p != out_n) return kErr;
  if (p > flushed) flush_block(flushed);  // the tail (the buffer is padded to 1 KB)
  {
    const int drop = nb & 7;
    bb >>= drop;
    nb -= drop;
    if (!refill()) return kErr;
    *adler = __builtin_bswap32((uint32_t)bb);
    nb -= 32;
    if (over || (64 * seg + li) * 4 - nb / 8 > in_n) return kErr;  // the stream ran past its bytes
  }
  return 0;
}

__global__ __launch_bounds__(64 * kInfWaves) void k_png_inflate(
    const uint8_t* __restrict__ zdata, const int64_t* __restrict__ z_off,
    const int32_t* __restrict__ z_len, int64_t n, int out_n, int64_t raw_stride,
    uint8_t* __restrict__ raw, int32_t* __restrict__ status) {
  __shared__ InfLds s_inf[kInfWaves];
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const int64_t k = (int64_t)blockIdx.x * kInfWaves + wave;
  if (k >= n) return;
  const int64_t off = z_off[k];
  const int len = z_len[k];
  uint32_t adler = 0;
  int st = kErr;
  if ((off & 255) == 0 && len >= 7)
    st = inflate_stream(zdata + off, len, raw + k * raw_stride, out_n, s_inf[wave], lane, &adler);
  if (lane == 0) {
    status[2 * k] = st;
    status[2 * k + 1] = (int32_t)adler;
  }
}

constexpr int kUnfWaves = 4;

__device__ __forceinline__ uint32_t unfilter_byte(int f, uint32_t x, uint32_t a, uint32_t b,
                                                  uint32_t c) {
  switch (f) {
    case 1:
      return (x + a) & 255;
    case 2:
      return (x + b) & 255;
    case 3:
      return (x + ((a + b) >> 1)) & 255;
    case 4: {
      const int pp = (int)a + (int)b - (int)c;
      const int pa = abs(pp - (int)a), pb = abs(pp - (int)b), pc = abs(pp - (int)c);
      return (x + (pa <= pb && pa <= pc ? a : pb <= pc ? b : c)) & 255;
    }
    default:
      return x;
  }
}

__global__ __launch_bounds__(64 * kUnfWaves) void k_png_unfilter(
    const uint8_t* __restrict__ raw, int64_t raw_stride, int64_t n, int H, int W,
    const float* __restrict__ scales, float* __restrict__ frames, int32_t* __restrict__ status) {
  __shared__ uint16_t s_carry[kUnfWaves][kPngMaxWidth];
  __shared__ uint16_t s_slot[kUnfWaves][64][4];
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const int64_t k = (int64_t)blockIdx.x * kUnfWaves + wave;
  if (k >= n) return;
  if (uni(status[2 * k]) != 0) return;
  const uint8_t* fr = raw + k * raw_stride;
  const uint32_t* fr32 = reinterpret_cast<const uint32_t*>(fr);
  const int64_t last_word = raw_stride / 4 - 5;  // a group's 5 words stay inside the frame
  const int rowb = 2 * W + 1;
  const uint64_t N = (uint64_t)H * rowb;
  const float scale = scales ? scales[k] : 1.0f;
  float* out = frames + k * (int64_t)H * W;
  uint16_t* carry = s_carry[wave];
  uint16_t(*slot)[4] = s_slot[wave];
  uint64_t A = 0, B = 0;
  bool bad = false;
  // a 16-bit pixel hi << 8 | lo as the pair hi << 16 | lo (and the raw pair
  // x = lo << 8 | hi alike), so both bytes of a step are filtered at once
  auto wide = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0C010C00u); };   // lo, 0, hi, 0
  auto wide_raw = [](uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0C000C01u); };  // hi, 0, lo, 0 from x
  auto narrow = [](uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0C0C0200u); };   // hi << 8 | lo
  for (int r0 = 0; r0 < H; r0 += 64) {
    const int row = r0 + lane;
    const bool act = row < H;
    const int64_t rb = (int64_t)(act ? row : H - 1) * rowb;
    int f = 0;
    if (act) {
      f = fr[rb];
      A += f;
      B += (N - rb) * f;
      bad |= f > 4;
    }
    // the filter types present in the pass (wave-uniform): a step computes
    // only those, and Paeth (rare in depth images) per byte
    const bool has1 = __any(f == 1), has2 = __any(f == 2), has3 = __any(f == 3),
               has4 = __any(f == 4);
    // lane k works on pixel c = t - 2k at step t; steps go in groups of 8, whose
    // 16 bytes start at rb + 1 + 16 g - 4 k (the same alignment for every group)
    const int64_t g0 = rb + 1 - 4 * lane;
    const int sh = (int)(g0 & 3);
    const int64_t d0 = (g0 - sh) >> 2;
    // (each word index clamped on its own: with 1-pixel rows (3 bytes) the
    // window of a lane's first groups starts before the frame, and clamping
    // the window would shift its alignment; the words before the frame only
    // feed steps with c < 0)
    auto load = [&](uint32_t(&w)[5], int g) {
      const int64_t d = min(d0 + 4 * (int64_t)g, last_word);
#pragma unroll
      for (int i = 0; i < 5; ++i) w[i] = fr32[max(d + i, (int64_t)0)];
    };
    uint32_t left = 0, upl = 0;  // this row's previous pixel, the row above's previous pixel
    // Adler-32 of the row's bytes: their sum and sum of (byte index in the row) x
    // byte, 32-bit within a group of 8 steps, 64-bit per group
    uint32_t rowA = 0;
    uint64_t rowS = 0;
    float* orow = out + (int64_t)(act ? row : 0) * W;
    auto group = [&](const uint32_t(&w)[5], int g) {
      uint32_t pl[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) pl[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
      const int c0 = 8 * g - 2 * lane;
      float fv[8];
      uint32_t gA = 0, gS = 0, gL = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t x = (pl[u >> 1] >> (16 * (u & 1))) & 0xFFFFu;
        const int c = c0 + u;
        const bool valid = act && c >= 0 && c < W;
        if (valid) {
          const uint32_t up = row == 0 ? 0u : lane == 0 ? carry[c] : slot[lane - 1][c & 3];
          const uint32_t wx = wide_raw(x), wa = wide(left), wb = wide(up);
          uint32_t r = wx;
          if (has1 && f == 1) r = wx + wa;
          if (has2 && f == 2) r = wx + wb;
          if (has3 && f == 3) r = wx + ((wa + wb) >> 1);
          uint32_t px = narrow(r & 0x00FF00FFu);
          if (has4 && f == 4) {
            const uint32_t xh = x & 255, xl = x >> 8;
            px = unfilter_byte(4, xh, left >> 8, up >> 8, upl >> 8) << 8 |
                 unfilter_byte(4, xl, left & 255, up & 255, upl & 255);
          }
          slot[lane][c & 3] = (uint16_t)px;
          if (lane == 63) carry[c] = (uint16_t)px;
          fv[u] = (float)px * scale;
          const uint32_t xh = x & 255, xl = x >> 8, sb = xh + xl;
          gA += sb;
          gS += (uint32_t)c * sb;  // byte 2c is xh, 2c + 1 is xl: 2 c (xh + xl) + xl
          gL += xl;
          left = px;
          upl = up;
        }
        wave_sync();
      }
      rowA += gA;
      rowS += 2 * (uint64_t)gS + gL;
      if (act && c0 >= 0 && c0 + 7 < W && (W & 1) == 0) {  // 8 pixels: four aligned 8-byte stores
        float2* o2 = reinterpret_cast<float2*>(orow + c0);
#pragma unroll
        for (int i = 0; i < 4; ++i) o2[i] = make_float2(fv[2 * i], fv[2 * i + 1]);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (act && c0 + u >= 0 && c0 + u < W) orow[c0 + u] = fv[u];
      }
    };
    const int nsteps = W + 2 * min(63, H - 1 - r0);
    const int ng = (nsteps + 7) >> 3;
    uint32_t wa[5], wb[5];  // groups in flight: even groups in wa, odd ones in wb
    load(wa, 0);
    for (int g = 0; g < ng; g += 2) {
      load(wb, g + 1);
      group(wa, g);
      if (g + 1 >= ng) break;
      load(wa, g + 2);
      group(wb, g + 1);
    }
    if (act) {  // byte j of the row is byte rb + 1 + j of the stream
      A += rowA;
      B += (N - (uint64_t)rb - 1) * rowA - rowS;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    A += __shfl_xor((unsigned long long)A, o, 64);
    B += __shfl_xor((unsigned long long)B, o, 64);
  }
  const uint32_t a = (uint32_t)((1 + A) % 65521u), b = (uint32_t)((N + B) % 65521u);
  const bool ok = !__any(bad) && (b << 16 | a) == (uint32_t)status[2 * k + 1];
  if (lane == 0 && !ok) status[2 * k] = kErr;
}

}  // namespace

hipError_t launch_png_decode(int64_t n, const uint8_t* zdata, const int64_t* z_off,
                             const int32_t* z_len, int H, int W, const float* scales, uint8_t* raw,
                             int64_t raw_stride, float* frames, int32_t* status, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int out_n = H * (2 * W + 1);
  const unsigned gi = (unsigned)((n + kInfWaves - 1) / kInfWaves);
  hipLaunchKernelGGL(k_png_inflate, dim3(gi), dim3(64 * kInfWaves), 0, s, zdata, z_off, z_len, n,
                     out_n, raw_stride, raw, status);
  if (hipError_t e = hipGetLastError()) return e;
  const unsigned gu = (unsigned)((n + kUnfWaves - 1) / kUnfWaves);
  hipLaunchKernelGGL(k_png_unfilter, dim3(gu), dim3(64 * kUnfWaves), 0, s, raw, raw_stride, n, H,
                     W, scales, frames, status);
  return hipGetLastError();
}

hipError_t preload_png_kernels() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_png_inflate));
}

}  // namespace bopx
