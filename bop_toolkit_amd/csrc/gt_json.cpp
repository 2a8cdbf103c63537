// Per-image instance lists of a BOP scene (scene_gt.json, scene_gt_info.json)
// into arrays, behind include/bopx_io.h (bopx_gt_lists_open / _take).
//
// The evaluation reads every scene's scene_gt.json (inout.load_scene_gt,
// bop_toolkit_lib/inout.py:182-198: json.load with integer image keys, then
// cam_R_m2c / cam_t_m2c as float64 arrays) for its error passes
// (scripts/eval_calc_errors.py:232-236) and, with scene_gt_info.json, for the
// scorer's GT table (scripts/eval_calc_scores.py:183-214). In Python that is
// ~40-50 ms per 8k-instance scene, under the GIL, on the thread that prepares
// the next scene while the error kernels of the current one are launched and
// saved on the main thread: the two serialise. Here one pass over the file,
// without the GIL, fills the fields the callers read.
//
// Only a strict form is taken: a JSON object whose keys are decimal integers
// (-? d+, at most 18 digits, no two equal) and whose values are arrays of
// objects; in every object each requested field appears once, as a number
// (width 1) or a flat array of exactly `width` numbers; other members may be
// any JSON value and are skipped. Numbers follow JSON's grammar and convert as
// Python's json module converts them and NumPy then stores them as float64
// (int(...) then float64, or float(...): both round the decimal value to
// nearest). Anything else (NaN / Infinity literals, escaped keys, duplicate
// keys or fields, another structure, malformed text) is declined and the
// caller parses the file with Python's json, which accepts what Python accepts
// or raises what the reference raises.
#include <sys/stat.h>

#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bopx_io.h"

namespace {

struct Lists {
  std::vector<int64_t> im, off;
  std::vector<std::vector<double>> vals;
};

struct Parser {
  const char* p;
  const char* e;
  int depth = 0;

  static bool digit(char c) { return c >= '0' && c <= '9'; }

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < e && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
  bool peek(char c) {
    ws();
    return p < e && *p == c;
  }
  // a string without escapes (keys): [s, se)
  bool key(const char*& s, const char*& se) {
    ws();
    if (p >= e || *p != '"') return false;
    s = ++p;
    while (p < e && *p != '"') {
      if (*p == '\\' || (unsigned char)*p < 0x20) return false;
      ++p;
    }
    if (p >= e) return false;
    se = p++;
    return true;
  }
  static bool hex(char c) {
    return digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
  }
  // a string member value that is skipped: JSON's escapes only (\" \\ \/ \b
  // \f \n \r \t \uXXXX), as Python's json accepts them; anything else is
  // declined (json raises on it). ADVICE r5.
  bool skip_string() {
    if (p >= e || *p != '"') return false;
    ++p;
    while (p < e && *p != '"') {
      if ((unsigned char)*p < 0x20) return false;
      if (*p == '\\') {
        if (++p >= e) return false;
        const char c = *p;
        if (c == 'u') {
          if (e - p < 5 || !hex(p[1]) || !hex(p[2]) || !hex(p[3]) || !hex(p[4])) return false;
          p += 4;
        } else if (!std::strchr("\"\\/bfnrt", c) || c == 0) {
          return false;
        }
      }
      ++p;
    }
    if (p >= e) return false;
    ++p;
    return true;
  }
  // JSON number: -?(0|[1-9]d*)(.d+)?([eE][+-]?d+)?
  bool number(double* out) {
    ws();
    const char* s = p;
    if (p < e && *p == '-') ++p;
    if (p >= e || !digit(*p)) return false;
    if (*p == '0') {
      ++p;
    } else {
      while (p < e && digit(*p)) ++p;
    }
    if (p < e && *p == '.') {
      ++p;
      if (p >= e || !digit(*p)) return false;
      while (p < e && digit(*p)) ++p;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (p >= e || !digit(*p)) return false;
      while (p < e && digit(*p)) ++p;
    }
    if (p < e && digit(*p)) return false;  // "01": Python's json stops after "0"
    if (!out) return true;
    const auto r = std::from_chars(s, p, *out);
    if (r.ec == std::errc() && r.ptr == p) return true;
    // out of range: strtod's inf / 0 / subnormal, as float() gives
    std::string buf(s, p);
    *out = std::strtod(buf.c_str(), nullptr);
    return true;
  }
  bool literal(const char* w) {
    const size_t n = std::strlen(w);
    if ((size_t)(e - p) < n || std::memcmp(p, w, n) != 0) return false;
    p += n;
    return true;
  }
  bool skip_value() {
    ws();
    if (p >= e) return false;
    const char c = *p;
    if (c == '"') return skip_string();
    if (c == '{' || c == '[') {
      if (++depth > 256) return false;
      const char close = c == '{' ? '}' : ']';
      ++p;
      if (eat(close)) {
        --depth;
        return true;
      }
      do {
        if (c == '{') {
          const char *s, *se;
          if (!key(s, se) || !eat(':')) return false;
        }
        if (!skip_value()) return false;
      } while (eat(','));
      if (!eat(close)) return false;
      --depth;
      return true;
    }
    if (c == 't') return literal("true");
    if (c == 'f') return literal("false");
    if (c == 'n') return literal("null");
    return number(nullptr);  // NaN / Infinity: declined here
  }
  // image key: -? d+ (at most 18 digits), Python's int(k) for the keys the
  // loader's hook converts
  static bool int_key(const char* s, const char* se, int64_t* v) {
    bool neg = false;
    if (s < se && *s == '-') {
      neg = true;
      ++s;
    }
    if (s == se || se - s > 18) return false;
    int64_t x = 0;
    for (; s < se; ++s) {
      if (!digit(*s)) return false;
      x = x * 10 + (*s - '0');
    }
    *v = neg ? -x : x;
    return true;
  }
};

// Well-formed UTF-8 (RFC 3629: shortest form, no surrogates, <= U+10FFFF):
// the reference opens the file as text (inout.py:66-82), so other bytes raise
// UnicodeDecodeError there; such a file is declined and Python raises it.
bool utf8_ok(const unsigned char* s, const unsigned char* e) {
  while (s < e) {
    const unsigned c = *s;
    if (c < 0x80) {
      ++s;
      continue;
    }
    int n;
    unsigned lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) {
      n = 1;
    } else if (c >= 0xE0 && c <= 0xEF) {
      n = 2;
      if (c == 0xE0) lo = 0xA0;
      if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      n = 3;
      if (c == 0xF0) lo = 0x90;
      if (c == 0xF4) hi = 0x8F;
    } else {
      return false;
    }
    if (e - s <= n) return false;
    if (s[1] < lo || s[1] > hi) return false;
    for (int k = 2; k <= n; ++k)
      if (s[k] < 0x80 || s[k] > 0xBF) return false;
    s += n + 1;
  }
  return true;
}

bool parse(const char* data, size_t n, int nf, const char* const* names, const int* widths,
           Lists& L) {
  if (!utf8_ok((const unsigned char*)data, (const unsigned char*)data + n)) return false;
  Parser P{data, data + n};
  std::vector<size_t> name_len(nf);
  for (int f = 0; f < nf; ++f) name_len[f] = std::strlen(names[f]);
  L.vals.assign(nf, {});
  L.off.push_back(0);
  std::vector<char> seen(nf);
  std::vector<double> tmp;
  if (!P.eat('{')) return false;
  if (!P.eat('}')) {
    do {
      const char *ks, *ke;
      int64_t im;
      if (!P.key(ks, ke) || !Parser::int_key(ks, ke, &im) || !P.eat(':')) return false;
      L.im.push_back(im);
      if (!P.eat('[')) return false;
      if (!P.eat(']')) {
        do {
          if (!P.eat('{')) return false;
          std::fill(seen.begin(), seen.end(), 0);
          if (!P.eat('}')) {
            do {
              const char *s, *se;
              if (!P.key(s, se) || !P.eat(':')) return false;
              int f = 0;
              for (; f < nf; ++f)
                if ((size_t)(se - s) == name_len[f] && std::memcmp(s, names[f], name_len[f]) == 0)
                  break;
              if (f == nf) {
                if (!P.skip_value()) return false;
                continue;
              }
              if (seen[f]) return false;  // a repeated field: Python keeps the last
              seen[f] = 1;
              std::vector<double>& v = L.vals[f];
              if (widths[f] == 1) {
                double x;
                if (P.peek('[') || !P.number(&x)) return false;
                v.push_back(x);
              } else {
                if (!P.eat('[')) return false;
                for (int k = 0; k < widths[f]; ++k) {
                  double x;
                  if ((k > 0 && !P.eat(',')) || !P.number(&x)) return false;
                  v.push_back(x);
                }
                if (!P.eat(']')) return false;
              }
            } while (P.eat(','));
            if (!P.eat('}')) return false;
          }
          for (int f = 0; f < nf; ++f)
            if (!seen[f]) return false;
        } while (P.eat(','));
        if (!P.eat(']')) return false;
      }
      L.off.push_back((int64_t)(L.vals.empty() ? 0 : L.vals[0].size() / widths[0]));
    } while (P.eat(','));
    if (!P.eat('}')) return false;
  }
  P.ws();
  if (P.p != P.e) return false;
  std::vector<int64_t> s = L.im;  // duplicate image keys: Python keeps the last list
  std::sort(s.begin(), s.end());
  return std::adjacent_find(s.begin(), s.end()) == s.end();
}

}  // namespace

extern "C" void* bopx_gt_lists_open(const char* path, int n_fields, const char* const* names,
                                    const int* widths, int64_t* n_im, int64_t* n_rec,
                                    int* status) {
  *status = BOPX_RES_OTHER;
  if (n_fields < 1 || n_fields > 16) return nullptr;
  for (int f = 0; f < n_fields; ++f)
    if (!names[f] || widths[f] < 1 || widths[f] > 64) return nullptr;
  FILE* fp = std::fopen(path, "rb");
  if (!fp) {
    *status = BOPX_RES_READ;
    return nullptr;
  }
  std::vector<char> buf;
  struct stat sb;
  bool ok = fstat(fileno(fp), &sb) == 0 && sb.st_size >= 0;
  if (ok) {
    buf.resize((size_t)sb.st_size);
    ok = std::fread(buf.data(), 1, buf.size(), fp) == buf.size() && std::fgetc(fp) == EOF;
  }
  std::fclose(fp);
  if (!ok) {
    *status = BOPX_RES_READ;
    return nullptr;
  }
  Lists* L = new Lists;
  if (!parse(buf.data(), buf.size(), n_fields, names, widths, *L)) {
    delete L;
    return nullptr;
  }
  *n_im = (int64_t)L->im.size();
  *n_rec = L->off.back();
  *status = 0;
  return L;
}

extern "C" void bopx_gt_lists_take(void* h, int64_t* im_ids, int64_t* off, double* const* vals) {
  Lists* L = static_cast<Lists*>(h);
  if (!L) return;
  if (im_ids && off && vals) {
    std::copy(L->im.begin(), L->im.end(), im_ids);
    std::copy(L->off.begin(), L->off.end(), off);
    for (size_t f = 0; f < L->vals.size(); ++f)
      std::copy(L->vals[f].begin(), L->vals[f].end(), vals[f]);
  }
  delete L;
}
