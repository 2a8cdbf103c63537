// BOP19 results CSV reader behind include/bopx_io.h (bopx_read_bop_results).
//
// The evaluation parses the whole results file once (inout.load_bop_results,
// bop_toolkit_lib/inout.py:221-261): per line int() of the three ids, float()
// of the score, the 9 R and 3 t numbers and the time. In Python that is ~0.6 s
// for 100k estimates. Here one pass over the file fills arrays; every number
// goes through std::from_chars (strtod when out of range), which round exactly
// as Python's float() for the decimal forms accepted below.
//
// Only a strict form is taken: '\n' line ends (no '\r'), an optional header
// first line, 7 comma-separated fields, ' ' / '\t' as the only blanks, decimal
// integers and decimal floating-point numbers (no inf / nan / underscores /
// hex), R with 9 numbers and t with 3. Anything else returns BOPX_RES_OTHER and
// the caller reads the file with the Python reader, which accepts what Python
// accepts or raises the reference's error for the first bad line.
#include <sys/stat.h>

#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/bopx_io.h"

namespace {

bool blank(char c) { return c == ' ' || c == '\t'; }
bool digit(char c) { return c >= '0' && c <= '9'; }

// [p, e) with surrounding blanks removed
void trim(const char*& p, const char*& e) {
  while (p < e && blank(*p)) ++p;
  while (e > p && blank(e[-1])) --e;
}

// decimal float: [+-]? (d+ (. d*)? | . d+) ([eE] [+-]? d+)?
bool parse_float(const char* p, const char* e, double* out) {
  const char* s = p;
  if (s < e && (*s == '+' || *s == '-')) ++s;
  int nd = 0;
  while (s < e && digit(*s)) ++s, ++nd;
  if (s < e && *s == '.') {
    ++s;
    while (s < e && digit(*s)) ++s, ++nd;
  }
  if (nd == 0) return false;
  if (s < e && (*s == 'e' || *s == 'E')) {
    ++s;
    if (s < e && (*s == '+' || *s == '-')) ++s;
    int ne = 0;
    while (s < e && digit(*s)) ++s, ++ne;
    if (ne == 0) return false;
  }
  if (s != e || e - p > 350) return false;
  // std::from_chars rounds to nearest like float(); out of range (and anything
  // it does not consume whole) goes through strtod, whose inf / 0 / subnormal
  // results are float()'s too
  const auto r = std::from_chars(*p == '+' ? p + 1 : p, e, *out);
  if (r.ec == std::errc() && r.ptr == e) return true;
  char buf[352];
  std::memcpy(buf, p, (size_t)(e - p));
  buf[e - p] = 0;
  *out = std::strtod(buf, nullptr);
  return true;
}

// decimal integer: [+-]? d+, at most 18 digits
bool parse_int(const char* p, const char* e, int64_t* out) {
  const char* s = p;
  bool neg = false;
  if (s < e && (*s == '+' || *s == '-')) neg = *s++ == '-';
  if (s == e || e - s > 18) return false;
  int64_t v = 0;
  for (; s < e; ++s) {
    if (!digit(*s)) return false;
    v = v * 10 + (*s - '0');
  }
  *out = neg ? -v : v;
  return true;
}

// exactly n blank-separated floats in [p, e)
bool parse_floats(const char* p, const char* e, int n, double* out) {
  int k = 0;
  while (true) {
    while (p < e && blank(*p)) ++p;
    if (p == e) break;
    const char* q = p;
    while (q < e && !blank(*q)) ++q;
    if (k == n || !parse_float(p, q, out + k)) return false;
    ++k;
    p = q;
  }
  return k == n;
}

}  // namespace

extern "C" int64_t bopx_read_bop_results(const char* path, int64_t cap, int64_t* ids,
                                         double* score, double* R, double* t, double* time,
                                         int64_t* need) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return BOPX_RES_READ;
  std::vector<char> buf;
  struct stat sb;
  bool ok = fstat(fileno(f), &sb) == 0 && sb.st_size >= 0;
  if (ok) {
    buf.resize((size_t)sb.st_size);
    ok = std::fread(buf.data(), 1, buf.size(), f) == buf.size() && std::fgetc(f) == EOF;
  }
  std::fclose(f);
  if (!ok) return BOPX_RES_READ;
  for (char ch : buf)  // '\r' line ends and non-ASCII text: the Python reader
    if (ch == '\r' || (unsigned char)ch >= 0x80) return BOPX_RES_OTHER;
  static const char kHeader[] = "scene_id,im_id,obj_id,score,R,t,time";
  const char* p = buf.data();
  const char* end = p + buf.size();
  // lines as Python iterates them: split after each '\n', no empty last line
  std::vector<std::pair<const char*, const char*>> lines;
  while (p < end) {
    const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
    const char* le = nl ? nl : end;
    lines.emplace_back(p, le);
    p = nl ? nl + 1 : end;
  }
  size_t first = 0;
  if (!lines.empty()) {
    const std::string l0(lines[0].first, lines[0].second);
    if (l0.find(kHeader) != std::string::npos) first = 1;
  }
  const int64_t n = (int64_t)(lines.size() - first);
  if (need) *need = n;
  if (cap < n || (n > 0 && (!ids || !score || !R || !t || !time))) return BOPX_RES_CAP;
  for (int64_t k = 0; k < n; ++k) {
    const char* a = lines[first + k].first;
    const char* b = lines[first + k].second;
    const char* fld[8];
    int nf = 0;
    fld[nf++] = a;
    for (const char* s = a; s < b; ++s)
      if (*s == ',') {
        if (nf == 7) return BOPX_RES_OTHER;
        fld[nf++] = s + 1;
      }
    if (nf != 7) return BOPX_RES_OTHER;
    fld[7] = b + 1;
    auto field = [&](int i, const char*& fp, const char*& fe) {
      fp = fld[i];
      fe = fld[i + 1] - 1;
    };
    const char *fp, *fe;
    for (int i = 0; i < 3; ++i) {
      field(i, fp, fe);
      trim(fp, fe);
      if (!parse_int(fp, fe, ids + 3 * k + i)) return BOPX_RES_OTHER;
    }
    field(3, fp, fe);
    trim(fp, fe);
    if (!parse_float(fp, fe, score + k)) return BOPX_RES_OTHER;
    field(4, fp, fe);
    if (!parse_floats(fp, fe, 9, R + 9 * k)) return BOPX_RES_OTHER;
    field(5, fp, fe);
    if (!parse_floats(fp, fe, 3, t + 3 * k)) return BOPX_RES_OTHER;
    field(6, fp, fe);
    trim(fp, fe);
    if (!parse_float(fp, fe, time + k)) return BOPX_RES_OTHER;
  }
  return n;
}
