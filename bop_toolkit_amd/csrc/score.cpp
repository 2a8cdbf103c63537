// score.cpp — native BOP scoring of one errors folder (include/bopx_score.h).
//
// The reference scores each (errors folder, threshold) pair in its own Python
// interpreter (scripts/eval_bop19_pose.py:150-213 -> scripts/eval_calc_scores.py):
// it parses the folder's errors_*.json, normalises the errors, matches the
// estimates of every image to its valid GT instances (bop_toolkit_lib/
// pose_matching.py:9-160) and writes one record per GT instance. Here one call
// parses the folder once and scores all its threshold settings (in parallel
// threads), writing the same matches_*.json bytes. Host code only.
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/bopx_score.h"

namespace {

// ---------------------------------------------------------------- numbers
// A JSON number as Python's json module returns it: int (arbitrary size; here
// int64) or float.
struct Num {
  double d = 0.0;
  int64_t i = 0;
  bool is_int = false;
  double as_double() const { return is_int ? (double)i : d; }
};

// float.__repr__: the shortest digit string that round-trips (std::to_chars
// gives the same digits as CPython's dtoa mode 0), laid out as Python does:
// exponent form when the decimal exponent is < -4 or >= 16 (decpt <= -4 or
// decpt > 16), "e" + sign + at least two digits; otherwise positional with
// at least one digit after the point.
int py_repr(double v, char* out) {
  if (std::isnan(v)) return (int)(std::strcpy(out, "NaN"), 3);
  if (std::isinf(v)) {
    std::strcpy(out, v > 0 ? "Infinity" : "-Infinity");
    return v > 0 ? 8 : 9;
  }
  char buf[64];
  const auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  *r.ptr = '\0';
  const char* p = buf;
  int n = 0;
  if (*p == '-') out[n++] = *p++;
  char dig[32] = {0};
  int nd = 0;
  for (; *p && *p != 'e'; ++p)
    if (*p != '.') dig[nd++] = *p;
  const int e10 = std::atoi(p + 1);  // value = d.ddd x 10^e10
  const int decpt = e10 + 1;         // value = 0.ddd x 10^decpt
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      out[n++] = '0';
      out[n++] = '.';
      for (int k = 0; k < -decpt; ++k) out[n++] = '0';
      for (int k = 0; k < nd; ++k) out[n++] = dig[k];
    } else if (decpt >= nd) {
      for (int k = 0; k < nd; ++k) out[n++] = dig[k];
      for (int k = nd; k < decpt; ++k) out[n++] = '0';
      out[n++] = '.';
      out[n++] = '0';
    } else {
      for (int k = 0; k < decpt; ++k) out[n++] = dig[k];
      out[n++] = '.';
      for (int k = decpt; k < nd; ++k) out[n++] = dig[k];
    }
  } else {
    out[n++] = dig[0];
    if (nd > 1) {
      out[n++] = '.';
      for (int k = 1; k < nd; ++k) out[n++] = dig[k];
    }
    n += std::snprintf(out + n, 16, "e%c%02d", e10 < 0 ? '-' : '+', e10 < 0 ? -e10 : e10);
  }
  out[n] = '\0';
  return n;
}

void put_num(std::string& s, const Num& x) {
  char b[40];
  if (x.is_int) {
    const auto r = std::to_chars(b, b + sizeof(b), x.i);
    s.append(b, r.ptr);
  } else {
    s.append(b, py_repr(x.d, b));
  }
}

void put_int(std::string& s, int64_t v) {
  char b[24];
  const auto r = std::to_chars(b, b + sizeof(b), v);
  s.append(b, r.ptr);
}

// ----------------------------------------------------------------- parsing
// The errors files: a JSON list of records {"errors": {"<gt id>": [e, ...]},
// "est_id": int, "im_id": int, "obj_id": int, "score": number} (other keys are
// skipped). Python's json module also reads NaN / Infinity / -Infinity.
struct ErrEntry {
  int64_t gt;
  int64_t v0;  // first value in Folder::vals
  int nv;
};
struct Rec {
  int64_t im = 0, obj = 0, est = 0;
  Num score;
  int64_t e0 = 0;  // first entry in Folder::ents
  int ne = 0;
  bool has_im = false, has_obj = false, has_est = false, has_score = false, has_errors = false;
};

struct Parser {
  const char* p;
  const char* end;
  std::string err;

  bool fail(const char* what) {
    if (err.empty()) err = what;
    return false;
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool lit(char c) {
    ws();
    if (p < end && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
  bool string(std::string& out) {
    ws();
    if (p >= end || *p != '"') return fail("string expected");
    ++p;
    out.clear();
    while (p < end && *p != '"') {
      if (*p == '\\') return fail("escaped strings are not supported");
      out.push_back(*p++);
    }
    if (p >= end) return fail("unterminated string");
    ++p;
    return true;
  }
  bool number(Num& x) {
    ws();
    if (end - p >= 3 && !std::strncmp(p, "NaN", 3)) {
      p += 3;
      x = Num{NAN, 0, false};
      return true;
    }
    if (end - p >= 8 && !std::strncmp(p, "Infinity", 8)) {
      p += 8;
      x = Num{INFINITY, 0, false};
      return true;
    }
    if (end - p >= 9 && !std::strncmp(p, "-Infinity", 9)) {
      p += 9;
      x = Num{-INFINITY, 0, false};
      return true;
    }
    const char* q = p;
    if (q < end && *q == '-') ++q;
    bool is_int = true;
    while (q < end && ((*q >= '0' && *q <= '9') || *q == '.' || *q == 'e' || *q == 'E' ||
                       *q == '+' || *q == '-')) {
      if (*q == '.' || *q == 'e' || *q == 'E') is_int = false;
      ++q;
    }
    if (q == p) return fail("number expected");
    x.is_int = is_int;
    if (is_int) {
      const auto r = std::from_chars(p, q, x.i);
      if (r.ec != std::errc() || r.ptr != q) return fail("integer out of range");
      x.d = (double)x.i;
    } else {
      const auto r = std::from_chars(p, q, x.d);
      if (r.ec != std::errc() || r.ptr != q) return fail("bad number");
    }
    p = q;
    return true;
  }
  // skip any value
  bool skip() {
    ws();
    if (p >= end) return fail("value expected");
    if (*p == '"') {
      std::string s;
      return string(s);
    }
    if (*p == '{' || *p == '[') {
      const char open = *p, close = open == '{' ? '}' : ']';
      ++p;
      if (lit(close)) return true;
      do {
        if (open == '{') {
          std::string k;
          if (!string(k) || !lit(':')) return fail("bad object");
        }
        if (!skip()) return false;
      } while (lit(','));
      return lit(close) || fail("bad container");
    }
    if (end - p >= 4 && (!std::strncmp(p, "true", 4) || !std::strncmp(p, "null", 4))) {
      p += 4;
      return true;
    }
    if (end - p >= 5 && !std::strncmp(p, "false", 5)) {
      p += 5;
      return true;
    }
    Num x;
    return number(x);
  }
};

struct Folder {
  std::vector<Rec> recs;  // every file's records, file by file
  std::vector<ErrEntry> ents;
  std::vector<Num> vals;
  std::vector<int64_t> file_r0;  // first record of each file (+ end)
};

bool int_key(const std::string& k, int64_t& v) {
  // keys_to_int (inout.py:66-82): k.lstrip("-").isdigit() -> int(k)
  size_t i = 0;
  while (i < k.size() && k[i] == '-') ++i;
  if (i == k.size()) return false;
  for (size_t j = i; j < k.size(); ++j)
    if (k[j] < '0' || k[j] > '9') return false;
  if (i > 1) return false;  // "--1": isdigit() true but int() raises
  const auto r = std::from_chars(k.data(), k.data() + k.size(), v);
  return r.ec == std::errc() && r.ptr == k.data() + k.size();
}

int parse_file(const char* path, Folder& f, std::string& msg) {
  FILE* fp = std::fopen(path, "rb");
  if (!fp) {
    msg = std::string("cannot read ") + path;
    return BOPX_SCORE_READ;
  }
  std::string text;
  char buf[1 << 16];
  size_t k;
  while ((k = std::fread(buf, 1, sizeof(buf), fp)) > 0) text.append(buf, k);
  std::fclose(fp);
  Parser P{text.data(), text.data() + text.size(), {}};
  auto bad = [&](const char* what) {
    msg = std::string(path) + ": " + (P.err.empty() ? what : P.err);
    return BOPX_SCORE_PARSE;
  };
  if (!P.lit('[')) return bad("list expected");
  if (!P.lit(']')) {
    do {
      if (!P.lit('{')) return bad("record expected");
      Rec r;
      r.e0 = (int64_t)f.ents.size();
      if (!P.lit('}')) {
        do {
          std::string key;
          if (!P.string(key) || !P.lit(':')) return bad("key expected");
          Num x;
          if (key == "errors") {
            if (r.has_errors) return BOPX_SCORE_UNSUPPORTED;  // duplicate key
            r.has_errors = true;
            if (!P.lit('{')) return bad("errors dict expected");
            if (!P.lit('}')) {
              do {
                std::string g;
                if (!P.string(g) || !P.lit(':')) return bad("GT id expected");
                ErrEntry e;
                if (!int_key(g, e.gt)) return BOPX_SCORE_UNSUPPORTED;
                for (int64_t q = r.e0; q < (int64_t)f.ents.size(); ++q)
                  if (f.ents[q].gt == e.gt) return BOPX_SCORE_UNSUPPORTED;  // duplicate key
                e.v0 = (int64_t)f.vals.size();
                if (!P.lit('[')) return BOPX_SCORE_UNSUPPORTED;  // not a list of errors
                if (!P.lit(']')) {
                  do {
                    if (!P.number(x)) return BOPX_SCORE_UNSUPPORTED;
                    f.vals.push_back(x);
                  } while (P.lit(','));
                  if (!P.lit(']')) return bad("bad error list");
                }
                e.nv = (int)((int64_t)f.vals.size() - e.v0);
                f.ents.push_back(e);
              } while (P.lit(','));
              if (!P.lit('}')) return bad("bad errors dict");
            }
          } else if (key == "im_id" || key == "obj_id" || key == "est_id") {
            if (!P.number(x)) return bad("number expected");
            if (!x.is_int) return BOPX_SCORE_UNSUPPORTED;
            bool& has = key == "im_id" ? r.has_im : key == "obj_id" ? r.has_obj : r.has_est;
            if (has) return BOPX_SCORE_UNSUPPORTED;
            has = true;
            (key == "im_id" ? r.im : key == "obj_id" ? r.obj : r.est) = x.i;
          } else if (key == "score") {
            if (r.has_score || !P.number(r.score)) return BOPX_SCORE_UNSUPPORTED;
            r.has_score = true;
          } else if (!P.skip()) {
            return bad("bad value");
          }
        } while (P.lit(','));
        if (!P.lit('}')) return bad("bad record");
      }
      r.ne = (int)((int64_t)f.ents.size() - r.e0);
      if (!(r.has_im && r.has_obj && r.has_est && r.has_score && r.has_errors))
        return BOPX_SCORE_UNSUPPORTED;  // the Python path raises its KeyError
      f.recs.push_back(r);
    } while (P.lit(','));
    if (!P.lit(']')) return bad("bad list");
  }
  P.ws();
  if (P.p != P.end) return bad("trailing data");
  return BOPX_SCORE_OK;
}

// ----------------------------------------------------------------- scoring
struct Match {
  int64_t rec = -1;  // matched error record (-1: none)
  int64_t ent = -1;  // its errors entry for this GT
};

// (image, object) groups of each image: record indices in match order
// (decreasing score, stable), the first n_top when n_top > 0.
struct Groups {
  std::vector<int64_t> order;      // record indices, group by group
  std::vector<int64_t> grp_off;    // per group: [grp_off[g], grp_off[g + 1]) in order
  std::vector<int64_t> im_grp;     // per image: its groups [im_grp[i], im_grp[i + 1])
};

// Text of n items formatted once (fmt(i, buf) appends item i), in chunks of
// kTextChunk items on `threads` threads; item i is bufs[i / kTextChunk] at
// [off[i], off[i] + len[i]).
constexpr int64_t kTextChunk = 4096;
struct TextTable {
  std::vector<std::string> bufs;
  std::vector<uint32_t> off, len;
  void append_to(std::string& out, int64_t i) const {
    out.append(bufs[(size_t)(i / kTextChunk)], off[(size_t)i], len[(size_t)i]);
  }
};

template <class F>
TextTable build_text(int64_t n, int threads, F fmt) {
  TextTable t;
  const int64_t nc = (n + kTextChunk - 1) / kTextChunk;
  t.bufs.resize((size_t)nc);
  t.off.resize((size_t)n);
  t.len.resize((size_t)n);
  std::atomic<int64_t> nx{0};
  auto work = [&]() {
    for (int64_t c; (c = nx.fetch_add(1)) < nc;) {
      std::string& b = t.bufs[(size_t)c];
      for (int64_t i = c * kTextChunk; i < std::min(n, (c + 1) * kTextChunk); ++i) {
        const size_t o = b.size();
        fmt(i, b);
        t.off[(size_t)i] = (uint32_t)o;
        t.len[(size_t)i] = (uint32_t)(b.size() - o);
      }
    }
  };
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(threads, nc));
  std::vector<std::thread> pool;
  for (int k = 1; k < nt; ++k) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return t;
}

}  // namespace

extern "C" int bopx_py_float_repr(double v, char* out) { return py_repr(v, out); }

extern "C" int bopx_write_errors(const char* const* paths, int n_values, int64_t n_rec,
                                 const int64_t* rec_im, const int64_t* rec_obj,
                                 const int64_t* rec_est, const double* rec_score,
                                 const int64_t* pair_off, const int64_t* pair_gt,
                                 const double* values) {
  if (n_values <= 0 || n_rec < 0) return BOPX_SCORE_INVALID;
  std::atomic<int> next{0}, status{BOPX_SCORE_OK};
  // the record text around its values (shared by the n_values files)
  std::vector<std::string> tail((size_t)n_rec);
  for (int64_t r = 0; r < n_rec; ++r) {
    std::string& t = tail[(size_t)r];
    t += pair_off[r + 1] > pair_off[r] ? "]}, \"est_id\": " : "}, \"est_id\": ";
    put_int(t, rec_est[r]);
    t += ", \"im_id\": ";
    put_int(t, rec_im[r]);
    t += ", \"obj_id\": ";
    put_int(t, rec_obj[r]);
    t += ", \"score\": ";
    put_num(t, Num{rec_score[r], 0, false});
    t += '}';
  }
  auto work = [&]() {
    std::string out;
    char b[40];
    for (int k; (k = next.fetch_add(1)) < n_values;) {
      out.clear();
      out += n_rec ? "[\n  " : "[\n";
      for (int64_t r = 0; r < n_rec; ++r) {
        if (r) out += ",\n  ";
        out += "{\"errors\": {";
        for (int64_t q = pair_off[r]; q < pair_off[r + 1]; ++q) {
          out += q > pair_off[r] ? "], \"" : "\"";
          put_int(out, pair_gt[q]);
          out += "\": [";
          out.append(b, py_repr(values[q * n_values + k], b));
        }
        out += tail[(size_t)r];
      }
      out += n_rec ? "\n]" : "]";
      FILE* fp = std::fopen(paths[k], "wb");
      if (!fp || std::fwrite(out.data(), 1, out.size(), fp) != out.size()) status = BOPX_SCORE_READ;
      if (fp) std::fclose(fp);
    }
  };
  const int nt = std::max(1, std::min(n_values, 4));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return status.load();
}

extern "C" int bopx_score_folder(const bopx_score_args* a, char* msg_out, int msg_len) {
  std::string msg;
  auto ret = [&](int code) {
    if (msg_out && msg_len > 0) {
      std::snprintf(msg_out, (size_t)msg_len, "%s", msg.c_str());
    }
    return code;
  };
  if (!a || a->n_gt < 0 || a->n_im < 0 || a->n_files < 0 || a->n_settings < 0 || a->n_th < 1 ||
      (a->norm == BOPX_NORM_DIAMETER && (!a->diam || a->n_diam <= 0))) {
    msg = "invalid arguments";
    return ret(BOPX_SCORE_INVALID);
  }
  // 1. parse every errors file, normalise (eval_calc_scores.py:221-233)
  // the files on a->threads threads, each into its own part (part-relative
  // entry / value indices), then concatenated in file order; the first file in
  // order that fails sets the status and message, as a sequential parse would
  Folder f;
  {
    const int nf = a->n_files;
    std::vector<Folder> parts((size_t)nf);
    std::vector<int> st((size_t)nf, BOPX_SCORE_OK);
    std::vector<std::string> msgs((size_t)nf);
    std::atomic<int> nx{0};
    auto parse = [&]() {
      for (int i; (i = nx.fetch_add(1)) < nf;)
        st[(size_t)i] = parse_file(a->err_paths[i], parts[(size_t)i], msgs[(size_t)i]);
    };
    const int npt = std::max(1, std::min(a->threads, nf));
    std::vector<std::thread> pp;
    for (int t = 1; t < npt; ++t) pp.emplace_back(parse);
    parse();
    for (auto& t : pp) t.join();
    size_t nr = 0, ne = 0, nv = 0;
    for (int i = 0; i < nf; ++i) {
      if (st[(size_t)i] != BOPX_SCORE_OK) {
        msg = msgs[(size_t)i];
        if (st[(size_t)i] == BOPX_SCORE_UNSUPPORTED && msg.empty())
          msg = std::string(a->err_paths[i]) + ": handled by the Python path";
        return ret(st[(size_t)i]);
      }
      nr += parts[(size_t)i].recs.size();
      ne += parts[(size_t)i].ents.size();
      nv += parts[(size_t)i].vals.size();
    }
    f.recs.reserve(nr);
    f.ents.reserve(ne);
    f.vals.reserve(nv);
    for (int i = 0; i < nf; ++i) {
      Folder& q = parts[(size_t)i];
      f.file_r0.push_back((int64_t)f.recs.size());
      const int64_t eo = (int64_t)f.ents.size(), vo = (int64_t)f.vals.size();
      for (Rec r : q.recs) {
        r.e0 += eo;
        f.recs.push_back(r);
      }
      for (ErrEntry e : q.ents) {
        e.v0 += vo;
        f.ents.push_back(e);
      }
      f.vals.insert(f.vals.end(), q.vals.begin(), q.vals.end());
      Folder().recs.swap(q.recs);
    }
  }
  f.file_r0.push_back((int64_t)f.recs.size());
  for (const Rec& r : f.recs) {
    if (std::isnan(r.score.as_double())) {
      msg = "NaN score";
      return ret(BOPX_SCORE_UNSUPPORTED);
    }
    for (int e = 0; e < r.ne; ++e) {
      const ErrEntry& en = f.ents[r.e0 + e];
      if (en.nv != a->n_th) {
        msg = "error list length differs from the threshold count";
        return ret(BOPX_SCORE_UNSUPPORTED);
      }
      for (int v = 0; v < en.nv; ++v) {
        Num& x = f.vals[en.v0 + v];
        if (a->norm == BOPX_NORM_DIAMETER) {
          if (r.obj < 0 || r.obj >= a->n_diam || !(a->diam[r.obj] == a->diam[r.obj]) ||
              a->diam[r.obj] == 0.0) {
            msg = "object without a diameter";
            return ret(BOPX_SCORE_UNSUPPORTED);
          }
          x = Num{x.as_double() / a->diam[r.obj], 0, false};
        } else if (a->norm == BOPX_NORM_WIDTH) {
          x = Num{a->width_factor * x.as_double(), 0, false};
        }
      }
    }
  }
  // 2. per image: its error records grouped by object, in match order
  Groups G;
  G.im_grp.push_back(0);
  {
    // records of each file by image id (file order kept)
    std::vector<std::unordered_map<int64_t, std::vector<int64_t>>> by_im(a->n_files);
    for (int i = 0; i < a->n_files; ++i)
      for (int64_t r = f.file_r0[i]; r < f.file_r0[i + 1]; ++r) by_im[i][f.recs[r].im].push_back(r);
    std::vector<int64_t> objs;
    for (int64_t im = 0; im < a->n_im; ++im) {
      const int64_t g0 = a->im_off[im], g1 = a->im_off[im + 1];
      const int fi = a->im_file[im];
      if (fi < 0 || fi >= a->n_files || g1 < g0) {
        msg = "bad image table";
        return ret(BOPX_SCORE_INVALID);
      }
      objs.clear();
      for (int64_t g = g0; g < g1; ++g)
        if (std::find(objs.begin(), objs.end(), (int64_t)a->gt_obj[g]) == objs.end())
          objs.push_back(a->gt_obj[g]);
      // the image's id is its GT records' (an image without GT instances has no match)
      const auto it = g1 > g0 ? by_im[fi].find(a->gt_im[g0]) : by_im[fi].end();
      if (it != by_im[fi].end()) {
        for (const int64_t o : objs) {
          const int64_t s0 = (int64_t)G.order.size();
          for (const int64_t r : it->second)
            if (f.recs[r].obj == o) G.order.push_back(r);
          // decreasing score, stable (sorted(..., key=score, reverse=True))
          std::stable_sort(G.order.begin() + s0, G.order.end(), [&](int64_t x, int64_t y) {
            return f.recs[x].score.as_double() > f.recs[y].score.as_double();
          });
          if (a->n_top > 0 && (int64_t)G.order.size() - s0 > a->n_top)
            G.order.resize((size_t)(s0 + a->n_top));
          G.grp_off.push_back(s0);
        }
      }
      G.im_grp.push_back((int64_t)G.grp_off.size());
    }
    G.grp_off.push_back((int64_t)G.order.size());
  }
  // every error entry of a matched image must index its image's GT list
  for (int64_t im = 0; im < a->n_im; ++im) {
    const int64_t ng = a->im_off[im + 1] - a->im_off[im];
    for (int64_t gi = G.im_grp[im]; gi < G.im_grp[im + 1]; ++gi)
      for (int64_t q = G.grp_off[gi]; q < G.grp_off[gi + 1]; ++q) {
        const Rec& r = f.recs[G.order[q]];
        for (int e = 0; e < r.ne; ++e)
          if (f.ents[r.e0 + e].gt < 0 || f.ents[r.e0 + e].gt >= ng) {
            msg = "GT id outside its image";
            return ret(BOPX_SCORE_UNSUPPORTED);
          }
      }
  }

  // 3. the matches files' text that every setting shares, formatted once: each
  // GT's id fields, each errors entry's values, each record's score
  const bool write = a->matches_paths != nullptr;
  const int nth = std::max(1, a->threads);
  TextTable gt_txt, ent_txt, score_txt;
  if (write) {
    gt_txt = build_text(a->n_gt, nth, [&](int64_t g, std::string& b) {
      b += ", \"gt_id\": ";
      put_int(b, a->gt_id[g]);
      b += ", \"im_id\": ";
      put_int(b, a->gt_im[g]);
      b += ", \"obj_id\": ";
      put_int(b, a->gt_obj[g]);
      b += ", \"scene_id\": ";
      put_int(b, a->gt_scene[g]);
      b += ", \"score\": ";
    });
    ent_txt = build_text((int64_t)f.ents.size(), nth, [&](int64_t e, std::string& b) {
      const ErrEntry& en = f.ents[(size_t)e];
      for (int k = 0; k < en.nv; ++k) {
        if (k) b += ", ";
        put_num(b, f.vals[(size_t)(en.v0 + k)]);
      }
    });
    score_txt = build_text((int64_t)f.recs.size(), nth,
                           [&](int64_t r, std::string& b) { put_num(b, f.recs[(size_t)r].score); });
  }
  // 4. every setting: greedy matching (pose_matching.py:9-90) + matches file
  std::atomic<int> next{0}, status{BOPX_SCORE_OK};
  std::vector<std::string> errs(a->n_settings);
  auto work = [&]() {
    std::vector<Match> m;
    std::vector<uint8_t> taken;
    std::string out;
    for (int s; (s = next.fetch_add(1)) < a->n_settings;) {
      const double* th = a->th + (size_t)s * a->n_th;
      m.assign((size_t)a->n_gt, Match{});
      for (int64_t im = 0; im < a->n_im; ++im) {
        const int64_t g0 = a->im_off[im];
        const int64_t ng = a->im_off[im + 1] - g0;
        for (int64_t gi = G.im_grp[im]; gi < G.im_grp[im + 1]; ++gi) {
          taken.assign((size_t)ng, 0);
          for (int64_t q = G.grp_off[gi]; q < G.grp_off[gi + 1]; ++q) {
            const int64_t ri = G.order[q];
            const Rec& r = f.recs[ri];
            int64_t best_e = -1;
            const Num* best_v = nullptr;
            for (int e = 0; e < r.ne; ++e) {
              const ErrEntry& en = f.ents[r.e0 + e];
              // pose_matching.py: skip invalid (when the image has a mask) and taken GTs
              if (ng > 0 && !a->gt_valid[g0 + en.gt]) continue;
              if (taken[(size_t)en.gt]) continue;
              const Num* v = &f.vals[en.v0];
              bool below = true;
              for (int k = 0; k < a->n_th; ++k)
                below = below && v[k].as_double() < (best_v ? best_v[k].as_double() : th[k]);
              if (below) {
                best_e = r.e0 + e;
                best_v = v;
              }
            }
            if (best_e >= 0) {
              const int64_t gt = f.ents[best_e].gt;
              taken[(size_t)gt] = 1;
              m[(size_t)(g0 + gt)] = Match{ri, best_e};
            }
          }
        }
      }
      uint8_t* mk = a->matched ? a->matched + (size_t)s * a->n_gt : nullptr;
      for (int64_t g = 0; g < a->n_gt; ++g)
        if (mk) mk[g] = m[(size_t)g].rec >= 0;
      if (!a->matches_paths || !a->matches_paths[s]) continue;
      // matches_{sign}.json: save_json's one-record-per-line list, sorted keys
      out.clear();
      out.reserve((size_t)a->n_gt * 150 + 8);
      out += a->n_gt ? "[\n  " : "[\n";
      for (int64_t g = 0; g < a->n_gt; ++g) {
        if (g) out += ",\n  ";
        const Match& mt = m[(size_t)g];
        out += "{\"error\": ";
        if (mt.rec < 0) {
          out += "-1, \"error_norm\": -1, \"est_id\": -1";
        } else {
          const ErrEntry& en = f.ents[mt.ent];
          out += '[';
          ent_txt.append_to(out, mt.ent);
          out += "], \"error_norm\": [";
          for (int k = 0; k < en.nv; ++k) {
            if (k) out += ", ";
            put_num(out, Num{f.vals[en.v0 + k].as_double() / th[k], 0, false});
          }
          out += "], \"est_id\": ";
          put_int(out, f.recs[mt.rec].est);
        }
        gt_txt.append_to(out, g);  // , "gt_id": .. "scene_id": .., "score":
        if (mt.rec < 0)
          out += "-1";
        else
          score_txt.append_to(out, mt.rec);
        out += a->gt_valid[g] ? ", \"valid\": true}" : ", \"valid\": false}";
      }
      out += a->n_gt ? "\n]" : "]";
      FILE* fp = std::fopen(a->matches_paths[s], "wb");
      if (!fp || std::fwrite(out.data(), 1, out.size(), fp) != out.size()) {
        errs[s] = std::string("cannot write ") + a->matches_paths[s];
        status = BOPX_SCORE_READ;
      }
      if (fp) std::fclose(fp);
    }
  };
  const int nt = std::max(1, std::min(a->threads, a->n_settings));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  for (const std::string& e : errs)
    if (!e.empty()) msg = e;
  return ret(status.load());
}
