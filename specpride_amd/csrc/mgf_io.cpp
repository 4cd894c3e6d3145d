// Native clustered-MGF ingest and emit for the bin-mean CLI path
// (reference: src/binning.py:122-167 parser,
// src/binning.py:234-245 writer).  Host C++ (no GPU), built into
// specpride_amd/lib/libspx_mgf.so with g++ -O3 -pthread.
//
// Parser contract = the reference's line loop, restricted to the well-formed
// subset whose Python meaning is unambiguous:
//   TITLE=<id;usi> starts a spectrum; PEPMASS=<float>; CHARGE=<int>[+];
//   a line whose first char is an ASCII digit is "mz intensity" (single space,
//   extra fields ignored); a stripped "END IONS" stores the spectrum.
// Numbers use the plain decimal grammar [+-]digits[.digits][e[+-]digits]; the
// values equal Python float(): both are correctly rounded (Clinger's exact fast
// path for short decimals, an x87 extended-precision step for up to 19 digits,
// strtod otherwise).  Any
// line outside that subset (underscores in numbers, inf/nan, tabs between
// fields, non-ASCII text, PEPMASS before the first TITLE, a repeated END IONS,
// a TITLE without ';') makes the parse report "fallback: ..." and the caller
// re-reads the file with the Python line loop, which then behaves (or raises)
// exactly like the reference.
//
// Files are split into per-thread byte ranges that begin at a "TITLE=" line:
// the reference's state is reset at every TITLE, so the ranges parse
// independently and concatenate in order.
//
// Writer: Python repr() of a float64 (numpy's str() of np.float64 is the same):
// shortest round-trip digits (std::to_chars), positional for 1e-4 <= |x| < 1e16,
// else d.ddde+XX.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <string_view>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/spx_mgf.h"

namespace {

// One thread's parse of a byte range (either grammar): per spectrum its peak
// count, precursor fields and title; the peaks in file order.
struct Chunk {
  std::vector<int64_t> npk;     // peaks per spectrum
  std::vector<double> mz, it, prec, rt;  // rt: general reader only
  std::vector<int64_t> charge;
  std::vector<int32_t> flags;   // bit0 PEPMASS, bit1 CHARGE (general: bit2 RTINSECONDS, bit3 TITLE)
  std::string titles;           // '\n'-joined
  std::string error;
  void reserve_for(size_t bytes) {  // a peak line is >= ~8 bytes; most are ~18
    mz.reserve(bytes / 16);
    it.reserve(bytes / 16);
  }
};
using GenChunk = Chunk;

// A parse: the threads' chunks kept as they are (no merge copy); the accessors
// copy them out in parallel.
struct Result {
  std::vector<Chunk> parts;
  std::vector<int64_t> s_base, p_base;  // first spectrum / peak of each part
  int64_t S = 0, P = 0;
  bool with_rt = false;
  std::string error;
  std::string titles;  // joined on first request
  bool titles_built = false;
  std::vector<int64_t> title_off;  // [S+1] offsets into `titles` (with the '\n's)
  std::string group_ids;           // '\n'-joined ids of the last spx_mgf_group
};

inline bool is_py_space(unsigned char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\x0b' || c == '\x0c' || (c >= 0x1c && c <= 0x1f);
}

inline void strip(const char*& b, const char*& e) {
  while (b < e && is_py_space((unsigned char)*b)) ++b;
  while (e > b && is_py_space((unsigned char)e[-1])) --e;
}

// Plain decimal float grammar [+-]digits[.digits][e[+-]digits] in ONE pass that
// also accumulates the significand; returns false on anything else.  Clinger's
// exact fast path: an integer significand w <= 2^53 scaled by an exactly
// representable 10^k (|k| <= 22) is ONE correctly rounded IEEE multiply or divide
// of exact operands -- the correctly rounded value of the decimal, i.e. what
// strtod and Python's float() return.  m/z and intensity lines ("1234.56789
// 17.25") take it; 16-19 digit ones take the extended-precision step below;
// anything longer (> 19 significant digits, large exponents) falls to strtod.
// The value of the decimal w * 10^k (w: its significant digits, `fast` false when
// there were more than 19), correctly rounded; [b, e) is the token for strtod.
inline double decimal_value(bool neg, uint64_t w, bool fast, int k, const char* b, const char* e) {
  static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                    1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  if (fast && w <= (uint64_t(1) << 53) && k >= -22 && k <= 22) {
    const double v = k < 0 ? (double)w / kPow10[-k] : (double)w * kPow10[k];
    return neg ? -v : v;
  }
  // Significands of 54..64 bits (the repr of an arbitrary double has 16-17 digits):
  // one x87 extended-precision divide or multiply of exact operands (w < 2^64 and
  // 10^|k| <= 10^27 are exact in a 64-bit significand) gives the decimal correctly
  // rounded to 64 bits.  Rounding that to 53 bits is the correct rounding of the
  // decimal itself unless a double's rounding midpoint lies within one extended
  // unit of it -- low 11 significand bits 0x3FF..0x401 -- which strtod decides.
  if (fast && k >= -27 && k <= 27) {
    static const long double kPow10L[28] = {1e0L,  1e1L,  1e2L,  1e3L,  1e4L,  1e5L,  1e6L,  1e7L,  1e8L,  1e9L,
                                            1e10L, 1e11L, 1e12L, 1e13L, 1e14L, 1e15L, 1e16L, 1e17L, 1e18L, 1e19L,
                                            1e20L, 1e21L, 1e22L, 1e23L, 1e24L, 1e25L, 1e26L, 1e27L};
    static_assert(sizeof(long double) >= 10 && std::numeric_limits<long double>::digits == 64,
                  "x87 extended precision");
    const long double L = k < 0 ? (long double)w / kPow10L[-k] : (long double)w * kPow10L[k];
    uint64_t sig;
    std::memcpy(&sig, &L, sizeof(sig));  // the 64-bit significand (explicit integer bit)
    const unsigned lo = (unsigned)(sig & 0x7FFu);
    if (lo < 0x3FFu || lo > 0x401u) {
      const double v = (double)L;
      return neg ? -v : v;
    }
  }
  char buf[128];
  const size_t n = (size_t)(e - b);
  if (n >= sizeof(buf)) {
    std::string s(b, e);
    return std::strtod(s.c_str(), nullptr);
  }
  std::memcpy(buf, b, n);
  buf[n] = 0;
  return std::strtod(buf, nullptr);
}

// digits [. digits] from p (no sign, no exponent): the significand, its digit
// count and fraction length, as parse_float accumulates them; p stops at the
// first byte of neither.  Returns whether any digit was seen.
inline bool scan_unsigned(const char*& p, const char* e, uint64_t& w, bool& fast, int& frac) {
  bool digits = false;
  int nd = 0;
  for (; p < e && (unsigned)(*p - '0') <= 9u; ++p) {
    digits = true;
    const unsigned d = (unsigned)(*p - '0');
    if (w == 0 && d == 0) continue;  // leading zeros: no significant digit
    if (++nd > 19) fast = false;
    else w = w * 10 + d;
  }
  if (p < e && *p == '.') {
    ++p;
    for (; p < e && (unsigned)(*p - '0') <= 9u; ++p) {
      digits = true;
      const unsigned d = (unsigned)(*p - '0');
      ++frac;
      if (w == 0 && d == 0) continue;
      if (++nd > 19) fast = false;
      else w = w * 10 + d;
    }
  }
  return digits;
}

bool parse_float(const char* b, const char* e, double& out) {
  const char* p = b;
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) { neg = *p == '-'; ++p; }
  uint64_t w = 0;
  int frac = 0;
  bool fast = true;
  if (!scan_unsigned(p, e, w, fast, frac)) return false;
  int ex = 0;
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '+' || *p == '-')) { eneg = *p == '-'; ++p; }
    const char* x0 = p;
    for (; p < e && (unsigned)(*p - '0') <= 9u; ++p)
      if (ex < 100000) ex = ex * 10 + (*p - '0');
    if (p == x0) return false;
    if (eneg) ex = -ex;
  }
  if (p != e) return false;
  out = decimal_value(neg, w, fast, ex - frac, b, e);
  return true;
}

// The common peak line "<digits>[.digits]<sep><digits>[.digits]" + \n, \r\n, \r or
// the end, parsed in one pass from its first byte (a digit) at p: the two values
// and p past the line terminator.  `single`: the separator is exactly one space
// (the binning reader's split(' ')), else one or more spaces/tabs (the general
// reader's whitespace split).  Any other shape -- a sign, an exponent, a third
// field, trailing blanks -- returns false with p unchanged, and the caller's
// line-by-line path decides; the values are parse_float's for the same tokens.
inline bool fast_peak_line(const char*& p, const char* e, bool single, double& a, double& v) {
  const char* q = p;
  uint64_t w1 = 0, w2 = 0;
  int f1 = 0, f2 = 0;
  bool k1 = true, k2 = true;
  const char* b1 = q;
  if (!scan_unsigned(q, e, w1, k1, f1)) return false;
  const char* e1 = q;
  if (q >= e || (*q != ' ' && (single || *q != '\t'))) return false;
  ++q;
  if (!single)
    while (q < e && (*q == ' ' || *q == '\t')) ++q;
  if (q >= e || (unsigned)(*q - '0') > 9u) return false;
  const char* b2 = q;
  if (!scan_unsigned(q, e, w2, k2, f2)) return false;
  const char* e2 = q;
  if (q < e) {
    if (*q == '\n') ++q;
    else if (*q == '\r') { ++q; if (q < e && *q == '\n') ++q; }
    else return false;
  }
  a = decimal_value(false, w1, k1, -f1, b1, e1);
  v = decimal_value(false, w2, k2, -f2, b2, e2);
  p = q;
  return true;
}

// One line of [p, e): [ls, le) without its terminator (\n, \r\n or \r: Python's
// universal newlines), p advanced past it; false if the line holds a non-ASCII
// or a NUL byte (one pass over the bytes; titles cross the ABI as NUL-terminated
// text, so a NUL inside one would cut every later title short).
inline bool next_line(const char*& p, const char* e, const char*& ls, const char*& le) {
  ls = p;
  const char* q = p;
  unsigned char hi = 0;
  bool nul = false;
  for (; q < e; ++q) {
    const unsigned char c = (unsigned char)*q;
    if (c == '\n' || c == '\r') break;
    hi |= c;
    nul |= c == 0;
  }
  le = q;
  if (q < e) {
    if (*q == '\r') {
      ++q;
      if (q < e && *q == '\n') ++q;
    } else {
      ++q;
    }
  }
  p = q;
  return hi < 0x80 && !nul;
}

bool parse_charge(const char* b, const char* e, int64_t& out) {
  strip(b, e);
  while (b < e && *b == '+') ++b;  // .strip("+")
  while (e > b && e[-1] == '+') --e;
  strip(b, e);                     // int() tolerates surrounding whitespace
  const char* p = b;
  bool neg = false;
  if (p < e && (*p == '-' || *p == '+')) { neg = *p == '-'; ++p; }
  if (p == e || e - p > 17) return false;
  int64_t v = 0;
  for (; p < e; ++p) {
    if (*p < '0' || *p > '9') return false;
    v = v * 10 + (*p - '0');
  }
  out = neg ? -v : v;
  return true;
}

void parse_range(const char* b, const char* e, Chunk& C) {
  C.reserve_for((size_t)(e - b));
  bool have = false, stored = true;  // `stored`: END IONS already taken for this TITLE
  int64_t cur_np = 0;
  double cur_prec = 0.0;
  int64_t cur_z = 0;
  int32_t cur_f = 0;
  std::string cur_title;
  size_t mark = 0;  // peaks of the current spectrum start at C.mz[mark]
  const char* p = b;
  auto fail = [&](const char* why) { if (C.error.empty()) C.error = std::string("fallback: ") + why; };
  while (p < e && C.error.empty()) {
    if (have && !stored && (unsigned)(*p - '0') <= 9u) {  // the common peak line in one pass
      double a, v;
      if (fast_peak_line(p, e, true, a, v)) {
        C.mz.push_back(a);
        C.it.push_back(v);
        ++cur_np;
        continue;
      }
    }
    const char *ls, *le;  // universal newlines, like Python text mode: \n, \r\n or \r
    if (!next_line(p, e, ls, le)) { fail("non-ASCII or NUL text"); break; }
    const size_t n = (size_t)(le - ls);
    // peak lines first (most lines; none of the keywords below starts with a digit)
    if (n >= 1 && *ls >= '0' && *ls <= '9') {
      if (!have || stored) { fail("peak outside a spectrum"); break; }
      const char *vb = ls, *ve = le;
      strip(vb, ve);
      const char* sp = (const char*)std::memchr(vb, ' ', (size_t)(ve - vb));
      if (!sp) { fail("peak line without ' '"); break; }
      const char* t1 = sp + 1;
      const char* sp2 = (const char*)std::memchr(t1, ' ', (size_t)(ve - t1));
      const char* t1e = sp2 ? sp2 : ve;
      double a, v;
      if (!parse_float(vb, sp, a) || !parse_float(t1, t1e, v)) { fail("peak value"); break; }
      C.mz.push_back(a);
      C.it.push_back(v);
      ++cur_np;
      continue;
    }
    if (n >= 6 && std::memcmp(ls, "TITLE=", 6) == 0) {
      const char *tb = ls + 6, *te = le;
      strip(tb, te);
      if (!std::memchr(tb, ';', (size_t)(te - tb))) { fail("TITLE without ';'"); break; }
      // a new spectrum: drop the previous one's un-stored peaks
      C.mz.resize(mark);
      C.it.resize(mark);
      have = true;
      stored = false;
      cur_np = 0;
      cur_f = 0;
      cur_title.assign(tb, te);
      continue;
    }
    if (n >= 8 && std::memcmp(ls, "PEPMASS=", 8) == 0) {
      if (!have || stored) { fail("PEPMASS outside a spectrum"); break; }
      const char *vb = ls + 8, *ve = le;
      strip(vb, ve);
      if (!parse_float(vb, ve, cur_prec)) { fail("PEPMASS value"); break; }
      cur_f |= 1;
      continue;
    }
    if (n >= 7 && std::memcmp(ls, "CHARGE=", 7) == 0) {
      if (!have || stored) { fail("CHARGE outside a spectrum"); break; }
      if (!parse_charge(ls + 7, le, cur_z)) { fail("CHARGE value"); break; }
      cur_f |= 2;
      continue;
    }
    const char *sb = ls, *se = le;
    strip(sb, se);
    if (se - sb == 8 && std::memcmp(sb, "END IONS", 8) == 0) {
      if (!have || stored) { fail("END IONS without a new TITLE"); break; }
      C.npk.push_back(cur_np);
      C.prec.push_back(cur_prec);
      C.charge.push_back(cur_z);
      C.flags.push_back(cur_f);
      C.titles += cur_title;
      C.titles += '\n';
      mark = C.mz.size();
      stored = true;
    }
  }
  C.mz.resize(mark);
  C.it.resize(mark);
}

// ---------------------------------------------------- general MGF (pyteomics shape)
// The subset of specpride_amd.mgf.iter_mgf (the gap-average and medoid CLIs'
// reader, pyteomics-shaped) whose meaning is unambiguous: stripped lines;
// BEGIN IONS / END IONS blocks; inside, a line starting with a digit (or +-.
// then a digit) is "mz [intensity]" split on spaces/tabs; KEY=value params with
// TITLE (string), PEPMASS (mz [intensity]), CHARGE (one charge, "2+", "3-", "2"),
// RTINSECONDS (float); other params are ignored (the writers do not emit them).
// Anything else (several charges, non-decimal numbers, non-ASCII) -> fallback.
inline bool is_ws(unsigned char c) { return c == ' ' || c == '\t'; }

bool parse_one_charge(const char* b, const char* e, int64_t& out) {
  strip(b, e);
  if (b == e) return false;
  int sign = 1;
  if (e[-1] == '+') --e;
  else if (e[-1] == '-') { sign = -1; --e; }
  while (b < e && *b == '+') ++b;
  if (b == e || e - b > 17) return false;
  int64_t v = 0;
  for (const char* p = b; p < e; ++p) {
    if (*p < '0' || *p > '9') return false;  // "2+ and 3+", "2,3": several charges
    v = v * 10 + (*p - '0');
  }
  out = sign * v;
  return true;
}

void parse_range_general(const char* b, const char* e, GenChunk& C) {
  C.reserve_for((size_t)(e - b));
  bool inside = false;
  int64_t cur_np = 0;
  double cur_prec = 0.0, cur_rt = 0.0;
  int64_t cur_z = 0;
  int32_t cur_f = 0;
  std::string cur_title;
  size_t mark = 0;
  const char* p = b;
  auto fail = [&](const char* why) { if (C.error.empty()) C.error = std::string("fallback: ") + why; };
  while (p < e && C.error.empty()) {
    if (inside && (unsigned)(*p - '0') <= 9u) {  // the common peak line in one pass
      double a, v;
      if (fast_peak_line(p, e, false, a, v)) {
        C.mz.push_back(a);
        C.it.push_back(v);
        ++cur_np;
        continue;
      }
    }
    const char *ls, *le;
    if (!next_line(p, e, ls, le)) { fail("non-ASCII or NUL text"); break; }
    const char *sb = ls, *se = le;
    strip(sb, se);
    const size_t n = (size_t)(se - sb);
    if (n == 0) continue;
    if (n == 10 && std::memcmp(sb, "BEGIN IONS", 10) == 0) {
      C.mz.resize(mark);
      C.it.resize(mark);
      inside = true;
      cur_np = 0;
      cur_f = 0;
      cur_z = 0;
      cur_title.clear();
      continue;
    }
    if (n == 8 && std::memcmp(sb, "END IONS", 8) == 0) {
      if (!inside) { fail("END IONS outside a block"); break; }
      C.npk.push_back(cur_np);
      C.prec.push_back((cur_f & 1) ? cur_prec : std::nan(""));
      C.rt.push_back((cur_f & 4) ? cur_rt : std::nan(""));
      C.charge.push_back(cur_z);
      C.flags.push_back(cur_f);
      C.titles += cur_title;
      C.titles += '\n';
      mark = C.mz.size();
      inside = false;
      continue;
    }
    if (!inside) continue;
    const unsigned char c0 = (unsigned char)sb[0];
    const bool digit0 = c0 >= '0' && c0 <= '9';
    const bool signed0 = (c0 == '+' || c0 == '-' || c0 == '.') && n > 1 && sb[1] >= '0' && sb[1] <= '9';
    if (digit0 || signed0) {
      const char* t0 = sb;
      const char* t0e = t0;
      while (t0e < se && !is_ws((unsigned char)*t0e)) ++t0e;
      const char* t1 = t0e;
      while (t1 < se && is_ws((unsigned char)*t1)) ++t1;
      const char* t1e = t1;
      while (t1e < se && !is_ws((unsigned char)*t1e)) ++t1e;
      double a, v = 0.0;
      if (!parse_float(t0, t0e, a) || (t1 < t1e && !parse_float(t1, t1e, v))) { fail("peak value"); break; }
      C.mz.push_back(a);
      C.it.push_back(v);
      ++cur_np;
      continue;
    }
    const char* eq = (const char*)std::memchr(sb, '=', n);
    if (!eq) continue;  // iter_mgf ignores lines that are neither peaks nor params
    const size_t kl = (size_t)(eq - sb);
    auto key_is = [&](const char* k) {
      const size_t m = std::strlen(k);
      if (m != kl) return false;
      for (size_t i = 0; i < m; ++i)
        if (std::tolower((unsigned char)sb[i]) != k[i]) return false;
      return true;
    };
    const char *vb = eq + 1, *ve = se;
    if (key_is("title")) {
      cur_title.assign(vb, ve);
      cur_f |= 8;
    } else if (key_is("pepmass")) {
      const char* a = vb;
      while (a < ve && is_ws((unsigned char)*a)) ++a;
      const char* ae = a;
      while (ae < ve && !is_ws((unsigned char)*ae)) ++ae;
      if (!parse_float(a, ae, cur_prec)) { fail("PEPMASS value"); break; }
      const char* b2 = ae;
      while (b2 < ve && is_ws((unsigned char)*b2)) ++b2;
      const char* b2e = b2;
      while (b2e < ve && !is_ws((unsigned char)*b2e)) ++b2e;
      double pint;
      if (b2 < b2e && !parse_float(b2, b2e, pint)) { fail("PEPMASS intensity"); break; }
      cur_f |= 1;
    } else if (key_is("charge")) {
      if (!parse_one_charge(vb, ve, cur_z)) { fail("CHARGE value"); break; }
      cur_f |= 2;
    } else if (key_is("rtinseconds")) {
      const char *a = vb, *ae = ve;
      strip(a, ae);
      if (!parse_float(a, ae, cur_rt)) { fail("RTINSECONDS value"); break; }
      cur_f |= 4;
    }
  }
  C.mz.resize(mark);
  C.it.resize(mark);
}

// Read-only mapping of a whole file: pages are read on first touch, so a rank
// that indexes one byte stripe of a large MGF reads only that stripe.
struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  std::string error;
  explicit MappedFile(const char* path) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) { error = std::string("cannot open ") + path; return; }
    struct stat st;
    if (::fstat(fd, &st) != 0) { error = "fstat failed"; ::close(fd); return; }
    size = (size_t)st.st_size;
    if (size > 0) {
      void* m = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m == MAP_FAILED) { error = "mmap failed"; size = 0; }
      else data = static_cast<const char*>(m);
    }
    ::close(fd);
  }
  ~MappedFile() {
    if (data) ::munmap(const_cast<char*>(data), size);
  }
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
};

// ------------------------------------------------------------ repr writer
// Python repr(float) into out; returns bytes written.
int py_repr(double x, char* out) {
  if (std::isnan(x)) { std::memcpy(out, "nan", 3); return 3; }
  if (std::isinf(x)) {
    if (x < 0) { std::memcpy(out, "-inf", 4); return 4; }
    std::memcpy(out, "inf", 3);
    return 3;
  }
  char sci[64];
  auto r = std::to_chars(sci, sci + sizeof(sci) - 1, x, std::chars_format::scientific);
  *r.ptr = '\0';  // atoi below reads the exponent up to the terminator
  const char* s = sci;
  const char* end = r.ptr;
  char* o = out;
  if (*s == '-') { *o++ = '-'; ++s; }
  // digits: s[0] [. s[2..epos)] e[+-]XX
  char digs[32];
  int nd = 0;
  const char* ep = (const char*)std::memchr(s, 'e', (size_t)(end - s));
  for (const char* q = s; q < ep; ++q)
    if (*q != '.') digs[nd++] = *q;
  int exp10 = std::atoi(ep + 1);
  while (nd > 1 && digs[nd - 1] == '0') --nd;  // to_chars gives shortest already; be safe
  if (exp10 >= -4 && exp10 < 16) {
    if (exp10 >= nd - 1) {            // integer valued: digits, zeros, ".0"
      for (int i = 0; i < nd; ++i) *o++ = digs[i];
      for (int i = nd - 1; i < exp10; ++i) *o++ = '0';
      *o++ = '.';
      *o++ = '0';
    } else if (exp10 < 0) {           // 0.000ddd
      *o++ = '0';
      *o++ = '.';
      for (int i = -1; i > exp10; --i) *o++ = '0';
      for (int i = 0; i < nd; ++i) *o++ = digs[i];
    } else {                          // ddd.ddd
      for (int i = 0; i <= exp10; ++i) *o++ = digs[i];
      *o++ = '.';
      for (int i = exp10 + 1; i < nd; ++i) *o++ = digs[i];
    }
  } else {
    *o++ = digs[0];
    if (nd > 1) {
      *o++ = '.';
      for (int i = 1; i < nd; ++i) *o++ = digs[i];
    }
    *o++ = 'e';
    *o++ = exp10 < 0 ? '-' : '+';
    int a = exp10 < 0 ? -exp10 : exp10;
    if (a < 10) *o++ = '0';
    char tmp[8];
    int k = std::snprintf(tmp, sizeof(tmp), "%d", a);
    std::memcpy(o, tmp, (size_t)k);
    o += k;
  }
  return (int)(o - out);
}

int64_t format_binning(char* buf, int64_t cap, const char* cid, const char* charge_str, double prec,
                       const double* mz, const double* it, int64_t n, int skip_nan) {
  // worst case per peak: two 24-byte floats + space + newline
  const size_t need = 64 + std::strlen(cid) + std::strlen(charge_str) + (size_t)n * 52;
  if ((int64_t)need > cap) return -1;
  char* o = buf;
  auto put = [&](const char* s) { size_t k = std::strlen(s); std::memcpy(o, s, k); o += k; };
  put("BEGIN IONS\nTITLE=");
  put(cid);
  put("\nPEPMASS=");
  o += py_repr(prec, o);
  put("\nCHARGE=");
  put(charge_str);
  put("+\n");
  for (int64_t k = 0; k < n; ++k) {
    if (skip_nan && std::isnan(it[k])) continue;
    o += py_repr(mz[k], o);
    *o++ = ' ';
    o += py_repr(it[k], o);
    *o++ = '\n';
  }
  put("END IONS\n\n");
  return (int64_t)(o - buf);
}

// ------------------------------------------------------------ record writers
// One output record per cluster, in three text styles:
//   0  binning.py:234-245 -- TITLE=<id>, PEPMASS=repr, CHARGE=<int>+, peaks with
//      NaN intensities skipped (the f-string of numpy floats);
//   1  the gap-average CLI (average_spectrum_clustering.py:207-208 via the shims'
//      write_pyteomics_style): TITLE (if non-empty), PEPMASS, RTINSECONDS,
//      CHARGE=<|z|><+|->, every peak;
//   2  the medoid CLI (most_similar_representative.py:115 via write_record):
//      TITLE, PEPMASS, CHARGE, RTINSECONDS, every peak.
// flags[c] (styles 1-2): bit0 PEPMASS, bit1 CHARGE, bit2 RTINSECONDS, bit3 TITLE
// present (absent fields are omitted).  Floats are Python repr().
struct RecordsIn {
  int style = 0;
  std::vector<const char*> tp;
  std::vector<size_t> tl;
  const int32_t* flags = nullptr;
  const double* prec = nullptr;
  const int64_t* charge = nullptr;
  const double* rt = nullptr;
  const int64_t* off = nullptr;
  const double* mz = nullptr;
  const double* it = nullptr;
};

inline char* put(char* o, const char* s, size_t k) {
  std::memcpy(o, s, k);
  return o + k;
}
inline char* put_int(char* o, long long v) {
  auto r = std::to_chars(o, o + 24, v);
  return r.ptr;
}
inline char* put_repr(char* o, double x) { return o + py_repr(x, o); }

size_t record_cap(size_t title_len, int64_t n) { return 192 + title_len + (size_t)n * 52; }

char* format_record(const RecordsIn& R, int64_t c, char* o) {
  const size_t tl = R.tl[(size_t)c];
  const char* t = R.tp[(size_t)c];
  const int32_t f = R.flags ? R.flags[c] : 0xf;
  const int64_t a = R.off[c], b = R.off[c + 1];
  o = put(o, "BEGIN IONS\n", 11);
  auto title = [&]() { o = put(o, "TITLE=", 6); o = put(o, t, tl); *o++ = '\n'; };
  auto pepmass = [&]() { o = put(o, "PEPMASS=", 8); o = put_repr(o, R.prec[c]); *o++ = '\n'; };
  auto rtsec = [&]() { o = put(o, "RTINSECONDS=", 12); o = put_repr(o, R.rt[c]); *o++ = '\n'; };
  auto charge = [&]() {  // format_charge: |z| then the sign
    const int64_t z = R.charge[c];
    o = put(o, "CHARGE=", 7);
    o = put_int(o, z < 0 ? -z : z);
    *o++ = z < 0 ? '-' : '+';
    *o++ = '\n';
  };
  if (R.style == 0) {
    title();
    pepmass();
    o = put(o, "CHARGE=", 7);
    o = put_int(o, R.charge[c]);
    o = put(o, "+\n", 2);
  } else if (R.style == 1) {
    if ((f & 8) && tl > 0) title();
    if (f & 1) pepmass();
    if (f & 4) rtsec();
    if (f & 2) charge();
  } else {
    if (f & 8) title();
    if (f & 1) pepmass();
    if (f & 2) charge();
    if (f & 4) rtsec();
  }
  const bool skip_nan = R.style == 0;
  for (int64_t k = a; k < b; ++k) {
    if (skip_nan && std::isnan(R.it[k])) continue;
    o = put_repr(o, R.mz[k]);
    *o++ = ' ';
    o = put_repr(o, R.it[k]);
    *o++ = '\n';
  }
  return put(o, "END IONS\n\n", 10);
}

// '\n'-joined strings -> pointers and lengths (C entries)
void split_lines(const char* s, int64_t C, std::vector<const char*>& p, std::vector<size_t>& l) {
  p.resize((size_t)C);
  l.resize((size_t)C);
  for (int64_t c = 0; c < C; ++c) {
    const char* nl = std::strchr(s, '\n');
    p[(size_t)c] = s;
    l[(size_t)c] = nl ? (size_t)(nl - s) : std::strlen(s);
    s = nl ? nl + 1 : s + l[(size_t)c];
  }
}

// Format clusters [0, C) on T threads in blocks, write them in order; the write
// of one round overlaps the formatting of the next.  0, or -1 on an I/O error.
int write_records(FILE* f, const RecordsIn& R, int64_t C, int T) {
  constexpr int64_t kBlock = 2048;
  std::vector<std::string> parts[2];
  parts[0].resize((size_t)T);
  parts[1].resize((size_t)T);
  std::thread writer;
  int rc = 0;
  int cur = 0;
  for (int64_t c0 = 0; c0 < C; c0 += kBlock * T, cur ^= 1) {
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) {
      pool.emplace_back([&, t, c0, cur]() {
        const int64_t a = std::min(C, c0 + t * kBlock), b = std::min(C, a + kBlock);
        std::string& out = parts[cur][(size_t)t];
        size_t cap = 0;
        for (int64_t c = a; c < b; ++c) cap += record_cap(R.tl[(size_t)c], R.off[c + 1] - R.off[c]);
        out.resize(cap);
        char* o = &out[0];
        for (int64_t c = a; c < b; ++c) o = format_record(R, c, o);
        out.resize((size_t)(o - out.data()));
      });
    }
    for (auto& th : pool) th.join();
    if (writer.joinable()) writer.join();
    writer = std::thread([&, cur]() {
      for (auto& s : parts[cur])
        if (!s.empty() && std::fwrite(s.data(), 1, s.size(), f) != s.size()) rc = -1;
    });
  }
  if (writer.joinable()) writer.join();
  return rc;
}

// Spectrum record start lines: "TITLE=" (binning.py's parser starts a peaklist
// there) or a stripped "BEGIN IONS" (general MGF).
inline bool record_start(const char* q, const char* e, int general) {
  if (!general) return e - q >= 6 && std::memcmp(q, "TITLE=", 6) == 0;
  const char* a = q;
  const char* le = (const char*)std::memchr(q, '\n', (size_t)(e - q));
  const char* b = le ? le : e;
  strip(a, b);
  return b - a == 10 && std::memcmp(a, "BEGIN IONS", 10) == 0;
}

// Per-thread byte ranges of [b, e) that begin at record starts.
std::vector<const char*> split_records(const char* b, const char* e, int T, int general) {
  std::vector<const char*> cuts{b};
  const size_t size = (size_t)(e - b);
  for (int t = 1; t < T; ++t) {
    const char* q = b + size * (size_t)t / (size_t)T;
    if (q <= cuts.back()) continue;
    while (q < e) {
      const char* nl = (const char*)std::memchr(q, '\n', (size_t)(e - q));
      if (!nl) { q = e; break; }
      q = nl + 1;
      if (record_start(q, e, general)) break;
    }
    if (q < e && q > cuts.back()) cuts.push_back(q);
  }
  cuts.push_back(e);
  return cuts;
}

// Take the threads' chunks as the result (first error wins; no copy).
void adopt(std::vector<Chunk>&& chunks, Result* R, bool with_rt) {
  for (auto& c : chunks)
    if (!c.error.empty()) { R->error = c.error; return; }
  R->parts = std::move(chunks);
  R->with_rt = with_rt;
  R->s_base.assign(R->parts.size() + 1, 0);
  R->p_base.assign(R->parts.size() + 1, 0);
  for (size_t i = 0; i < R->parts.size(); ++i) {
    R->s_base[i + 1] = R->s_base[i] + (int64_t)R->parts[i].npk.size();
    R->p_base[i + 1] = R->p_base[i] + (int64_t)R->parts[i].mz.size();
  }
  R->S = R->s_base.back();
  R->P = R->p_base.back();
}

// f(part index) on one thread per part
template <class F>
void for_parts(const Result* R, F&& f) {
  std::vector<std::thread> pool;
  for (size_t i = 0; i < R->parts.size(); ++i) pool.emplace_back(f, i);
  for (auto& th : pool) th.join();
}

void build_titles(Result* R) {
  if (R->titles_built) return;
  size_t n = 0;
  for (auto& c : R->parts) n += c.titles.size();
  R->titles.reserve(n);
  for (auto& c : R->parts) R->titles += c.titles;
  R->title_off.assign((size_t)R->S + 1, 0);
  int64_t s = 0;
  for (size_t k = 0; k < R->titles.size(); ++k)
    if (R->titles[k] == '\n') R->title_off[(size_t)++s] = (int64_t)k + 1;
  R->titles_built = true;
}

int default_threads(int threads) {
  return threads > 0 ? threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// Record index: where each spectrum record starts and ends, its title, peaks.
struct Index {
  std::vector<int64_t> begin, end, npk;
  std::string titles, error;
};

// Is `q` (inside [b, e)) the start of a line?  Lines end at \n, \r\n or \r
// (Python's universal newlines, as the parsers split them).
inline bool line_start(const char* b, const char* e, const char* q) {
  if (q == b) return true;
  if (q[-1] == '\n') return true;
  return q[-1] == '\r' && (q == e || *q != '\n');
}

// Index the records whose start line begins in [b + lo, b + hi) of the file
// [b, b + size); a record runs to the next record start (possibly past hi) or EOF.
void index_span(const char* b, size_t size, size_t lo, size_t hi, int general, Index& X) {
  const char* e = b + size;
  const char* p = b + lo;
  const char* stop = b + hi;
  while (p < e && !line_start(b, e, p)) ++p;  // resync to a line start
  int64_t rb = -1, np = 0;
  bool has_end = false;
  std::string title;
  auto close = [&](int64_t at) {
    if (rb >= 0 && has_end) {
      X.begin.push_back(rb);
      X.end.push_back(at);
      X.npk.push_back(np);
      X.titles += title;
      X.titles += '\n';
    }
  };
  while (p < e) {
    const char* ls = p;
    const char* le = p;
    while (le < e && *le != '\n' && *le != '\r') ++le;
    p = le;
    if (p < e) {
      if (*p == '\r') { ++p; if (p < e && *p == '\n') ++p; }
      else ++p;
    }
    if (record_start(ls, le, general)) {
      if (ls >= stop) { close(ls - b); return; }  // the next stripe's first record
      close(ls - b);
      rb = ls - b;
      np = 0;
      has_end = false;
      title.clear();
    }
    if (rb < 0) continue;  // before this stripe's first record: the previous stripe's
    const char *sb = ls, *se = le;
    strip(sb, se);
    if (!has_end && se - sb >= 6 && (general ? (std::tolower((unsigned char)sb[0]) == 't' && std::tolower((unsigned char)sb[1]) == 'i' &&
                                    std::tolower((unsigned char)sb[2]) == 't' && std::tolower((unsigned char)sb[3]) == 'l' &&
                                    std::tolower((unsigned char)sb[4]) == 'e' && sb[5] == '=')
                                 : std::memcmp(ls, "TITLE=", 6) == 0)) {
      const char *tb = (general ? sb : ls) + 6, *te = general ? se : le;
      if (!general) strip(tb, te);
      title.assign(tb, te);
      // titles cross the ABI NUL-terminated and '\n'-joined: a NUL would cut the rest
      if (std::memchr(tb, 0, (size_t)(te - tb)) && X.error.empty()) X.error = "fallback: NUL byte in a TITLE";
    } else if (se - sb == 8 && std::memcmp(sb, "END IONS", 8) == 0) {
      has_end = true;
    } else if (se > sb && ((*(general ? sb : ls) >= '0' && *(general ? sb : ls) <= '9') ||
                           (general && (*sb == '+' || *sb == '-' || *sb == '.') && se - sb > 1 && sb[1] >= '0' &&
                            sb[1] <= '9'))) {
      ++np;
    }
  }
  close(e - b);
}

// [lo, hi) indexed by T threads over sub-stripes (they compose: every record is
// listed by the sub-stripe its start line lies in), merged in file order.
void index_stripes(const char* b, size_t size, size_t lo, size_t hi, int general, int T, Index& X) {
  T = std::max(1, T);
  std::vector<Index> parts((size_t)T);
  std::vector<std::thread> pool;
  for (int t = 0; t < T; ++t) {
    const size_t a = lo + (hi - lo) * (size_t)t / (size_t)T, z = lo + (hi - lo) * (size_t)(t + 1) / (size_t)T;
    if (T == 1) index_span(b, size, a, z, general, parts[0]);
    else pool.emplace_back(index_span, b, size, a, z, general, std::ref(parts[(size_t)t]));
  }
  for (auto& th : pool) th.join();
  for (auto& x : parts) {
    X.begin.insert(X.begin.end(), x.begin.begin(), x.begin.end());
    X.end.insert(X.end.end(), x.end.begin(), x.end.end());
    X.npk.insert(X.npk.end(), x.npk.begin(), x.npk.end());
    X.titles += x.titles;
    if (X.error.empty()) X.error = x.error;
  }
}

}  // namespace

extern "C" {

void* spx_mgf_parse(const char* path, int threads) {
  Result* R = new Result();
  MappedFile mf(path);
  if (!mf.error.empty()) { R->error = mf.error; return R; }
  const char* b = mf.data;
  const char* e = b + mf.size;
  int T = default_threads(threads);
  if (mf.size < (1u << 20)) T = 1;
  // per-thread ranges start at "TITLE=" lines (the reference resets its state there)
  const std::vector<const char*> cuts = split_records(b, e, T, 0);
  const int nc = (int)cuts.size() - 1;
  std::vector<Chunk> chunks((size_t)nc);
  std::vector<std::thread> pool;
  for (int i = 0; i < nc; ++i) pool.emplace_back(parse_range, cuts[i], cuts[i + 1], std::ref(chunks[(size_t)i]));
  for (auto& th : pool) th.join();
  adopt(std::move(chunks), R, false);
  return R;
}

const char* spx_mgf_error(void* h) {
  Result* R = static_cast<Result*>(h);
  return R->error.empty() ? nullptr : R->error.c_str();
}
int64_t spx_mgf_n_spectra(void* h) { return static_cast<Result*>(h)->S; }
int64_t spx_mgf_n_peaks(void* h) { return static_cast<Result*>(h)->P; }
void spx_mgf_copy(void* h, int64_t* spec_off, double* mz, double* it, double* prec, int64_t* charge, int32_t* flags) {
  Result* R = static_cast<Result*>(h);
  spec_off[0] = 0;
  for_parts(R, [&](size_t i) {  // each part straight into its slice of the caller's arrays
    const Chunk& c = R->parts[i];
    const int64_t sb = R->s_base[i], pb = R->p_base[i];
    int64_t o = pb;
    for (size_t k = 0; k < c.npk.size(); ++k) spec_off[sb + (int64_t)k + 1] = (o += c.npk[k]);
    if (!c.mz.empty()) {
      std::memcpy(mz + pb, c.mz.data(), c.mz.size() * sizeof(double));
      std::memcpy(it + pb, c.it.data(), c.it.size() * sizeof(double));
    }
    std::copy(c.prec.begin(), c.prec.end(), prec + sb);
    std::copy(c.charge.begin(), c.charge.end(), charge + sb);
    std::copy(c.flags.begin(), c.flags.end(), flags + sb);
  });
}
const char* spx_mgf_titles(void* h) {
  Result* R = static_cast<Result*>(h);
  build_titles(R);
  return R->titles.c_str();
}
void spx_mgf_free(void* h) { delete static_cast<Result*>(h); }
void spx_mgf_copy_rt(void* h, double* rt) {
  Result* R = static_cast<Result*>(h);
  for (size_t i = 0; i < R->parts.size(); ++i) {
    const Chunk& c = R->parts[i];
    if (R->with_rt) std::copy(c.rt.begin(), c.rt.end(), rt + R->s_base[i]);
    else std::fill(rt + R->s_base[i], rt + R->s_base[i + 1], std::nan(""));
  }
}

// The three CLIs' cluster groupings of a parse, from the titles' cluster ids
// (TITLE up to the first ';'), without handing every title to the
// caller.  key[s] per spectrum:
//   mode 0 (binning.py:160-165): the id's ordinal in first-appearance order;
//   mode 1 (average_spectrum_clustering.py:158, itertools.groupby): the ordinal of
//          the consecutive run s is in;
//   mode 2 (most_similar_representative.py:49-75): the id's ordinal if s lies in the
//          id's FIRST contiguous run (the run the reference's range_start scan finds:
//          ids are taken in first-appearance order, so each scan starts before that
//          id's first appearance), else -1.
// Returns the number of groups (ids available from spx_mgf_group_ids), -1 on a bad mode.
int64_t spx_mgf_group(void* h, int mode, int64_t* key) {
  Result* R = static_cast<Result*>(h);
  if (mode < 0 || mode > 2) return -1;
  build_titles(R);
  R->group_ids.clear();
  std::unordered_map<std::string_view, int64_t> seen;
  seen.reserve((size_t)R->S / 4 + 16);
  std::string_view prev;
  int64_t n = 0, cur = -1, run = -1;
  for (int64_t s = 0; s < R->S; ++s) {
    const char* t = R->titles.data() + R->title_off[(size_t)s];
    const size_t len = (size_t)(R->title_off[(size_t)s + 1] - R->title_off[(size_t)s] - 1);
    const char* semi = static_cast<const char*>(std::memchr(t, ';', len));
    const std::string_view id(t, semi ? (size_t)(semi - t) : len);
    if (mode == 1) {
      if (s == 0 || id != prev) {
        ++run;
        R->group_ids.append(id.data(), id.size());
        R->group_ids += '\n';
      }
      key[s] = run;
      prev = id;
      continue;
    }
    auto it = seen.find(id);
    if (it == seen.end()) {
      it = seen.emplace(id, n++).first;
      R->group_ids.append(id.data(), id.size());
      R->group_ids += '\n';
      cur = it->second;  // a new id's first run starts here
      key[s] = it->second;
    } else if (mode == 0) {
      key[s] = it->second;
    } else if (it->second == cur) {
      key[s] = cur;  // its first run goes on
    } else {
      key[s] = -1;  // a later run: the reference never reaches it
      cur = -1;
    }
  }
  return mode == 1 ? run + 1 : n;
}
const char* spx_mgf_group_ids(void* h) { return static_cast<Result*>(h)->group_ids.c_str(); }
// Title offsets into spx_mgf_titles' string: title s = [off[s], off[s+1] - 1).
void spx_mgf_title_offsets(void* h, int64_t* off) {
  Result* R = static_cast<Result*>(h);
  build_titles(R);
  std::copy(R->title_off.begin(), R->title_off.end(), off);
}

// General MGF (pyteomics-shaped subset, see parse_range_general): same result
// accessors as spx_mgf_parse, plus spx_mgf_copy_rt (NaN where absent); prec is
// NaN without PEPMASS; flags bit0 PEPMASS, bit1 CHARGE, bit2 RTINSECONDS, bit3 TITLE.
void* spx_mgf_parse_general(const char* path, int threads) {
  Result* R = new Result();
  MappedFile mf(path);
  if (!mf.error.empty()) { R->error = mf.error; return R; }
  const char* b = mf.data;
  const char* e = b + mf.size;
  int T = default_threads(threads);
  if (mf.size < (1u << 20)) T = 1;
  const std::vector<const char*> cuts = split_records(b, e, T, 1);
  const int nc = (int)cuts.size() - 1;
  std::vector<GenChunk> chunks((size_t)nc);
  std::vector<std::thread> pool;
  for (int i = 0; i < nc; ++i)
    pool.emplace_back(parse_range_general, cuts[i], cuts[i + 1], std::ref(chunks[(size_t)i]));
  for (auto& th : pool) th.join();
  adopt(std::move(chunks), R, true);
  return R;
}

// Record index of an MGF without parsing numbers (the sharded CLIs' planning
// pass): record r = bytes [begin[r], end[r]) from its start line ("TITLE=" for
// general == 0, binning.py's reader; "BEGIN IONS" for general == 1) to the next
// record's start, its title (the TITLE= value, stripped) and its peak-line count.
// Only records holding an END IONS line are listed (the ones a parser stores).
// threads <= 0: min(16, hardware threads); the file is indexed in byte stripes.
void* spx_mgf_index(const char* path, int general) {
  Index* X = new Index();
  MappedFile mf(path);
  if (!mf.error.empty()) { X->error = mf.error; return X; }
  index_stripes(mf.data, mf.size, 0, mf.size, general, mf.size < (1u << 20) ? 1 : default_threads(0), *X);
  return X;
}

// The records of spx_mgf_index whose start line begins in bytes [lo, hi) -- a
// rank-local slice of the index: ranks indexing [k*size/W, (k+1)*size/W) list
// every record exactly once, and each reads its stripe plus the tail of its last
// record.  hi is clamped to the file size.
void* spx_mgf_index_range(const char* path, int general, int64_t lo, int64_t hi, int threads) {
  Index* X = new Index();
  MappedFile mf(path);
  if (!mf.error.empty()) { X->error = mf.error; return X; }
  if (lo < 0 || hi < lo) { X->error = "bad byte range"; return X; }
  const size_t l = std::min((size_t)lo, mf.size), h = std::min((size_t)hi, mf.size);
  index_stripes(mf.data, mf.size, l, h, general, (h - l) < (1u << 20) ? 1 : default_threads(threads), *X);
  return X;
}

const char* spx_mgf_index_error(void* h) {
  Index* X = static_cast<Index*>(h);
  return X->error.empty() ? nullptr : X->error.c_str();
}
int64_t spx_mgf_index_n(void* h) { return (int64_t)static_cast<Index*>(h)->begin.size(); }
void spx_mgf_index_copy(void* h, int64_t* begin, int64_t* end, int64_t* npk) {
  Index* X = static_cast<Index*>(h);
  std::copy(X->begin.begin(), X->begin.end(), begin);
  std::copy(X->end.begin(), X->end.end(), end);
  std::copy(X->npk.begin(), X->npk.end(), npk);
}
const char* spx_mgf_index_titles(void* h) { return static_cast<Index*>(h)->titles.c_str(); }
void spx_mgf_index_free(void* h) { delete static_cast<Index*>(h); }

// Parse only the records [begin[r], end[r]) (any order: the result follows it),
// with the binning (general == 0) or the general parser.  A rank of a sharded CLI
// reads its own clusters' spectra this way and nothing else.
void* spx_mgf_parse_ranges(const char* path, const int64_t* begin, const int64_t* end, int64_t n, int general,
                           int threads) {
  Result* R = new Result();
  FILE* f = std::fopen(path, "rb");
  if (!f) { R->error = std::string("cannot open ") + path; return R; }
  // read the records into one buffer (in the requested order)
  std::vector<int64_t> at((size_t)n + 1, 0);
  for (int64_t r = 0; r < n; ++r) {
    if (begin[r] < 0 || end[r] < begin[r]) { std::fclose(f); R->error = "bad record range"; return R; }
    at[(size_t)r + 1] = at[(size_t)r] + (end[r] - begin[r]);
  }
  std::string data((size_t)at[(size_t)n], '\0');
  for (int64_t r = 0; r < n && R->error.empty();) {
    int64_t q = r + 1;  // coalesce records adjacent in the file into one read
    while (q < n && begin[q] == end[q - 1]) ++q;
    const int64_t len = end[q - 1] - begin[r];
    if (len > 0 && (std::fseek(f, (long)begin[r], SEEK_SET) != 0 ||
                    std::fread(&data[(size_t)at[(size_t)r]], 1, (size_t)len, f) != (size_t)len))
      R->error = "short read";
    r = q;
  }
  std::fclose(f);
  if (!R->error.empty()) return R;
  int T = default_threads(threads);
  if (data.size() < (1u << 20)) T = 1;
  T = (int)std::min<int64_t>(T, std::max<int64_t>(n, 1));
  // thread t parses whole records [rs[t], rs[t+1])
  std::vector<const char*> cuts{data.data()};
  for (int t = 1; t < T; ++t) {
    const int64_t r = n * t / T;
    const char* q = data.data() + at[(size_t)r];
    if (q > cuts.back()) cuts.push_back(q);
  }
  cuts.push_back(data.data() + data.size());
  const int nc = (int)cuts.size() - 1;
  std::vector<std::thread> pool;
  if (general) {
    std::vector<GenChunk> chunks((size_t)nc);
    for (int i = 0; i < nc; ++i)
      pool.emplace_back(parse_range_general, cuts[i], cuts[i + 1], std::ref(chunks[(size_t)i]));
    for (auto& th : pool) th.join();
    adopt(std::move(chunks), R, true);
  } else {
    std::vector<Chunk> chunks((size_t)nc);
    for (int i = 0; i < nc; ++i) pool.emplace_back(parse_range, cuts[i], cuts[i + 1], std::ref(chunks[(size_t)i]));
    for (auto& th : pool) th.join();
    adopt(std::move(chunks), R, false);
  }
  if (R->error.empty() && R->S != n) R->error = "fallback: records and parsed spectra differ";
  return R;
}

int64_t spx_mgf_format_binning(char* buf, int64_t cap, const char* cid, const char* charge_str, double prec,
                               const double* mz, const double* it, int64_t n, int skip_nan) {
  return format_binning(buf, cap, cid, charge_str, prec, mz, it, n, skip_nan);
}

int spx_py_repr(double x, char* out) { return py_repr(x, out); }

// Write C consensus spectra (dense layout: cluster c = peaks [off[c], off[c+1]))
// as binning.py:234-245 text, formatted in parallel, written in order.
// ids: '\n'-joined cluster ids.  Returns 0, or -1 on an I/O error.
int spx_mgf_write_binning_batch(const char* path, int64_t C, const char* ids, const int64_t* charge,
                                const double* prec, const int64_t* off, const double* mz, const double* it,
                                int threads) {
  return spx_mgf_write_records(path, 0, 0, C, ids, nullptr, prec, charge, nullptr, off, mz, it, threads);
}

// C records in one of the styles of format_record (0 binning, 1 gap-average,
// 2 medoid), titles '\n'-joined, record c's peaks [off[c], off[c+1]) of mz / it.
// append: open with "ab" (the gap-average CLI's --append).  0, or -1 on an I/O
// error or a bad argument.
int spx_mgf_write_records(const char* path, int append, int style, int64_t C, const char* titles,
                          const int32_t* flags, const double* prec, const int64_t* charge, const double* rt,
                          const int64_t* off, const double* mz, const double* it, int threads) {
  if (C < 0 || style < 0 || style > 2 || (C > 0 && (!titles || !prec || !charge || !off || !mz || !it)) ||
      (style != 0 && C > 0 && (!flags || !rt)))
    return -1;
  RecordsIn R;
  R.style = style;
  split_lines(titles ? titles : "", C, R.tp, R.tl);
  R.flags = flags;
  R.prec = prec;
  R.charge = charge;
  R.rt = rt;
  R.off = off;
  R.mz = mz;
  R.it = it;
  FILE* f = std::fopen(path, append ? "ab" : "wb");
  if (!f) return -1;
  int rc = write_records(f, R, C, default_threads(threads));
  if (std::fclose(f) != 0) rc = -1;
  return rc;
}

}  // extern "C"
