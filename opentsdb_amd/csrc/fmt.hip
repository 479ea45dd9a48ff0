// fmt.hip — host-side output formatting of SpanGroup results (SURVEY.md §8(f)
// rank 4): the text the reference's consumers write for every DataPoint.
//
//   TSDBHIP_FMT_ASCII    GraphHandler.respondAsciiQuery (GraphHandler.java:785-808):
//                        metric ' ' timestamp ' ' value tags '\n'
//   TSDBHIP_FMT_GNUPLOT  Plot.dumpToFiles (Plot.java:190-204):
//                        (timestamp + utc_offset) ' ' value '\n'
//   TSDBHIP_FMT_CLI      CliQuery (CliQuery.java:161-170):
//                        metric ' ' timestamp ' ' value ' ' tagz '\n',
//                        doubles as String.format("%f")
//
// Longs print as Long.toString. Doubles print as Double.toString (ASCII,
// GNUPLOT): the shortest decimal of at least two significant digits that
// rounds to the double (the closest one on ties of length), plain notation for
// 1e-3 <= |v| < 1e7 with at least one fractional digit, else d.dddE[-]n —
// the JDK 19+ specification of Double.toString. For CLI, "%f" rounds that
// decimal half-up to six fractional digits (java.util.Formatter). The tag
// strings come from the caller (UID lookups and HashMap order stay in Java).
// Runs on the host cores: chunks of points formatted by parallel threads
// into per-chunk buffers, then concatenated.
#include <charconv>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace fmtq {

// shortest round-trip digits of |v| (v finite, nonzero): digits, exponent E
// with |v| ~ d1.d2d3... x 10^E
static void shortest(double v, char* dig, int* nd, int* E, bool min2) {
  char b[64];
  auto r = std::to_chars(b, b + sizeof b, std::fabs(v), std::chars_format::scientific);
  *r.ptr = 0;
  // b = "d[.ddd]e[+-]xx"
  int n = 0;
  const char* p = b;
  for (; *p && *p != 'e'; p++)
    if (*p != '.') dig[n++] = *p;
  *E = atoi(p + 1);
  if (n == 1 && min2) {
    // length >= 2: the 2-digit decimal closest to v (rounds to v, since the
    // 1-digit one does and it is at least as close)
    auto r2 = std::to_chars(b, b + sizeof b, std::fabs(v), std::chars_format::scientific, 1);
    *r2.ptr = 0;
    n = 0;
    for (p = b; *p && *p != 'e'; p++)
      if (*p != '.') dig[n++] = *p;
    *E = atoi(p + 1);
  }
  while (n > 1 && dig[n - 1] == '0') n--;  // "1.0E10" keeps its one digit; zeros come back below
  *nd = n;
}

// Double.toString
static void java_double(double v, std::string& o) {
  if (v != v) { o += "NaN"; return; }
  if (std::isinf(v)) { o += v > 0 ? "Infinity" : "-Infinity"; return; }
  if (v == 0) { o += std::signbit(v) ? "-0.0" : "0.0"; return; }
  if (v < 0) o += '-';
  char dig[40];
  int n, E;
  shortest(v, dig, &n, &E, true);
  const double a = std::fabs(v);
  if (a >= 1e-3 && a < 1e7) {
    if (E >= 0) {
      for (int i = 0; i <= E; i++) o += i < n ? dig[i] : '0';
      o += '.';
      if (n > E + 1) o.append(dig + E + 1, n - E - 1);
      else o += '0';
    } else {
      o += "0.";
      for (int i = 0; i < -E - 1; i++) o += '0';
      o.append(dig, n);
    }
  } else {
    o += dig[0];
    o += '.';
    if (n > 1) o.append(dig + 1, n - 1);
    else o += '0';
    o += 'E';
    o += std::to_string(E);
  }
}

// String.format("%f", v): the decimal digits rounded HALF_UP to 6 places
static void java_pct_f(double v, std::string& o) {
  if (v != v) { o += "NaN"; return; }
  if (std::isinf(v)) { o += v > 0 ? "Infinity" : "-Infinity"; return; }
  if (std::signbit(v)) o += '-';
  if (v == 0) { o += "0.000000"; return; }
  char dig[40];
  int n, E;
  shortest(v, dig, &n, &E, false);
  // fixed digits: integer part (E+1 digits, >= 1) and 6 fractional digits
  std::vector<int> d;  // all digits from the highest integer digit down to 10^-7
  const int hi = std::max(E, 0);
  for (int pos = hi; pos >= -7; pos--) {
    const int idx = E - pos;  // index into dig
    d.push_back(idx >= 0 && idx < n ? dig[idx] - '0' : 0);
  }
  // any nonzero digit below 10^-7 does not matter for HALF_UP at 10^-6 except
  // through the 10^-7 digit itself (>= 5 rounds up)
  const int last = (int)d.size() - 1;  // the 10^-7 digit
  bool up = d[last] >= 5;
  d.pop_back();
  for (int i = (int)d.size() - 1; up && i >= 0; i--) {
    if (++d[i] == 10) d[i] = 0; else up = false;
  }
  if (up) o += '1';
  const int nint = hi + 1;
  for (int i = 0; i < (int)d.size(); i++) {
    if (i == nint) o += '.';
    o += (char)('0' + d[i]);
  }
}

static void append_long(int64_t x, std::string& o) {
  char b[24];
  auto r = std::to_chars(b, b + sizeof b, (long long)x);
  o.append(b, r.ptr - b);
}

}  // namespace fmtq

extern "C" int64_t tsdbhip_format_points(int32_t mode, const char* metric, const char* tags, int64_t utc_offset,
                                         const int64_t* ts, const uint8_t* is_int, const int64_t* bits, uint64_t n,
                                         char* buf, uint64_t cap) {
  if (mode < TSDBHIP_FMT_ASCII || mode > TSDBHIP_FMT_CLI || (n && (!ts || !is_int || !bits)) || (cap && !buf))
    return TSDBHIP_E_INVALID_ARG;
  if (mode != TSDBHIP_FMT_GNUPLOT && !metric) return TSDBHIP_E_INVALID_ARG;
  // GraphHandler / Plot throw IllegalStateException on NaN / Infinity
  if (mode != TSDBHIP_FMT_CLI)
    for (uint64_t i = 0; i < n; i++)
      if (!is_int[i]) {
        double v;
        std::memcpy(&v, &bits[i], 8);
        if (v != v || std::isinf(v)) return TSDBHIP_E_NAN_INF;
      }
  const uint64_t chunk = 1u << 16;
  const uint64_t nch = (n + chunk - 1) / chunk;
  std::vector<std::string> parts(nch);
  auto work = [&](uint64_t c0, uint64_t c1) {
    for (uint64_t c = c0; c < c1; c++) {
      std::string& o = parts[c];
      o.reserve(48 * chunk);
      const uint64_t e = std::min(n, (c + 1) * chunk);
      for (uint64_t i = c * chunk; i < e; i++) {
        if (mode != TSDBHIP_FMT_GNUPLOT) {
          o += metric;
          o += ' ';
        }
        fmtq::append_long(mode == TSDBHIP_FMT_GNUPLOT ? (int64_t)((uint64_t)ts[i] + (uint64_t)utc_offset) : ts[i], o);
        o += ' ';
        if (is_int[i]) {
          fmtq::append_long(bits[i], o);
        } else {
          double v;
          std::memcpy(&v, &bits[i], 8);
          if (mode == TSDBHIP_FMT_CLI) fmtq::java_pct_f(v, o);
          else fmtq::java_double(v, o);
        }
        if (mode == TSDBHIP_FMT_ASCII && tags) o += tags;
        if (mode == TSDBHIP_FMT_CLI) {
          o += ' ';
          if (tags) o += tags;
        }
        o += '\n';
      }
    }
  };
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned nt = (unsigned)std::min<uint64_t>(hw, nch);
  if (nt <= 1) {
    work(0, nch);
  } else {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++) th.emplace_back(work, nch * t / nt, nch * (t + 1) / nt);
    for (auto& x : th) x.join();
  }
  uint64_t total = 0;
  for (auto& p : parts) total += p.size();
  if (total > cap) return TSDBHIP_E_CAPACITY;
  uint64_t off = 0;
  for (auto& p : parts) {
    std::memcpy(buf + off, p.data(), p.size());
    off += p.size();
  }
  return (int64_t)total;
}
