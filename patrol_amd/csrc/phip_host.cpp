// Host-side pieces of the drop-in boundary that need no GPU: Patrol's rate
// parser, the wire encoder used for egress (unicast replies / broadcast), and
// the API.takeBucket handler logic running over the engine.
//
// ParseRate (bucket.go:102-123) is only ever used with its error ignored
// (api.go:61), so what matters is the Rate value Go returns beside each
// error; this file reproduces strconv.Atoi / time.ParseDuration closely
// enough to return the same values (tests/test_host.py checks every case of
// tests/golden/parse_rate.json).
#include <cstdint>
#include <cstring>
#include <string>

#include "patrolhip.h"
#include "phip_host.hpp"

namespace {

using u64 = uint64_t;
using i64 = int64_t;

struct Cursor {
  const char* p;
  const char* end;
  bool done() const { return p == end; }
  char peek() const { return *p; }
  bool digit() const { return p != end && *p >= '0' && *p <= '9'; }
};

// strconv.Atoi for 64-bit int: {value, ok}.  Syntax errors give 0, range
// errors the clamped bound (strconv.ParseInt semantics).
bool atoi64(const char* s, size_t n, i64* out) {
  *out = 0;
  if (n == 0) return false;
  size_t k = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; k = 1; }
  if (k == n) return false;
  // Unsigned accumulate with left-to-right error detection (ParseUint).
  u64 acc = 0;
  bool range = false;
  for (; k < n; ++k) {
    unsigned d = (unsigned char)s[k] - '0';
    if (d > 9) return false;                       // syntax error -> 0
    if (acc > (UINT64_MAX - d) / 10) { range = true; break; }
    acc = acc * 10 + d;
  }
  // The short fast path of Atoi (len < 19) can neither overflow nor differ.
  const u64 lim = 1ull << 63;
  if (range || (!neg && acc >= lim) || (neg && acc > lim)) {
    *out = neg ? INT64_MIN : INT64_MAX;
    return false;
  }
  *out = neg ? (i64)(0 - acc) : (i64)acc;
  return true;
}

u64 unit_ns(const char* u, size_t n, bool* ok) {
  struct { const char* s; u64 v; } tab[] = {
      {"ns", 1ull}, {"us", 1000ull}, {"\xC2\xB5s", 1000ull}, {"\xCE\xBCs", 1000ull},
      {"ms", 1000000ull}, {"s", 1000000000ull}, {"m", 60000000000ull}, {"h", 3600000000000ull}};
  for (auto& e : tab)
    if (strlen(e.s) == n && memcmp(e.s, u, n) == 0) { *ok = true; return e.v; }
  *ok = false;
  return 0;
}

// time.ParseDuration: {ns, ok}; every error yields 0.
bool parse_duration(const char* s, size_t n, i64* out) {
  *out = 0;
  Cursor c{s, s + n};
  bool neg = false;
  if (!c.done() && (c.peek() == '-' || c.peek() == '+')) { neg = c.peek() == '-'; ++c.p; }
  if (c.end - c.p == 1 && c.peek() == '0') return true;
  if (c.done()) return false;
  const u64 two63 = 1ull << 63;
  u64 total = 0;
  while (!c.done()) {
    if (!(c.peek() == '.' || c.digit())) return false;
    u64 whole = 0;
    const char* start = c.p;
    while (c.digit()) {
      if (whole > two63 / 10) return false;
      whole = whole * 10 + (u64)(c.peek() - '0');
      if (whole > two63) return false;
      ++c.p;
    }
    bool had_whole = c.p != start;
    u64 frac = 0;
    double scale = 1.0;
    bool had_frac = false;
    if (!c.done() && c.peek() == '.') {
      ++c.p;
      const char* fs = c.p;
      bool stop = false;
      while (c.digit()) {
        if (!stop) {
          u64 nx = frac * 10 + (u64)(c.peek() - '0');
          if (frac > (two63 - 1) / 10 || nx > two63) stop = true;
          else { frac = nx; scale *= 10; }
        }
        ++c.p;
      }
      had_frac = c.p != fs;
    }
    if (!had_whole && !had_frac) return false;
    const char* us = c.p;
    while (!c.done() && c.peek() != '.' && !c.digit()) ++c.p;
    if (c.p == us) return false;
    bool uok;
    u64 unit = unit_ns(us, (size_t)(c.p - us), &uok);
    if (!uok) return false;
    if (whole > two63 / unit) return false;
    whole *= unit;
    if (frac > 0) {
      whole += (u64)((double)frac * ((double)unit / scale));
      if (whole > two63) return false;
    }
    total += whole;
    if (total > two63) return false;
  }
  if (neg) { *out = (i64)(0 - total); return true; }
  if (total > two63 - 1) return false;
  *out = (i64)total;
  return true;
}

// strconv.ParseUint(s, 10, 64): syntax error 0, range error MaxUint64.
u64 parse_count(const char* s, size_t n) {
  if (n == 0) return 0;
  u64 acc = 0;
  for (size_t k = 0; k < n; ++k) {
    unsigned d = (unsigned char)s[k] - '0';
    if (d > 9) return 0;
    if (acc > (UINT64_MAX - d) / 10) return UINT64_MAX;
    acc = acc * 10 + d;
  }
  return acc;
}

}  // namespace

namespace phip_host {

int api_prepare(const uint8_t* name, uint32_t len, const char* rate, uint32_t rate_len,
                const char* count, uint32_t count_len, int64_t* freq, int64_t* per, uint64_t* n,
                char* body, uint32_t* body_len) {
  (void)name;
  if (len > PHIP_MAX_NAME_LEN) {                                  // api.go:55-58
    static const char msg[] = "bucket name larger than 231";
    memcpy(body, msg, sizeof msg - 1);
    *body_len = sizeof msg - 1;
    return 400;
  }
  phip_parse_rate(rate, rate_len, freq, per);                     // api.go:61, error ignored
  *n = parse_count(count, count_len);                             // api.go:62-65
  if (*n == 0) *n = 1;
  return 0;
}

}  // namespace phip_host

extern "C" {

int phip_parse_rate(const char* s, uint32_t len, int64_t* freq, int64_t* per) {
  *freq = 0;
  *per = 0;
  if (!s && len) return PHIP_ERR_INVALID;
  const char* colon = len ? (const char*)memchr(s, ':', len) : nullptr;
  size_t flen = colon ? (size_t)(colon - s) : len;
  if (!atoi64(s, flen, freq)) return PHIP_ERR_INVALID;
  std::string unit = colon ? std::string(colon + 1, s + len) : std::string("1s");
  // bucket.go:117: a bare unit means one of it (micro sign U+00B5 only).
  static const char* bare[] = {"ns", "us", "\xC2\xB5s", "ms", "s", "m", "h"};
  for (const char* b : bare)
    if (unit == b) { unit = "1" + unit; break; }
  return parse_duration(unit.data(), unit.size(), per) ? PHIP_OK : PHIP_ERR_INVALID;
}

int phip_marshal(const uint8_t* name, uint32_t len, const phip_state* st, uint8_t* out) {
  if (!st || !out || (!name && len)) return PHIP_ERR_INVALID;
  if (len > PHIP_MAX_NAME_LEN) return PHIP_ERR_NAME_TOO_LARGE;   // bucket.go:54-57
  const u64 words[3] = {st->added, st->taken, (u64)st->elapsed};
  for (int w = 0; w < 3; ++w)
    for (int b = 0; b < 8; ++b) out[w * 8 + b] = (uint8_t)(words[w] >> (56 - 8 * b));
  out[24] = (uint8_t)len;
  if (len) memcpy(out + PHIP_BUCKET_FIXED_SIZE, name, len);
  return PHIP_BUCKET_FIXED_SIZE + (int)len;
}

int phip_api_take(phip_handle* h, const uint8_t* name, uint32_t len, const char* rate,
                  uint32_t rate_len, const char* count, uint32_t count_len, int64_t now,
                  char* body, uint32_t* body_len) {
  if (!body || !body_len) return PHIP_ERR_INVALID;
  int64_t freq, per;
  uint64_t n;
  const int pre = phip_host::api_prepare(name, len, rate, rate_len, count, count_len, &freq, &per,
                                         &n, body, body_len);
  if (pre) return pre;
  uint32_t offs[2] = {0, len};
  uint8_t empty = 0;
  uint64_t rem = 0;
  uint8_t ok = 0;
  int rc = phip_take(h, len ? name : &empty, offs, 1, &now, &freq, &per, &n, &rem, &ok, 0);
  if (rc < 0) return rc;
  std::string s = std::to_string(rem);                            // api.go:84-85
  memcpy(body, s.data(), s.size());
  *body_len = (uint32_t)s.size();
  return ok ? 200 : 429;
}

}  // extern "C"
