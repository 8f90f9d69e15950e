// ORACLE — test infrastructure only.  CPU restatement of calavera/patrol's
// bucket-state hot path (Go), used as the parity checker for libpatrolhip and
// as the CPU baseline (`cpu_baseline.kind = "port"`).  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
// product path (patrol_amd/, libpatrolhip) never does.
//
// Parity pinning: the Go reference cannot be built here (no Go toolchain), so
// this restatement is pinned against the reference's own known-answer tests
// (bucket_test.go:35-66 Take table, bucket_test.go:68-114 Merge laws,
// bucket_test.go:10-34 codec round-trip, api_test.go:34-73 HTTP table) and
// cross-checked bit-for-bit against an independent Python restatement
// (oracle/go_semantics.py) through tests/golden/.
//
// Every function cites the reference file:line it restates.  The data
// structure deliberately mirrors the Go one (global RWMutex around a map of
// heap Buckets, each with its own RWMutex: repo.go:171-235, bucket.go:20-32)
// so that the timed CPU baseline has the reference's locking shape.
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <chrono>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>
#include <algorithm>

namespace orc {

typedef uint64_t u64;
typedef int64_t i64;

static inline u64 f2b(double x) { u64 b; std::memcpy(&b, &x, 8); return b; }
static inline double b2f(u64 b) { double x; std::memcpy(&x, &b, 8); return x; }

// x86-64 CVTTSD2SQ: truncate toward zero; NaN or out of int64 range gives
// the "integer indefinite" 0x8000000000000000.
static inline i64 cvttsd2sq(double x) {
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
  return (i64)x;
}

// Go's uint64(float64) on amd64 (cmd/compile ssagen floatToUint: cutoff 2^63,
// result = x < 2^63 ? CVTTSD2SQ(x) : CVTTSD2SQ(x - 2^63) | 1<<63).  Used by
// bucket.go:217 `uint64(have)` and bucket.go:224 `uint64(b.added - b.taken)`.
static inline u64 go_f64_to_u64(double x) {
  if (x < 9223372036854775808.0) return (u64)cvttsd2sq(x);
  return (u64)cvttsd2sq(x - 9223372036854775808.0) | 0x8000000000000000ull;
}

// ---------------------------------------------------------------- Rate ----
// bucket.go:96-99
struct Rate { i64 freq; i64 per; };

// bucket.go:126-128
static inline bool rate_is_zero(Rate r) { return r.freq == 0 || r.per == 0; }

// bucket.go:146-148  (Go int64 division truncates; MinInt64 / -1 == MinInt64)
static inline i64 rate_interval(Rate r) {
  if (r.freq == -1 && r.per == INT64_MIN) return INT64_MIN;
  return r.per / r.freq;
}

// bucket.go:132-143
static inline double rate_tokens(Rate r, i64 d) {
  if (rate_is_zero(r)) return 0;
  i64 interval = rate_interval(r);
  if (interval == 0) return 0;
  return (double)d / (double)interval;
}

// ---- Go strconv / time restatements used by ParseRate (bucket.go:102-123)
// and the API handler (api.go:60-65).  Error => same value Go returns.

// strconv.ParseUint(s, 10, 64): syntax error -> 0, range error -> MaxUint64.
static int go_parse_uint10(std::string_view s, u64* out) {
  *out = 0;
  if (s.empty()) return -1;
  u64 n = 0;
  const u64 cutoff = UINT64_MAX / 10 + 1;
  for (char c : s) {
    if (c < '0' || c > '9') { *out = 0; return -1; }
    if (n >= cutoff) { *out = UINT64_MAX; return -2; }
    n *= 10;
    u64 n1 = n + (u64)(c - '0');
    if (n1 < n) { *out = UINT64_MAX; return -2; }
    n = n1;
  }
  *out = n;
  return 0;
}

// strconv.Atoi on a 64-bit platform (fast path for len<19, else ParseInt(s,10,0)).
// Syntax error -> 0; range error -> clamped to [MinInt64, MaxInt64].
static int go_atoi(std::string_view s, i64* out) {
  *out = 0;
  size_t n = s.size();
  if (n > 0 && n < 19) {
    std::string_view t = s;
    if (t[0] == '-' || t[0] == '+') {
      t.remove_prefix(1);
      if (t.empty()) return -1;
    }
    i64 v = 0;
    for (char c : t) {
      unsigned d = (unsigned char)c - '0';
      if (d > 9) return -1;
      v = v * 10 + (i64)d;
    }
    *out = s[0] == '-' ? -v : v;
    return 0;
  }
  if (n == 0) return -1;
  bool neg = false;
  std::string_view t = s;
  if (t[0] == '+') t.remove_prefix(1);
  else if (t[0] == '-') { neg = true; t.remove_prefix(1); }
  u64 un;
  int rc = go_parse_uint10(t, &un);
  if (rc == -1) { *out = 0; return -1; }
  const u64 cutoff = 1ull << 63;
  if (!neg && un >= cutoff) { *out = INT64_MAX; return -2; }
  if (neg && un > cutoff) { *out = INT64_MIN; return -2; }
  if (rc == -2) { *out = neg ? INT64_MIN : INT64_MAX; return -2; }
  *out = neg ? (i64)(0 - un) : (i64)un;
  return 0;
}

// time.ParseDuration (Go >= 1.15 restatement): any error returns 0.
static int go_parse_duration(std::string_view s, i64* out) {
  *out = 0;
  u64 d = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) { neg = s[0] == '-'; s.remove_prefix(1); }
  if (s == "0") return 0;
  if (s.empty()) return -1;
  while (!s.empty()) {
    u64 v = 0, f = 0;
    double scale = 1;
    if (!(s[0] == '.' || (s[0] >= '0' && s[0] <= '9'))) return -1;
    // leadingInt
    size_t pl = s.size(), i = 0;
    for (; i < s.size(); ++i) {
      char c = s[i];
      if (c < '0' || c > '9') break;
      if (v > (1ull << 63) / 10) return -1;
      v = v * 10 + (u64)(c - '0');
      if (v > (1ull << 63)) return -1;
    }
    s.remove_prefix(i);
    bool pre = pl != s.size();
    bool post = false;
    if (!s.empty() && s[0] == '.') {
      s.remove_prefix(1);
      size_t pl2 = s.size(), j = 0;
      bool overflow = false;
      for (; j < s.size(); ++j) {
        char c = s[j];
        if (c < '0' || c > '9') break;
        if (overflow) continue;
        if (f > ((1ull << 63) - 1) / 10) { overflow = true; continue; }
        u64 y = f * 10 + (u64)(c - '0');
        if (y > (1ull << 63)) { overflow = true; continue; }
        f = y;
        scale *= 10;
      }
      s.remove_prefix(j);
      post = pl2 != s.size();
    }
    if (!pre && !post) return -1;
    size_t k = 0;
    for (; k < s.size(); ++k) {
      char c = s[k];
      if (c == '.' || (c >= '0' && c <= '9')) break;
    }
    if (k == 0) return -1;
    std::string_view u = s.substr(0, k);
    s.remove_prefix(k);
    u64 unit;
    if (u == "ns") unit = 1;
    else if (u == "us" || u == "\xC2\xB5s" || u == "\xCE\xBCs") unit = 1000;
    else if (u == "ms") unit = 1000000;
    else if (u == "s") unit = 1000000000ull;
    else if (u == "m") unit = 60000000000ull;
    else if (u == "h") unit = 3600000000000ull;
    else return -1;
    if (v > (1ull << 63) / unit) return -1;
    v *= unit;
    if (f > 0) {
      v += (u64)((double)f * ((double)unit / scale));
      if (v > (1ull << 63)) return -1;
    }
    d += v;
    if (d > (1ull << 63)) return -1;
  }
  if (neg) { *out = (i64)(0 - d); return 0; }
  if (d > (1ull << 63) - 1) return -1;
  *out = (i64)d;
  return 0;
}

// bucket.go:102-123 ParseRate.  Returns the Rate Go returns alongside err
// (api.go:61 ignores err and uses the value).
static int parse_rate(std::string_view v, Rate* r) {
  r->freq = 0; r->per = 0;
  std::string_view f = v, p = "1s";
  size_t colon = v.find(':');
  if (colon != std::string_view::npos) { f = v.substr(0, colon); p = v.substr(colon + 1); }
  int rc = go_atoi(f, &r->freq);
  if (rc != 0) return rc;  // Per stays 0
  std::string tmp(p);
  // bucket.go:117 lists only U+00B5 (micro sign), not U+03BC (Greek mu).
  if (p == "ns" || p == "us" || p == "\xC2\xB5s" || p == "ms" || p == "s" || p == "m" ||
      p == "h")
    tmp = "1" + tmp;
  return go_parse_duration(tmp, &r->per);
}

// -------------------------------------------------------------- Bucket ----
// bucket.go:20-32.  `created` is int64 ns since the Unix epoch (the clock the
// C-ABI hands in); time.Time arithmetic below is restated for that domain.
struct Bucket {
  mutable std::shared_mutex mu;
  std::string name;
  double added = 0;
  double taken = 0;
  i64 elapsed = 0;
  i64 created = 0;
};

// bucket.go:165-170
static inline bool is_zero(const Bucket& b) {
  std::shared_lock<std::shared_mutex> l(b.mu);
  return b.added == 0 && b.taken == 0 && b.elapsed == 0;
}

// bucket.go:240-263 (one `other`)
static inline void merge(Bucket& b, const Bucket& o) {
  if (&o == &b) return;
  std::unique_lock<std::shared_mutex> lb(b.mu);
  std::shared_lock<std::shared_mutex> lo(o.mu);
  if (b.added < o.added) b.added = o.added;
  if (b.taken < o.taken) b.taken = o.taken;
  if (b.elapsed < o.elapsed) b.elapsed = o.elapsed;
}

// Raw field merge without locks (same semantics, used by unit helpers).
static inline void merge_fields(double& a, double& t, i64& e, double oa, double ot, i64 oe) {
  if (a < oa) a = oa;
  if (t < ot) t = ot;
  if (e < oe) e = oe;
}

struct TakeOut { u64 remaining; bool ok; double have; };

// bucket.go:186-225.  Time model: created/now are int64 ns; Go's time.Time
// has a far wider range, so `created.Add(elapsed)` is computed exactly in
// 128 bits, `now.Sub(last)` saturates like time.Time.Sub, and
// `b.elapsed += elapsed` wraps like Go int64 arithmetic.
static inline TakeOut take_fields(double& added, double& taken, i64& elapsed, i64 created,
                                  i64 now, Rate r, u64 n) {
  double capacity = (double)r.freq;                       // :192
  if (added == 0) added = capacity;                        // :194-196
  __int128 last = (__int128)created + (__int128)elapsed;   // :198
  if ((__int128)now < last) last = now;                    // :199-201
  double tokens = added - taken;                           // :204
  __int128 dd = (__int128)now - last;                      // :207
  i64 dt = dd > (__int128)INT64_MAX ? INT64_MAX : (dd < (__int128)INT64_MIN ? INT64_MIN : (i64)dd);
  double add = rate_tokens(r, dt);                         // :210
  double missing = capacity - tokens;                      // :211
  if (add > missing) add = missing;                        // :211-213
  double t = (double)n;                                    // :215
  double have = tokens + add;                              // :216
  if (t > have) return {go_f64_to_u64(have), false, have}; // :216-218
  elapsed = (i64)((u64)elapsed + (u64)dt);                 // :220
  added += add;                                            // :221
  taken += t;                                              // :222
  double rem = added - taken;
  return {go_f64_to_u64(rem), true, rem};                  // :224
}

static inline TakeOut take(Bucket& b, i64 now, Rate r, u64 n) {
  std::unique_lock<std::shared_mutex> l(b.mu);
  return take_fields(b.added, b.taken, b.elapsed, b.created, now, r, n);
}

// bucket.go:34-48
static const int kFixed = 25, kPacket = 256, kMaxName = kPacket - kFixed;

static inline void put_be64(uint8_t* p, u64 v) { for (int i = 7; i >= 0; --i) { p[i] = (uint8_t)v; v >>= 8; } }
static inline u64 get_be64(const uint8_t* p) { u64 v = 0; for (int i = 0; i < 8; ++i) v = (v << 8) | p[i]; return v; }

// bucket.go:51-68.  Returns bytes written or -1 (ErrNameTooLarge).
static int marshal(const std::string& name, double a, double t, i64 e, uint8_t* out) {
  if ((int)name.size() > kMaxName) return -1;
  put_be64(out, f2b(a));
  put_be64(out + 8, f2b(t));
  put_be64(out + 16, (u64)e);
  out[24] = (uint8_t)name.size();
  std::memcpy(out + 25, name.data(), name.size());
  return kFixed + (int)name.size();
}

// bucket.go:71-91.  0 ok, -1 io.ErrShortBuffer (before any field is set),
// -2 io.ErrShortBuffer after the numeric fields were set (truncated name).
static int unmarshal(const uint8_t* d, size_t n, Bucket& b) {
  if (n < (size_t)kFixed) return -1;
  std::unique_lock<std::shared_mutex> l(b.mu);
  b.added = b2f(get_be64(d));
  b.taken = b2f(get_be64(d + 8));
  b.elapsed = (i64)get_be64(d + 16);
  size_t nl = d[24];
  if (n - 25 < nl) return -2;
  b.name.assign((const char*)d + 25, nl);
  return 0;
}

// ----------------------------------------------------------- LocalRepo ----
struct SvHash {
  using is_transparent = void;
  size_t operator()(std::string_view s) const { return std::hash<std::string_view>{}(s); }
};

// repo.go:171-177
struct LocalRepo {
  mutable std::shared_mutex mu;
  std::unordered_map<std::string, Bucket*, SvHash, std::equal_to<>> buckets;
  ~LocalRepo() { for (auto& kv : buckets) delete kv.second; }

  // repo.go:189-211 (clock() is the caller-supplied now)
  Bucket* get_bucket(std::string_view name, i64 clock, bool* existed) {
    {
      std::shared_lock<std::shared_mutex> l(mu);
      auto it = buckets.find(name);
      if (it != buckets.end()) { *existed = true; return it->second; }
    }
    std::unique_lock<std::shared_mutex> l(mu);
    auto it = buckets.find(name);
    if (it != buckets.end()) { *existed = true; return it->second; }
    Bucket* b = new Bucket;
    b->name.assign(name);
    b->created = clock;
    buckets.emplace(b->name, b);
    *existed = false;
    return b;
  }

  // repo.go:215-235.  `b` is a distinct, caller-owned state; on a miss a
  // heap copy is inserted (the Go code inserts the pointer itself).
  Bucket* upsert_bucket(const Bucket& b, i64 clock, bool* merged) {
    Bucket* prev = nullptr;
    {
      std::shared_lock<std::shared_mutex> l(mu);
      auto it = buckets.find(b.name);
      if (it != buckets.end()) prev = it->second;
    }
    if (prev == &b) { *merged = true; return prev; }
    {
      std::unique_lock<std::shared_mutex> l(mu);
      auto it = buckets.find(b.name);
      if (it == buckets.end()) {
        Bucket* nb = new Bucket;
        nb->name = b.name;
        { std::shared_lock<std::shared_mutex> lb(b.mu); nb->added = b.added; nb->taken = b.taken; nb->elapsed = b.elapsed; }
        nb->created = clock;
        buckets.emplace(nb->name, nb);
        *merged = false;
        return nb;
      }
      prev = it->second;
    }
    merge(*prev, b);
    *merged = true;
    return prev;
  }
};

}  // namespace orc

using namespace orc;

// ---------------------------------------------------------------- C ABI ----
// Status codes per message, shared with include/patrolhip.h.
enum {
  ST_MERGED = 1,          // !remote.IsZero(): local.Merge(&remote)        repo.go:78-79
  ST_INCAST_REPLY = 2,    // zero remote, existed && !local.IsZero()      repo.go:86-90
  ST_INCAST_NOREPLY = 3,  // zero remote, otherwise
  ST_SHORT = 4,           // io.ErrShortBuffer: Receive returns            repo.go:72-73
  ST_NOT_PROCESSED = 5,   // after a ST_SHORT (the Go loop has exited)
  ST_TAKE_OK = 6,
  ST_TAKE_DENIED = 7,
  ST_UPSERT_INSERTED = 8, // UpsertBucket inserted the state as-is          repo.go:225-230
  ST_CREATED = 0x80,      // flag: this op created the bucket (GetBucket miss)
};

extern "C" {

void* orc_repo_new() { return new LocalRepo; }
void orc_repo_free(void* r) { delete (LocalRepo*)r; }

size_t orc_repo_len(void* r) { return ((LocalRepo*)r)->buckets.size(); }

// NewLocalRepo(clock, bs...) (repo.go:179-185): buckets inserted as given.
void orc_repo_seed(void* r, const uint8_t* names, const uint32_t* offs, uint32_t n,
                   const double* added, const double* taken, const int64_t* elapsed,
                   const int64_t* created) {
  LocalRepo* repo = (LocalRepo*)r;
  for (uint32_t i = 0; i < n; ++i) {
    std::string name((const char*)names + offs[i], offs[i + 1] - offs[i]);
    auto it = repo->buckets.find(name);
    Bucket* b;
    if (it == repo->buckets.end()) { b = new Bucket; b->name = name; repo->buckets.emplace(name, b); }
    else b = it->second;
    b->added = added[i]; b->taken = taken[i]; b->elapsed = elapsed[i]; b->created = created[i];
  }
}

// ReplicatedRepo.Receive over a batch of datagrams (repo.go:54-92), the local
// clock reading `now` for every GetBucket create.  Per message: status,
// and for ST_INCAST_REPLY the marshalled local state at that moment
// (repo.go:160-169) as (added bits, taken bits, elapsed).
// Returns the index of the first ST_SHORT or n.
uint32_t orc_receive(void* r, const uint8_t* bytes, const uint64_t* offs, uint32_t n, int64_t now,
                     uint8_t* status, uint64_t* reply_added, uint64_t* reply_taken,
                     int64_t* reply_elapsed) {
  LocalRepo* repo = (LocalRepo*)r;
  Bucket remote;
  uint32_t stop = n;
  for (uint32_t i = 0; i < n; ++i) {
    if (stop != n) { status[i] = ST_NOT_PROCESSED; continue; }
    int rc = unmarshal(bytes + offs[i], offs[i + 1] - offs[i], remote);
    if (rc != 0) { status[i] = ST_SHORT; stop = i; continue; }
    bool existed;
    Bucket* local = repo->get_bucket(remote.name, now, &existed);
    uint8_t st;
    if (!is_zero(remote)) { merge(*local, remote); st = ST_MERGED; }
    else if (existed && !is_zero(*local)) {
      st = ST_INCAST_REPLY;
      std::shared_lock<std::shared_mutex> l(local->mu);
      if (reply_added) reply_added[i] = f2b(local->added);
      if (reply_taken) reply_taken[i] = f2b(local->taken);
      if (reply_elapsed) reply_elapsed[i] = local->elapsed;
    } else st = ST_INCAST_NOREPLY;
    status[i] = st | (existed ? 0 : ST_CREATED);
  }
  return stop;
}

// Same as orc_receive on pre-decoded messages (names blob + offsets).
void orc_receive_soa(void* r, const uint8_t* names, const uint32_t* offs, uint32_t n,
                     const uint64_t* added, const uint64_t* taken, const int64_t* elapsed,
                     int64_t now, uint8_t* status, uint64_t* reply_added, uint64_t* reply_taken,
                     int64_t* reply_elapsed) {
  LocalRepo* repo = (LocalRepo*)r;
  Bucket remote;
  for (uint32_t i = 0; i < n; ++i) {
    remote.added = b2f(added[i]); remote.taken = b2f(taken[i]); remote.elapsed = elapsed[i];
    std::string_view name((const char*)names + offs[i], offs[i + 1] - offs[i]);
    bool existed;
    Bucket* local = repo->get_bucket(name, now, &existed);
    uint8_t st;
    if (!is_zero(remote)) { merge(*local, remote); st = ST_MERGED; }
    else if (existed && !is_zero(*local)) {
      st = ST_INCAST_REPLY;
      if (reply_added) reply_added[i] = f2b(local->added);
      if (reply_taken) reply_taken[i] = f2b(local->taken);
      if (reply_elapsed) reply_elapsed[i] = local->elapsed;
    } else st = ST_INCAST_NOREPLY;
    if (status) status[i] = st | (existed ? 0 : ST_CREATED);
  }
}

// LocalRepo.UpsertBucket for each decoded state (repo.go:215-235).
void orc_upsert_soa(void* r, const uint8_t* names, const uint32_t* offs, uint32_t n,
                    const uint64_t* added, const uint64_t* taken, const int64_t* elapsed,
                    int64_t now, uint8_t* merged_out) {
  LocalRepo* repo = (LocalRepo*)r;
  Bucket b;
  for (uint32_t i = 0; i < n; ++i) {
    b.name.assign((const char*)names + offs[i], offs[i + 1] - offs[i]);
    b.added = b2f(added[i]); b.taken = b2f(taken[i]); b.elapsed = elapsed[i];
    bool merged;
    repo->upsert_bucket(b, now, &merged);
    if (merged_out) merged_out[i] = merged;
  }
}

// Mixed ordered stream: kind 0 = Take (api.go:67-74 minus HTTP), kind 1 =
// received replica state (repo.go:78-90), kind 2 = UpsertBucket (repo.go:215-235).  Ops apply in index order; each op
// carries its own clock reading `now`, also used as `created` on a miss.
// reply_* (any may be null) receive the bucket's state right after the op
// for a Take (what UpsertBucket broadcasts next, api.go:74 -> repo.go:123-127),
// an Upsert (the upserted bucket, repo.go:123-127) and an incast (the local
// state: the unicast payload of repo.go:86-90 when it is sent); merged
// replicas leave them untouched.
static inline void put_reply(const Bucket* b, uint32_t i, uint64_t* ra, uint64_t* rt, int64_t* re,
                             int64_t* rc) {
  std::shared_lock<std::shared_mutex> l(b->mu);
  if (ra) ra[i] = f2b(b->added);
  if (rt) rt[i] = f2b(b->taken);
  if (re) re[i] = b->elapsed;
  if (rc) rc[i] = b->created;
}

void orc_apply_mixed(void* r, const uint8_t* kind, const uint8_t* names, const uint32_t* offs,
                     uint32_t n, const int64_t* now, const int64_t* freq, const int64_t* per,
                     const uint64_t* count, const uint64_t* added, const uint64_t* taken,
                     const int64_t* elapsed, uint8_t* status, uint64_t* remaining,
                     uint64_t* have_bits, uint64_t* reply_added, uint64_t* reply_taken,
                     int64_t* reply_elapsed, int64_t* reply_created) {
  LocalRepo* repo = (LocalRepo*)r;
  Bucket remote;
  for (uint32_t i = 0; i < n; ++i) {
    std::string_view name((const char*)names + offs[i], offs[i + 1] - offs[i]);
    if (kind[i] == 2) {   // LocalRepo.UpsertBucket of a distinct state (repo.go:215-235)
      Bucket up;
      up.name.assign(name);
      up.added = b2f(added[i]); up.taken = b2f(taken[i]); up.elapsed = elapsed[i];
      bool merged;
      const Bucket* got = repo->upsert_bucket(up, now[i], &merged);
      status[i] = merged ? ST_MERGED : (ST_UPSERT_INSERTED | ST_CREATED);
      if (remaining) remaining[i] = 0;
      if (have_bits) have_bits[i] = 0;
      put_reply(got, i, reply_added, reply_taken, reply_elapsed, reply_created);
      continue;
    }
    bool existed;
    Bucket* b = repo->get_bucket(name, now[i], &existed);
    uint8_t st;
    if (kind[i] == 0) {
      TakeOut t = take(*b, now[i], Rate{freq[i], per[i]}, count[i]);
      st = t.ok ? ST_TAKE_OK : ST_TAKE_DENIED;
      if (remaining) remaining[i] = t.remaining;
      if (have_bits) have_bits[i] = f2b(t.have);
      put_reply(b, i, reply_added, reply_taken, reply_elapsed, reply_created);
    } else {
      remote.added = b2f(added[i]); remote.taken = b2f(taken[i]); remote.elapsed = elapsed[i];
      if (!is_zero(remote)) { merge(*b, remote); st = ST_MERGED; }
      else {
        st = existed && !is_zero(*b) ? ST_INCAST_REPLY : ST_INCAST_NOREPLY;
        put_reply(b, i, reply_added, reply_taken, reply_elapsed, reply_created);
      }
      if (remaining) remaining[i] = 0;
      if (have_bits) have_bits[i] = 0;
    }
    status[i] = st | (existed ? 0 : ST_CREATED);
  }
}

// Fetch one bucket.  Returns 1 if found.
int orc_get(void* r, const uint8_t* name, uint32_t len, uint64_t* added, uint64_t* taken,
            int64_t* elapsed, int64_t* created) {
  LocalRepo* repo = (LocalRepo*)r;
  auto it = repo->buckets.find(std::string_view((const char*)name, len));
  if (it == repo->buckets.end()) return 0;
  Bucket* b = it->second;
  *added = f2b(b->added); *taken = f2b(b->taken); *elapsed = b->elapsed; *created = b->created;
  return 1;
}

// Dump all buckets sorted by name: names concatenated into `names`
// (capacity `cap` bytes), offsets[n+1].  Returns bucket count, or -needed
// when buffers are too small (pass null to size).
int64_t orc_dump(void* r, uint8_t* names, uint64_t cap, uint64_t* offs, uint64_t* added,
                 uint64_t* taken, int64_t* elapsed, int64_t* created, uint64_t max_n) {
  LocalRepo* repo = (LocalRepo*)r;
  std::vector<const Bucket*> v;
  v.reserve(repo->buckets.size());
  uint64_t total = 0;
  for (auto& kv : repo->buckets) { v.push_back(kv.second); total += kv.first.size(); }
  if (!names || total > cap || v.size() > max_n) return -(int64_t)total - 1;
  std::sort(v.begin(), v.end(), [](const Bucket* a, const Bucket* b) { return a->name < b->name; });
  uint64_t o = 0;
  for (size_t i = 0; i < v.size(); ++i) {
    offs[i] = o;
    std::memcpy(names + o, v[i]->name.data(), v[i]->name.size());
    o += v[i]->name.size();
    added[i] = f2b(v[i]->added); taken[i] = f2b(v[i]->taken);
    elapsed[i] = v[i]->elapsed; created[i] = v[i]->created;
  }
  offs[v.size()] = o;
  return (int64_t)v.size();
}

// Compare a table dump (any order; names blob + u64 offsets[n+1], float64
// bits, elapsed, created) with this repo, for full-size parity checks where
// a per-bucket Python comparison would be too slow.  Returns the number of
// differences: an entry whose name is absent here or whose state differs,
// a name listed twice, and (once) a bucket count that differs.  *first_bad
// receives the index of the first differing entry (n if none).
uint64_t orc_check_dump(void* r, const uint8_t* names, const uint64_t* offs, uint64_t n,
                        const uint64_t* added, const uint64_t* taken, const int64_t* elapsed,
                        const int64_t* created, uint64_t* first_bad) {
  LocalRepo* repo = (LocalRepo*)r;
  std::unordered_map<const Bucket*, uint64_t> seen;
  seen.reserve(n);
  uint64_t bad = 0;
  *first_bad = n;
  for (uint64_t i = 0; i < n; ++i) {
    auto it = repo->buckets.find(std::string_view((const char*)names + offs[i], offs[i + 1] - offs[i]));
    bool ok = it != repo->buckets.end();
    if (ok) {
      const Bucket* b = it->second;
      ok = f2b(b->added) == added[i] && f2b(b->taken) == taken[i] && b->elapsed == elapsed[i] &&
           b->created == created[i] && seen.emplace(b, i).second;
    }
    if (!ok) {
      if (*first_bad == n) *first_bad = i;
      ++bad;
    }
  }
  if (n != repo->buckets.size()) ++bad;
  return bad;
}

// ------------------------------------------------------- scalar helpers ----
int orc_parse_rate(const char* s, uint32_t len, int64_t* freq, int64_t* per) {
  Rate r;
  int rc = parse_rate(std::string_view(s, len), &r);
  *freq = r.freq; *per = r.per;
  return rc;
}
int orc_parse_uint10(const char* s, uint32_t len, uint64_t* out) {
  return go_parse_uint10(std::string_view(s, len), out);
}
uint64_t orc_go_f64_to_u64(double x) { return go_f64_to_u64(x); }
int64_t orc_rate_interval(int64_t freq, int64_t per) {
  if (freq == 0) return 0;  // Go panics; never reached from Tokens (IsZero guard)
  return rate_interval(Rate{freq, per});
}
double orc_rate_tokens(int64_t freq, int64_t per, int64_t d) { return rate_tokens(Rate{freq, per}, d); }

// Single Take on raw fields; state updated in place.  Returns ok.
int orc_take_fields(double* added, double* taken, int64_t* elapsed, int64_t created, int64_t now,
                    int64_t freq, int64_t per, uint64_t n, uint64_t* remaining, double* have) {
  TakeOut t = take_fields(*added, *taken, *elapsed, created, now, Rate{freq, per}, n);
  *remaining = t.remaining; *have = t.have;
  return t.ok;
}
void orc_merge_fields(double* a, double* t, int64_t* e, double oa, double ot, int64_t oe) {
  merge_fields(*a, *t, *e, oa, ot, oe);
}
int orc_marshal(const uint8_t* name, uint32_t len, double a, double t, int64_t e, uint8_t* out) {
  return marshal(std::string((const char*)name, len), a, t, e, out);
}
int orc_unmarshal(const uint8_t* d, uint32_t n, double* a, double* t, int64_t* e, uint8_t* name,
                  uint32_t* name_len) {
  Bucket b;
  int rc = unmarshal(d, n, b);
  if (rc == -1) return rc;
  *a = b.added; *t = b.taken; *e = b.elapsed;
  if (rc == 0) { std::memcpy(name, b.name.data(), b.name.size()); *name_len = (uint32_t)b.name.size(); }
  return rc;
}

// API.takeBucket (api.go:51-86) over this repo: name-length check, rate and
// count parsing with Go's error values, GetBucket/Take/UpsertBucket.
// Writes the response body; returns the HTTP status code.
int orc_api_take(void* r, const uint8_t* name, uint32_t len, const char* rate, uint32_t rate_len,
                 const char* count, uint32_t count_len, int64_t now, char* body, uint32_t* body_len) {
  LocalRepo* repo = (LocalRepo*)r;
  if ((int)len > kMaxName) {
    static const char msg[] = "bucket name larger than 231";
    std::memcpy(body, msg, sizeof(msg) - 1);
    *body_len = sizeof(msg) - 1;
    return 400;
  }
  Rate rt;
  parse_rate(std::string_view(rate, rate_len), &rt);
  u64 n;
  go_parse_uint10(std::string_view(count, count_len), &n);
  if (n == 0) n = 1;
  bool existed;
  Bucket* b = repo->get_bucket(std::string_view((const char*)name, len), now, &existed);
  TakeOut t = take(*b, now, rt, n);
  bool merged;
  (void)merged;  // UpsertBucket(bucket) with the same pointer: repo.go:220-222 fast path
  std::string s = std::to_string(t.remaining);
  std::memcpy(body, s.data(), s.size());
  *body_len = (uint32_t)s.size();
  return t.ok ? 200 : 429;
}

// ------------------------------------------------------- CPU baseline -----
// Times the Receive hot loop (repo.go:78-79: GetBucket + Merge) over
// pre-decoded messages with `threads` workers, each owning a contiguous
// share of the messages and its own reused `remote` (repo.go:56).  The repo
// must already hold the buckets (C2 is pre-populated).  Returns seconds.
double orc_bench_receive(void* r, const uint8_t* names, const uint32_t* offs, uint64_t n,
                         const uint64_t* added, const uint64_t* taken, const int64_t* elapsed,
                         int64_t now, int threads) {
  LocalRepo* repo = (LocalRepo*)r;
  if (threads < 1) threads = 1;
  std::vector<std::thread> th;
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  auto worker = [&](uint64_t lo, uint64_t hi) {
    Bucket remote;
    ready.fetch_add(1);
    while (!go.load(std::memory_order_acquire)) {}
    for (uint64_t i = lo; i < hi; ++i) {
      {
        std::unique_lock<std::shared_mutex> l(remote.mu);  // UnmarshalBinary locks (bucket.go:76)
        remote.added = b2f(added[i]); remote.taken = b2f(taken[i]); remote.elapsed = elapsed[i];
      }
      std::string_view name((const char*)names + offs[i], offs[i + 1] - offs[i]);
      bool existed;
      Bucket* local = repo->get_bucket(name, now, &existed);
      if (!is_zero(remote)) merge(*local, remote);
    }
  };
  for (int t = 0; t < threads; ++t)
    th.emplace_back(worker, n * t / threads, n * (t + 1) / threads);
  while (ready.load() < threads) {}
  auto t0 = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

// Times the ordered mixed stream (single goroutine per op sequence).
double orc_bench_mixed(void* r, const uint8_t* kind, const uint8_t* names, const uint32_t* offs,
                       uint32_t n, const int64_t* now, const int64_t* freq, const int64_t* per,
                       const uint64_t* count, const uint64_t* added, const uint64_t* taken,
                       const int64_t* elapsed, uint8_t* status, uint64_t* remaining) {
  auto t0 = std::chrono::steady_clock::now();
  orc_apply_mixed(r, kind, names, offs, n, now, freq, per, count, added, taken, elapsed, status,
                  remaining, nullptr, nullptr, nullptr, nullptr, nullptr);
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

// Times the ordered mixed stream on `threads` workers the way concurrent Go
// handlers run it: every op takes the global map lock (GetBucket,
// repo.go:189-211) and its bucket's mutex (bucket.go:186-225, 240-263);
// per-bucket order is the stream's, because each bucket's ops are given to
// one worker (by a hash of the name, assigned before the timed region) and
// that worker runs them in stream order.  Returns seconds.
double orc_bench_mixed_mt(void* r, const uint8_t* kind, const uint8_t* names, const uint32_t* offs,
                          uint32_t n, const int64_t* now, const int64_t* freq, const int64_t* per,
                          const uint64_t* count, const uint64_t* added, const uint64_t* taken,
                          const int64_t* elapsed, uint8_t* status, uint64_t* remaining,
                          int threads) {
  LocalRepo* repo = (LocalRepo*)r;
  if (threads < 1) threads = 1;
  std::vector<std::vector<uint32_t>> part(threads);
  for (uint32_t i = 0; i < n; ++i) {
    std::string_view name((const char*)names + offs[i], offs[i + 1] - offs[i]);
    part[std::hash<std::string_view>{}(name) % (size_t)threads].push_back(i);
  }
  std::vector<std::thread> th;
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  auto worker = [&](int t) {
    Bucket remote;
    ready.fetch_add(1);
    while (!go.load(std::memory_order_acquire)) {}
    for (uint32_t i : part[t]) {
      std::string_view name((const char*)names + offs[i], offs[i + 1] - offs[i]);
      if (kind[i] == 2) {
        Bucket up;
        up.name.assign(name);
        up.added = b2f(added[i]); up.taken = b2f(taken[i]); up.elapsed = elapsed[i];
        bool merged;
        repo->upsert_bucket(up, now[i], &merged);
        status[i] = merged ? ST_MERGED : (ST_UPSERT_INSERTED | ST_CREATED);
        continue;
      }
      bool existed;
      Bucket* b = repo->get_bucket(name, now[i], &existed);
      uint8_t st;
      if (kind[i] == 0) {
        TakeOut o = take(*b, now[i], Rate{freq[i], per[i]}, count[i]);
        st = o.ok ? ST_TAKE_OK : ST_TAKE_DENIED;
        remaining[i] = o.remaining;
      } else {
        {
          std::unique_lock<std::shared_mutex> l(remote.mu);
          remote.added = b2f(added[i]); remote.taken = b2f(taken[i]); remote.elapsed = elapsed[i];
        }
        if (!is_zero(remote)) { merge(*b, remote); st = ST_MERGED; }
        else st = existed && !is_zero(*b) ? ST_INCAST_REPLY : ST_INCAST_NOREPLY;
      }
      status[i] = st | (existed ? 0 : ST_CREATED);
    }
  };
  for (int t = 0; t < threads; ++t) th.emplace_back(worker, t);
  while (ready.load() < threads) {}
  auto t0 = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

// FNV-1a 64 (the device table's key hash; not part of the reference).
uint64_t orc_fnv1a64(const uint8_t* p, uint32_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ull; }
  return h;
}

}  // extern "C"
