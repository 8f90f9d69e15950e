// Device-side building blocks of libpatrolhip (gfx950).
//
//  * the order-preserving 64-bit key encoding ("E-encoding") that lets one
//    unsigned atomicMax reproduce Go's asymmetric `if b.x < o.x { b.x = o.x }`
//    merge (bucket.go:250-256) for every stored value and every replica value
//    except -0.0 (DESIGN.md §3.2 has the proof sketch);
//  * the op-for-op restatement of Bucket.Take (bucket.go:186-225) on doubles,
//    including Go's time.Time saturation and amd64 uint64(float64) rules;
//  * the slot record of the device hash table and name canonicalisation.
//
// Compiled with -ffp-contract=off: every + - / below is one IEEE-754 binary64
// operation, exactly as the Go compiler emits them on amd64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "patrolhip.h"

namespace phip {

typedef unsigned long long u64;
typedef long long i64;
typedef unsigned int u32;
typedef unsigned char u8;
typedef unsigned short u16;

constexpr u64 kSign = 0x8000000000000000ull;
constexpr u64 kInfBits = 0x7FF0000000000000ull;      // +Inf
constexpr u64 kNanBase = 0xFFE0000000000002ull;      // first E-code of a NaN
constexpr u64 kNanPerSign = (1ull << 52) - 1;        // NaN payloads per sign
constexpr u64 kEPosZero = kInfBits;                  // E(+0.0)
constexpr u64 kENegZero = kInfBits + 1;              // E(-0.0)

__host__ __device__ inline bool is_nan_bits(u64 b) { return (b & ~kSign) > kInfBits; }
__host__ __device__ inline bool is_zero_bits(u64 b) { return (b & ~kSign) == 0; }

// E: float64 bits -> u64 such that unsigned order is
//   negatives (by value) < +0 < -0 < positives (by value) < NaNs.
// It is a bijection on all 2^64 patterns.  Placing -0 just above +0 makes
// max(E(b), E(o)) equal E(Go's merge result) for every stored b and every
// replica o != -0.0 (a NaN replica is mapped to 0 = E(-Inf), a no-op).
__host__ __device__ inline u64 enc_f64(u64 b) {
  u64 mag = b & ~kSign;
  if (mag > kInfBits) {                            // NaN
    u64 idx = mag - kInfBits - 1;
    if (b & kSign) idx += kNanPerSign;
    return kNanBase + idx;
  }
  if (b & kSign) return mag == 0 ? kENegZero : kInfBits - mag;
  return mag == 0 ? kEPosZero : kInfBits + 1 + mag;
}

__host__ __device__ inline u64 dec_f64(u64 e) {
  if (e < kInfBits) return kSign | (kInfBits - e);
  if (e == kEPosZero) return 0;
  if (e == kENegZero) return kSign;
  if (e < kNanBase) return e - kInfBits - 1;
  u64 idx = e - kNanBase;
  if (idx < kNanPerSign) return kInfBits + 1 + idx;
  return kSign | (kInfBits + 1 + idx - kNanPerSign);
}

// Replica value as an atomicMax operand (NaN is never adopted by Go's `<`).
__host__ __device__ inline u64 enc_replica(u64 b) { return is_nan_bits(b) ? 0ull : enc_f64(b); }

__host__ __device__ inline double as_f64(u64 b) { return __builtin_bit_cast(double, b); }
__host__ __device__ inline u64 as_bits(double x) { return __builtin_bit_cast(u64, x); }

// ------------------------------------------------------------- Take -----
// x86-64 CVTTSD2SQ (what Go's amd64 backend uses for float->int).
__device__ inline i64 cvttsd2sq(double x) {
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return (i64)kSign;
  return (i64)x;
}
// Go uint64(float64) on amd64: cutoff at 2^63 (ssagen floatToUint).
__device__ inline u64 go_u64(double x) {
  if (x < 9223372036854775808.0) return (u64)cvttsd2sq(x);
  return (u64)cvttsd2sq(x - 9223372036854775808.0) | kSign;
}

// Rate.Interval (bucket.go:146-148) folded with the zero tests of
// Rate.Tokens (bucket.go:132-137): 0 means "Tokens() returns 0".  Computed
// once per op when the ordered stream is gathered (k_gather_ops).
__host__ __device__ inline i64 rate_interval(i64 freq, i64 per) {
  if (freq == 0 || per == 0) return 0;
  if (freq == -1 && per == (i64)kSign) return (i64)kSign;   // Go's MinInt64 / -1 wraps
  return per / freq;
}

// Go float64 + and - as amd64 executes them (ADDSD/SUBSD, the left Go
// operand in the destination register), down to the NaN bits: a NaN operand
// comes back quieted with its sign and payload, the left one first, and an
// invalid operation (Inf - Inf) gives the x86 default NaN 0xFFF8000000000000.
// gfx950 computes a - b as a + (-b), which flips the sign of a NaN b and
// returns the positive default NaN, so results that are NaN are rebuilt here.
constexpr u64 kQuietBit = 0x0008000000000000ull;
constexpr u64 kX86DefaultNaN = 0xFFF8000000000000ull;

__device__ inline double x86_nan_fix(double r, double a, double b) {
  if (__builtin_expect(r == r, 1)) return r;
  const u64 ab = as_bits(a), bb = as_bits(b);
  if (is_nan_bits(ab)) return as_f64(ab | kQuietBit);
  if (is_nan_bits(bb)) return as_f64(bb | kQuietBit);
  return as_f64(kX86DefaultNaN);
}
__device__ inline double go_add(double a, double b) { return x86_nan_fix(a + b, a, b); }
__device__ inline double go_sub(double a, double b) { return x86_nan_fix(a - b, a, b); }

// dt of Take (bucket.go:198-207): last = created.Add(elapsed) (exact),
// clamped to now, then now.Sub(last) saturating to the int64 range.  The
// int64 fast path is exact whenever created + elapsed does not overflow.
__device__ inline i64 take_dt(i64 created, i64 elapsed, i64 now) {
  i64 last;
  if (__builtin_expect(!__builtin_add_overflow(created, elapsed, &last), 1)) {
    if (now < last) return 0;
    i64 d;
    return __builtin_sub_overflow(now, last, &d) ? 0x7FFFFFFFFFFFFFFFll : d;
  }
  __int128 l = (__int128)created + (__int128)elapsed;
  if ((__int128)now < l) return 0;
  __int128 dd = (__int128)now - l;
  return dd > (__int128)0x7FFFFFFFFFFFFFFFll ? 0x7FFFFFFFFFFFFFFFll : (i64)dd;
}

struct TakeResult {
  u64 remaining;
  u64 have_bits;
  bool ok;
};

// Bucket.Take (bucket.go:186-225), in the reference's exact operation order,
// with Rate.Interval precomputed (rate_interval).  `created` and `now` are
// int64 ns; created.Add(elapsed) is exact (128-bit, as time.Time cannot
// overflow here), now.Sub(last) saturates like time.Time.Sub, and
// elapsed += dt wraps like Go int64.
// capacity = float64(Freq) and t = float64(n) come precomputed (k_pack_ops).
__device__ inline TakeResult take_step(double& added, double& taken, i64& elapsed, i64 created,
                                       i64 now, i64 interval, double capacity, double t) {
  //                                                              :192 capacity
  if (added == 0) added = capacity;                            // :194-196
  const i64 dt = take_dt(created, elapsed, now);                // :198-207
  double tokens = go_sub(added, taken);                        // :204
  // :210, bucket.go:132-143; 0/interval is a zero with interval's sign
  double add = !interval ? 0.0 : dt ? (double)dt / (double)interval : (interval < 0 ? -0.0 : 0.0);
  double missing = go_sub(capacity, tokens);                   // :211
  if (add > missing) add = missing;                            // :211-213
  //                                                              :215 t
  double have = go_add(tokens, add);                           // :216
  if (t > have) return TakeResult{go_u64(have), as_bits(have), false};   // :216-218
  elapsed = (i64)((u64)elapsed + (u64)dt);                     // :220
  added = go_add(added, add);                                  // :221
  taken = go_add(taken, t);                                    // :222
  double rem = go_sub(added, taken);
  return TakeResult{go_u64(rem), as_bits(rem), true};          // :224
}

// Bucket.Merge for one `other` (bucket.go:250-260) on raw values.
__device__ inline void go_merge(double& a, double& t, i64& e, double oa, double ot, i64 oe) {
  if (a < oa) a = oa;
  if (t < ot) t = ot;
  if (e < oe) e = oe;
}

// Bucket.IsZero (bucket.go:165-170): -0.0 == 0 is true.
__host__ __device__ inline bool state_is_zero(u64 a_bits, u64 t_bits, i64 e) {
  return is_zero_bits(a_bits) && is_zero_bits(t_bits) && e == 0;
}

// ------------------------------------------------------------ table -----
// One 64-byte slot record = one HBM burst holding everything a lookup and a
// merge touch, ordered so that the Receive fast path reads only the first
// 48 bytes (three 16-byte loads) for names of up to 14 bytes:
//   [ 0,16) tag, added     tag = FNV-1a 64 of the name (0 = empty; a 0 hash is stored as 1)
//   [16,32) taken, elapsed added/taken are E-encoded float64
//   [32,48) name0, name1   canonical name words 0-1
//   [48,64) created, name2 canonical name word 2
// Canonical name (24 bytes, words name0..name2): byte 0 = len, byte 1 = flags
// (kRec*), then len <= 22: bytes 2..2+len = the name, zero padded (names of
// up to 14 bytes end in name1, so name2 = 0); len > 22: bytes 4..7 = arena
// offset, bytes 8..23 = the first 16 bytes (fast reject), full name in the arena.
struct alignas(64) Rec {
  u64 tag;
  u64 added;
  u64 taken;
  i64 elapsed;
  u64 name0;
  u64 name1;
  i64 created;
  u64 name2;
};
static_assert(sizeof(Rec) == 64, "slot record must be one 64-byte burst");

constexpr u32 kInlineName = 22;
constexpr u32 kShortName = 14;     // fits name0/name1: the 48-byte fast path
constexpr u64 kRecPublished = 1u;   // name and state written (visible after a kernel boundary)
constexpr u64 kRecNew = 2u;         // created by the current batch

__host__ __device__ inline u32 rec_flags(const Rec& r) { return (u32)((r.name0 >> 8) & 0xFFu); }
__host__ __device__ inline u64 with_flags(u64 w0, u64 f) { return (w0 & ~0xFF00ull) | (f << 8); }

constexpr u64 kFnvOffset = 0xcbf29ce484222325ull;
constexpr u64 kFnvPrime = 0x100000001b3ull;

// h * 0x100000001b3 == h * 0x1b3 + (h << 40)
__host__ __device__ inline u64 fnv_step(u64 h, u8 c) {
  h ^= c;
  return h * 0x1b3ull + (h << 40);
}

__host__ __device__ inline u64 tag_of(u64 h) { return h ? h : 1ull; }

struct Name {
  u64 w0, w1, w2;   // canonical 24-byte field (see Rec), flags byte 0
  u64 h;            // FNV-1a 64
  u64 off;          // byte offset of the name in its source blob
  u32 len;
};

__host__ __device__ inline void put_name_byte(Name& nm, u32 pos, u8 c) {
  u64 v = (u64)c << ((pos & 7) * 8);
  if (pos < 8) nm.w0 |= v;
  else if (pos < 16) nm.w1 |= v;
  else nm.w2 |= v;
}

// Reads name bytes src[off .. off+len), hashes and canonicalises them.
__host__ __device__ inline void load_name(const u8* src, u64 off, u32 len, Name& nm) {
  nm.w0 = len & 0xFFu; nm.w1 = 0; nm.w2 = 0; nm.h = kFnvOffset; nm.off = off; nm.len = len;
  const bool inl = len <= kInlineName;
  for (u32 k = 0; k < len; ++k) {
    u8 c = src[off + k];
    nm.h = fnv_step(nm.h, c);
    if (inl) put_name_byte(nm, k + 2, c);
    else if (k < 16) put_name_byte(nm, k + 8, c);
  }
}

}  // namespace phip
