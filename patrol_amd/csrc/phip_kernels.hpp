// HIP kernels of libpatrolhip (gfx950).  Host orchestration: phip_engine.hip.
//
// Table: recs[2^L] 64-byte slot records (tag, state and name in one HBM
// burst) + aux[2^L] u32 scratch used only by inserting/seeding batches.
// Home slot = top L bits of seeded_mix(tag, seed) (a per-handle seed, as Go
// seeds its map hash), linear probing; a lookup touches one 64-byte record
// per probe step.
#pragma once
#include <type_traits>

#include "phip_device.hpp"

namespace phip {

constexpr int kBlock = 256;

// Streaming loads, optionally non-temporal (read-once batch data should not
// push hot slot records out of the XCD's L2).
template <bool NT, class T>
__device__ inline T ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

__device__ inline u64 load_be64(const u8* p) {
  u64 v = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) v = (v << 8) | p[k];
  return v;
}

// ---------------------------------------------------------- name sources --
// Decoded messages: names[offs[i] .. offs[i+1]).  lim: the blob's byte
// length as the caller gave it (phip_msgs / phip_ops names_len), 0 when the
// caller did not (unchecked).  With lim, an entry that is not
// offs[i] <= offs[i+1] <= lim with at most PHIP_MAX_NAME_LEN bytes reads as
// the empty name at offset 0 (get() returns true): no kernel reads the blob
// at a wild offset, and the passes that check (k_classify_soa2,
// k_resolve_batch) report the entry, so the call returns PHIP_ERR_INVALID
// (bucket.go:71-91: malformed input is an error, not a crash).
struct NamesOffs {
  const u8* blob;
  const u32* offs;
  u32 lim = 0;
  __device__ inline bool bad(u32 a, u32 b) const {
    return lim != 0 && (b < a || b - a > PHIP_MAX_NAME_LEN || b > lim);
  }
  template <bool NT = false>
  __device__ inline bool get(u32 i, u64& off, u32& len) const {
    u32 a = ld<NT>(offs + i), b = ld<NT>(offs + i + 1);
    const bool x = bad(a, b);
    if (x) a = b = 0;
    off = a;
    len = b - a;
    return x;
  }
};
// Raw datagrams after decode: name at (off[i], len[i]) inside the datagram blob.
struct NamesPairs {
  const u8* blob;
  const uint64_t* off;
  const u8* len;
  template <bool NT = false>
  __device__ inline bool get(u32 i, u64& o, u32& l) const {
    o = ld<NT>(off + i);
    l = ld<NT>(len + i);
    return false;
  }
};

// Raw datagrams (bucket.go:59-64) read in place: name at offs[i] + 25, its
// length byte at offs[i] + 24, clamped to the datagram so that a malformed
// one never sends a name read past its end.
struct Datagrams {
  const u8* blob;
  const uint64_t* offs;
  template <bool NT = false>
  __device__ inline bool get(u32 i, u64& o, u32& l) const {
    const u64 a = ld<NT>(offs + i), b = ld<NT>(offs + i + 1);
    o = a + 25;
    const u64 room = b > o ? b - o : 0;
    const u32 want = b >= a + 25 ? blob[a + 24] : 0;
    l = want < room ? want : (u32)room;
    return false;
  }
};

// Bytes [8k, 8k + 8) of a byte string that starts `sh` bits into the
// aligned word p[0], assembled from aligned 8-byte loads; `lastw` is the
// word holding the string's last byte, so no load runs past it (bytes past
// the string come back as garbage: callers mask them).
// Device-scope coherent load (past the CU's L1): for data other threads of
// the same kernel may have just written (k_small_mixed's inserts).
__device__ inline u64 ld_co(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool Co = false>
__device__ inline u64 str_word(const u64* p, u32 sh, u32 k, u32 lastw) {
  const u64* a = p + (k < lastw ? k : lastw);
  const u64* b = p + (k + 1 < lastw ? k + 1 : lastw);
  const u64 lo = Co ? ld_co(a) : *a, hi = Co ? ld_co(b) : *b;
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}
__device__ inline u64 low_bytes(u64 w, u32 n) { return n >= 8 ? w : (w & ((1ull << (8 * n)) - 1)); }

// One FNV-1a step on the hash held as 32-bit halves:
// h*0x100000001b3 = h*0x1b3 + (h << 40), so hi' = hi*0x1b3 + carry + (lo << 8).
__device__ inline void fnv_step32(u32& lo, u32& hi, u32 c) {
  lo ^= c;
  const u64 p = (u64)lo * 0x1b3u;
  hi = (u32)((u64)hi * 0x1b3u + (p >> 32)) + (lo << 8);
  lo = (u32)p;
}
// FNV-1a over the low n (<= 8) bytes of w.
__device__ inline void fnv_word32(u32& lo, u32& hi, u64 w, u32 n) {
#pragma unroll
  for (u32 b = 0; b < 8; ++b)
    if (b < n) fnv_step32(lo, hi, (u32)(w >> (8 * b)) & 0xFFu);
}

// A name longer than kInlineName bytes read with aligned 8-byte loads (any
// alignment): FNV-1a and the canonical words of a long name (Rec: len in
// word 0, the first 16 bytes in words 1-2; the arena offset is the
// record's).
__device__ inline void load_name_long(const u8* src, u64 off, u32 len, Name& nm) {
  const u64* p = reinterpret_cast<const u64*>(src + (off & ~7ull));
  const u32 sh = (u32)(off & 7) * 8;
  const u32 lastw = ((u32)(off & 7) + len - 1) >> 3;
  u32 lo = (u32)kFnvOffset, hi = (u32)(kFnvOffset >> 32);
  const u64 w1 = str_word(p, sh, 0, lastw), w2 = str_word(p, sh, 1, lastw);   // len > 16
  fnv_word32(lo, hi, w1, 8);
  fnv_word32(lo, hi, w2, 8);
  for (u32 k = 16; k < len; k += 8) {
    const u32 n = len - k < 8 ? len - k : 8;
    fnv_word32(lo, hi, str_word(p, sh, k >> 3, lastw), n);
  }
  nm.h = ((u64)hi << 32) | lo; nm.len = len; nm.off = off;
  nm.w0 = len; nm.w1 = w1; nm.w2 = w2;
}

// Bytes [16, len) of a long name equal the arena copy at aoff (both read as
// words from aligned loads; Co: the arena side coherently).
template <bool Co = false>
__device__ inline bool long_tail_equal(const u8* arena, u64 aoff, const u8* src, u64 off, u32 len) {
  const u64 a0 = aoff + 16, s0 = off + 16;
  const u32 n = len - 16;
  const u64* pa = reinterpret_cast<const u64*>(arena + (a0 & ~7ull));
  const u64* ps = reinterpret_cast<const u64*>(src + (s0 & ~7ull));
  const u32 sha = (u32)(a0 & 7) * 8, shs = (u32)(s0 & 7) * 8;
  const u32 la = ((u32)(a0 & 7) + n - 1) >> 3, ls = ((u32)(s0 & 7) + n - 1) >> 3;
  for (u32 k = 0; k < n; k += 8) {
    const u32 m = n - k < 8 ? n - k : 8;
    if (low_bytes(str_word<Co>(pa, sha, k >> 3, la), m) != low_bytes(str_word(ps, shs, k >> 3, ls), m))
      return false;
  }
  return true;
}

// Name read with aligned 8-byte loads (up to 4 per name) instead of one
// byte load per character.  Needs the blob 8-byte aligned and readable up to
// the next 8-byte boundary past its last name (the ABI's slack rule).
template <bool NT>
__device__ inline void load_name_wide(const u8* src, u64 off, u32 len, Name& nm) {
  if (len > kInlineName) { load_name_long(src, off, len, nm); return; }
  const u32 sh = (u32)(off & 7) * 8;
  const u32 nw = ((u32)(off & 7) + len + 7) >> 3;
  const u64* p = reinterpret_cast<const u64*>(src + (off & ~7ull));
  const u64 w0 = nw > 0 ? ld<NT>(p) : 0, w1 = nw > 1 ? ld<NT>(p + 1) : 0;
  const u64 w2 = nw > 2 ? ld<NT>(p + 2) : 0, w3 = nw > 3 ? ld<NT>(p + 3) : 0;
  u64 b0 = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  u64 b1 = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
  u64 b2 = sh ? (w2 >> sh) | (w3 << (64 - sh)) : w2;
  if (len < 8) { b0 = len ? b0 & ((1ull << (8 * len)) - 1) : 0; b1 = 0; b2 = 0; }
  else if (len < 16) { b1 = len > 8 ? b1 & ((1ull << (8 * (len - 8))) - 1) : 0; b2 = 0; }
  else if (len < 24) { b2 = len > 16 ? b2 & ((1ull << (8 * (len - 16))) - 1) : 0; }
  u32 lo = (u32)kFnvOffset, hi = (u32)(kFnvOffset >> 32);
  fnv_word32(lo, hi, b0, len);
  if (len > 8) fnv_word32(lo, hi, b1, len - 8);
  if (len > 16) fnv_word32(lo, hi, b2, len - 16);
  nm.h = ((u64)hi << 32) | lo; nm.len = len; nm.off = off;
  nm.w0 = (u64)len | (b0 << 16);           // name byte k sits at canonical byte k+2
  nm.w1 = (b0 >> 48) | (b1 << 16);
  nm.w2 = (b1 >> 48) | (b2 << 16);
}

// Wave-aggregated append: returns this lane's position in `list`.
__device__ inline u32 wave_append(u32* counter, bool pred) {
  u64 mask = __ballot(pred);
  if (!pred) return 0;
  u32 lane = __lane_id();
  u32 leader = __ffsll((long long)mask) - 1;
  u32 rank = __popcll(mask & ((1ull << lane) - 1));
  u32 base = 0;
  if (lane == leader) base = atomicAdd(counter, (u32)__popcll(mask));
  base = __shfl(base, leader);
  return base + rank;
}

// Sharded append list.  A list that every wave of a large grid appends to
// through ONE counter serialises on that word once most waves have an entry
// (an insert-heavy batch: 1.5M appends per 100M messages, ~11 ns each).
// Instead, unit u (a wave's chunk, or a block) appends to shard u % kShards,
// whose region holds the entries of at most ceil(units / kShards) units;
// k_shard_scan + k_shard_compact then pack the shards into one list.
constexpr u32 kShards = 256;
__host__ __device__ inline u32 shard_cap(u32 units, u32 per_unit) {
  return per_unit * ((units + kShards - 1) / kShards);
}
struct Sharded {
  u32* base = nullptr;   // kShards regions of `cap` entries (nullptr: no list)
  u32* cnt = nullptr;    // kShards counters (zeroed before the kernel)
  u32 cap = 0;
  __device__ inline void append(u32 unit, bool pred, u32 v) const {
    const u32 sh = unit & (kShards - 1);
    const u32 pos = wave_append(&cnt[sh], pred);
    if (pred) base[(size_t)sh * cap + pos] = v;
  }
};

// A batch's counters in one launch: ctr[16] zero except ctr[5] (first
// malformed datagram) and ctr[kCtrDirty] (first dirty message), which start
// at "none"; and, when given, a sharded list's kShards counters.
__global__ __launch_bounds__(kShards) void k_batch_reset(u32* ctr, u32* shard_cnt) {
  const u32 t = threadIdx.x;
  if (t < 16) ctr[t] = (t == 5 || t == 12) ? ~0u : 0u;
  if (shard_cnt) shard_cnt[t] = 0;
}

// One workgroup of kShards lanes over a sharded list's counters: exclusive
// offsets of the shards (into cnt[kShards + s]), the total into ctr[tot] and
// the largest shard into ctr[13].  With `host` (the handle's pinned counter
// mirror, mapped into the device's address space), the first `words` counter
// words are then stored there, which ends a fast batch without a copy; with
// `next`, the next batch's counters (next_ctr: the other fast set) and its
// shard counters are reset as k_batch_reset does, so a queued batch's
// successor needs no reset launch.
__device__ inline void shard_scan(u32* cnt, u32* ctr, u32 tot, u32* host, u32 words, u32* next,
                                  u32* next_ctr);
__global__ __launch_bounds__(kShards) void k_shard_scan(u32* cnt, u32* ctr, u32 tot, u32* host,
                                                        u32 words, u32* next, u32* next_ctr) {
  shard_scan(cnt, ctr, tot, host, words, next, next_ctr);
}
__device__ inline void shard_scan(u32* cnt, u32* ctr, u32 tot, u32* host, u32 words, u32* next,
                                  u32* next_ctr) {
  __shared__ u32 v[kShards];
  __shared__ u32 wmax[kShards / 64];
  const u32 t = threadIdx.x, c = cnt[t];
  v[t] = c;
  u32 m = c;
  for (u32 d = 32; d; d >>= 1) m = max(m, (u32)__shfl_xor((int)m, d));
  if ((t & 63) == 0) wmax[t >> 6] = m;
  __syncthreads();
  for (u32 off = 1; off < kShards; off <<= 1) {
    const u32 x = t >= off ? v[t - off] : 0u;
    __syncthreads();
    v[t] += x;
    __syncthreads();
  }
  cnt[kShards + t] = v[t] - c;
  const u32 total = v[kShards - 1];
  u32 mx = 0;
  for (u32 w = 0; w < kShards / 64; ++w) mx = max(mx, wmax[w]);
  if (t == 0) {
    ctr[tot] = total;
    ctr[13] = mx;
  }
  if (host && t < words) {
    const u32 w = t == tot ? total : t == 13 ? mx : ctr[t];
    __hip_atomic_store(&host[t], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (next) {
    if (t < 16) next_ctr[t] = (t == 5 || t == 12) ? ~0u : 0u;
    next[t] = 0;
  }
}

// grid (ceil(max shard count / 256), kShards): shard s's entries, in order,
// to out[offset(s) ...].
__global__ __launch_bounds__(256) void k_shard_compact(const u32* __restrict__ base, u32 cap,
                                                       const u32* __restrict__ cnt,
                                                       u32* __restrict__ out) {
  const u32 s = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
  if (j < cnt[s]) out[cnt[kShards + s] + j] = base[(size_t)s * cap + j];
}

// Full-name equality for a candidate record (names > 22 bytes live in the arena).
template <bool Co = false>
__device__ inline bool name_equal(const Rec& r, const Name& nm, const u8* src, const u8* arena) {
  const u64 r0 = r.name0 & ~0xFF00ull;   // drop the flags byte
  if ((r0 & 0xFFu) != (nm.w0 & 0xFFu)) return false;
  if (nm.len <= kInlineName) return r0 == nm.w0 && r.name1 == nm.w1 && r.name2 == nm.w2;
  if (r.name1 != nm.w1 || r.name2 != nm.w2) return false;
  return long_tail_equal<Co>(arena, r.name0 >> 32, src, nm.off, nm.len);
}

enum ProbeResult : int { kFound = 0, kMiss = 1, kPending = 2, kFull = 3 };

// Seeded placement mix of a tag: murmur3's 64-bit finaliser of tag ^ seed
// (a bijection whose every output bit depends on every input bit), so that
// names crafted to share a home under one seed scatter under another.  The
// seed is per handle (phip_config.hash_seed / the OS), as Go's map seeds its
// hash per process (repo.go:175).
__host__ __device__ inline u64 seeded_mix(u64 tag, u64 seed) {
  u64 x = tag ^ seed;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// The device table, passed to kernels by value.
struct Table {
  Rec* recs;
  u32* aux;
  const u8* arena;
  u32 L;
  u64 tag_mask;   // all ones; narrower only in collision tests (phip_config.debug_tag_bits)
  u64 seed;       // placement seed (seeded_mix)
  __device__ inline u64 tag(u64 h) const { return tag_of(h & tag_mask); }
  __device__ inline u32 home(u64 tag) const { return (u32)(seeded_mix(tag, seed) >> (64 - L)); }
  __device__ inline u32 mask() const { return (u32)((1ull << L) - 1); }
};

// Whole-record load: four 16-byte loads issued together (one 64-byte burst),
// so tag, state and name arrive in one memory round trip.
__device__ inline Rec load_rec(const Rec* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1], c = q[2], d = q[3];
  Rec r;
  r.tag = ((u64)a.y << 32) | a.x;
  r.added = ((u64)a.w << 32) | a.z;
  r.taken = ((u64)b.y << 32) | b.x;
  r.elapsed = (i64)(((u64)b.w << 32) | b.z);
  r.name0 = ((u64)c.y << 32) | c.x;
  r.name1 = ((u64)c.w << 32) | c.z;
  r.created = (i64)(((u64)d.y << 32) | d.x);
  r.name2 = ((u64)d.w << 32) | d.z;
  return r;
}

// The first 48 bytes only (tag, state, name words 0-1); name2 and created
// are left 0.  Enough to find and merge a name of <= kShortName bytes.
#ifndef PHIP_REC48_X2
#define PHIP_REC48_X2 1   // (k_receive_fast 1.765 / 1.762 against 1.770 / 1.773 ms, one box)
#endif
__device__ inline Rec load_rec48(const Rec* p) {
  // (plain loads: the kernel lives on L2 / Infinity Cache retention of warm
  // records; non-temporal record loads made it 65% slower, DESIGN.md §4:
  // an nt load does not allocate, so the three loads of a record fetch its
  // 128-byte line ~2 times, tools/ubench_req)
#if PHIP_REC48_X2
  // six 8-byte loads (tools/ubench_req: random 48-byte records 2.27 ms per
  // 100M as dwordx2, 3.30 as dwordx4, the same one 128-byte request each)
  const u64* w = reinterpret_cast<const u64*>(p);
  const u64 w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4], w5 = w[5];
  const uint4 a{(u32)w0, (u32)(w0 >> 32), (u32)w1, (u32)(w1 >> 32)};
  const uint4 b{(u32)w2, (u32)(w2 >> 32), (u32)w3, (u32)(w3 >> 32)};
  const uint4 c{(u32)w4, (u32)(w4 >> 32), (u32)w5, (u32)(w5 >> 32)};
#else
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1], c = q[2];
#endif
  Rec r;
  r.tag = ((u64)a.y << 32) | a.x;
  r.added = ((u64)a.w << 32) | a.z;
  r.taken = ((u64)b.y << 32) | b.x;
  r.elapsed = (i64)(((u64)b.w << 32) | b.z);
  r.name0 = ((u64)c.y << 32) | c.x;
  r.name1 = ((u64)c.w << 32) | c.z;
  r.created = 0;
  r.name2 = 0;
  return r;
}

// Look the name up.  kFound: *slot = its slot and *rec = its contents (for
// names of <= kShortName bytes only the first 48 bytes: created/name2 = 0).
// kMiss: not present.  kPending: a same-tag slot is claimed but not yet
// published (only seen by insert rounds).
__device__ inline int probe(const Table& T, const Name& nm, const u8* src, u32* slot, Rec* rec) {
  const u64 tag = T.tag(nm.h);
  const u32 mask = T.mask();
  u32 s = T.home(tag);
  const bool shortname = nm.len <= kShortName;
  for (u32 k = 0; k <= mask; ++k) {
    Rec r = shortname ? load_rec48(&T.recs[s]) : load_rec(&T.recs[s]);
    if (r.tag == 0) return kMiss;
    if (r.tag == tag) {
      if (!(rec_flags(r) & kRecPublished)) return kPending;
      if (name_equal(r, nm, src, T.arena)) { *slot = s; *rec = r; return kFound; }
    }
    s = (s + 1) & mask;
  }
  return kFull;
}

// ----------------------------------------------------------- classify ----
// Counter slot of the first dirty message of a Receive batch: an incast
// (an all-zero state asks for a reply, repo.go:78,86-90) or a -0.0 field (Go's
// `>` and the E order disagree on +-0), the two things only the ordered path
// handles.  The fast path applies the clean prefix before it (merges commute),
// the ordered path the rest.
constexpr u32 kCtrDirty = 12;
constexpr u32 kCtrBadName = 1;   // an ordered batch's malformed name entry (k_resolve_batch)

// Min-reduce the index of a wave's first dirty lane (lanes hold increasing
// indices, so the lowest set lane has the lowest index).
__device__ inline void note_min(bool d, u32 i, u32* word) {
  const u64 m = __ballot(d);
  if (m && __lane_id() == (u32)(__ffsll((long long)m) - 1)) atomicMin(word, i);
}
__device__ inline void note_dirty(bool d, u32 i, u32* ctr) { note_min(d, i, &ctr[kCtrDirty]); }

// Dirty buckets (round 6).  Go's Receive loop is per bucket in effect: a
// message's result depends only on the messages before it that name the same
// bucket (repo.go:54-92, bucket.go:240-263).  And between two dirty messages
// (incast, -0.0 field: the ones whose place matters) of a bucket, its clean
// messages commute: their effect is one merge of their field-wise maximum.
// So a batch with a few dirty messages is not sent through the ordered path
// from its first dirty message on (a batch with one early incast was 5x
// slower than a clean one); instead the classification lists the dirty
// messages, k_dirty_build makes a set of the buckets they name, sorted
// per bucket, and the fast kernel
//   - merges every message of a clean bucket, and every message of a dirty
//     bucket before that bucket's first dirty message, as before;
//   - folds each later clean message of a dirty bucket into a cell, the
//     maximum of the clean messages between one of its dirty messages and
//     the next (E-encoded, as the table's fields);
// and dirty_finish turns the dirty messages and the non-empty cells into an
// ordered sub-batch of at most 3 * kDirtyCap entries (a dirty message, then
// the merge of its cell), which the ordered path applies after the rest of
// the batch.  Exact: every bucket sees the Go loop's sequence of states at
// its dirty messages.  Up to kDirtyCap dirty messages with names of at most
// kShortName bytes (the names the set compares exactly); otherwise the batch
// keeps the prefix rule.
constexpr u32 kCtrNDirty = 0;        // dirty messages listed (> kDirtyCap: the prefix rule)
constexpr u32 kCtrNDefer = 18;       // entries of the ordered sub-batch (dirty_finish)
constexpr u32 kCtrNSorted = 19;      // dirty messages in the set (before the batch's stop)
constexpr u32 kDirtyCap = 4096;
constexpr u32 kDirtySlots = 2 * kDirtyCap;
constexpr u64 kRecDirty = 4u;        // record flag: its bucket is in the batch's dirty set
__device__ inline void note_dirty_list(bool d, u32 i, u32* ctr, u32* dlist) {
  const u32 pos = wave_append(&ctr[kCtrNDirty], d);
  if (d && pos < kDirtyCap) dlist[pos] = i;
}
// The dirty buckets: open addressing over kDirtySlots keys (FNV-1a, 0 stored
// as 1; 0 = empty) with the canonical words beside them (exact for short
// names); per bucket its first dirty message, its dirty messages' range in
// `idx` (sorted by (set slot, message)) and its table slot.
struct DirtySet {
  u64* key;     // [kDirtySlots]
  u64* w;       // [2 * kDirtySlots]: w0, w1 of slot s at 2s, 2s + 1
  u32* ready;   // [kDirtySlots] w written
  u32* first;   // [kDirtySlots]
  u32* start;   // [kDirtySlots]
  u32* cnt;     // [kDirtySlots]
  u32* rslot;   // [kDirtySlots] table slot marked kRecDirty (~0: none)
  u32* idx;     // [kDirtyCap] dirty messages by (set slot, message)
  u32* dslot;   // [kDirtyCap] their set slots
  u64* cell;    // [3 * 2 * kDirtyCap] cell j < kDirtyCap: maxima of the clean messages
                //   after idx[j]; kDirtyCap + j: the bucket's messages before idx[j], its
                //   first (its "pre" cell, j the bucket's start)
  u32* premin;  // [kDirtyCap] the first message of the pre cell of start j
  static constexpr size_t kWords = 3 * (size_t)kDirtySlots + 5 * (size_t)kDirtySlots / 2 +
                                   (size_t)kDirtyCap + 6 * (size_t)kDirtyCap +
                                   (size_t)kDirtyCap / 2;
  __host__ __device__ static DirtySet at(u64* b) {
    DirtySet d;
    d.key = b;
    d.w = b + kDirtySlots;
    u32* u = reinterpret_cast<u32*>(b + 3 * (size_t)kDirtySlots);
    d.ready = u;
    d.first = u + kDirtySlots;
    d.start = u + 2 * kDirtySlots;
    d.cnt = u + 3 * kDirtySlots;
    d.rslot = u + 4 * kDirtySlots;
    d.idx = u + 5 * kDirtySlots;
    d.dslot = d.idx + kDirtyCap;
    d.cell = b + 3 * (size_t)kDirtySlots + 5 * (size_t)kDirtySlots / 2 + kDirtyCap;
    d.premin = reinterpret_cast<u32*>(d.cell + 6 * (size_t)kDirtyCap);
    return d;
  }
};
__device__ inline u32 dirty_home(u64 h) { return (u32)(h ^ (h >> 31)) & (kDirtySlots - 1); }
// The set slot of a (short) name, or -1.
__device__ inline int dirty_find(const DirtySet& D, const Name& nm) {
  const u64 k = nm.h ? nm.h : 1;
  for (u32 s = dirty_home(k);; s = (s + 1) & (kDirtySlots - 1)) {
    const u64 x = D.key[s];
    if (x == 0) return -1;
    if (x == k && D.w[2 * s] == nm.w0 && D.w[2 * s + 1] == nm.w1) return (int)s;
  }
}
// A cell field back to its replica bits: 0 (no clean message, or only NaN /
// -Inf, which never win Go's `<`) reads NaN, which never wins either.
__device__ inline u64 dec_replica_max(u64 x) {
  if (x == 0) return 0x7FF8000000000000ull;
  if (x == kInfBits) return 0;                    // +-0 (a clean batch's are +0)
  if (x > kInfBits) return x - kInfBits - 1;
  return kSign | (kInfBits - x);
}

__device__ inline bool replica_dirty(u64 ab, u64 tb, i64 e) {
  const bool inc = is_zero_bits(ab) && is_zero_bits(tb) && e == 0;
  return inc || ab == kSign || tb == kSign;
}

// ------------------------------------------------------- fast receive ----
// The batched Receive loop (repo.go:54-92) for a batch with no incast and no
// -0.0: GetBucket(name) + Merge(&remote) for every message.
//
// One lane per message.  The kernel is bound by memory latency, so every
// lane issues its loads in as few dependent rounds as possible:
//   round 1  name offsets + the three replica fields (all independent);
//   round 2  the name as three aligned 8-byte words, each address clamped to
//            the name's own last word (always in bounds, so no branches);
//   round 3  the home slot's first 48 bytes (tag, state, name words 0-1).
// Names of more than kShortName bytes and probe chains longer than one slot
// take a divergent slow path (rare: C2's names are <= 8 bytes, load 0.3).
//
// The lane then compares the replica against the state it just read.  Only
// fields that would grow go further: they are max-combined per slot in an LDS
// table shared by the workgroup, and one lane per distinct slot issues the
// device-scope atomicMax for the combined value.  State only grows
// (E-encoding, phip_device.hpp), so a stale read can only cause a redundant
// atomic, never a lost update; combining keeps a Zipf-hot bucket at one
// atomic per workgroup instead of one per message, and a workgroup in which
// no field grows skips the flush.  Misses are appended to `miss` (insert
// pipeline, then this kernel again on the miss list with `track_new`).
constexpr u32 kCombEmpty = 0xFFFFFFFFu;
constexpr u32 kCombSlots = 256;
constexpr u32 kCombBits = 8;
static_assert((1u << kCombBits) == kCombSlots, "combining table size");

// Name words for a name of <= kShortName bytes: the three aligned words that
// can hold it, with each address clamped to the word holding its last byte
// (so all three loads issue unconditionally and stay inside the name).
template <bool NT>
__device__ inline void load_words3(const u8* blob, u64 off, u32 len, u64& w0, u64& w1, u64& w2) {
  const u64* p = reinterpret_cast<const u64*>(blob);
  const u64 wb = off >> 3;
  const u64 we = (off + (len ? len : 1u) - 1) >> 3;
  w0 = ld<NT>(p + wb);
  w1 = ld<NT>(p + (wb + 1 < we ? wb + 1 : we));
  w2 = ld<NT>(p + (wb + 2 < we ? wb + 2 : we));
}

// FNV-1a and the canonical words of a name of <= kShortName bytes from the
// words load_words3 returned (bytes past the name's end are ignored).
__device__ inline void short_name(u64 w0, u64 w1, u64 w2, u64 off, u32 len, Name& nm) {
  const u32 sh = (u32)(off & 7) * 8;
  u64 b0 = (w0 >> sh) | ((w1 << 1) << (63 - sh));
  u64 b1 = (w1 >> sh) | ((w2 << 1) << (63 - sh));
  b0 = len >= 8 ? b0 : (b0 & ((1ull << (8 * len)) - 1));
  b1 = len > 8 ? (b1 & ((1ull << (8 * (len - 8))) - 1)) : 0;
  u32 lo = (u32)kFnvOffset, hi = (u32)(kFnvOffset >> 32);
  const u32 q[4] = {(u32)b0, (u32)(b0 >> 32), (u32)b1, (u32)(b1 >> 32)};
  // A wave whose names all fit in 8 bytes (most of a batch of short names)
  // hashes 8 bytes, not 14 (a wave-uniform branch on one ballot).
  if (__builtin_amdgcn_ballot_w64(len > 8) == 0) {
#pragma unroll
    for (u32 k = 0; k < 8; ++k)
      if (k < len) fnv_step32(lo, hi, (q[k >> 2] >> (8 * (k & 3))) & 0xFFu);
  } else
  {
#pragma unroll
    for (u32 k = 0; k < kShortName; ++k)
      if (k < len) fnv_step32(lo, hi, (q[k >> 2] >> (8 * (k & 3))) & 0xFFu);
  }
  nm.h = ((u64)hi << 32) | lo; nm.len = len; nm.off = off;
  nm.w0 = (u64)len | (b0 << 16);     // name byte k sits at canonical byte k+2
  nm.w1 = (b0 >> 48) | (b1 << 16);
  nm.w2 = 0;
}

// FNV-1a and canonical words of an inline name of kShortName < len <=
// kInlineName bytes from the words the fast kernel already loaded (w0..w2 as
// load_words3 returns them) and the next word w3 (clamped like them).
__device__ inline void inline_name(u64 w0, u64 w1, u64 w2, u64 w3, u64 off, u32 len, Name& nm) {
  const u32 sh = (u32)(off & 7) * 8;
  const u64 b0 = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  u64 b1 = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
  u64 b2 = sh ? (w2 >> sh) | (w3 << (64 - sh)) : w2;
  b1 = low_bytes(b1, len - 8);
  b2 = len > 16 ? low_bytes(b2, len - 16) : 0;
  u32 lo = (u32)kFnvOffset, hi = (u32)(kFnvOffset >> 32);
  fnv_word32(lo, hi, b0, 8);
  fnv_word32(lo, hi, b1, len - 8);
  if (len > 16) fnv_word32(lo, hi, b2, len - 16);
  nm.h = ((u64)hi << 32) | lo; nm.len = len; nm.off = off;
  nm.w0 = (u64)len | (b0 << 16);     // name byte k sits at canonical byte k+2
  nm.w1 = (b0 >> 48) | (b1 << 16);
  nm.w2 = (b1 >> 48) | (b2 << 16);
}

// enc_replica for a replica field that is not -0.0 (the fast path's batches
// hold none), without branches.
__device__ inline u64 enc_replica_nz(u64 b) {
  const u64 mag = b & ~kSign;
  const u64 e = (b >> 63) ? kInfBits - mag : kInfBits + mag + (mag != 0);
  return mag > kInfBits ? 0ull : e;
}

// ------------------------------------------------- hot-bucket directory --
// Zipf-skewed batches put most messages on a few buckets (C2: the 732
// hottest of 10M buckets carry 63% of the messages).  Before the fast kernel runs, a
// strided sample of the batch is resolved and counted; the (at most kHotMax)
// buckets sampled most often form the batch's hot directory.  Every fast
// workgroup keeps the directory in LDS and folds the messages of those
// buckets into per-workgroup maxima there, with no record read, flushing them
// with one atomicMax per field at the end.  Merge is an order-free max on the
// fast path, so this is exact; the directory only decides which messages skip
// the table read.
// (PHIP_HOT_MAX / PHIP_HOT_LDS / PHIP_FAST_BLOCK / PHIP_FAST_PER_CU override
// the defaults for tuning builds, tools/build_variants.sh.)
// 736 entries in a 4096-slot lookup (18% load) with two 1024-lane
// workgroups a CU fill its 160 KB of LDS; against 384 in 1024 slots with
// four 512-lane workgroups: k_receive_fast 1.78-1.79 vs 1.85 ms on C2
// (DESIGN.md §4 round 5).  The lookup's load matters as much as the size:
// 640 entries in 1024 slots ran 2.06 ms.
#ifndef PHIP_HOT_MAX
#define PHIP_HOT_MAX 736
#endif
#ifndef PHIP_HOT_LDS
#define PHIP_HOT_LDS 4096
#endif
constexpr u32 kHotMax = PHIP_HOT_MAX;     // directory entries
constexpr u32 kHotLds = PHIP_HOT_LDS;     // LDS lookup slots (power of 2, >= 1.5 * kHotMax)
// The sender-side combine's directory (phip_route_pack): its own size, as its
// kernels hold less per entry in LDS than k_receive_fast.
constexpr u32 kRouteHotMax = 512;
static_assert(kHotLds * 2 >= kRouteHotMax * 3 && kHotLds * 2 >= kHotMax * 3, "LDS lookup load");
constexpr u32 kHotCntBits = 18;       // sample count table: 2^18 (slot+1, count) pairs
constexpr u32 kHotSampleMax = 1u << 17;   // samples per batch (half the count table)
constexpr u32 kHotSamplePerBlock = 1024;   // 128 workgroups: the chain runs beside k_classify on stream2 (512 one-sample workgroups queued behind its blocks and delayed the join)
constexpr u32 kHotHist = 4096;        // histogram bins of sample counts
constexpr u32 kHotMinCount = 8;       // sample hits for a bucket to qualify
// Smaller batches skip the directory.  2^16, not larger: a skewed batch of a
// few 100k messages (C1: 1M into 100k buckets, 13% of them on one bucket)
// otherwise sends every message of its hottest bucket to one record as a
// device-scope atomicMax, and those serialise at the memory side.
constexpr u32 kHotMinBatch = 1u << 16;
constexpr u32 kRouteMinBatch = 1u << 20;   // the route combine's (phip_route_pack)
// A fast batch with this many misses creates its buckets from one message per
// name and merges by a second fast pass (finish_many_misses); fewer go
// through k_receive_list.
#ifndef PHIP_MANY_MISSES
#define PHIP_MANY_MISSES (1u << 16)
#endif
constexpr u32 kManyMisses = PHIP_MANY_MISSES;

// Hot names of up to kHotTailName bytes are matched from LDS alone: the
// directory also holds bytes [16, len) of an arena name (tail words).
constexpr u32 kHotTailName = 40;
constexpr u32 kHotTailWords = (kHotTailName - 16) / 8;
struct HotEntry {
  u64 tag, w0, w1, w2;   // table tag and canonical name words (flags byte and arena offset cleared)
  u64 tail[kHotTailWords];   // arena names of <= kHotTailName bytes: bytes [16, len), zero-padded
  u32 slot, aoff;        // record slot; arena offset of a name longer than kInlineName
};
struct HotHdr {
  u32 n;             // directory entries
  u32 thresh;        // sample count threshold that selected them
  u32 pad[14];
};

__device__ inline u32 hot_home(u64 tag) { return (u32)(tag ^ (tag >> 29)) & (kHotLds - 1); }

// Sample j = message j*stride: resolve it and count its
// slot, aggregated per workgroup in LDS first (a hot slot is sampled by most
// lanes; one global atomic per workgroup and slot keeps it off one address).
template <class Src>
__global__ __launch_bounds__(256) void k_hot_sample(Src src, u32 n, u32 stride, u32 nsample, Table T,
                                                    u32* __restrict__ ckeys, u32* __restrict__ ccnt) {
  constexpr u32 kPer = kHotSamplePerBlock / 256;
  constexpr u32 kL = 2 * kHotSamplePerBlock;
  __shared__ u32 lkey[kL], lcnt[kL];
  for (u32 e = threadIdx.x; e < kL; e += 256) { lkey[e] = 0; lcnt[e] = 0; }
  __syncthreads();
  for (u32 r = 0; r < kPer; ++r) {
    const u32 j = blockIdx.x * kHotSamplePerBlock + r * 256 + threadIdx.x;
    const u64 i = (u64)j * stride;
    if (j >= nsample || i >= n) continue;
    u64 off; u32 len;
    src.template get<true>((u32)i, off, len);
    Name nm;
    load_name_wide<true>(src.blob, off, len, nm);
    u32 s;
    Rec rec;
    if (probe(T, nm, src.blob, &s, &rec) != kFound) continue;
    u32 h = (s * 2654435761u) & (kL - 1);
    for (;;) {   // at most kHotSamplePerBlock distinct keys in 2x as many entries
      const u32 old = atomicCAS(&lkey[h], 0u, s + 1);
      if (old == 0 || old == s + 1) { atomicAdd(&lcnt[h], 1u); break; }
      h = (h + 1) & (kL - 1);
    }
  }
  __syncthreads();
  constexpr u32 mask = (1u << kHotCntBits) - 1;
  for (u32 e = threadIdx.x; e < kL; e += 256) {
    const u32 key = lkey[e];
    if (!key) continue;
    u32 h = ((key - 1) * 2654435761u) >> (32 - kHotCntBits);
    for (u32 k = 0; k <= mask; ++k) {
      const u32 old = atomicCAS(&ckeys[h], 0u, key);
      if (old == 0 || old == key) { atomicAdd(&ccnt[h], lcnt[e]); break; }
      h = (h + 1) & mask;
    }
  }
}

__global__ void k_hot_hist(const u32* __restrict__ ccnt, u32* __restrict__ hist) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (1u << kHotCntBits)) return;
  const u32 c = ccnt[e];
  if (c >= kHotMinCount) atomicAdd(&hist[c < kHotHist ? c : kHotHist - 1], 1u);
}

// One workgroup of 256: the lowest threshold t >= kHotMinCount with at most
// maxn sampled slots counted t or more times (maxn: the directory's size).
__global__ __launch_bounds__(256) void k_hot_select(const u32* __restrict__ hist, HotHdr* hdr,
                                                    u32 maxn) {
  constexpr u32 kPer = kHotHist / 256;
  __shared__ u32 part[256];
  __shared__ u32 best;
  const u32 t = threadIdx.x;
  u32 s = 0;
  for (u32 k = 0; k < kPer; ++k) s += hist[t * kPer + k];
  part[t] = s;
  if (t == 0) best = kHotHist;
  __syncthreads();
  u32 run = 0;   // slots counted in later chunks
  for (u32 u = t + 1; u < 256; ++u) run += part[u];
  u32 lo = kHotHist;
  for (int b = (int)kPer - 1; b >= 0; --b) {
    run += hist[t * kPer + b];
    if (run <= maxn) lo = t * kPer + b;
  }
  atomicMin(&best, lo);
  __syncthreads();
  if (t == 0) {
    hdr->n = 0;
    hdr->thresh = best > kHotMinCount ? best : kHotMinCount;
  }
}

__global__ void k_hot_build(const u32* __restrict__ ckeys, const u32* __restrict__ ccnt, HotHdr* hdr,
                            Table T, HotEntry* __restrict__ dir) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (1u << kHotCntBits)) return;
  const u32 c = ccnt[e];
  if (c < kHotMinCount || c < hdr->thresh) return;
  const u32 idx = atomicAdd(&hdr->n, 1u);
  if (idx >= kHotMax) return;   // cannot happen: the threshold bounds the count
  const u32 s = ckeys[e] - 1;
  const Rec r = load_rec(&T.recs[s]);
  HotEntry d;
  const bool arena = (r.name0 & 0xFFu) > kInlineName;
  d.tag = r.tag;
  d.w0 = arena ? (r.name0 & 0xFFu) : (r.name0 & ~0xFF00ull);
  d.w1 = r.name1;
  d.w2 = r.name2;
  d.slot = s;
  d.aoff = arena ? (u32)(r.name0 >> 32) : 0u;
  const u32 len = (u32)(r.name0 & 0xFFu);
  for (u32 k = 0; k < kHotTailWords; ++k) d.tail[k] = 0;
  if (arena && len <= kHotTailName) {
    const u64 a0 = (r.name0 >> 32) + 16;
    const u64* p = reinterpret_cast<const u64*>(T.arena + (a0 & ~7ull));
    const u32 sh = (u32)(a0 & 7) * 8, lastw = ((u32)(a0 & 7) + len - 17) >> 3;
    for (u32 k = 0; 8 * k < len - 16; ++k) {
      const u32 m = len - 16 - 8 * k;
      d.tail[k] = low_bytes(str_word(p, sh, k, lastw), m);
    }
  }
  dir[idx] = d;
}

// ----------------------------------------------------- fast receive --------
// Statuses: the caller's status column is filled with PHIP_ST_MERGED
// before the kernel (by k_classify_soa2, or a fill beside k_classify); every
// message the kernel does not merge is written again later (misses by the
// miss path, dirty buckets by the ordered path).
// Persistent workgroups; every wave walks its own 64-message chunks
// (grid-stride over waves, no workgroup barrier inside the loop, so a wave
// waiting on a table read never holds up another).  Per message:
//   hot directory hit  -> fold into the workgroup's LDS maxima (no table read);
//   otherwise          -> read the home slot's first 48 bytes, compare, and
//                         atomicMax the fields that grow.
// Cold buckets almost never repeat inside a chunk once the hot ones are in
// the directory, so there is no workgroup-wide combining table.  State only
// grows (E-encoding, phip_device.hpp), so a stale read can only cause a
// redundant atomic, never a lost update.  Misses are appended to `miss`; the
// insert pipeline then creates their buckets and k_receive_list merges them.
#ifndef PHIP_FAST_BLOCK
#define PHIP_FAST_BLOCK 1024
#endif
#ifndef PHIP_FAST_PER_CU
#define PHIP_FAST_PER_CU 2
#endif
constexpr u32 kFastBlock = PHIP_FAST_BLOCK;
constexpr u32 kFastPerCU = PHIP_FAST_PER_CU;   // resident workgroups per CU (LDS-bound)

// Batch inputs of the fast kernel.  load() issues a message's loads in two
// dependent rounds (offsets, then everything they address) and returns the
// name's offset/length, the three words that can hold a short name, and the
// replica fields as Go's UnmarshalBinary would hand them over.
template <class Src>
struct SoaIn {   // decoded messages (phip_receive_soa / decoded datagrams)
  Src src;
  const uint64_t* ma;
  const uint64_t* mt;
  const int64_t* me;
  static constexpr bool kSoa = true;
  __device__ inline const u8* blob() const { return src.blob; }
  // Round 1 of a message on its own (the name's offset and length), so the
  // fast kernel can issue it one chunk ahead.
  // (NamesOffs: the two u32 offsets as loaded, two registers; other name
  // sources: offset and length.)
  struct PreOffs { u32 a, b; };
  struct PreGen { u64 off; u32 len; };
  static constexpr bool kOffs = std::is_same<Src, NamesOffs>::value;
  using Pre = typename std::conditional<kOffs, PreOffs, PreGen>::type;
  __device__ inline Pre pre(u32 i) const {
    Pre p;
    if constexpr (kOffs) {
      p.a = ld<true>(src.offs + i);
      p.b = ld<true>(src.offs + i + 1);
    } else {
      src.template get<true>(i, p.off, p.len);
    }
    return p;
  }
  // Round 2 given round 1: the name words and the replica fields.
  __device__ inline void load(u32 i, const Pre& p, u64& off, u32& len, u64& w0, u64& w1, u64& w2,
                              u64& ra, u64& rt, i64& re) const {
    if constexpr (kOffs) { off = p.a; len = p.b - p.a; }
    else { off = p.off; len = p.len; }
    ra = ld<true>(ma + i); rt = ld<true>(mt + i); re = ld<true>(me + i);
    load_words3<false>(src.blob, off, len, w0, w1, w2);
  }
  // Classification (elapsed matters only when both floats are zero, so it is
  // read only then: a third of the pass's bytes on a clean batch).  A
  // malformed name entry (NamesOffs::bad, checked names only) min-reduces its
  // index into ctr[5], as a short datagram does: the batch stops there.
  __device__ inline bool dirty(u32 i, u32* ctr) const {
    if constexpr (kOffs) {
      if (src.lim && src.bad(src.offs[i], src.offs[i + 1])) {
        atomicMin(&ctr[5], i);
        return false;
      }
    }
    const u64 ab = __builtin_nontemporal_load(ma + i), tb = __builtin_nontemporal_load(mt + i);
    if (is_zero_bits(ab) && is_zero_bits(tb)) return me[i] == 0 || ab == kSign || tb == kSign;
    return ab == kSign || tb == kSign;
  }
};

// Raw datagrams (bucket.go:59-64): bytes[offs[i] .. offs[i+1]) = added,
// taken, elapsed (big-endian 8-byte words), one length byte, the name.  Read
// in place: the header as four aligned words and the name as three, every
// address clamped into the datagram, all issued in the second round (the
// name words are placed from the datagram's end, not its length byte).  Only
// datagrams before the first malformed one are merged (k_classify_wire).
__device__ inline u64 funnel8(u64 lo, u64 hi, u32 sb) {   // bytes sb..sb+7 of hi:lo, sb < 8
  return sb ? (lo >> (8 * sb)) | (hi << (64 - 8 * sb)) : lo;
}
struct WireIn {
  const u8* bytes;
  const uint64_t* offs;
  static constexpr bool kSoa = false;
  __device__ inline const u8* blob() const { return bytes; }
  struct Pre { u64 o; u32 sz; };   // round 1: the datagram's start and size
  __device__ inline Pre pre(u32 i) const {
    const u64 o = ld<true>(offs + i), end = ld<true>(offs + i + 1);
    return Pre{o, (u32)min(end - o, (u64)0xFFFFFFFFu)};
  }
  __device__ inline void load(u32 i, const Pre& pr, u64& off, u32& len, u64& w0, u64& w1, u64& w2,
                              u64& ra, u64& rt, i64& re) const {
    const u64 o = pr.o, end = pr.o + pr.sz;
    const u64* p = reinterpret_cast<const u64*>(bytes);
    const u64 last = (end > o ? end - 1 : o) >> 3;   // word of the datagram's last byte
    const u64 hb = o >> 3;
    // Plain (L1-allocating) loads: the seven words of a lane and its
    // neighbours' share cache lines, so only the first touch of a line goes
    // to L2.
    u64 h[4];
#pragma unroll
    for (u32 k = 0; k < 4; ++k) h[k] = ld<false>(p + (hb + k < last ? hb + k : last));
    off = o + 25;
    const u64 nb = off >> 3;
    const u64 nb0 = nb < last ? nb : last, nb1 = nb + 1 < last ? nb + 1 : last;
    const u64 nb2 = nb + 2 < last ? nb + 2 : last;
    w0 = ld<false>(p + nb0); w1 = ld<false>(p + nb1); w2 = ld<false>(p + nb2);
    const u32 sb = (u32)(o & 7);
    ra = __builtin_bswap64(funnel8(h[0], h[1], sb));
    rt = __builtin_bswap64(funnel8(h[1], h[2], sb));
    re = (i64)__builtin_bswap64(funnel8(h[2], h[3], sb));
    len = (u32)(h[3] >> (8 * sb)) & 0xFFu;
  }
  // Classification from the header words: a malformed datagram
  // (io.ErrShortBuffer, bucket.go:72,84) min-reduces its index into ctr[5]
  // (the Go loop stops there); otherwise incast / -0.0 as SoaIn::dirty.
  __device__ inline bool dirty(u32 i, u32* ctr) const {
    const u64 o = offs[i], end = offs[i + 1], sz = end - o;
    const u64* p = reinterpret_cast<const u64*>(bytes);
    const u64 last = (end > o ? end - 1 : o) >> 3, hb = o >> 3;
    u64 h[4];
#pragma unroll
    for (u32 k = 0; k < 4; ++k) h[k] = p[hb + k < last ? hb + k : last];
    const u32 sb = (u32)(o & 7);
    const u32 len = (u32)(h[3] >> (8 * sb)) & 0xFFu;
    if (sz < PHIP_BUCKET_FIXED_SIZE || sz - PHIP_BUCKET_FIXED_SIZE < len) {
      atomicMin(&ctr[5], i);
      return false;
    }
    return replica_dirty(__builtin_bswap64(funnel8(h[0], h[1], sb)),
                         __builtin_bswap64(funnel8(h[1], h[2], sb)),
                         (i64)__builtin_bswap64(funnel8(h[2], h[3], sb)));
  }
};

// Classification of a fast batch: the first dirty message into
// ctr[kCtrDirty], the first malformed datagram into ctr[5].  One atomic per
// wave that finds one, none on a clean batch.
template <class In>
__global__ __launch_bounds__(kBlock) void k_classify(In in, u32 n, u32* ctr, u32* dlist) {
  const u32 i = blockIdx.x * kBlock + threadIdx.x;
  const bool d = i < n && in.dirty(i, ctr);
  note_dirty(d, i, ctr);
  if (dlist && __ballot(d)) note_dirty_list(d, i, ctr, dlist);
}

// The dirty set of a classified batch (one workgroup, behind the
// classification; a batch without a dirty message returns at once): every
// listed dirty message's bucket, its dirty messages sorted, its record marked
// kRecDirty (the fast kernel reads that flag with the record it loads anyway:
// no set lookup for a clean bucket's message), its cells cleared.  A batch
// with more than kDirtyCap dirty messages, or one with a name longer than
// kShortName, is marked (ctr[kCtrNDirty] = ~0) before anything is marked: it
// keeps the prefix rule.  Dirty messages at or past the batch's stop (a
// checked batch's first malformed entry) are not read.
template <class In>
__global__ __launch_bounds__(1024) void k_dirty_build(In in, u32 n, u32* ctr, const u32* dlist,
                                                      DirtySet D, Table T) {
  __shared__ u64 sk[kDirtyCap];   // (set slot, message) keys
  __shared__ u32 longname, nvalid;
  const u32 nd = ctr[kCtrNDirty];
  if (nd == 0 || nd > kDirtyCap) return;
  const u32 tid = threadIdx.x;
  for (u32 s = tid; s < kDirtySlots; s += 1024) {
    D.key[s] = 0;
    D.ready[s] = 0;
    D.first[s] = ~0u;
  }
  if (tid == 0) { longname = 0; nvalid = 0; }
  __syncthreads();
  const u32 stop = min(n, ctr[5]);
  u32 valid = 0;
  for (u32 j = tid; j < nd; j += 1024) {
    const u32 i = dlist[j];
    sk[j] = ~0ull;
    if (i >= stop) continue;
    u64 off, w0, w1, w2, ra, rt;
    u32 len;
    i64 re;
    const typename In::Pre p = in.pre(i);
    in.load(i, p, off, len, w0, w1, w2, ra, rt, re);
    if (len > kShortName) {
      longname = 1;
      continue;
    }
    Name nm;
    short_name(w0, w1, w2, off, len, nm);
    const u64 k = nm.h ? nm.h : 1;
    // One slot per bucket: the lane that claims a key writes its words and
    // then `ready`; a lane that finds the same key waits for `ready` by
    // trying again (in the same loop, so lanes of one wave never wait on
    // each other across a branch).
    u32 s = dirty_home(k);
    for (;;) {
      const u64 old = atomicCAS(&D.key[s], 0ull, k);
      if (old == 0ull) {
        D.w[2 * s] = nm.w0;
        D.w[2 * s + 1] = nm.w1;
        __threadfence_block();
        atomicExch(&D.ready[s], 1u);
        break;
      }
      if (old == k) {
        if (__hip_atomic_load(&D.ready[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
          continue;
        if (D.w[2 * s] == nm.w0 && D.w[2 * s + 1] == nm.w1) break;
      }
      s = (s + 1) & (kDirtySlots - 1);
    }
    atomicMin(&D.first[s], i);
    sk[j] = ((u64)s << 32) | i;
    ++valid;
  }
  if (valid) atomicAdd(&nvalid, valid);
  __syncthreads();
  if (longname) {
    if (tid == 0) ctr[kCtrNDirty] = ~0u;
    return;
  }
  // bitonic sort of the keys (the unused ones, ~0, last)
  u32 P = 1;
  while (P < nd) P <<= 1;
  for (u32 j = nd + tid; j < P; j += 1024) sk[j] = ~0ull;
  __syncthreads();
  for (u32 k = 2; k <= P; k <<= 1) {
    for (u32 j = k >> 1; j > 0; j >>= 1) {
      for (u32 t = tid; t < P; t += 1024) {
        const u32 u = t ^ j;
        if (u > t) {
          const u64 x = sk[t], y = sk[u];
          if ((x > y) == ((t & k) == 0)) { sk[t] = y; sk[u] = x; }
        }
      }
      __syncthreads();
    }
  }
  const u32 nv = nvalid;
  for (u32 j = tid; j < nv; j += 1024) {
    const u32 s = (u32)(sk[j] >> 32);
    D.idx[j] = (u32)sk[j];
    D.dslot[j] = s;
    D.cell[3 * j] = 0; D.cell[3 * j + 1] = 0; D.cell[3 * j + 2] = 0;
    u64* pc = D.cell + 3 * ((size_t)kDirtyCap + j);
    pc[0] = 0; pc[1] = 0; pc[2] = 0;
    D.premin[j] = ~0u;
    if (j == 0 || (u32)(sk[j - 1] >> 32) != s) D.start[s] = j;
  }
  __syncthreads();
  for (u32 j = tid; j < nv; j += 1024) {
    const u32 s = (u32)(sk[j] >> 32);
    if (j + 1 == nv || (u32)(sk[j + 1] >> 32) != s) D.cnt[s] = j + 1 - D.start[s];
    if (j == 0 || (u32)(sk[j - 1] >> 32) != s) {
      // the bucket's record, if it has one: marked for the fast kernel
      const u32 i = (u32)sk[j];
      u64 off, w0, w1, w2, ra, rt;
      u32 len;
      i64 re;
      const typename In::Pre p = in.pre(i);
      in.load(i, p, off, len, w0, w1, w2, ra, rt, re);
      Name nm;
      short_name(w0, w1, w2, off, len, nm);
      u32 slot;
      Rec cur;
      if (probe(T, nm, in.blob(), &slot, &cur) == kFound) {
        D.rslot[s] = slot;
        atomicOr(reinterpret_cast<unsigned long long*>(&T.recs[slot].name0),
                 (unsigned long long)(kRecDirty << 8));
      } else {
        D.rslot[s] = ~0u;
      }
    }
  }
  if (tid == 0) {
    ctr[kCtrNSorted] = nv;
    if (nv == 0) ctr[kCtrNDirty] = 0;   // (every dirty message past the stop)
  }
}

// The same for decoded messages with 16-byte aligned replica columns: two
// messages per lane, one 16-byte load per column (the pass is a pure stream
// of 16 bytes per message; elapsed is read only when both floats are zero).
// Lane l holds messages 2l, 2l+1 of its wave's 128, so the lowest dirty lane
// still holds the lowest dirty index.  With `status`, the pass also fills the
// status column with PHIP_ST_MERGED (2 bytes per lane), which the fast kernel
// relies on: it writes no status for the messages it merges.
// With names.lim (a caller-given blob length), the pass also checks the name
// offsets (two more 4-byte loads per lane) and min-reduces the first
// malformed entry into ctr[5]: the fast kernel stops there (its gate), and so
// does the batch (PHIP_ERR_INVALID).  Unchecked batches read no offsets (the
// check costs the C2 step ~0.1 ms per 100M messages: a 0.4 GB stream).
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(kBlock) void k_classify_soa2(const uint64_t* __restrict__ ma,
                                                          const uint64_t* __restrict__ mt,
                                                          const int64_t* __restrict__ me, u32 n,
                                                          u32* ctr, u8* status, NamesOffs names,
                                                          u32* dlist) {
  const u32 i0 = 2 * (blockIdx.x * kBlock + threadIdx.x);
  if (names.lim) {   // (uniform)
    bool b0 = false, b1 = false;
    if (i0 < n) {
      const u32 o0 = names.offs[i0], o1 = names.offs[i0 + 1];
      const u32 o2 = i0 + 1 < n ? names.offs[i0 + 2] : o1;
      b0 = names.bad(o0, o1);
      b1 = i0 + 1 < n && names.bad(o1, o2);
    }
    note_min(b0 || b1, b0 ? i0 : i0 + 1, &ctr[5]);
  }
  if (status) {   // every status starts as merged (the fast pass writes none)
    if (i0 + 1 < n && ((uintptr_t)status & 1) == 0)
      *reinterpret_cast<u16*>(status + i0) = (u16)(PHIP_ST_MERGED | (PHIP_ST_MERGED << 8));
    else {
      if (i0 < n) status[i0] = PHIP_ST_MERGED;
      if (i0 + 1 < n) status[i0 + 1] = PHIP_ST_MERGED;
    }
  }
  bool d = false, e0 = false, e1 = false;
  u32 at = i0;
  if (i0 + 1 < n) {
    const u64x2 a = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(ma + i0));
    const u64x2 t = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(mt + i0));
    const bool z0 = is_zero_bits(a.x) && is_zero_bits(t.x);
    const bool z1 = is_zero_bits(a.y) && is_zero_bits(t.y);
    const bool d0 = (z0 && me[i0] == 0) || a.x == kSign || t.x == kSign;
    const bool d1 = (z1 && me[i0 + 1] == 0) || a.y == kSign || t.y == kSign;
    d = d0 || d1;
    at = d0 ? i0 : i0 + 1;
    e0 = d0;
    e1 = d1;
  } else if (i0 < n) {
    const u64 a = ma[i0], t = mt[i0];
    d = (is_zero_bits(a) && is_zero_bits(t) && me[i0] == 0) || a == kSign || t == kSign;
    e0 = d;
  }
  note_dirty(d, at, ctr);
  if (dlist && __ballot(d)) {   // (rare: the dirty messages, listed)
    note_dirty_list(e0, i0, ctr, dlist);
    note_dirty_list(e1, i0 + 1, ctr, dlist);
  }
}

// load_name_long for kInlineName < len <= kHotTailName, also returning the
// tail words (bytes [16, len), zero-padded).
__device__ inline void load_name_tail(const u8* src, u64 off, u32 len, Name& nm, u64 (&tail)[kHotTailWords]) {
  const u64* p = reinterpret_cast<const u64*>(src + (off & ~7ull));
  const u32 sh = (u32)(off & 7) * 8;
  const u32 lastw = ((u32)(off & 7) + len - 1) >> 3;
  u32 lo = (u32)kFnvOffset, hi = (u32)(kFnvOffset >> 32);
  const u64 w1 = str_word(p, sh, 0, lastw), w2 = str_word(p, sh, 1, lastw);
  fnv_word32(lo, hi, w1, 8);
  fnv_word32(lo, hi, w2, 8);
#pragma unroll
  for (u32 k = 0; k < kHotTailWords; ++k) {
    const u32 m = len > 16 + 8 * k ? len - 16 - 8 * k : 0;
    const u64 w = m ? low_bytes(str_word(p, sh, k + 2, lastw), m) : 0;
    fnv_word32(lo, hi, w, m);
    tail[k] = w;
  }
  nm.h = ((u64)hi << 32) | lo; nm.len = len; nm.off = off;
  nm.w0 = len; nm.w1 = w1; nm.w2 = w2;
}
__device__ inline bool tail_match(const u64 (&htail)[kHotTailWords][kHotMax], u32 j,
                                  const u64 (&tail)[kHotTailWords]) {
  bool eq = true;
#pragma unroll
  for (u32 k = 0; k < kHotTailWords; ++k) eq &= htail[k][j] == tail[k];
  return eq;
}

// Mark byte of a message k_dirty_pass completes (in the status column,
// whose statuses are < 0x40 or carry 0x80).
constexpr u8 kMarkDirty = 0x40;

// Messages [lo, n) of the batch (lo a multiple of 64: a segment of a batch
// classified segment by segment, or 0).
template <class In>
__global__ __launch_bounds__(kFastBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_receive_fast(
    In in, u32 lo, u32 n, Table T, Sharded miss, u32* ctr,
    const HotHdr* __restrict__ hot, const HotEntry* __restrict__ hot_dir, const u64* dtab,
    u8* __restrict__ mark) {
  __shared__ u32 hslot[kHotLds];        // directory index + 1 (0 = empty)
  __shared__ u64 htag[kHotMax], hw0[kHotMax], hw1[kHotMax], hw2[kHotMax];
  __shared__ u32 hrec[kHotMax], haoff[kHotMax];
  __shared__ u64 htail[kHotTailWords][kHotMax];
  __shared__ u64 hmax[3][kHotMax];      // per-workgroup maxima (elapsed biased by 2^63)
  __shared__ u32 hhits;

  // Gate (k_classify ran before, over every message up to n): only the clean
  // prefix is applied, the messages before the first dirty one
  // (ctr[kCtrDirty]) and before the first malformed datagram (ctr[5]); none:
  // ~0.
  // (dirty buckets, decoded batches: with a dirty set, the whole batch up to
  // the first malformed message; the messages that may name a dirty bucket
  // are marked for k_dirty_pass)
  const u32 ndr = dtab ? ctr[kCtrNDirty] : 0u;
  const bool iso = ndr != 0 && ndr <= kDirtyCap;
  n = min(n, iso ? ctr[5] : min(ctr[5], ctr[kCtrDirty]));
  if (n <= lo) return;
  const u32 nh = hot ? min(hot->n, kHotMax) : 0u;
  for (u32 j = threadIdx.x; j < kHotLds; j += kFastBlock) hslot[j] = 0;
  for (u32 j = threadIdx.x; j < kHotMax; j += kFastBlock) {
    hmax[0][j] = 0; hmax[1][j] = 0; hmax[2][j] = 0;
  }
  if (threadIdx.x == 0) hhits = 0;
  __syncthreads();
  for (u32 j = threadIdx.x; j < nh; j += kFastBlock) {
    const HotEntry d = hot_dir[j];
    htag[j] = d.tag; hw0[j] = d.w0; hw1[j] = d.w1; hw2[j] = d.w2;
    // (bit 31: a dirty bucket's entry, its record marked by k_dirty_build)
    hrec[j] = d.slot | (iso && (rec_flags(T.recs[d.slot]) & kRecDirty) ? 0x80000000u : 0u);
    haoff[j] = d.aoff;
    for (u32 k = 0; k < kHotTailWords; ++k) htail[k][j] = d.tail[k];
    u32 hs = hot_home(d.tag);
    while (atomicCAS(&hslot[hs], 0u, j + 1) != 0) hs = (hs + 1) & (kHotLds - 1);
  }
  __syncthreads();

  constexpr u32 kWaves = kFastBlock / 64;
  const u32 lane = threadIdx.x & 63;
  u32 nchunks = (n + 63) / 64;
  u32 hits = 0;
  // Round 1 (the name offsets) runs one chunk ahead: a chunk's dependent
  // chain is then name words -> home slot, and the next chunk's offsets
  // arrive meanwhile.
  // wave-uniform (in SGPRs): the chunk index, its shard of the miss list
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  // The workgroups that share an XCD (blockIdx % 8 labels them) walk one
  // eighth of the batch, so the lines two neighbouring chunks share (names,
  // offsets) are fetched into one L2: 1.770 against 1.79 ms on C2
  // (DESIGN.md §4 round 5).
  u32 cstride, chunk;
  if (gridDim.x % 8 == 0) {
    const u32 per = (nchunks - lo / 64 + 7) / 8;
    const u32 c0 = lo / 64 + (blockIdx.x % 8) * per;
    nchunks = min(nchunks, c0 + per);
    cstride = gridDim.x / 8 * kWaves;
    chunk = c0 + blockIdx.x / 8 * kWaves + wave;
  } else {
    cstride = gridDim.x * kWaves;
    chunk = lo / 64 + blockIdx.x * kWaves + wave;
  }
  typename In::Pre pre{};
  if (chunk < nchunks) pre = in.pre(min(chunk * 64 + lane, n - 1));
  for (; chunk < nchunks; chunk += cstride) {
    const u32 tid = chunk * 64 + lane;
    const bool valid = tid < n;
    const u32 i = tid < n ? tid : n - 1;
    // round 2: the name words and replica fields
    u64 off, w0, w1, w2, ra, rt;
    u32 len;
    i64 re;
    in.load(i, pre, off, len, w0, w1, w2, ra, rt, re);
    if (chunk + cstride < nchunks) pre = in.pre(min((chunk + cstride) * 64 + lane, n - 1));
    Name nm;
    short_name(w0, w1, w2, off, len, nm);
    const bool shortname = len <= kShortName;
    // Longer names (rare on the headline batches, all of a 32-byte-name
    // batch): the full canonical words and hash, word loads from the blob;
    // an arena name of <= kHotTailName bytes also keeps its tail words for
    // the directory match.
    u64 tail[kHotTailWords] = {};
    if (!shortname) {
      if (len <= kInlineName) {   // one more word than round 2 loaded
        const u64* bw = reinterpret_cast<const u64*>(in.blob());
        const u64 last = (off + len - 1) >> 3, w3i = (off >> 3) + 3;
        inline_name(w0, w1, w2, bw[w3i < last ? w3i : last], off, len, nm);
      } else if (In::kSoa && len <= kHotTailName) {
        // (decoded batches only: the datagram form keeps its registers
        // for the wire decode)
        load_name_tail(in.blob(), off, len, nm, tail);
      } else {
        load_name_wide<true>(in.blob(), off, len, nm);
      }
    }
    const u64 tag = T.tag(nm.h);
    const u64 ea = enc_replica_nz(ra), et = enc_replica_nz(rt), ee = (u64)re ^ kSign;

    bool missed = false;
    if (valid) {
      int hidx = -1;
      if (nh) {
        for (u32 hs = hot_home(tag);; hs = (hs + 1) & (kHotLds - 1)) {
          const u32 e = hslot[hs];
          if (!e) break;
          if (htag[e - 1] == tag && hw0[e - 1] == nm.w0 && hw1[e - 1] == nm.w1 &&
              (shortname || (hw2[e - 1] == nm.w2 &&
                             (len <= kInlineName ||
                              (In::kSoa && len <= kHotTailName
                                   ? tail_match(htail, e - 1, tail)
                                   : long_tail_equal(T.arena, haoff[e - 1], in.blob(), off, len)))))) {
            hidx = (int)e - 1;
            break;
          }
        }
      }
      // A message of a dirty bucket (iso only: its directory entry or record
      // marked), or a short-named miss that may be one, is marked and left
      // to k_dirty_pass (a byte store; doing that work here cost this kernel
      // its registers: 11 spilled, 1.78 -> 2.54 ms on a clean C2 batch).
      if (hidx >= 0) {
        if (iso && (hrec[hidx] >> 31)) {
          mark[i] = kMarkDirty;
        } else {
          ++hits;
          if (ea > hmax[0][hidx]) atomicMax(&hmax[0][hidx], ea);
          if (et > hmax[1][hidx]) atomicMax(&hmax[1][hidx], et);
          if (ee > hmax[2][hidx]) atomicMax(&hmax[2][hidx], ee);
        }
      } else {
        // round 3: the home slot
        u32 s = T.home(tag);
        Rec cur = load_rec48(&T.recs[s]);
        const bool hit = shortname && cur.tag == tag && (cur.name0 & ~0xFF00ull) == nm.w0 &&
                         cur.name1 == nm.w1 && (rec_flags(cur) & kRecPublished);
        int pr = kFound;
        if (!hit) {
          if (shortname && cur.tag == 0) {
            pr = kMiss;
          } else {
            pr = probe(T, nm, in.blob(), &s, &cur);
          }
        }
        if (pr == kFound) {
          if (iso && (rec_flags(cur) & kRecDirty)) {
            mark[i] = kMarkDirty;
          } else {
            Rec* r = &T.recs[s];
            if (ea > cur.added) atomicMax(&r->added, ea);
            if (et > cur.taken) atomicMax(&r->taken, et);
            if (ee > ((u64)cur.elapsed ^ kSign)) atomicMax(&r->elapsed, (i64)(ee ^ kSign));
          }
        } else if (iso && shortname) {
          mark[i] = kMarkDirty;
        } else {
          missed = true;
          if (pr == kFull) atomicOr(&ctr[8], 1u);
        }
      }
    }
    miss.append(chunk, missed, i);
  }
  if (hits) atomicAdd(&hhits, hits);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (hhits) atomicAdd(&ctr[10], hhits);
    if (blockIdx.x == 0) ctr[11] = nh;
  }

  // Directory flush: the workgroup's maxima, skipping fields already beaten.
  for (u32 j = threadIdx.x; j < nh; j += kFastBlock) {
    const u64 xa = hmax[0][j], xt = hmax[1][j], xe = hmax[2][j];
    if (!(xa | xt | xe)) continue;
    Rec* r = &T.recs[hrec[j] & 0x7FFFFFFFu];
    const u64 ca = r->added, ct = r->taken, ce = (u64)r->elapsed ^ kSign;
    if (xa > ca) atomicMax(&r->added, xa);
    if (xt > ct) atomicMax(&r->taken, xt);
    if (xe > ce) atomicMax(&r->elapsed, (i64)(xe ^ kSign));
  }
}

// The marked messages of an isolated batch (after k_receive_fast, before the
// launch that ends the batch; a grid-stride pass over the mark bytes, one
// message a lane): each names a dirty bucket or is a short-named miss.
//   - not in the dirty set: a miss (appended to the miss list, as the fast
//     kernel would have);
//   - dirty itself: left to the ordered sub-batch (dirty_finish);
//   - before its bucket's first dirty message: folded into the bucket's pre
//     cell (its first message kept: its merge may create the bucket);
//   - after it: folded into the cell of the last dirty message of its bucket
//     before it (the sorted dirty messages, at most 16 KB, searched in LDS).
// Cells fold in an LDS cache first (a hot bucket's cells take millions of
// messages: device atomics on one line serialise, 3.8 ms per C2 dirty
// batch), flushed with one atomic per field per workgroup; a cell the cache
// has no room for folds in device memory.
// Every mark is put back to PHIP_ST_MERGED (the status every fast-path
// message starts with; the miss path and the sub-batch write theirs after).
constexpr u32 kCellCacheBits = 10;
constexpr u32 kCellCache = 1u << kCellCacheBits;
template <class In>
__global__ __launch_bounds__(1024) void k_dirty_pass(In in, u32 n, u32* ctr, u8* mark,
                                                     const u64* dtab, Table T, Sharded miss) {
  __shared__ u32 sidx[kDirtyCap];
  __shared__ u32 ckey[kCellCache], cmin[kCellCache];
  __shared__ u64 cmax[3][kCellCache];
  __shared__ u32 queue[16][128];   // per wave: marked messages waiting for a full wave
  const u32 ndr = ctr[kCtrNDirty];
  if (ndr == 0 || ndr > kDirtyCap) return;
  n = min(n, ctr[5]);
  const DirtySet D = DirtySet::at(const_cast<u64*>(dtab));
  const u32 nv = ctr[kCtrNSorted];
  for (u32 j = threadIdx.x; j < nv; j += 1024) sidx[j] = D.idx[j];
  for (u32 j = threadIdx.x; j < kCellCache; j += 1024) {
    ckey[j] = 0; cmin[j] = ~0u;
    cmax[0][j] = 0; cmax[1][j] = 0; cmax[2][j] = 0;
  }
  __syncthreads();
  auto process = [&](u32 i) {
    u64 off, w0, w1, w2, ra, rt;
    u32 len;
    i64 re;
    const typename In::Pre p = in.pre(i);
    in.load(i, p, off, len, w0, w1, w2, ra, rt, re);
    Name nm;
    short_name(w0, w1, w2, off, len, nm);
    mark[i] = PHIP_ST_MERGED;
    const int s = dirty_find(D, nm);
    if (s < 0) {   // a miss of a clean bucket
      const u32 sh = (i / 64) & (kShards - 1);
      miss.base[(size_t)sh * miss.cap + atomicAdd(&miss.cnt[sh], 1u)] = i;
      return;
    }
    if (replica_dirty(ra, rt, re)) return;
    u32 lo = D.start[s];
    u32 cid;
    if (i < D.first[s]) {
      cid = kDirtyCap + lo;   // the pre cell
    } else {
      u32 hi = lo + D.cnt[s];
      while (hi - lo > 1) {   // the last dirty message before i (sidx[lo] < i)
        const u32 mid = (lo + hi) / 2;
        if (sidx[mid] < i) lo = mid; else hi = mid;
      }
      cid = lo;
    }
    const u64 ea = enc_replica_nz(ra), et = enc_replica_nz(rt), ee = (u64)re ^ kSign;
    u32 h = (cid * 2654435761u) >> (32 - kCellCacheBits);
    int slot = -1;
    for (u32 k = 0; k < 16; ++k, h = (h + 1) & (kCellCache - 1)) {
      const u32 old = atomicCAS(&ckey[h], 0u, cid + 1);
      if (old == 0u || old == cid + 1) { slot = (int)h; break; }
    }
    if (slot >= 0) {
      if (ea > cmax[0][slot]) atomicMax(&cmax[0][slot], ea);
      if (et > cmax[1][slot]) atomicMax(&cmax[1][slot], et);
      if (ee > cmax[2][slot]) atomicMax(&cmax[2][slot], ee);
      if (cid >= kDirtyCap && i < cmin[slot]) atomicMin(&cmin[slot], i);
    } else {
      u64* cl = D.cell + 3 * (size_t)cid;
      atomicMax(reinterpret_cast<unsigned long long*>(&cl[0]), ea);
      atomicMax(reinterpret_cast<unsigned long long*>(&cl[1]), et);
      atomicMax(reinterpret_cast<unsigned long long*>(&cl[2]), ee);
      if (cid >= kDirtyCap) atomicMin(&D.premin[cid - kDirtyCap], i);
    }
  };
  // Each wave walks 64-message chunks and queues its marked messages in LDS;
  // a full queue is processed a message a lane (a dirty batch marks a third
  // of its messages, scattered: processed in place, two lanes in three idle).
  const u32 w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u64 below = (1ull << lane) - 1;
  u32* q = queue[w];
  u32 qn = 0;
  const u32 stride = gridDim.x * 1024;
  for (u32 base = blockIdx.x * 1024 + w * 64; base < n; base += stride) {
    const u32 i = base + lane;
    const bool mk = i < n && mark[i] == kMarkDirty;
    const u64 m = __ballot(mk);
    if (mk) q[qn + __popcll(m & below)] = i;
    qn += (u32)__popcll(m);
    if (qn >= 64) {
      __builtin_amdgcn_wave_barrier();
      const u32 mine = q[lane];
      const u32 rest = qn - 64;
      const u32 tail = lane < rest ? q[64 + lane] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (lane < rest) q[lane] = tail;
      qn = rest;
      process(mine);
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (lane < qn) process(q[lane]);
  __syncthreads();
  for (u32 j = threadIdx.x; j < kCellCache; j += 1024) {
    const u32 k = ckey[j];
    if (!k) continue;
    const u32 cid = k - 1;
    u64* cl = D.cell + 3 * (size_t)cid;
    atomicMax(reinterpret_cast<unsigned long long*>(&cl[0]), cmax[0][j]);
    atomicMax(reinterpret_cast<unsigned long long*>(&cl[1]), cmax[1][j]);
    atomicMax(reinterpret_cast<unsigned long long*>(&cl[2]), cmax[2][j]);
    if (cid >= kDirtyCap) atomicMin(&D.premin[cid - kDirtyCap], cmin[j]);
  }
}


// The messages of a list (the fast batch's misses, after the insert
// pipeline created their buckets): GetBucket + Merge with creator tracking
// (the lowest-seq message of a bucket created by this batch is recorded in
// aux[] for PHIP_ST_CREATED).
template <class Src>
__global__ __launch_bounds__(kBlock) void k_receive_list(
    Src src, const uint64_t* __restrict__ ma, const uint64_t* __restrict__ mt,
    const int64_t* __restrict__ me, u32 n, const u32* __restrict__ list, Table T,
    u8* __restrict__ status, u32* miss, u32* ctr) {
  const u32 tid = blockIdx.x * kBlock + threadIdx.x;
  bool missed = false;
  u32 i = 0;
  if (tid < n) {
    i = list[tid];
    u64 off; u32 len;
    src.get(i, off, len);
    Name nm;
    load_name_wide<false>(src.blob, off, len, nm);
    u32 s;
    Rec cur;
    const int pr = probe(T, nm, src.blob, &s, &cur);
    if (pr == kFound) {
      const u64 ea = enc_replica_nz(ma[i]), et = enc_replica_nz(mt[i]), ee = (u64)me[i] ^ kSign;
      Rec* r = &T.recs[s];
      if (ea > cur.added) atomicMax(&r->added, ea);
      if (et > cur.taken) atomicMax(&r->taken, et);
      if (ee > ((u64)cur.elapsed ^ kSign)) atomicMax(&r->elapsed, (i64)(ee ^ kSign));
      // Creator tracking: the lowest index wins.  aux only falls, so a stale
      // read costs at most a redundant atomic; reading first keeps the
      // messages of a hot new bucket from serialising on one word.
      if ((rec_flags(cur) & kRecNew) && i < __hip_atomic_load(&T.aux[s], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT))
        atomicMin(&T.aux[s], i);
      if (status) status[i] = PHIP_ST_MERGED;
    } else {
      missed = true;
      if (pr == kFull) atomicOr(&ctr[8], 1u);
    }
  }
  const u32 pos = wave_append(&ctr[2], missed);
  if (missed) miss[pos] = i;
}

// Distinct names of a (large) miss list, for the insert pipeline: one
// message per name hash goes on (a set of 64-bit table tags in `set`, probed
// linearly; the load before the CAS keeps a hot name's messages from
// serialising on its word).  Two names that share a tag keep only one
// message: the other name then misses the fast pass that follows and takes
// the general insert path (finish_misses), so dropping it is safe.
template <class Src>
__global__ __launch_bounds__(kBlock) void k_dedupe(Src src, u32 n, const u32* __restrict__ list,
                                                   Table T, u64* set, u32 setbits, Sharded out) {
  const u32 tid = blockIdx.x * kBlock + threadIdx.x;
  bool keep = false;
  u32 i = 0;
  if (tid < n) {
    i = list[tid];
    u64 off; u32 len;
    src.get(i, off, len);
    Name nm;
    load_name_wide<false>(src.blob, off, len, nm);
    const u64 tag = T.tag(nm.h);
    const u64 mask = (1ull << setbits) - 1;
    u64 h = seeded_mix(tag, T.seed) >> (64 - setbits);
    keep = true;   // no free entry found (cannot happen at <= 50% load): keep it
    for (u64 k = 0; k <= mask; ++k, h = (h + 1) & mask) {
      u64 v = __hip_atomic_load(&set[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == 0) v = atomicCAS(&set[h], 0ull, tag);
      if (v == 0) break;                      // first of its name: keep
      if (v == tag) { keep = false; break; }  // a message of this name went on
    }
  }
  out.append(blockIdx.x, keep, i);
}

// Creator tracking without merging (the large-miss path merges by a second
// fast pass): aux[s] = the lowest index among the list's messages of every
// bucket this batch created.
template <class Src>
__global__ __launch_bounds__(kBlock) void k_first_seen(Src src, u32 n, const u32* __restrict__ list,
                                                       Table T) {
  const u32 tid = blockIdx.x * kBlock + threadIdx.x;
  if (tid >= n) return;
  const u32 i = list[tid];
  u64 off; u32 len;
  src.get(i, off, len);
  Name nm;
  load_name_wide<false>(src.blob, off, len, nm);
  u32 s;
  Rec cur;
  if (probe(T, nm, src.blob, &s, &cur) != kFound) return;
  if ((rec_flags(cur) & kRecNew) &&
      i < __hip_atomic_load(&T.aux[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMin(&T.aux[s], i);
}

// PHIP_ST_CREATED from the claimed slots: status[aux[s]] of each.
__global__ void k_mark_created_slots(const u32* __restrict__ cslot, u32 n, Table T, u8* status) {
  const u32 j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const u32 i = T.aux[cslot[j]];
  if (i != 0xFFFFFFFFu) status[i] |= 0x80;
}

// Status of the messages that went through the insert pipeline: the first
// (lowest-seq) message of a created bucket gets PHIP_ST_CREATED
// (repo.go:189-211 creates on the first GetBucket).
template <class Src>
__global__ void k_mark_created(Src src, u32 n, const u32* __restrict__ list, Table T, u8* status) {
  u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n || !status) return;
  u32 i = list[tid];
  u64 off; u32 len;
  src.get(i, off, len);
  Name nm;
  load_name_wide<false>(src.blob, off, len, nm);
  u32 s;
  Rec r;
  if (probe(T, nm, src.blob, &s, &r) != kFound) return;
  if ((rec_flags(r) & kRecNew) && T.aux[s] == i) status[i] |= 0x80;
}

// -------------------------------------------------------------- resolve --
// The ordered path's sort values (op index | kind << kOpIdxBits), written by
// the first full resolve (val == nullptr: none).
struct SortVals {
  const u8* kind; u32 kind0;
  u32* val;
};
constexpr u32 kSortValKindShift = 30;

// Name -> slot for every op (ordered path, seed, get).  Misses appended.
template <class Src>
__global__ __launch_bounds__(kBlock) void k_resolve(Src src, u32 n, const u32* __restrict__ list,
                                                    Table T, u32* __restrict__ slot_out, Sharded miss,
                                                    u32* ctr, SortVals sv) {
  u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
  bool missed = false;
  u32 i = 0;
  if (tid < n) {
    i = list ? list[tid] : tid;
    if (sv.val) sv.val[i] = i | ((u32)(sv.kind ? sv.kind[i] : sv.kind0) << kSortValKindShift);
    u64 off; u32 len;
    src.get(i, off, len);
    Name nm;
    load_name_wide<false>(src.blob, off, len, nm);
    u32 s;
    Rec r;
    int pr = probe(T, nm, src.blob, &s, &r);
    if (pr == kFound) slot_out[i] = s;
    else {
      missed = true;
      if (pr == kFull) atomicOr(&ctr[8], 1u);
    }
  }
  if (miss.base) miss.append(blockIdx.x, missed, i);
}

// k_resolve over a whole batch (no list; the ordered path's first resolve):
// kResPer ops per thread, every round's loads of all of them issued together
// (name offsets, name words, home record), so a thread keeps kResPer
// dependent chains in flight at the same occupancy; a short name found in
// its home slot needs no probe loop (k_receive_fast's test).  Same results
// as k_resolve.
constexpr u32 kResPer = 2;   // (3: 78 VGPRs, 6 waves a SIMD; 4: 100, 4 waves; both slower)
template <class Src>
__global__ __launch_bounds__(kBlock) void k_resolve_batch(Src src, u32 n, Table T,
                                                          u32* __restrict__ slot_out, Sharded miss,
                                                          u32* ctr, SortVals sv) {
  const u32 i0 = blockIdx.x * (kBlock * kResPer) + threadIdx.x;
  u64 off[kResPer], w0[kResPer], w1[kResPer], w2[kResPer];
  u32 len[kResPer];
  bool bad = false;
#pragma unroll
  for (u32 k = 0; k < kResPer; ++k) bad |= src.get(min(i0 + k * kBlock, n - 1), off[k], len[k]);
  // a malformed name entry (checked names only): the batch is refused before
  // anything is created (check_flags)
  const u64 bm = __ballot(bad);
  if (bm && __lane_id() == (u32)(__ffsll((long long)bm) - 1)) atomicOr(&ctr[kCtrBadName], 1u);
#pragma unroll
  for (u32 k = 0; k < kResPer; ++k) load_words3<false>(src.blob, off[k], len[k], w0[k], w1[k], w2[k]);
  Name nm[kResPer];
  u64 tag[kResPer];
  u32 s[kResPer];
  Rec cur[kResPer];
#pragma unroll
  for (u32 k = 0; k < kResPer; ++k) {
    if (len[k] <= kShortName) short_name(w0[k], w1[k], w2[k], off[k], len[k], nm[k]);
    else load_name_wide<false>(src.blob, off[k], len[k], nm[k]);
    tag[k] = T.tag(nm[k].h);
    s[k] = T.home(tag[k]);
    cur[k] = load_rec48(&T.recs[s[k]]);
  }
#pragma unroll
  for (u32 k = 0; k < kResPer; ++k) {
    const u32 i = i0 + k * kBlock;
    bool missed = false;
    if (i < n) {
      if (sv.val) sv.val[i] = i | ((u32)(sv.kind ? sv.kind[i] : sv.kind0) << kSortValKindShift);
      const bool shortname = len[k] <= kShortName;
      const bool hit = shortname && cur[k].tag == tag[k] &&
                       (cur[k].name0 & ~0xFF00ull) == nm[k].w0 && cur[k].name1 == nm[k].w1 &&
                       (rec_flags(cur[k]) & kRecPublished);
      int pr = kFound;
      u32 sk = s[k];
      if (!hit) {
        if (shortname && cur[k].tag == 0) {
          pr = kMiss;
        } else {
          Rec r;
          pr = probe(T, nm[k], src.blob, &sk, &r);
        }
      }
      if (pr == kFound) {
        slot_out[i] = sk;
      } else {
        missed = true;
        if (pr == kFull) atomicOr(&ctr[8], 1u);
      }
    }
    if (miss.base) miss.append(blockIdx.x * kResPer + k, missed, i);
  }
}

// ------------------------------------------------------------- inserts ---
// Round of the insert pipeline.  Claim: CAS an empty tag slot.  A same-tag
// slot claimed in this round (not yet published) cannot be name-checked, so
// the message waits for the next round (retry list); after the publish
// kernel the name is visible and the retry either finds it or keeps probing.
template <class Src>
__global__ __launch_bounds__(kBlock) void k_claim(Src src, u32 n, const u32* __restrict__ list,
                                                  Table T, u32* claimed_slot, u32* claimed_msg,
                                                  u32* retry, u32* ctr) {
  u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
  bool won = false, again = false;
  u32 i = 0, s = 0;
  if (tid < n) {
    i = list[tid];
    u64 off; u32 len;
    src.get(i, off, len);
    Name nm;
    load_name_wide<false>(src.blob, off, len, nm);
    const u64 tag = T.tag(nm.h);
    const u32 mask = T.mask();
    s = T.home(tag);
    u32 k = 0;
    for (; k <= mask; ++k) {
      u64 t = __hip_atomic_load(&T.recs[s].tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == 0) {
        t = atomicCAS(&T.recs[s].tag, 0ull, tag);
        if (t == 0) { won = true; break; }
      }
      if (t == tag) {
        Rec r = load_rec(&T.recs[s]);
        if (!(rec_flags(r) & kRecPublished)) { again = true; break; }
        if (name_equal(r, nm, src.blob, T.arena)) break;   // inserted by an earlier round
      }
      s = (s + 1) & mask;
    }
    if (k > mask) atomicOr(&ctr[8], 1u);
  }
  u32 p = wave_append(&ctr[3], won);
  if (won) { claimed_slot[p] = s; claimed_msg[p] = i; }
  u32 q = wave_append(&ctr[4], again);
  if (again) retry[q] = i;
}

// Publish claimed slots: canonical name (+arena for long names), zero state
// (a GetBucket-created Bucket, repo.go:208), created clock, NEW flag.
template <class Src>
__global__ void k_publish(Src src, u32 base, u32 n, const u32* __restrict__ claimed_slot,
                          const u32* __restrict__ claimed_msg, Table T, u8* arena,
                          u64 arena_cap, u64* arena_cursor, const int64_t* __restrict__ now_arr,
                          i64 now0, u32* ctr) {
  u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n) return;
  u32 s = claimed_slot[base + tid], i = claimed_msg[base + tid];
  u64 off; u32 len;
  src.get(i, off, len);
  Name nm;
  load_name_wide<false>(src.blob, off, len, nm);
  Rec r;
  r.tag = T.tag(nm.h);
  r.added = kEPosZero;
  r.taken = kEPosZero;
  r.elapsed = 0;
  r.created = now_arr ? now_arr[i] : now0;
  r.name0 = nm.w0; r.name1 = nm.w1; r.name2 = nm.w2;
  if (len > kInlineName) {
    u64 a = atomicAdd(arena_cursor, (u64)len);
    if (a + len > arena_cap) { atomicOr(&ctr[7], 1u); a = 0; }
    else for (u32 k = 0; k < len; ++k) arena[a + k] = src.blob[off + k];
    r.name0 = (nm.w0 & 0xFFu) | (a << 32);
  }
  r.name0 = with_flags(r.name0, kRecPublished | kRecNew);
  T.recs[s] = r;
  T.aux[s] = 0xFFFFFFFFu;
}

__global__ void k_clear_new(const u32* __restrict__ claimed_slot, u32 n, Table T) {
  u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n) return;
  u32 s = claimed_slot[tid];
  Rec* r = &T.recs[s];
  r->name0 = with_flags(r->name0, kRecPublished);
  T.aux[s] = 0;
}

// Error paths: the NEW flag (and creator scratch) of every slot, whatever
// list claimed it, so a refused batch leaves no bucket marked as created.
__global__ void k_clear_new_all(Table T, u64 cap) {
  const u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= cap) return;
  Rec* r = &T.recs[s];
  if (r->tag && (rec_flags(*r) & kRecNew)) r->name0 = with_flags(r->name0, kRecPublished);
  T.aux[s] = 0;
}

// Arena bytes the names of a list could need (names > kInlineName bytes;
// duplicates counted once each, so an upper bound), summed into *out.
template <class Src>
__global__ __launch_bounds__(kBlock) void k_list_long_bytes(Src src, u32 n,
                                                            const u32* __restrict__ list,
                                                            u64* out) {
  const u32 tid = blockIdx.x * kBlock + threadIdx.x;
  u64 b = 0;
  if (tid < n) {
    u64 off; u32 len;
    src.get(list[tid], off, len);
    b = len > kInlineName ? len : 0;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) b += (u64)__shfl_xor((long long)b, d);
  if (__lane_id() == 0 && b) atomicAdd((unsigned long long*)out, (unsigned long long)b);
}

// Table growth (Go's map never refuses a bucket, repo.go:204-207,225-227):
// every record of the old table moves to its home in the new one (2x the
// slots) by linear probing.  Names are distinct, so a slot is claimed by a
// CAS on its tag and no name is compared; the record (state, name words,
// created, flags) and its aux word move as they are, arena offsets included.
__global__ __launch_bounds__(kBlock) void k_rehash(const Rec* __restrict__ old,
                                                   const u32* __restrict__ old_aux, u64 old_cap,
                                                   Table T, u32* ctr) {
  const u64 s = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (s >= old_cap) return;
  const Rec r = load_rec(&old[s]);
  if (!r.tag) return;
  const u32 mask = T.mask();
  u32 d = T.home(r.tag);
  u32 k = 0;
  for (; k <= mask; ++k, d = (d + 1) & mask)
    if (atomicCAS(&T.recs[d].tag, 0ull, r.tag) == 0ull) break;
  if (k > mask) { atomicOr(&ctr[8], 1u); return; }
  Rec* q = &T.recs[d];
  q->added = r.added; q->taken = r.taken; q->elapsed = r.elapsed;
  q->name0 = r.name0; q->name1 = r.name1; q->created = r.created; q->name2 = r.name2;
  T.aux[d] = old_aux[s];
}

// Placement quality (phip_table_stats): every bucket's probe distance from
// its home slot; out[0] the longest (atomicMax), out[1] the sum.
__global__ __launch_bounds__(kBlock) void k_table_stats(Table T, u64 cap, u64* out) {
  const u64 s = (u64)blockIdx.x * kBlock + threadIdx.x;
  u64 d = 0;
  if (s < cap) {
    const u64 tag = T.recs[s].tag;
    if (tag) d = ((u32)s - T.home(tag)) & T.mask();
  }
  // a wave's maximum and sum first: one atomic pair per wave
  u64 mx = d, sm = d;
  for (int o = 32; o > 0; o >>= 1) {
    const u64 x = __shfl_down(mx, o), y = __shfl_down(sm, o);
    mx = x > mx ? x : mx;
    sm += y;
  }
  if (__lane_id() == 0 && sm) {
    atomicMax(&out[0], mx);
    atomicAdd(&out[1], sm);
  }
}

// --------------------------------------------------------------- decode --
// UnmarshalBinary (bucket.go:71-91) for a batch of raw datagrams: big-endian
// fields, name length byte, io.ErrShortBuffer when < 25 bytes or the name is
// truncated; trailing bytes are ignored.  The first short datagram index is
// min-reduced into ctr[5] (the Go loop stops there, repo.go:72-73).

__global__ void k_decode(const u8* __restrict__ bytes, const uint64_t* __restrict__ offs, u32 n,
                         uint64_t* __restrict__ a, uint64_t* __restrict__ t,
                         int64_t* __restrict__ e, uint64_t* __restrict__ noff,
                         u8* __restrict__ nlen, u32* ctr) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    u64 o = offs[i], sz = offs[i + 1] - o;
    bool bad = sz < 25;
    if (!bad) {
      const u8* p = bytes + o;
      u64 ab = load_be64(p), tb = load_be64(p + 8);
      i64 eb = (i64)load_be64(p + 16);
      u32 l = p[24];
      bad = sz - 25 < l;
      a[i] = ab; t[i] = tb; e[i] = eb;
      noff[i] = o + 25;
      nlen[i] = (u8)l;
    }
    if (bad) {
      nlen[i] = 0; noff[i] = o;
      atomicMin(&ctr[5], i);
    }
  }
}

// After the fast kernel (one workgroup): the dirty buckets' records
// unmarked, and the ordered sub-batch built -- per dirty bucket, in
// (bucket, message) order: its pre cell as one merge (its messages before its
// first dirty message), then each of its dirty messages followed by its
// cell as one merge (a cell whose maxima read +0, +0, 0 would read as an
// incast: it is split in two merges, (+0, +0, min) and (NaN, NaN, 0), the
// same effect).  Entries name their bucket by its dirty message's name (in
// place in the batch's blob); map2 holds the message an entry's status and
// reply go back to: the message itself, a pre cell's first message (its
// merge may create the bucket: PHIP_ST_CREATED), ~0 for a later cell's merge
// (its messages keep PHIP_ST_MERGED: the bucket exists by then).
// The entry count lands in ctr[kCtrNDefer].
// (one workgroup of kShards lanes; k_batch_end runs it before the batch's
// shard scan, in one launch)
struct SubOut {
  uint64_t* off;
  u8* len;
  uint64_t* a;
  uint64_t* t;
  int64_t* e;
  u32* map;
};
template <class In>
__device__ inline void dirty_finish(const In& in, u32* ctr, const DirtySet& D, const Table& T,
                                    const SubOut& so) {
  __shared__ u32 part[kShards];
  uint64_t* __restrict__ off2 = so.off;
  u8* __restrict__ len2 = so.len;
  uint64_t* __restrict__ a2 = so.a;
  uint64_t* __restrict__ t2 = so.t;
  int64_t* __restrict__ e2 = so.e;
  u32* __restrict__ map2 = so.map;
  const u32 tid = threadIdx.x;
  const u32 nd = ctr[kCtrNDirty];
  if (nd == 0 || nd > kDirtyCap) {
    if (tid == 0) ctr[kCtrNDefer] = 0;
    return;
  }
  const u32 nv = ctr[kCtrNSorted];
  // thread tid: set entries [j0, j1), up to three sub-batch entries each
  const u32 per = (nv + kShards - 1) / kShards;
  const u32 j0 = min(nv, tid * per), j1 = min(nv, j0 + per);
  // entries of a cell's merge: 0 (empty), 1, or 2 (maxima +0, +0, 0 read
  // as an incast: split in two merges of the same effect)
  auto cell_n = [&](const u64* c) -> u32 {
    if (!(c[0] | c[1] | c[2])) return 0u;
    return c[0] == kInfBits && c[1] == kInfBits && c[2] == kSign ? 2u : 1u;
  };
  auto is_start = [&](u32 j) { return j == 0 || D.dslot[j - 1] != D.dslot[j]; };
  u32 c = 0;
  for (u32 j = j0; j < j1; ++j) {
    c += 1 + cell_n(D.cell + 3 * j);
    if (is_start(j)) {
      c += cell_n(D.cell + 3 * ((size_t)kDirtyCap + j));
      const u32 s = D.dslot[j];
      if (D.rslot[s] != ~0u)
        atomicAnd(reinterpret_cast<unsigned long long*>(&T.recs[D.rslot[s]].name0),
                  ~(unsigned long long)(kRecDirty << 8));
    }
  }
  part[tid] = c;
  __syncthreads();
  for (u32 off = 1; off < kShards; off <<= 1) {   // inclusive scan
    const u32 v = tid >= off ? part[tid - off] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  u32 o = part[tid] - c;
  auto emit_cell = [&](const u64* cl, u64 off, u32 len, u32 to) {
    const u32 k = cell_n(cl);
    if (k == 0) return;
    off2[o] = off; len2[o] = (u8)len; map2[o] = to;
    if (k == 2) {
      a2[o] = 0; t2[o] = 0; e2[o] = (int64_t)kSign;
      ++o;
      off2[o] = off; len2[o] = (u8)len; map2[o] = ~0u;
      a2[o] = 0x7FF8000000000000ull; t2[o] = 0x7FF8000000000000ull; e2[o] = 0;
    } else {
      a2[o] = dec_replica_max(cl[0]); t2[o] = dec_replica_max(cl[1]);
      e2[o] = (int64_t)(cl[2] ^ kSign);
    }
    ++o;
  };
  for (u32 j = j0; j < j1; ++j) {
    const u32 i = D.idx[j];
    u64 off, w0, w1, w2, ra, rt;
    u32 len;
    i64 re;
    const typename In::Pre pr = in.pre(i);
    in.load(i, pr, off, len, w0, w1, w2, ra, rt, re);   // (decoded or wire form)
    // the bucket's messages before its first dirty message: one merge, whose
    // status (it may create the bucket) goes to the first of them
    if (is_start(j)) emit_cell(D.cell + 3 * ((size_t)kDirtyCap + j), off, len, D.premin[j]);
    off2[o] = off; len2[o] = (u8)len;
    a2[o] = ra; t2[o] = rt; e2[o] = re;
    map2[o] = i;
    ++o;
    emit_cell(D.cell + 3 * j, off, len, ~0u);
  }
  if (tid == kShards - 1) ctr[kCtrNDefer] = part[kShards - 1];
}

// The end of a decoded fast batch in one launch: dirty_finish (an isolated
// batch's sub-batch; nothing otherwise), then the miss list's shard scan
// (k_shard_scan: counters to the host mirror, the next batch's reset).
template <class In>
__global__ __launch_bounds__(kShards) void k_batch_end(In in, u32* ctr, const u64* dtab, Table T,
                                                       SubOut so, u32* cnt, u32* host, u32 words,
                                                       u32* next, u32* next_ctr) {
  dirty_finish(in, ctr, DirtySet::at(const_cast<u64*>(dtab)), T, so);
  __threadfence_block();
  __syncthreads();
  shard_scan(cnt, ctr, 2, host, words, next, next_ctr);
}

// ------------------------------------------------------------ ordered ----
// A view of a mixed op stream as the ABI hands it over; null arrays mean
// "uniform value" (kind0 / now0).
struct OpView {
  const u8* kind; u32 kind0;
  const int64_t* now; i64 now0;
  const int64_t* freq; const int64_t* per; const uint64_t* count;
  const uint64_t* a; const uint64_t* t; const int64_t* e;
};

struct OutView {
  u8* status;
  uint64_t* remaining;
  uint64_t* have;
  phip_state* reply;
};

// The ordered sub-batch's statuses and replies back to their messages
// (dirty_finish's map2; ~0: a cell's merge, no output).
__global__ void k_defer_scatter(const u32* __restrict__ map2, u32 nd, const u8* __restrict__ st2,
                                const phip_state* __restrict__ rep2, OutView ow) {
  const u32 j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nd) return;
  const u32 i = map2[j];
  if (i == ~0u) return;
  if (ow.status) ow.status[i] = st2[j];
  if (ow.reply) ow.reply[i] = rep2[j];
}

// Lane l's value when l is wave-uniform (a ballot's first set lane): a
// v_readlane into a scalar register instead of an LDS permute.
__device__ inline u64 lane_u64(u64 v, u32 l) {
  const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)v, (int)l);
  const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), (int)l);
  return ((u64)hi << 32) | lo;
}

// One op packed into 32 bytes (one aligned sector), in original order:
//   TAKE:            x = Rate.Interval (0 = Tokens() is always 0),
//                    y = float64(Freq) bits (capacity), z = float64(n) bits
//   RECEIVE/UPSERT:  x = added bits, y = taken bits, z = elapsed
// The op kind rides in the top 2 bits of the radix-sort value (kOpIdxMask
// below it is the op index), so a fold reads the sorted value stream
// coalesced and then one 32-byte record per op.
struct alignas(32) OpRec {
  i64 now;
  u64 x, y, z;
};
constexpr u32 kOpIdxBits = 30;
static_assert(kOpIdxBits == kSortValKindShift, "k_resolve's sort values");
constexpr u32 kOpIdxMask = (1u << kOpIdxBits) - 1;
constexpr u32 kMaxOrderedOps = 1u << kOpIdxBits;

struct SOp {
  i64 now;
  u64 x, y, z;
  u32 idx;
  u32 kind;
};

__device__ inline OpRec load_oprec(const OpRec* p) {
  const ulonglong2* q = reinterpret_cast<const ulonglong2*>(p);
  ulonglong2 a = q[0], b = q[1];
  return OpRec{(i64)a.x, a.y, b.x, b.y};
}
__device__ inline SOp make_sop(const OpRec& r, u32 v) {
  return SOp{r.now, r.x, r.y, r.z, v & kOpIdxMask, v >> kOpIdxBits};
}
__device__ inline SOp load_sop(const OpRec* ops, u32 v) {
  return make_sop(load_oprec(ops + (v & kOpIdxMask)), v);
}

// Pack: op i -> ops[i] (coalesced reads of the ABI columns, coalesced
// 32-byte writes).  The per-op integer division of Rate.Interval happens
// here, once, not in every fold round.  kPackPer ops per thread, every
// column load of all of them issued before the first is used (a stream
// kernel needs the loads in flight: one op per thread left it at ~3 TB/s);
// a column the view does not have is not read.
constexpr u32 kPackPer = 4;
__global__ __launch_bounds__(kBlock) void k_pack_ops(OpView ov, u32 n, OpRec* __restrict__ ops) {
  const u32 i0 = blockIdx.x * (kBlock * kPackPer) + threadIdx.x;
  u32 kd[kPackPer];
  i64 nw[kPackPer], f[kPackPer], p[kPackPer];
  u64 c[kPackPer], x[kPackPer], y[kPackPer], z[kPackPer];
#pragma unroll
  for (u32 j = 0; j < kPackPer; ++j) {
    const u32 i = min(i0 + j * kBlock, n - 1);
    kd[j] = ov.kind ? (u32)ld<true>(ov.kind + i) : ov.kind0;
    nw[j] = ov.now ? ld<true>(ov.now + i) : ov.now0;
    f[j] = ov.freq ? ld<true>(ov.freq + i) : 0;
    p[j] = ov.per ? ld<true>(ov.per + i) : 0;
    c[j] = ov.count ? ld<true>(ov.count + i) : 0;
    x[j] = ov.a ? ld<true>(ov.a + i) : 0;
    y[j] = ov.t ? ld<true>(ov.t + i) : 0;
    z[j] = ov.e ? (u64)ld<true>(ov.e + i) : 0;
  }
#pragma unroll
  for (u32 j = 0; j < kPackPer; ++j) {
    const u32 i = i0 + j * kBlock;
    const bool take = i < n && kd[j] == PHIP_OP_TAKE;
    // Rate.Interval (an int64 division, a long instruction sequence): the
    // Takes of a wave usually share one rate, then it is divided once
    const u64 tm = __ballot(take);
    if (tm) {
      const u32 l0 = (u32)__ffsll((long long)tm) - 1;
      const i64 f0 = (i64)lane_u64((u64)f[j], l0), p0 = (i64)lane_u64((u64)p[j], l0);
      i64 iv;
      if (__ballot(take && (f[j] != f0 || p[j] != p0)) == 0) iv = rate_interval(f0, p0);
      else iv = rate_interval(f[j], p[j]);
      if (take) {
        x[j] = (u64)iv;
        y[j] = as_bits((double)f[j]);             // bucket.go:192
        z[j] = as_bits((double)c[j]);             // bucket.go:215
      }
    }
    if (i < n) {
      ulonglong2* q = reinterpret_cast<ulonglong2*>(ops + i);
      q[0] = ulonglong2{(u64)nw[j], x[j]};
      q[1] = ulonglong2{y[j], z[j]};
    }
  }
}

struct FState {
  double a, t;
  i64 e, c;
  bool existed;
};

struct OpOut {
  u8 st;
  bool has_reply;   // the op has a reply state: the bucket right after it
  u64 rem, have;
};

// One op of the ordered stream against state S (result state in S2).
// Returns whether S2 differs from S (bitwise, or existence).  kOut: also
// fill the op's results (the state test alone lets the compiler drop them).
template <bool kOut>
__device__ inline bool step_sop(const SOp& op, const FState& S, FState& S2, OpOut& out) {
  S2 = S;
  u8 cflag = 0;
  if (!S.existed) { S2.c = op.now; S2.existed = true; cflag = 0x80; }   // repo.go:208
  if (kOut) { out.has_reply = false; out.rem = 0; out.have = 0; }
  // Reply states (phip_results.reply): the bucket right after the op for a
  // Take (what UpsertBucket then broadcasts, api.go:74, repo.go:123-127), an
  // Upsert (repo.go:123-127 broadcasts the upserted bucket) and an incast
  // request (unchanged by it: the unicast payload of repo.go:86-90, and the
  // find-or-create result GetBucket returns); none for a merged replica.
  if (op.kind == PHIP_OP_TAKE) {
    TakeResult r = take_step(S2.a, S2.t, S2.e, S2.c, op.now, (i64)op.x, as_f64(op.y), as_f64(op.z));
    if (kOut) {
      out.st = (r.ok ? PHIP_ST_TAKE_OK : PHIP_ST_TAKE_DENIED) | cflag;
      out.rem = r.remaining; out.have = r.have_bits;
      out.has_reply = true;
    }
  } else {
    const u64 ab = op.x, tb = op.y;
    const i64 eb = (i64)op.z;
    if (op.kind == PHIP_OP_UPSERT && !S.existed) {               // repo.go:225-230
      S2.a = as_f64(ab); S2.t = as_f64(tb); S2.e = eb;
      if (kOut) { out.st = PHIP_ST_UPSERT_INSERTED | cflag; out.has_reply = true; }
    } else if (op.kind == PHIP_OP_RECEIVE && state_is_zero(ab, tb, eb)) {   // repo.go:86-90
      if (kOut) {
        bool reply = S.existed && !state_is_zero(as_bits(S.a), as_bits(S.t), S.e);
        out.st = (reply ? PHIP_ST_INCAST_REPLY : PHIP_ST_INCAST_NOREPLY) | cflag;
        out.has_reply = true;
      }
    } else {                                                      // bucket.go:240-263
      go_merge(S2.a, S2.t, S2.e, as_f64(ab), as_f64(tb), eb);
      if (kOut) {
        out.st = PHIP_ST_MERGED | cflag;
        out.has_reply = op.kind == PHIP_OP_UPSERT;
      }
    }
  }
  return !S.existed || as_bits(S2.a) != as_bits(S.a) || as_bits(S2.t) != as_bits(S.t) ||
         S2.e != S.e;
}
__device__ inline bool eval_sop(const SOp& op, const FState& S, FState& S2, OpOut& out) {
  return step_sop<true>(op, S, S2, out);
}
__device__ inline bool apply_sop(const SOp& op, const FState& S, FState& S2) {
  OpOut unused;
  return step_sop<false>(op, S, S2, unused);
}

// S is the bucket's state right after the op (its reply state, step_sop).
__device__ inline void write_out(const OutView& o, u32 i, const OpOut& r, const FState& S) {
  if (o.status) o.status[i] = r.st;
  if (o.remaining) o.remaining[i] = r.rem;
  if (o.have) o.have[i] = r.have;
  if (o.reply && r.has_reply) {
    phip_state st;
    st.added = as_bits(S.a); st.taken = as_bits(S.t); st.elapsed = S.e; st.created = S.c;
    o.reply[i] = st;
  }
}

// write_out with the outputs present fixed at compile time (kOut: kOutStatus
// | kOutRem | kOutHave | kOutReply): no branch around a store, so the loops
// that store have a fixed number of vector memory instructions per
// iteration and the compiler's vmcnt waits for a load need not wait for
// the stores issued after it (gfx9 counts loads and stores in one in-order
// counter: with a variable count it waits for everything, vmcnt(0)).
constexpr u32 kOutStatus = 1, kOutRem = 2, kOutHave = 4, kOutReply = 8;
inline u32 out_mask(const OutView& o) {
  return (o.status ? kOutStatus : 0) | (o.remaining ? kOutRem : 0) | (o.have ? kOutHave : 0) |
         (o.reply ? kOutReply : 0);
}
template <u32 kOut>
__device__ inline void write_out_m(const OutView& o, u32 i, const OpOut& r, const FState& S) {
  if constexpr ((kOut & kOutStatus) != 0) o.status[i] = r.st;
  if constexpr ((kOut & kOutRem) != 0) o.remaining[i] = r.rem;
  if constexpr ((kOut & kOutHave) != 0) o.have[i] = r.have;
  if constexpr ((kOut & kOutReply) != 0) {
    if (r.has_reply) {
      phip_state st;
      st.added = as_bits(S.a); st.taken = as_bits(S.t); st.elapsed = S.e; st.created = S.c;
      o.reply[i] = st;
    }
  }
}

// write_out_m for outputs prefilled with the defaults (status MERGED,
// remaining / have 0): only the values that differ are stored.  A hot
// segment's ops are scattered over the whole batch, so every store is a
// random write of its own; half of them are merges whose results are the
// defaults (k_huge_outputs).
template <u32 kOut>
__device__ inline void write_out_nd(const OutView& o, u32 i, const OpOut& r, const FState& S) {
  if constexpr ((kOut & kOutStatus) != 0) if (r.st != PHIP_ST_MERGED) o.status[i] = r.st;
  if constexpr ((kOut & kOutRem) != 0) if (r.rem) o.remaining[i] = r.rem;
  if constexpr ((kOut & kOutHave) != 0) if (r.have) o.have[i] = r.have;
  if constexpr ((kOut & kOutReply) != 0) {
    if (r.has_reply) {
      phip_state st;
      st.added = as_bits(S.a); st.taken = as_bits(S.t); st.elapsed = S.e; st.created = S.c;
      o.reply[i] = st;
    }
  }
}

__device__ inline FState load_state(const Rec& r) {
  FState S;
  S.a = as_f64(dec_f64(r.added));
  S.t = as_f64(dec_f64(r.taken));
  S.e = r.elapsed;
  S.c = r.created;
  S.existed = !(rec_flags(r) & kRecNew);
  return S;
}

__device__ inline void store_state(Rec* r, const FState& S) {
  r->added = enc_f64(as_bits(S.a));
  r->taken = enc_f64(as_bits(S.t));
  r->elapsed = S.e;
  r->created = S.c;
  r->name0 = with_flags(r->name0, kRecPublished);
}

constexpr u32 kLongSeg = 32;        // longer segments: one wave each (k_fold_wave)
#ifndef PHIP_HUGE_SEG
#define PHIP_HUGE_SEG 32768   // C3: 16384 7.04-7.10 ms, 32768 6.70-6.76, 65536 6.83
#endif
constexpr u32 kHugeSeg = PHIP_HUGE_SEG;   // longer still: one workgroup each (k_fold_block)
// The largest huge segments (at most this many) fold on a stream of their own.
#ifndef PHIP_HUGE_FIRST
#define PHIP_HUGE_FIRST 8
#endif
constexpr u32 kHugeFirstMax = 16;
static_assert(PHIP_HUGE_FIRST <= kHugeFirstMax, "PHIP_HUGE_FIRST");
#ifndef PHIP_FOLD_THREADS
#define PHIP_FOLD_THREADS 512
#endif
#ifndef PHIP_FOLD_PER
#define PHIP_FOLD_PER 1
#endif
constexpr u32 kFoldThreads = PHIP_FOLD_THREADS;   // k_fold_block: threads, ops per thread per window
constexpr u32 kFoldPer = PHIP_FOLD_PER;
constexpr u32 kFoldWin = kFoldThreads * kFoldPer;
constexpr u32 kBurstQuiet = 16;     // a sequential burst ends after this many unchanged ops

// One thread folds one short bucket segment in seq order.
template <u32 kOut>
__global__ __launch_bounds__(kBlock) void k_fold_thread(
    const u32* __restrict__ seg_slot, const u32* __restrict__ seg_start,
    const u32* __restrict__ seg_count, u32 nseg, const u32* __restrict__ sval,
    const OpRec* __restrict__ ops, Rec* recs, OutView ow) {
  u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nseg) return;
  const u32 cnt = seg_count[g];
  if (cnt > kLongSeg) return;
  Rec* r = &recs[seg_slot[g]];
  const u32 st = seg_start[g];
  SOp op = load_sop(ops, sval[st]);
  u32 v1 = sval[st + min(1u, cnt - 1)];
  FState S = load_state(load_rec(r)), S2;
  for (u32 j = 0; j < cnt; ++j) {
    // The next op in flight during this one and the sort value of the one
    // after (unconditional, clamped: see k_fold_block): the record load
    // never waits on a sort value loaded after this op's stores.
    const u32 v2 = sval[st + min(j + 2, cnt - 1)];
    SOp nx = load_sop(ops, v1);
    OpOut o;
    eval_sop(op, S, S2, o);
    write_out_m<kOut>(ow, op.idx, o, S2);
    S = S2;
    op = nx;
    v1 = v2;
  }
  store_state(r, S);
}

__device__ inline FState lane_state(const FState& x, u32 l) {
  FState y;
  y.a = as_f64(lane_u64(as_bits(x.a), l));
  y.t = as_f64(lane_u64(as_bits(x.t), l));
  y.e = (i64)lane_u64((u64)x.e, l);
  y.c = (i64)lane_u64((u64)x.c, l);
  y.existed = true;
  return y;
}

// One wave folds one long segment, 64 ops per window, the window held in
// registers (lane k owns op base+k), the next window's records and the
// sort values of the one after already in flight.  A round evaluates every
// unretired op of the window against the current state; every op up to and
// including the first one that changes the state is final (the ops before
// it saw exactly the state a sequential fold would have shown them), and
// that op's result state becomes the current one.  A round costs one op
// evaluation, so a change costs what a sequential fold step costs, and a run
// of unchanged ops (denied Takes, no-op merges) retires up to 64 ops at once.
template <u32 kOut>
__global__ __launch_bounds__(64) void k_fold_wave(
    const u32* __restrict__ long_list, u32 nlong, const u32* __restrict__ seg_slot,
    const u32* __restrict__ seg_start, const u32* __restrict__ seg_count,
    const u32* __restrict__ sval, const OpRec* __restrict__ ops, Rec* recs, OutView ow) {
  u32 w = blockIdx.x;
  if (w >= nlong) return;
  const u32 g = long_list[w];
  const u32 lane = threadIdx.x;
  Rec* r = &recs[seg_slot[g]];
  const u32 st = seg_start[g], cnt = seg_count[g];
  // unconditional loads, index clamped into the segment (see k_fold_block)
  const u32 last = st + cnt - 1;
  FState S = load_state(load_rec(r));
  SOp op = load_sop(ops, sval[min(st + lane, last)]);
  u32 v_nx = sval[min(st + 64 + lane, last)];
  // Each lane's result is kept in registers and stored at the top of the
  // next window, ahead of that window's loads, with no store inside the
  // round loop: every iteration issues the same stores before the same
  // loads, so the compiler's in-order wait for a window's records (gfx9
  // counts loads and stores in one counter) never waits for the stores
  // issued after them.  Window 0 starts with placeholder stores to its own
  // outputs, rewritten with its results.
  // (Reply states, when asked for, are stored where their op retires.)
  constexpr u32 kDefer = kOut & ~kOutReply;
  const FState none{};
  OpOut po{};
  u32 pidx = op.idx;
  for (u32 base = 0; base < cnt; base += 64) {
    write_out_m<kDefer>(ow, pidx, po, none);
    SOp nx = load_sop(ops, v_nx);
    v_nx = sval[min(st + base + 128 + lane, last)];
    const u32 lim = min(64u, cnt - base);
    OpOut mo{};
    u32 c = 0;
    while (c < lim) {
      const bool active = lane >= c && lane < lim;
      FState S2;
      OpOut o;
      bool ch = false;
      if (active) ch = eval_sop(op, S, S2, o);
      const u64 m = __ballot(ch);
      const u32 p = m ? (u32)(__ffsll((long long)m) - 1) : 64u;
      if (active && lane <= p) {
        mo = o;
        if constexpr ((kOut & kOutReply) != 0) {
          if (o.has_reply) write_out_m<kOutReply>(ow, op.idx, o, S2);
        }
      }
      if (p >= 64) break;
      S = lane_state(S2, p);
      c = p + 1;
    }
    if (lim < 64) {
      // lanes past the segment's end hold its last op (clamped loads): they
      // store lane lim-1's results again, so every lane stores (the reads
      // of lane q run on every lane, outside any branch)
      const u32 q = lim - 1;
      const bool past = lane > q;
      const u32 qst = (u32)__builtin_amdgcn_readlane((int)(u32)mo.st, (int)q);
      const u64 qrem = lane_u64(mo.rem, q), qhave = lane_u64(mo.have, q);
      mo.st = past ? (u8)qst : mo.st;
      mo.rem = past ? qrem : mo.rem;
      mo.have = past ? qhave : mo.have;
    }
    po = mo;
    pidx = op.idx;
    op = nx;
  }
  write_out_m<kDefer>(ow, pidx, po, none);
  if (lane == 0) store_state(r, S);
}

// ---- small ordered batches: one workgroup, one launch ------------------
// A batch of at most kSmallMax ops (the Take batcher's batches, single HTTP
// takes, small mixed streams) in one kernel instead of the ordered
// pipeline's dozen launches and host round trips: resolve every op, create
// the missing buckets, order the ops by (slot, seq) and fold every bucket's
// ops in that order with the same per-op code as the large path (eval_sop).
//   * resolve: probe() per op (the table is quiescent at kernel start);
//   * capacity: the host checked the bucket bound; the arena bytes the
//     missing long names could need are checked here, before any claim: if
//     they do not fit, hdr->fallback is set and nothing is written (the host
//     then runs the large path, which grows the arena);
//   * create: rounds of CAS claims from each missing name's home slot; a
//     claimer publishes its record (zero state, NEW flag) and a lookup that
//     meets an unpublished slot with its tag retries after the round's
//     barrier; later lookups read records and arena coherently (ld_co), as
//     other waves of this kernel wrote them;
//   * order: op i's rank among the (slot << 32 | i) keys, counted over LDS;
//   * fold: one thread per bucket with <= kLongSeg ops, one wave per longer
//     one (rounds of 64 ops against the current state, as k_fold_wave).
// The NEW flag of a created bucket is consumed by its fold (store_state), and
// the creating op gets PHIP_ST_CREATED from step_sop, as on the large path.
constexpr u32 kSmallMax = 1024;
struct SmallHdr {
  u32 created;    // buckets this launch created
  u32 fallback;   // 1: nothing was done, run the large path
  u32 full;       // a probe wrapped the table (cannot happen below the load limit)
  u32 pad;
};

__device__ inline Rec load_rec_co(const Rec* p) {
  const u64* q = reinterpret_cast<const u64*>(p);
  Rec r;
  r.tag = ld_co(q); r.added = ld_co(q + 1); r.taken = ld_co(q + 2); r.elapsed = (i64)ld_co(q + 3);
  r.name0 = ld_co(q + 4); r.name1 = ld_co(q + 5); r.created = (i64)ld_co(q + 6); r.name2 = ld_co(q + 7);
  return r;
}

__global__ __launch_bounds__(kSmallMax) void k_small_mixed(NamesOffs src, OpView ov, u32 n, Table T,
                                                         u8* arena, u64 arena_cap,
                                                         u64* arena_cursor, OutView ow,
                                                         SmallHdr* hdr) {
  __shared__ OpRec sop[kSmallMax];
  __shared__ u32 sval[kSmallMax];
  __shared__ u64 skey[kSmallMax];
  __shared__ u32 sorted[kSmallMax];
  __shared__ u32 lstart[kSmallMax / kLongSeg + 1], lcnt[kSmallMax / kLongSeg + 1];
  __shared__ u32 nlong, long_need, pending, created, full;
  const u32 i = threadIdx.x;
  const bool valid = i < n;
  if (i == 0) { nlong = 0; long_need = 0; pending = 0; created = 0; full = 0; }
  // 1. the op (k_pack_ops' record) and its name's slot
  Name nm{};
  u32 slot = 0;
  bool miss = false;
  if (valid) {
    const u32 kind = ov.kind ? ov.kind[i] : ov.kind0;
    OpRec r;
    r.now = ov.now ? ov.now[i] : ov.now0;
    if (kind == PHIP_OP_TAKE) {
      const i64 f = ov.freq[i], pr = ov.per[i];
      r.x = (u64)rate_interval(f, pr);
      r.y = as_bits((double)f);             // bucket.go:192
      r.z = as_bits((double)ov.count[i]);   // bucket.go:215
    } else {
      r.x = ov.a[i]; r.y = ov.t[i]; r.z = (u64)ov.e[i];
    }
    sop[i] = r;
    sval[i] = i | (kind << kOpIdxBits);
    u64 off; u32 len;
    src.get(i, off, len);
    load_name_wide<false>(src.blob, off, len, nm);
    Rec rr;
    const int pr = probe(T, nm, src.blob, &slot, &rr);
    miss = pr != kFound;
  }
  __syncthreads();
  // 2. arena room for the missing long names (an upper bound), before any claim
  if (miss && nm.len > kInlineName) atomicAdd(&long_need, nm.len);
  __syncthreads();
  if (long_need && ld_co(arena_cursor) + long_need > arena_cap) {
    if (i == 0) hdr->fallback = 1;
    return;
  }
  // 3. create the missing buckets, in rounds
  const u32 mask = T.mask();
  for (;;) {
    if (miss) {
      const u64 tag = T.tag(nm.h);
      u32 s = T.home(tag), k = 0;
      for (; k <= mask; ++k, s = (s + 1) & mask) {
        u64 t = ld_co(&T.recs[s].tag);
        if (t == 0) {
          t = atomicCAS(&T.recs[s].tag, 0ull, tag);
          if (t == 0) {   // claimed: publish (k_publish's record)
            Rec* q = &T.recs[s];
            q->added = kEPosZero; q->taken = kEPosZero; q->elapsed = 0;
            q->created = sop[i].now;
            q->name1 = nm.w1; q->name2 = nm.w2;
            u64 w0 = nm.w0;
            if (nm.len > kInlineName) {
              const u64 a = atomicAdd(arena_cursor, (u64)nm.len);   // room checked above
              u64 off; u32 len;
              src.get(i, off, len);
              for (u32 b = 0; b < len; ++b) arena[a + b] = src.blob[off + b];
              w0 = (nm.w0 & 0xFFu) | (a << 32);
            }
            T.aux[s] = 0;
            __threadfence();
            q->name0 = with_flags(w0, kRecPublished | kRecNew);
            atomicAdd(&created, 1u);
            slot = s;
            miss = false;
            break;
          }
        }
        if (t == tag) {
          const Rec r = load_rec_co(&T.recs[s]);
          if (!(rec_flags(r) & kRecPublished)) { pending = 1; break; }   // its claimer publishes this round
          if (name_equal<true>(r, nm, src.blob, T.arena)) { slot = s; miss = false; break; }
        }
      }
      if (k > mask) { full = 1; miss = false; }
    }
    __threadfence();
    __syncthreads();
    const bool again = pending != 0;
    __syncthreads();
    if (!again) break;
    if (i == 0) pending = 0;
    __syncthreads();
  }
  if (full) {   // cannot happen below the load limit the host checked; nothing is folded
    if (i == 0) { hdr->full = 1; hdr->created = created; }
    return;
  }
  // 4. order: rank of (slot, seq)
  const u64 key = valid ? ((u64)slot << 32 | i) : ~0ull;
  skey[i] = key;
  __syncthreads();
  if (valid) {
    u32 rank = 0;
    for (u32 j = 0; j < n; ++j) rank += skey[j] < key;
    sorted[rank] = i;
  }
  __syncthreads();
  // 5. fold: position r starts a bucket's segment when its slot differs
  //    from position r - 1's
  if (valid) {
    const u32 sl = (u32)(skey[sorted[i]] >> 32);
    if (i == 0 || (u32)(skey[sorted[i - 1]] >> 32) != sl) {
      u32 cnt = 1;
      while (i + cnt < n && (u32)(skey[sorted[i + cnt]] >> 32) == sl) ++cnt;
      if (cnt > kLongSeg) {
        const u32 l = atomicAdd(&nlong, 1u);
        lstart[l] = i;
        lcnt[l] = cnt;
      } else {
        Rec* rec = &T.recs[sl];
        FState S = load_state(load_rec_co(rec)), S2;
        for (u32 j = 0; j < cnt; ++j) {
          const u32 o = sorted[i + j];
          const SOp op = make_sop(sop[o], sval[o]);
          OpOut out;
          eval_sop(op, S, S2, out);
          write_out(ow, op.idx, out, S2);
          S = S2;
        }
        store_state(rec, S);
      }
    }
  }
  __syncthreads();
  const u32 lane = i & 63, wave = i >> 6;
  for (u32 l = wave; l < nlong; l += kSmallMax / 64) {
    const u32 r0 = lstart[l], cnt = lcnt[l];
    Rec* rec = &T.recs[(u32)(skey[sorted[r0]] >> 32)];
    FState S = load_state(load_rec_co(rec));
    for (u32 base = 0; base < cnt; base += 64) {
      const u32 lim = min(64u, cnt - base);
      const u32 o = sorted[r0 + base + min(lane, lim - 1)];
      const SOp op = make_sop(sop[o], sval[o]);
      u32 c = 0;
      while (c < lim) {   // k_fold_wave's round
        const bool active = lane >= c && lane < lim;
        FState S2;
        OpOut out;
        bool ch = false;
        if (active) ch = eval_sop(op, S, S2, out);
        const u64 m = __ballot(ch);
        const u32 p = m ? (u32)(__ffsll((long long)m) - 1) : 64u;
        if (active && lane <= p) write_out(ow, op.idx, out, S2);
        if (p >= 64) break;
        S = lane_state(S2, p);
        c = p + 1;
      }
    }
    if (lane == 0) store_state(rec, S);
  }
  if (i == 0) hdr->created = created;
}

// ---- window summaries: skip provably quiet windows of a hot bucket -------
// For window w of a huge segment (ops [w*kFoldWin, (w+1)*kFoldWin)):
//   merge-applied ops (RECEIVE of a non-zero state, UPSERT): field maxima in
//   replica E order (enc_replica, elapsed biased);
//   TAKE ops: the now range, and whether all share (interval, capacity, t).
// window_quiet(S) proves that no op of the window changes S:
//   * a merge changes nothing when E'(o) <= E(b) field by field (the
//     E-encoding identity of phip_device.hpp; for o = -0.0, E'(o) <= E(b)
//     means b is -0.0, positive or NaN, and Go's b < -0.0 is false);
//   * an incast request never changes an existing bucket;
//   * with added != 0 a denied Take changes nothing, and for one (interval,
//     capacity, t) Take's `have` is monotone in now (dt = now - last is, and
//     every later step is a correctly rounded monotone operation), so one
//     denial at the extreme now of the window (max now for interval >= 0,
//     min now for interval < 0) proves every Take of the window is denied.
struct alignas(16) WinSum {
  u64 ea, et, ee;        // maxima (0 = none)
  i64 now_min, now_max;
  u64 interval, cap, t;  // the shared Take parameters (kind bit kSumMixed if not shared)
  u32 flags, pad;
};
constexpr u32 kSumTake = 1, kSumMixed = 2, kSumMerge = 4;
constexpr u32 kSumDirty = 8;   // a merge with a -0.0 replica field (E max != Go's merge)

__device__ inline bool window_quiet(const WinSum& q, const FState& S) {
  if (!S.existed) return false;
  if (q.flags & kSumMerge) {
    if (q.ea > enc_f64(as_bits(S.a)) || q.et > enc_f64(as_bits(S.t)) ||
        q.ee > ((u64)S.e ^ kSign))
      return false;
  }
  if (q.flags & kSumTake) {
    if ((q.flags & kSumMixed) || S.a == 0) return false;
    double a = S.a, t = S.t;
    i64 e = S.e;
    const i64 now = (i64)q.interval < 0 ? q.now_min : q.now_max;
    TakeResult r = take_step(a, t, e, S.c, now, (i64)q.interval, as_f64(q.cap), as_f64(q.t));
    if (r.ok) return false;
  }
  return true;
}

template <u32 kDiv>
__device__ inline void huge_scan(const u32* __restrict__ huge_list, u32 nhuge,
                                 const u32* __restrict__ seg_count, u64* __restrict__ out,
                                 u64* part) {
  const u32 tid = threadIdx.x;
  const u32 per = (nhuge + 1023) / 1024;
  u64 sum = 0;
  for (u32 k = 0; k < per; ++k) {
    const u32 h = tid * per + k;
    if (h < nhuge) sum += (seg_count[huge_list[h]] + kDiv - 1) / kDiv;
  }
  part[tid] = sum;
  __syncthreads();
  for (u32 off = 1; off < 1024; off <<= 1) {
    u64 v = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  u64 base = part[tid] - sum;
  for (u32 k = 0; k < per; ++k) {
    const u32 h = tid * per + k;
    if (h < nhuge) { out[h] = base; base += (seg_count[huge_list[h]] + kDiv - 1) / kDiv; }
  }
  __syncthreads();
}

// The huge segment list with its nfirst largest segments moved to the front
// (the rest keep their order): the largest segments' folds are the step's
// longest sequential chains, so they get their own stream and start first
// (one block; out must not alias huge_list).
__global__ __launch_bounds__(1024) void k_huge_order(const u32* __restrict__ huge_list, u32 nhuge,
                                                     const u32* __restrict__ seg_count, u32 nfirst,
                                                     u32* __restrict__ out) {
  __shared__ u64 part[1024];
  __shared__ u32 sel[kHugeFirstMax];
  const u32 tid = threadIdx.x;
  for (u32 r = 0; r < nfirst; ++r) {
    u64 best = 0;   // (count, ~index): the largest count, then the lowest index
    for (u32 h = tid; h < nhuge; h += 1024) {
      bool taken = false;
      for (u32 q = 0; q < r; ++q) taken |= sel[q] == h;
      if (!taken) best = max(best, ((u64)seg_count[huge_list[h]] << 32) | (0xFFFFFFFFu - h));
    }
    part[tid] = best;
    __syncthreads();
    for (u32 off = 512; off; off >>= 1) {
      if (tid < off) part[tid] = max(part[tid], part[tid + off]);
      __syncthreads();
    }
    if (tid == 0) {
      const u32 h = 0xFFFFFFFFu - (u32)part[0];
      sel[r] = h;
      out[r] = huge_list[h];
    }
    __syncthreads();
  }
  for (u32 h = tid; h < nhuge; h += 1024) {
    u32 below = 0;
    bool taken = false;
    for (u32 q = 0; q < nfirst; ++q) {
      below += sel[q] < h;
      taken |= sel[q] == h;
    }
    if (!taken) out[nfirst + h - below] = huge_list[h];
  }
}

// Offsets of the huge segments in the contiguous staging arrays (ops) and in
// the window-summary array (one block).
__global__ __launch_bounds__(1024) void k_huge_offsets(const u32* __restrict__ huge_list, u32 nhuge,
                                                       const u32* __restrict__ seg_count,
                                                       u64* __restrict__ hoff, u64* __restrict__ woff) {
  __shared__ u64 part[1024];
  huge_scan<1>(huge_list, nhuge, seg_count, hoff, part);
  huge_scan<kFoldWin>(huge_list, nhuge, seg_count, woff, part);
  if (threadIdx.x == 0 && nhuge)
    woff[nhuge] = woff[nhuge - 1] + (seg_count[huge_list[nhuge - 1]] + kFoldWin - 1) / kFoldWin;
}

// Window b of the flat window index space -> (huge segment h, window w).
__device__ inline bool huge_window(const u64* __restrict__ woff, u32 nhuge, u32 b, u32& h, u32& w) {
  if (b >= woff[nhuge]) return false;
  u32 lo = 0, hi = nhuge - 1;   // last h with woff[h] <= b
  while (lo < hi) {
    const u32 mid = (lo + hi + 1) >> 1;
    if (woff[mid] <= b) lo = mid; else hi = mid - 1;
  }
  h = lo;
  w = b - (u32)woff[lo];
  return true;
}

// The ops of every huge segment gathered into contiguous (slot, seq) order
// by the whole chip, one block per fold window, so that the one workgroup
// folding a hot bucket streams its input instead of chasing one random
// record per op (a single CU cannot keep enough random misses in flight).
// The same pass writes the window's summary (WinSum).
constexpr u32 kGatherPer = kFoldWin / kBlock;

__global__ __launch_bounds__(kBlock) void k_gather_huge(
    const u32* __restrict__ huge_list, u32 nhuge, const u64* __restrict__ hoff,
    const u64* __restrict__ woff, const u32* __restrict__ seg_start,
    const u32* __restrict__ seg_count, const u32* __restrict__ sval,
    const OpRec* __restrict__ ops, OpRec* __restrict__ hop, u32* __restrict__ hval,
    WinSum* __restrict__ sums, u32 h_begin) {
  __shared__ u64 red[6][kBlock / 64];
  __shared__ u32 s_first;
  __shared__ u64 s_par[3];
  // segments [h_begin, nhuge) of the list: their windows follow
  // woff[h_begin]; a grid of a few blocks per CU walks them
  const u32 b_end = (u32)woff[nhuge];
  for (u32 b = (u32)woff[h_begin] + blockIdx.x; b < b_end; b += gridDim.x) {
  u32 h, w;
  huge_window(woff, nhuge, b, h, w);
  const u32 g = huge_list[h];
  const u32 st = seg_start[g], cnt = seg_count[g];
  const u64 dst = hoff[h];
  const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const u32 p0 = w * kFoldWin, p1 = min(cnt, p0 + kFoldWin);
  if (tid == 0) s_first = 0xFFFFFFFFu;
  u32 v[kGatherPer];
  OpRec r[kGatherPer];
#pragma unroll
  for (u32 k = 0; k < kGatherPer; ++k) v[k] = sval[st + min(p0 + k * kBlock + tid, p1 - 1)];
#pragma unroll
  for (u32 k = 0; k < kGatherPer; ++k) r[k] = load_oprec(ops + (v[k] & kOpIdxMask));
  u64 ea = 0, et = 0, ee = 0, nmin = ~0ull, nmax = 0;
  u32 first_take = 0xFFFFFFFFu;
  bool merge = false, dirty = false;
#pragma unroll
  for (u32 k = 0; k < kGatherPer; ++k) {
    const u32 j = p0 + k * kBlock + tid;
    if (j >= p1) continue;
    ulonglong2* q = reinterpret_cast<ulonglong2*>(hop + dst + j);
    q[0] = ulonglong2{(u64)r[k].now, r[k].x};
    q[1] = ulonglong2{r[k].y, r[k].z};
    hval[dst + j] = v[k];
    const u32 kind = v[k] >> kOpIdxBits;
    if (kind == PHIP_OP_TAKE) {
      const u64 nb = (u64)r[k].now ^ kSign;
      nmin = min(nmin, nb); nmax = max(nmax, nb);
      first_take = min(first_take, j);
    } else if (kind == PHIP_OP_UPSERT || !state_is_zero(r[k].x, r[k].y, (i64)r[k].z)) {
      merge = true;
      dirty |= r[k].x == kSign || r[k].y == kSign;
      ea = max(ea, enc_replica(r[k].x)); et = max(et, enc_replica(r[k].y));
      ee = max(ee, r[k].z ^ kSign);
    }
  }
  __syncthreads();
  if (first_take != 0xFFFFFFFFu) atomicMin(&s_first, first_take);
  __syncthreads();
  const u32 ft = s_first;
#pragma unroll
  for (u32 k = 0; k < kGatherPer; ++k)
    if (p0 + k * kBlock + tid == ft) { s_par[0] = r[k].x; s_par[1] = r[k].y; s_par[2] = r[k].z; }
  __syncthreads();
  bool mixed = false;
  if (ft != 0xFFFFFFFFu) {
    const u64 iv = s_par[0], cp = s_par[1], tb = s_par[2];
#pragma unroll
    for (u32 k = 0; k < kGatherPer; ++k) {
      const u32 j = p0 + k * kBlock + tid;
      if (j < p1 && (v[k] >> kOpIdxBits) == PHIP_OP_TAKE)
        mixed |= r[k].x != iv || r[k].y != cp || r[k].z != tb;
    }
  }
  u64 x[6] = {ea, et, ee, ~nmin, nmax, (u64)(merge ? 1 : 0) | (mixed ? 2 : 0) | (dirty ? 4 : 0)};
#pragma unroll
  for (int k = 0; k < 6; ++k)
    for (int off = 32; off >= 1; off >>= 1) {
      const u64 o = (u64)__shfl_xor((long long)x[k], off);
      x[k] = k == 5 ? (x[k] | o) : max(x[k], o);
    }
  if (lane == 0)
    for (int k = 0; k < 6; ++k) red[k][wv] = x[k];
  __syncthreads();
  if (tid == 0) {
    for (u32 y = 1; y < kBlock / 64; ++y) {
      for (int k = 0; k < 5; ++k) x[k] = max(x[k], red[k][y]);
      x[5] |= red[5][y];
    }
    WinSum q;
    q.ea = x[0]; q.et = x[1]; q.ee = x[2];
    q.now_min = (i64)(~x[3] ^ kSign); q.now_max = (i64)(x[4] ^ kSign);
    q.interval = ft != 0xFFFFFFFFu ? s_par[0] : 0;
    q.cap = ft != 0xFFFFFFFFu ? s_par[1] : 0;
    q.t = ft != 0xFFFFFFFFu ? s_par[2] : 0;
    q.flags = (ft != 0xFFFFFFFFu ? kSumTake : 0) | ((x[5] & 2) ? kSumMixed : 0) |
              ((x[5] & 1) ? kSumMerge : 0) | ((x[5] & 4) ? kSumDirty : 0);
    q.pad = 0;
    sums[woff[h] + w] = q;
  }
  __syncthreads();   // the window's shared arrays are reused by the next
  }
}

// The hot-bucket fold records the bucket's state history as runs instead of
// per-op results: run k says "ops [pos_k, pos_{k+1}) of the segment saw state
// state_k, raised by the merges between" (below).  k_huge_outputs then
// evaluates every op against its state on the whole chip and writes the
// results, so the one workgroup on the sequential critical path only streams
// ops and tests "does this op change the state?".
//
// Absorbing merges.  A hot bucket receives replica states all the time, and
// many raise it a little (replica `elapsed` values run close behind the local
// clock), while most of its Takes are denied (it is rate limited).  Treating
// every such merge as a sequential state change made the fold of a realistic
// stream 20x slower than its quiet-window fast path.  Instead, while the
// bucket's state only grows (E order, every field), the state an op sees is
//     X_k = max(R, G_k)
// with R the state after the last change that was not a merge (a successful
// Take) and G_k the running maximum of the replica states merged before op k
// (E' codes, phip_device.hpp): R already holds every merge before it, and a
// merge is the E max for replicas without -0.0 fields (kSumDirty).  A window
// whose Takes are all provably denied for every X_k between its first and last
// op (window_absorbable) then changes nothing but G, and needs no run.  If a
// change ever lowers a field (a Take whose refill is negative because tokens
// exceed capacity, a -0.0 replica) the identity fails from there on: the
// segment turns "exact" at that run (exact_from) and every later change,
// merges included, is a run of its own (window_quiet, the strict test).
struct RunState {
  u64 a, t;   // float64 bits
  i64 e, c;
};

__device__ inline void put_run(u32* run_pos, RunState* run_st, u32 k, u32 pos, const FState& S) {
  run_pos[k] = pos;
  run_st[k] = RunState{as_bits(S.a), as_bits(S.t), S.e, S.c};
}

// Maxima of merged replica states: E' codes of added and taken (enc_replica)
// and elapsed biased by 2^63, 0 = none.
struct GMax {
  u64 a, t, e;
};
__device__ inline GMax gmax(const GMax& x, const GMax& y) {
  return GMax{x.a > y.a ? x.a : y.a, x.t > y.t ? x.t : y.t, x.e > y.e ? x.e : y.e};
}
__device__ inline GMax gmax_of(const WinSum& q) { return GMax{q.ea, q.et, q.ee}; }
__device__ inline bool gmax_empty(const GMax& g) { return !(g.a | g.t | g.e); }

// X = max(R, G) in E order, field by field.
__device__ inline FState join_state(const FState& R, const GMax& g) {
  FState X = R;
  if (g.a > enc_f64(as_bits(R.a))) X.a = as_f64(dec_f64(g.a));
  if (g.t > enc_f64(as_bits(R.t))) X.t = as_f64(dec_f64(g.t));
  if (g.e > ((u64)R.e ^ kSign)) X.e = (i64)(g.e ^ kSign);
  return X;
}

// A change from S to S2 that keeps X_k = max(R, G_k) exact afterwards: no
// field is lowered in E order.
__device__ inline bool state_grew(const FState& S, const FState& S2) {
  return enc_f64(as_bits(S2.a)) >= enc_f64(as_bits(S.a)) &&
         enc_f64(as_bits(S2.t)) >= enc_f64(as_bits(S.t)) && S2.e >= S.e;
}

// Window q, whose ops see states between Xs (at its start) and Xe (Xs raised
// by the window's merge maxima): true when no Take of the window can succeed
// (then no op changes anything but G).  For every op the state lies between
// the two ends field by field, and with a shared (interval > 0, capacity, t)
// Take's `have` (bucket.go:198-216) is bounded by
//     (Xe.added - Xs.taken) + take_dt(created, Xs.elapsed, max now) / interval,
// every step being a correctly rounded monotone operation (a refill capped at
// `missing` is below the uncapped one, and + is monotone).  t > bound then
// means every Take of the window is denied; added > 0 at the start (it only
// grows) rules out the added = capacity write of bucket.go:194-196.
__device__ inline bool window_absorbable(const WinSum& q, const FState& Xs, const FState& Xe) {
  if (!Xs.existed || (q.flags & kSumDirty)) return false;
  if (!(q.flags & kSumTake)) return true;
  if (q.flags & kSumMixed) return false;
  const i64 iv = (i64)q.interval;
  if (iv <= 0) return false;
  if (!(Xs.a > 0.0) || !(Xe.a < __builtin_inf()) || !(Xs.t > -__builtin_inf()) ||
      !(Xs.t < __builtin_inf()))
    return false;
  const double tok = Xe.a - Xs.t;
  const double add = (double)take_dt(Xs.c, Xs.e, q.now_max) / (double)iv;
  return as_f64(q.t) > tok + add;
}

// One workgroup folds one very long segment (a Zipf-hot bucket) from the
// contiguous copy k_gather_huge made.  Windows are tested kSumChunk at a time
// from their summaries (quiet, absorbable, or quiet once the segment is
// exact), and only a window that may change the state is staged in LDS and
// folded (fold_window_absorb, or fold_window once exact):
//  * parallel round: every thread tests its unretired ops (k*kFoldThreads +
//    t, k < kFoldPer) against the state they see; a workgroup min finds the
//    first op that changes it; the ops before it saw exactly that state;
//  * burst from that op by wave 0, until the state stops changing.
// The window lives in LDS while it is folded; registers hold per-op values
// only, so the kernel keeps its working set without spilling.

constexpr u32 kSumChunk = kFoldThreads;   // window summaries staged in LDS at a time

struct FoldShared {
  OpRec op[kFoldWin];
  u32 val[kFoldWin];
  WinSum sum[kSumChunk];
  GMax pinc[kSumChunk];                   // inclusive merge-maxima prefix over the chunk
  GMax wtot[kFoldThreads / 64];
  GMax wtot4[kFoldPer][kFoldThreads / 64];
  u32 wave_min[2][kFoldThreads / 64];
  u32 quiet_min[kFoldThreads / 64];
  u64 state[8];
  u32 cur, nrun, exact_from;
  u32 n_burst, n_walk;   // diagnostics (k_fold_block's dbg)
  u32 n_iter, n_raise;   // burst iterations; those that stopped at a merge
  u64 prof[6];           // diagnostics: wall-clock ticks per phase (dbg only)
  u32 profiling;
};

// Phase timing of k_fold_block (PHIP_FOLD_STATS): thread 0 adds the ticks
// since *t to sh.prof[k] (the workgroup's threads run every phase together).
__device__ inline void prof_mark(FoldShared& sh, u32 k, u64& t) {
  if (sh.profiling && threadIdx.x == 0) {
    const u64 now = wall_clock64();
    sh.prof[k] += now - t;
    t = now;
  }
}

// Window [pos, pos + kFoldWin) of the segment into LDS (sh.op / sh.val, op k
// of the window at index k).  Loads are unconditional (index clamped into the
// segment) and issued together: a load under a runtime condition makes hipcc
// branch around it and wait for it on the spot (cdna_hip_programming.md,
// "traps that silently de-pipeline").
__device__ inline void fold_stage(const u32* __restrict__ sv, const OpRec* __restrict__ so, u32 pos,
                                  u32 last, u32 tid, FoldShared& sh) {
  u32 v[kFoldPer];
  OpRec r[kFoldPer];
#pragma unroll
  for (u32 k = 0; k < kFoldPer; ++k) {
    const u32 j = min(pos + k * kFoldThreads + tid, last);
    v[k] = sv[j];
    r[k] = load_oprec(so + j);
  }
#pragma unroll
  for (u32 k = 0; k < kFoldPer; ++k) {
    sh.op[k * kFoldThreads + tid] = r[k];
    sh.val[k * kFoldThreads + tid] = v[k];
  }
  __syncthreads();
}

__device__ inline SOp staged_sop(const FoldShared& sh, u32 i) { return make_sop(sh.op[i], sh.val[i]); }

__device__ inline void publish_state(FoldShared& sh, const FState& T) {
  sh.state[0] = as_bits(T.a); sh.state[1] = as_bits(T.t);
  sh.state[2] = (u64)T.e; sh.state[3] = (u64)T.c;
}
__device__ inline FState read_state(const FoldShared& sh) {
  FState S;
  S.a = as_f64(sh.state[0]); S.t = as_f64(sh.state[1]);
  S.e = (i64)sh.state[2]; S.c = (i64)sh.state[3]; S.existed = true;
  return S;
}

// Workgroup min of u32 (alternating buffers: one barrier per round).
__device__ inline u32 block_min(u32 m, FoldShared& sh, u32& round, u32 tid) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = min(m, (u32)__shfl_xor((int)m, off));
  u32* wm = sh.wave_min[round & 1];
  ++round;
  if ((tid & 63) == 0) wm[tid >> 6] = m;
  __syncthreads();
  u32 r = 0xFFFFFFFFu;
#pragma unroll
  for (u32 x = 0; x < kFoldThreads / 64; ++x) r = min(r, wm[x]);
  return r;
}

// Exact fold of a staged window: every change of the state is a run.
__device__ inline void fold_window(u32 pos, u32 lim, FState& S, u32& round, FoldShared& sh, u32* rp,
                                   RunState* rs, u32 tid) {
  const u32 lane = tid & 63, wv = tid >> 6;
  u32 cur = 0;
  while (cur < lim) {
    u32 my_first = 0xFFFFFFFFu;
    {
#pragma unroll 1
      for (u32 k = 0; k < kFoldPer; ++k) {
        const u32 w = k * kFoldThreads + tid;
        if (w >= cur && w < lim && my_first == 0xFFFFFFFFu) {
          FState S2;
          if (apply_sop(staged_sop(sh, w), S, S2)) my_first = w;
        }
      }
    }
    const u32 first = block_min(my_first, sh, round, tid);
    if (first == 0xFFFFFFFFu) return;
    // ---- sequential burst (wave 0) from `first`, which changes the state
    if (wv == 0) {
      FState T = S;
      u32 j = first, quiet = 0, nrun = sh.nrun;
      while (j < lim && quiet < kBurstQuiet) {
        FState T2;
        if (apply_sop(staged_sop(sh, j), T, T2)) {
          T = T2;
          if (lane == 0) put_run(rp, rs, nrun, pos + j + 1, T);
          ++nrun;
          quiet = 0;
        } else {
          ++quiet;
        }
        ++j;
      }
      if (lane == 0) {
        sh.n_burst += 1;
        sh.n_walk += j - first;
        publish_state(sh, T);
        sh.cur = j;
        sh.nrun = nrun;
      }
    }
    __syncthreads();
    S = read_state(sh);
    cur = sh.cur;
    __syncthreads();   // state / cur are rewritten by the next burst
  }
}

__device__ inline u64 shfl_up_u64(u64 v, u32 d) {
  const u32 lo = __shfl_up((u32)v, d), hi = __shfl_up((u32)(v >> 32), d);
  return ((u64)hi << 32) | lo;
}
__device__ inline GMax shfl_up_gmax(const GMax& g, u32 d) {
  return GMax{shfl_up_u64(g.a, d), shfl_up_u64(g.t, d), shfl_up_u64(g.e, d)};
}

// Wave-wide max scans of GMax with DPP moves (no LDS round trip per step:
// the fold runs one wave per SIMD, so every step's latency is exposed).
// Lanes with no source read 0, the identity of the unsigned max.  All 64
// lanes must be active.
template <int Ctrl, int RowMask = 0xF>
__device__ inline u64 dpp_u64(u64 v) {
  const u32 lo = (u32)__builtin_amdgcn_update_dpp(0, (int)(u32)v, Ctrl, RowMask, 0xF, true);
  const u32 hi = (u32)__builtin_amdgcn_update_dpp(0, (int)(u32)(v >> 32), Ctrl, RowMask, 0xF, true);
  return ((u64)hi << 32) | lo;
}
template <int Ctrl, int RowMask = 0xF>
__device__ inline GMax dpp_gmax(const GMax& g) {
  return GMax{dpp_u64<Ctrl, RowMask>(g.a), dpp_u64<Ctrl, RowMask>(g.t), dpp_u64<Ctrl, RowMask>(g.e)};
}
// inclusive: row_shr 1/2/4/8 within rows of 16, then row_bcast15 into rows
// 1 and 3, row_bcast31 into rows 2 and 3
__device__ inline GMax wave_incl_max(GMax x) {
  x = gmax(x, dpp_gmax<0x111>(x));
  x = gmax(x, dpp_gmax<0x112>(x));
  x = gmax(x, dpp_gmax<0x114>(x));
  x = gmax(x, dpp_gmax<0x118>(x));
  x = gmax(x, dpp_gmax<0x142, 0xA>(x));
  x = gmax(x, dpp_gmax<0x143, 0xC>(x));
  return x;
}
// the value of lane - 1 (wave_shr:1; lane 0 reads 0)
__device__ inline GMax wave_shr1(const GMax& x) { return dpp_gmax<0x138>(x); }

// Inclusive prefix max of x over the workgroup (kFoldThreads lanes, thread
// order) into sh.pinc[tid].
__device__ inline void block_prefix_gmax(GMax x, FoldShared& sh, u32 tid) {
  const u32 lane = tid & 63, wv = tid >> 6;
  x = wave_incl_max(x);
  if (lane == 63) sh.wtot[wv] = x;
  __syncthreads();
  for (u32 y = 0; y < wv; ++y) x = gmax(x, sh.wtot[y]);
  if (tid < kSumChunk) sh.pinc[tid] = x;
  __syncthreads();
}

// A merge op's contribution to the running replica maximum G (E' codes,
// elapsed biased; 0 for Takes and incast requests, which merge nothing).
__device__ inline GMax merge_contrib(const OpRec& r, u32 v) {
  const u32 kind = v >> kOpIdxBits;
  if (kind == PHIP_OP_TAKE || (kind == PHIP_OP_RECEIVE && state_is_zero(r.x, r.y, (i64)r.z)))
    return GMax{0, 0, 0};
  return GMax{enc_replica(r.x), enc_replica(r.y), r.z ^ kSign};
}

// g[k] = the replica maximum before op k*kFoldThreads + tid of the staged
// window (gstart, then the window's merges in op order); *gend after the
// whole window.  Four rows of kFoldThreads ops, each a wave scan plus the
// totals of the waves and rows before it.
__device__ inline void window_prefix(u32 lim, GMax gstart, GMax (&g)[kFoldPer], GMax& gend,
                                     FoldShared& sh, u32 tid) {
  const u32 lane = tid & 63, wv = tid >> 6;
  GMax inc[kFoldPer];
#pragma unroll
  for (u32 k = 0; k < kFoldPer; ++k) {
    const u32 i = k * kFoldThreads + tid;
    inc[k] = wave_incl_max(i < lim ? merge_contrib(sh.op[i], sh.val[i]) : GMax{0, 0, 0});
    if (lane == 63) sh.wtot4[k][wv] = inc[k];
  }
  __syncthreads();
  GMax acc = gstart;
#pragma unroll
  for (u32 k = 0; k < kFoldPer; ++k) {
    GMax before = acc;
    for (u32 y = 0; y < wv; ++y) before = gmax(before, sh.wtot4[k][y]);
    g[k] = gmax(before, wave_shr1(inc[k]));   // lane 0: 0, the identity
#pragma unroll
    for (u32 y = 0; y < kFoldThreads / 64; ++y) acc = gmax(acc, sh.wtot4[k][y]);
  }
  gend = acc;
  __syncthreads();   // wtot4 is rewritten by the next window
}

// g[k] for a runtime k without indexing the register array (a dynamic
// index would put it in scratch memory).
__device__ inline GMax pick(const GMax (&g)[kFoldPer], u32 k) {
  GMax r = g[0];
#pragma unroll
  for (u32 x = 1; x < kFoldPer; ++x) {
    const bool s = k == x;
    r.a = s ? g[x].a : r.a;
    r.t = s ? g[x].t : r.t;
    r.e = s ? g[x].e : r.e;
  }
  return r;
}

// Fold a staged window that neither window test could clear, in the
// absorbing model: merges only raise G, so the ops that need a run are those
// that change the state otherwise (a successful Take, a denied Take's added =
// capacity write, the op creating the bucket).  A parallel round evaluates
// every such op against its own X_k = max(R, G_k) and finds the first that
// changes it; the ops before it saw exactly those states.  Wave 0 then runs
// wave rounds from there carrying the true state X (lane l looks at op
// cur + l; the first op that changes X decides: a merge that raises it is
// applied with no run, a Take that changes it is applied and starts one)
// until two rounds in a row change nothing; the workgroup round follows.  A
// change that lowers a field ends the identity: the run it starts is exact
// (sh.exact_from) and the rest of the window is applied one op at a time,
// every change a run.  R and G are updated in place.
__device__ inline void fold_window_absorb(u32 pos, u32 lim, FState& R, GMax& G, u32& round,
                                          FoldShared& sh, u32* rp, RunState* rs, u32 tid) {
  const u32 lane = tid & 63, wv = tid >> 6;
  GMax g[kFoldPer], gend;
  u64 tp = sh.profiling ? wall_clock64() : 0;
  window_prefix(lim, G, g, gend, sh, tid);
  prof_mark(sh, 2, tp);
  u32 cur = 0;
  while (cur < lim) {
    u32 my_first = 0xFFFFFFFFu;
    {
#pragma unroll 1
      for (u32 k = 0; k < kFoldPer; ++k) {
        const u32 idx = k * kFoldThreads + tid;
        if (idx >= cur && idx < lim && my_first == 0xFFFFFFFFu) {
          const SOp op = staged_sop(sh, idx);
          const FState X = join_state(R, pick(g, k));
          if (op.kind == PHIP_OP_TAKE || !X.existed) {
            FState X2;
            if (apply_sop(op, X, X2)) my_first = idx;
          }
        }
      }
    }
    const u32 p = block_min(my_first, sh, round, tid);
    prof_mark(sh, 3, tp);
    if (p == 0xFFFFFFFFu) break;
    if (tid == p % kFoldThreads) {   // G before op p, for the burst
      const GMax gp = pick(g, p / kFoldThreads);
      sh.state[4] = gp.a; sh.state[5] = gp.t; sh.state[6] = gp.e;
    }
    __syncthreads();
    if (wv == 0) {
      FState X = join_state(R, GMax{sh.state[4], sh.state[5], sh.state[6]});
      u32 j = p, quiet = 0, nrun = sh.nrun, exact_from = sh.exact_from;
      const bool prof = sh.profiling;   // diagnostics counters only when asked (an LDS update per round)
      while (j < lim && quiet < 2 && exact_from == 0xFFFFFFFFu) {
        const u32 i = j + lane;
        const bool valid = i < lim;
        const SOp op = staged_sop(sh, min(i, lim - 1));
        const bool is_take = op.kind == PHIP_OP_TAKE || !X.existed;
        const bool is_merge = !is_take &&
                              (op.kind != PHIP_OP_RECEIVE || !state_is_zero(op.x, op.y, (i64)op.z));
        bool raise = false;
        FState X2 = X;
        if (valid && is_merge) {
          go_merge(X2.a, X2.t, X2.e, as_f64(op.x), as_f64(op.y), (i64)op.z);   // bucket.go:250-260
          raise = as_bits(X2.a) != as_bits(X.a) || as_bits(X2.t) != as_bits(X.t) || X2.e != X.e;
        }
        bool chg = false;
        if (valid && is_take) chg = apply_sop(op, X, X2);
        const u64 mb = __ballot(raise | chg);
        if (!mb) {
          j += 64;
          ++quiet;
          continue;
        }
        const u32 q = (u32)__ffsll((long long)mb) - 1;
        const FState Y = lane_state(X2, q);
        const bool q_chg = (__ballot(chg) >> q) & 1;
        if (prof && lane == 0) { ++sh.n_iter; sh.n_raise += !q_chg; }
        if (q_chg) {
          if (!state_grew(X, Y)) exact_from = nrun;
          if (lane == 0) put_run(rp, rs, nrun, pos + j + q + 1, Y);
          ++nrun;
          quiet = 0;
        }
        X = Y;
        j += q + 1;
      }
      if (exact_from != 0xFFFFFFFFu) {   // exact from here: one op at a time, every change a run
        for (; j < lim; ++j) {
          FState X2;
          if (apply_sop(staged_sop(sh, j), X, X2)) {
            X = X2;
            if (lane == 0) put_run(rp, rs, nrun, pos + j + 1, X);
            ++nrun;
          }
        }
      }
      j = min(j, lim);
      if (lane == 0) {
        sh.n_burst += 1;
        sh.n_walk += j - p;
        publish_state(sh, X);
        sh.cur = j;
        sh.nrun = nrun;
        sh.exact_from = exact_from;
      }
    }
    __syncthreads();
    R = read_state(sh);
    cur = sh.cur;
    __syncthreads();   // state / cur are rewritten by the next burst
    prof_mark(sh, 4, tp);
  }
  G = gend;
}

__global__ __launch_bounds__(kFoldThreads) void k_fold_block(
    const u32* __restrict__ huge_list, u32 nhuge, const u32* __restrict__ seg_slot,
    const u64* __restrict__ hoff, const u32* __restrict__ seg_count,
    const u32* __restrict__ hval, const OpRec* __restrict__ hop, Rec* recs,
    u32* __restrict__ run_pos, RunState* __restrict__ run_st, u32* __restrict__ run_n,
    u8* __restrict__ seg_existed, u32* __restrict__ seg_exact_from,
    const u64* __restrict__ woff, const WinSum* __restrict__ sums, u32* __restrict__ win_run,
    GMax* __restrict__ win_g, u64* __restrict__ dbg, u32 h_begin) {
  __shared__ FoldShared sh;
  const u32 hs = h_begin + blockIdx.x;   // segments [h_begin, nhuge) of the list
  if (hs >= nhuge) return;
  // A hot segment's fold is one sequential chain of dependent rounds beside
  // the bandwidth-bound wave and thread folds: its waves take the SIMD's
  // issue priority.
  __builtin_amdgcn_s_setprio(3);
  const u64 t_begin = wall_clock64();
  u32 n_folded = 0;
  const u32 g = huge_list[hs];
  const u32 tid = threadIdx.x;
  Rec* r = &recs[seg_slot[g]];
  const u32 cnt = seg_count[g], last = cnt - 1;
  const u64 base = hoff[hs];
  const u32* __restrict__ sv = hval + base;
  const OpRec* __restrict__ so = hop + base;
  // this segment's runs: at most one per op plus the initial one
  u32* rp = run_pos + base + hs;
  RunState* rs = run_st + base + hs;

  FState R = load_state(load_rec(r));   // run state (see the module comment)
  GMax G{0, 0, 0};                      // merges absorbed so far
  if (tid == 0) {
    put_run(rp, rs, 0, 0, R);
    seg_existed[hs] = R.existed;
    sh.nrun = 1;
    sh.exact_from = 0xFFFFFFFFu;
    sh.n_burst = 0;
    sh.n_walk = 0;
    sh.n_iter = 0;
    sh.n_raise = 0;
    sh.profiling = dbg != nullptr;
    for (u32 k = 0; k < 6; ++k) sh.prof[k] = 0;
  }
  __syncthreads();
  u64 tp = dbg ? wall_clock64() : 0;
  const u32 nwin = (cnt + kFoldWin - 1) / kFoldWin;
  const WinSum* __restrict__ ws = sums + woff[hs];
  u32* __restrict__ wr = win_run + woff[hs];
  GMax* __restrict__ wg = win_g + woff[hs];
  u32 round = 0;
  // Windows are tested kSumChunk at a time: every thread tests one window's
  // summary (with the merge maxima of the windows before it in the chunk)
  // and a workgroup min picks the first window that may change the state.
  // The windows before it change nothing but G, so a long rate-limited
  // stretch costs one test per thread; only the found window is folded.
  u32 staged = 0xFFFFFFFFu;
  for (u32 w = 0; w < nwin;) {
    const u32 cb = w - w % kSumChunk;
    if (cb != staged) {
      __syncthreads();   // previous chunk's readers are done
      if (cb + tid < nwin) sh.sum[tid] = ws[cb + tid];
      staged = cb;
      __syncthreads();
    }
    const u32 lim = min(cb + kSumChunk, nwin);
    const u32 mine = cb + tid;
    const bool in = mine >= w && mine < lim;
    const bool exact = sh.exact_from != 0xFFFFFFFFu;
    block_prefix_gmax(in ? gmax_of(sh.sum[tid]) : GMax{0, 0, 0}, sh, tid);
    const GMax gs = gmax(G, (in && mine > w) ? sh.pinc[tid - 1] : GMax{0, 0, 0});
    bool quiet = false;
    if (in) {
      if (exact) {
        quiet = window_quiet(sh.sum[tid], R);
      } else {
        // merges that raise nothing and Takes denied at the extreme clock
        // (the strict test), or Takes denied for every state the window's
        // merges lead through (the absorbing bound)
        const FState Xs = join_state(R, gs);
        quiet = window_quiet(sh.sum[tid], Xs) ||
                window_absorbable(sh.sum[tid], Xs, join_state(R, gmax(G, sh.pinc[tid])));
      }
    }
    const u32 first = block_min((in && !quiet) ? mine : 0xFFFFFFFFu, sh, round, tid);
    const u32 stop = first == 0xFFFFFFFFu ? lim : first;
    const u32 run_now = sh.nrun - 1;   // run in effect at each such window's first op
    if (in && mine <= stop && mine < lim) {
      wr[mine] = run_now;
      wg[mine] = gs;
    }
    // G after the windows before `stop` (their merges are absorbed)
    if (stop > w) G = gmax(G, sh.pinc[stop - 1 - cb]);
    __syncthreads();   // wave_min, pinc and nrun are rewritten below
    if (first == 0xFFFFFFFFu) {
      w = lim;
      continue;
    }
    const u32 pos = first * kFoldWin;
    const u32 wlim = min(kFoldWin, cnt - pos);
    if (!exact && (sh.sum[first - cb].flags & kSumDirty)) {
      // A -0.0 replica: Go's merge is not the E max for it, so the segment is
      // exact from here on, starting with a run that holds the true state.
      // Nothing absorbed yet (G empty): the current run is already exact
      // (and may be the bucket's not-yet-created initial state, which a new
      // run could not express).
      const FState X = join_state(R, G);
      if (tid == 0) {
        if (!gmax_empty(G)) {
          put_run(rp, rs, sh.nrun, pos, X);
          sh.exact_from = sh.nrun;
          ++sh.nrun;
        } else {
          sh.exact_from = sh.nrun - 1;
        }
      }
      R = X;
      __syncthreads();
    }
    const GMax gw = gmax_of(sh.sum[first - cb]);
    prof_mark(sh, 0, tp);
    fold_stage(sv, so, pos, last, tid, sh);
    prof_mark(sh, 1, tp);
    ++n_folded;
    if (sh.exact_from == 0xFFFFFFFFu) {
      fold_window_absorb(pos, wlim, R, G, round, sh, rp, rs, tid);
    } else {
      fold_window(pos, wlim, R, round, sh, rp, rs, tid);   // R: the exact state after
      G = gmax(G, gw);
    }
    if (sh.profiling && tid == 0) tp = wall_clock64();
    w = first + 1;
  }
  prof_mark(sh, 0, tp);
  if (tid == 0) {
    store_state(r, join_state(R, sh.exact_from == 0xFFFFFFFFu ? G : GMax{0, 0, 0}));
    run_n[hs] = sh.nrun;
    seg_exact_from[hs] = sh.exact_from;
    if (dbg) {
      u64* d = dbg + (u64)hs * 16;
      d[0] = cnt; d[1] = nwin; d[2] = n_folded; d[3] = round; d[4] = sh.n_burst;
      d[5] = sh.n_walk; d[6] = sh.nrun; d[7] = wall_clock64() - t_begin;
      for (u32 k = 0; k < 5; ++k) d[8 + k] = sh.prof[k];
      d[13] = sh.n_iter;
      d[14] = sh.n_raise;
    }
  }
}

// Results of every op of the huge segments: op j of segment h saw the state
// of the last run of h starting at or before j, raised by the merges before
// j (G: the window's starting maximum k_fold_block recorded, then a prefix
// max over the window) unless that run is exact.  One block per fold
// window; each thread takes kFoldWin / kBlock consecutive ops, so the
// in-window prefix is a thread-local scan plus a workgroup scan of thread
// totals.  The fold recorded the run in effect at each window start, so the
// run search only spans the runs that begin inside the window (usually none).
constexpr u32 kOutPer = kFoldWin / kBlock;

template <u32 kOut>
__global__ __launch_bounds__(kBlock) void k_huge_outputs(
    const u32* __restrict__ huge_list, u32 nhuge, const u64* __restrict__ hoff,
    const u64* __restrict__ woff, const u32* __restrict__ seg_count,
    const u32* __restrict__ hval, const OpRec* __restrict__ hop,
    const u32* __restrict__ run_pos, const RunState* __restrict__ run_st,
    const u32* __restrict__ run_n, const u8* __restrict__ seg_existed,
    const u32* __restrict__ seg_exact_from, const u32* __restrict__ win_run,
    const GMax* __restrict__ win_g, OutView ow, u32 h_begin) {
  __shared__ GMax wtot[kBlock / 64];
  // segments [h_begin, nhuge) of the list: their windows follow
  // woff[h_begin]; a grid of a few blocks per CU walks them
  const u32 b_end = (u32)woff[nhuge];
  for (u32 b = (u32)woff[h_begin] + blockIdx.x; b < b_end; b += gridDim.x) {
  u32 h, w;
  huge_window(woff, nhuge, b, h, w);
  const u32 cnt = seg_count[huge_list[h]];
  const u64 base = hoff[h];
  const u32* rp = run_pos + base + h;
  const RunState* rs = run_st + base + h;
  const u32 nwin = (u32)(woff[h + 1] - woff[h]);
  const u32 k0 = win_run[woff[h] + w];
  const u32 k1 = w + 1 < nwin ? win_run[woff[h] + w + 1] : run_n[h] - 1;
  const bool existed0 = seg_existed[h];
  const u32 exact_from = seg_exact_from[h];
  const GMax g0 = win_g[woff[h] + w];
  const u32 p0 = w * kFoldWin, p1 = min(cnt, p0 + kFoldWin);
  const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const u32 j0 = p0 + tid * kOutPer;
  OpRec op[kOutPer];
  u32 val[kOutPer];
  GMax tot{0, 0, 0};
#pragma unroll
  for (u32 k = 0; k < kOutPer; ++k) {
    const u32 j = min(j0 + k, p1 - 1);
    op[k] = load_oprec(hop + base + j);
    val[k] = hval[base + j];
    if (j0 + k < p1) tot = gmax(tot, merge_contrib(op[k], val[k]));
  }
  // exclusive prefix of the thread totals over the workgroup
  GMax inc = tot;
#pragma unroll
  for (u32 d = 1; d < 64; d <<= 1) {
    const GMax y = shfl_up_gmax(inc, d);
    if (lane >= d) inc = gmax(inc, y);
  }
  if (lane == 63) wtot[wv] = inc;
  GMax exc = shfl_up_gmax(inc, 1);
  if (lane == 0) exc = GMax{0, 0, 0};
  __syncthreads();
  for (u32 y = 0; y < wv; ++y) exc = gmax(exc, wtot[y]);
  GMax gj = gmax(g0, exc);
  // Every op's run first (its loads), then the evaluations, then the
  // stores: with the stores last and specialised on the outputs present
  // (write_out_m), no run load waits for an earlier op's stores (gfx9's
  // in-order vmcnt).
  u32 lo[kOutPer];
  RunState q[kOutPer];
#pragma unroll
  for (u32 k = 0; k < kOutPer; ++k) {
    const u32 j = min(j0 + k, p1 - 1);
    u32 l = k0, hi = k1;   // last run in [k0, k1] with rp[run] <= j
    while (l < hi) {
      const u32 mid = (l + hi + 1) >> 1;
      if (rp[mid] <= j) l = mid; else hi = mid - 1;
    }
    lo[k] = l;
    q[k] = rs[l];
  }
  OpOut o[kOutPer];
  FState seen[kOutPer];
#pragma unroll
  for (u32 k = 0; k < kOutPer; ++k) {
    FState S;
    S.a = as_f64(q[k].a); S.t = as_f64(q[k].t); S.e = q[k].e; S.c = q[k].c;
    S.existed = lo[k] > 0 || existed0;
    if (lo[k] < exact_from) S = join_state(S, gj);
    const SOp sop = make_sop(op[k], val[k]);
    FState S2;
    eval_sop(sop, S, S2, o[k]);
    seen[k] = S2;   // the reply state: the bucket right after the op
    if (j0 + k < p1) gj = gmax(gj, merge_contrib(op[k], val[k]));
  }
  // (status, remaining and have were prefilled with the defaults, ordered())
#pragma unroll
  for (u32 k = 0; k < kOutPer; ++k)
    if (j0 + k < p1) write_out_nd<kOut>(ow, val[k] & kOpIdxMask, o[k], seen[k]);
  __syncthreads();   // the window's shared arrays are reused by the next
  }
}

// Segment classes for rocprim::select (segments are folded by k_fold_thread
// unless listed here).
struct LongSeg {
  const u32* cnt;
  __device__ bool operator()(u32 g) const { return cnt[g] > kLongSeg && cnt[g] <= kHugeSeg; }
};
struct HugeSeg {
  const u32* cnt;
  __device__ bool operator()(u32 g) const { return cnt[g] > kHugeSeg; }
};
// Long segments whose wave fold starts first (k_fold_wave takes the list in
// block order): a segment's fold is a sequential chain, so the longest ones
// must not start last.
constexpr u32 kBigLongSeg = 1024;
struct BigLongSeg {
  const u32* cnt;
  __device__ bool operator()(u32 g) const { return cnt[g] > kBigLongSeg; }
};

// Per-bucket segments of the sorted ops in three passes over the sorted slots
// (run_length_encode + exclusive_scan + two selects before: 0.31 ms and a
// host round trip on C3): k_seg_count counts the segment heads of every tile
// of kSegTile sorted ops, a scan of the tile counts places them, k_seg_write
// writes each head's slot and start, and k_seg_finish derives the counts and
// appends the long (ctr[6]) and huge (ctr[9]) segments; ctr[15] = segments.
// The long / huge lists come out in no particular order: every segment is
// folded on its own, so the order only schedules.
constexpr u32 kSegTile = 4096;
constexpr u32 kSegPer = kSegTile / 256;
constexpr u32 kCtrSegs = 15;

__device__ inline bool seg_head(const u32* __restrict__ key, u64 k) {
  return k == 0 || key[k] != key[k - 1];
}

__global__ __launch_bounds__(256) void k_seg_count(const u32* __restrict__ key, u32 n,
                                                   u32* __restrict__ tile_cnt, u32* ctr) {
  __shared__ u32 part[4];
  const u32 wave = threadIdx.x / 64, lane = threadIdx.x & 63;
  const u64 k0 = (u64)blockIdx.x * kSegTile;
  u32 c = 0;
#pragma unroll 4
  for (u32 r = 0; r < kSegPer; ++r) {
    const u64 k = k0 + r * 256 + threadIdx.x;
    c += (u32)__popcll(__ballot(k < n && seg_head(key, k)));
  }
  if (lane == 0) part[wave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    tile_cnt[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
    if (blockIdx.x == 0) { ctr[6] = 0; ctr[9] = 0; tile_cnt[gridDim.x] = 0; }
  }
}

__global__ __launch_bounds__(256) void k_seg_write(const u32* __restrict__ key, u32 n,
                                                   const u32* __restrict__ tile_base,
                                                   u32* __restrict__ uslot, u32* __restrict__ sstart) {
  __shared__ u32 wtot[kSegPer][4];
  const u32 wave = threadIdx.x / 64, lane = threadIdx.x & 63;
  const u64 k0 = (u64)blockIdx.x * kSegTile;
  bool hd[kSegPer];
  u32 rank[kSegPer];
#pragma unroll
  for (u32 r = 0; r < kSegPer; ++r) {
    const u64 k = k0 + r * 256 + threadIdx.x;
    hd[r] = k < n && seg_head(key, k);
    const u64 m = __ballot(hd[r]);
    rank[r] = (u32)__popcll(m & ((1ull << lane) - 1));
    if (lane == 0) wtot[r][wave] = (u32)__popcll(m);
  }
  __syncthreads();
  u32 base = tile_base[blockIdx.x];
#pragma unroll
  for (u32 r = 0; r < kSegPer; ++r) {
    u32 pre = 0;
    for (u32 w = 0; w < wave; ++w) pre += wtot[r][w];
    const u64 k = k0 + r * 256 + threadIdx.x;
    if (hd[r]) {
      const u32 j = base + pre + rank[r];
      uslot[j] = key[k];
      sstart[j] = (u32)k;
    }
    base += wtot[r][0] + wtot[r][1] + wtot[r][2] + wtot[r][3];
  }
}

// Each workgroup takes a contiguous range of the segments (their number is on
// the device only) and appends its long / huge ones through LDS lists, with
// one global atomic per list and flush: a wave-level atomic on ctr[6] per
// 64 segments serialised ~10^5 same-address atomics (0.41 ms on C3).
constexpr u32 kSegListCap = 1024;
__device__ inline void seg_flush(u32* lst, u32& cnt, u32* gcnt, u32* out, u32* base_sh) {
  __syncthreads();
  const u32 c = cnt;
  if (threadIdx.x == 0) *base_sh = c ? atomicAdd(gcnt, c) : 0u;
  __syncthreads();
  const u32 b = *base_sh;
  for (u32 k = threadIdx.x; k < c; k += 256) out[b + k] = lst[k];
  __syncthreads();
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_seg_finish(const u32* __restrict__ tile_base, u32 ntiles,
                                                    const u32* __restrict__ sstart, u32 n,
                                                    u32* __restrict__ scnt, u32* __restrict__ lng,
                                                    u32* __restrict__ huge, u32* ctr) {
  __shared__ u32 llist[kSegListCap], hlist[kSegListCap];
  __shared__ u32 lcnt, hcnt, base_sh;
  const u32 nseg = tile_base[ntiles];
  if (blockIdx.x == 0 && threadIdx.x == 0) ctr[kCtrSegs] = nseg;
  if (threadIdx.x == 0) { lcnt = 0; hcnt = 0; }
  const u32 per = (nseg + gridDim.x - 1) / gridDim.x;
  const u32 g0 = min(nseg, blockIdx.x * per), g1 = min(nseg, g0 + per);
  __syncthreads();
  for (u32 j0 = g0; j0 < g1; j0 += 256) {
    const u32 j = j0 + threadIdx.x;
    u32 c = 0;
    if (j < g1) {
      c = (j + 1 < nseg ? sstart[j + 1] : n) - sstart[j];
      scnt[j] = c;
    }
    const bool lo = c > kLongSeg && c <= kHugeSeg, hu = c > kHugeSeg;
    if (lo) llist[atomicAdd(&lcnt, 1u)] = j;
    if (hu) hlist[atomicAdd(&hcnt, 1u)] = j;
    __syncthreads();
    const u32 lc = lcnt, hc = hcnt;   // the same in every thread: read between barriers
    __syncthreads();
    // room for the next 256 in both lists
    if (lc > kSegListCap - 256) seg_flush(llist, lcnt, &ctr[6], lng, &base_sh);
    if (hc > kSegListCap - 256) seg_flush(hlist, hcnt, &ctr[9], huge, &base_sh);
  }
  seg_flush(llist, lcnt, &ctr[6], lng, &base_sh);
  seg_flush(hlist, hcnt, &ctr[9], huge, &base_sh);
}

// Sorted-slot segments from run-length output (counts -> starts is a scan).
__global__ void k_seg_mark(const u32* __restrict__ sorted_slot, u32 n, u32* head) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) head[i] = (i == 0 || sorted_slot[i] != sorted_slot[i - 1]) ? 1u : 0u;
}

// ------------------------------------------------------------ seed/dump --
// NewLocalRepo(clock, bs...): last entry of a name wins (map assignment).
__global__ void k_seed_pick(const u32* __restrict__ slot_of, u32 n, Table T) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicMax(&T.aux[slot_of[i]], i + 1);
}
__global__ void k_seed_apply(const u32* __restrict__ slot_of, u32 n, const phip_state* st,
                             Table T) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Rec* r = &T.recs[slot_of[i]];
  if (T.aux[slot_of[i]] != i + 1) return;
  phip_state s = st[i];
  r->added = enc_f64(s.added);
  r->taken = enc_f64(s.taken);
  r->elapsed = s.elapsed;
  r->created = s.created;
}
__global__ void k_seed_finish(const u32* __restrict__ slot_of, u32 n, Table T) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u32 s = slot_of[i];
  T.aux[s] = 0;
  T.recs[s].name0 = with_flags(T.recs[s].name0, kRecPublished);
}

// Occupied slots into list (list == nullptr: count only, into ctr[2]).
__global__ void k_dump_collect(const Rec* __restrict__ recs, u64 cap, u32* list, u32* ctr) {
  u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  bool occ = s < cap && recs[s].tag != 0;
  u32 p = wave_append(&ctr[2], occ);
  if (occ && list) list[p] = (u32)s;
}
__global__ void k_dump_gather(const u32* __restrict__ list, u32 n, const Rec* __restrict__ recs,
                              Rec* out) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = recs[list[i]];
}

// FNV-1a 64 of every name (phip_hash_names): the probe key and the shard map.
// Owner routing: the one exchange step of a sharded merge.
// owner(name) = ((fnv1a64(name) >> 32) * world) >> 32 (patrol_amd.shard).
//
// Layout: every workgroup owns a contiguous tile of `span` messages.  The
// count pass fills cells [owner][tile] with message and name-byte counts;
// their exclusive scans are each (owner, tile)'s base in the owner-major
// send buffers, so an owner's segment holds its messages tile after tile,
// each tile's in their original order (a stable partition).  The scatter
// walks its tile in steps of kRouteStep messages, all eight waves together:
// each wave ranks its own lanes per owner (ballots / DPP sums, a running
// place per owner in the wave's LDS row), one barrier makes every wave's
// totals visible, and a wave's messages for owner o follow those of the
// waves before it.  So each step writes one contiguous run per owner and
// column from the whole workgroup: a chip-wide handful of open output lines
// per owner, where per-wave tiles kept ~30k partly written lines per XCD and
// the L2 wrote them back in 32-byte pieces (2.4x the bytes, round 3).
//
// Sender-side combine (flag PHIP_ROUTE_COMBINE): a Zipf batch
// puts most messages on a few names, and in the clean domain (no incast, no
// -0.0: k_classify) merges commute, so a workgroup's messages for one hot
// name can leave as ONE message carrying the field-wise maxima (E order).
// The hot names are the most sampled names of a strided sample, counted by
// name hash (the buckets live on other ranks: there is no slot to count).
// A message whose three fields are all <= 0 (or NaN) is never combined: the
// maxima of such messages alone could be the all-zero state, which its owner
// would read as an incast request; every combined message thus has a field
// > 0.  A workgroup's combined messages follow its last wave's tile.
constexpr u32 kRouteMaxWorld = 64;
constexpr u32 kRouteBlock = 512;
constexpr u32 kRouteWaves = kRouteBlock / 64;
constexpr u16 kRouteHot = 0x8000;   // route code: combined into hot entry (low bits)
#ifndef PHIP_ROUTE_UNROLL
#define PHIP_ROUTE_UNROLL 1   // chunks per wave and scatter step: 1 1.81 ms, 2 2.01 ms (100M, 8 owners)
#endif
constexpr u32 kRU = PHIP_ROUTE_UNROLL;   // chunks of 64 messages per wave step
#ifndef PHIP_ROUTE_COUNT_UNROLL
#define PHIP_ROUTE_COUNT_UNROLL 2
#endif
constexpr u32 kRUC = PHIP_ROUTE_COUNT_UNROLL;   // k_route_count's (it holds less per message)
#ifndef PHIP_ROUTE_COUNT_CONTIG
#define PHIP_ROUTE_COUNT_CONTIG 0   // waves count contiguous eighths of the tile (else interleaved): 0.71 vs 0.70 ms
#endif
#ifndef PHIP_ROUTE_COUNT_PACKED
#define PHIP_ROUTE_COUNT_PACKED 0   // world <= 8: packed wave sums (else LDS atomics): 0.86 vs 0.70 ms
#endif
constexpr u32 kRouteStep = kRouteWaves * 64 * kRU;   // messages a scatter step takes

__device__ inline u32 owner_of_hash(u64 h, u32 world) {
  return (u32)(((h >> 32) * (u64)world) >> 32);
}

struct RouteHot {   // a hot name: FNV-1a, canonical words (short names only), owner
  u64 h, w0, w1;
  u32 owner, pad;
};

// Strided sample of the batch, counted by name hash (k_hot_sample's shape:
// LDS aggregation per workgroup, then the global count table).  cidx keeps
// one sampled message of each key, the name the directory takes.
template <class Src>
__global__ __launch_bounds__(256) void k_route_sample(Src src, u32 n, u32 stride, u32 nsample,
                                                     u32* __restrict__ ckeys, u32* __restrict__ ccnt,
                                                     u32* __restrict__ cidx) {
  constexpr u32 kPer = kHotSamplePerBlock / 256;
  constexpr u32 kL = 2 * kHotSamplePerBlock;
  __shared__ u32 lkey[kL], lcnt[kL], lidx[kL];
  for (u32 e = threadIdx.x; e < kL; e += 256) { lkey[e] = 0; lcnt[e] = 0; }
  __syncthreads();
  for (u32 r = 0; r < kPer; ++r) {
    const u32 j = blockIdx.x * kHotSamplePerBlock + r * 256 + threadIdx.x;
    const u64 i = (u64)j * stride;
    if (j >= nsample || i >= n) continue;
    u64 off; u32 len;
    src.template get<true>((u32)i, off, len);
    if (len > kShortName) continue;
    Name nm;
    load_name_wide<true>(src.blob, off, len, nm);
    const u32 key = (u32)(nm.h ^ (nm.h >> 32)) | 1u;
    u32 hs = (key * 2654435761u) & (kL - 1);
    for (;;) {   // at most kHotSamplePerBlock distinct keys in 2x as many entries
      const u32 old = atomicCAS(&lkey[hs], 0u, key);
      if (old == 0) lidx[hs] = (u32)i;
      if (old == 0 || old == key) { atomicAdd(&lcnt[hs], 1u); break; }
      hs = (hs + 1) & (kL - 1);
    }
  }
  __syncthreads();
  constexpr u32 mask = (1u << kHotCntBits) - 1;
  for (u32 e = threadIdx.x; e < kL; e += 256) {
    const u32 key = lkey[e];
    if (!key) continue;
    u32 hs = (key * 2654435761u) >> (32 - kHotCntBits);
    for (u32 k = 0; k <= mask; ++k) {
      const u32 old = atomicCAS(&ckeys[hs], 0u, key);
      if (old == 0) cidx[hs] = lidx[e];
      if (old == 0 || old == key) { atomicAdd(&ccnt[hs], lcnt[e]); break; }
      hs = (hs + 1) & mask;
    }
  }
}

// The sampled keys at or above k_hot_select's threshold, named by their
// sampled message.
template <class Src>
__global__ void k_route_dir_build(const u32* __restrict__ ckeys, const u32* __restrict__ ccnt,
                                  const u32* __restrict__ cidx, HotHdr* hdr, Src src, u32 world,
                                  RouteHot* __restrict__ dir) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (1u << kHotCntBits)) return;
  const u32 c = ccnt[e];
  if (!ckeys[e] || c < kHotMinCount || c < hdr->thresh) return;
  const u32 idx = atomicAdd(&hdr->n, 1u);
  if (idx >= kRouteHotMax) return;   // cannot happen: the threshold bounds the count
  u64 off; u32 len;
  src.get(cidx[e], off, len);
  Name nm;
  load_name_wide<false>(src.blob, off, len, nm);
  dir[idx] = RouteHot{nm.h, nm.w0, nm.w1, owner_of_hash(nm.h, world), 0};
}

// The hot directory in LDS, open-addressed by name hash at a quarter load:
// each slot holds the entry + 1 (low 16 bits) and 16 bits of the hash, so a
// probe is one LDS read and a name that is not hot (most of a batch) ends
// after ~1.2 slots (k_route_count probed a half-full table of bare indices,
// two LDS reads a step, the wave waiting for its longest chain).
constexpr u32 kRouteLds = 2048;
static_assert(kRouteLds >= 4 * kRouteHotMax && kRouteHotMax < 0xFFFF, "route directory load");
struct RouteLds {
  u32 slot[kRouteLds];   // (hash >> 48) << 16 | (entry + 1); 0 = empty
  u64 h[kRouteHotMax], w0[kRouteHotMax], w1[kRouteHotMax];
  u32 owner[kRouteHotMax];
};

__device__ inline u32 route_home(u64 h) { return (u32)(h ^ (h >> 29)) & (kRouteLds - 1); }

// Entries used by this launch: none without a directory or on a dirty batch.
__device__ inline u32 route_hot_n(const HotHdr* hot, const u32* ctr) {
  return (hot && ctr[kCtrDirty] == ~0u) ? min(hot->n, kRouteHotMax) : 0u;
}

__device__ inline void route_lds_load(RouteLds& L, const RouteHot* dir, u32 nh) {
  for (u32 j = threadIdx.x; j < kRouteLds; j += kRouteBlock) L.slot[j] = 0;
  __syncthreads();
  for (u32 j = threadIdx.x; j < nh; j += kRouteBlock) {
    const RouteHot d = dir[j];
    L.h[j] = d.h; L.w0[j] = d.w0; L.w1[j] = d.w1; L.owner[j] = d.owner;
    const u32 v = (u32)(d.h >> 48) << 16 | (j + 1);
    u32 hs = route_home(d.h);
    while (atomicCAS(&L.slot[hs], 0u, v) != 0) hs = (hs + 1) & (kRouteLds - 1);
  }
}

// What the scatter needs of the directory: the combined messages' names and
// owners (it reads the route codes the count pass wrote, not the hash table).
struct RouteNames {
  u64 w0[kRouteHotMax], w1[kRouteHotMax];
  u32 owner[kRouteHotMax];
};
__device__ inline void route_names_load(RouteNames& D, const RouteHot* dir, u32 nh) {
  for (u32 j = threadIdx.x; j < nh; j += kRouteBlock) {
    const RouteHot d = dir[j];
    D.w0[j] = d.w0; D.w1[j] = d.w1; D.owner[j] = d.owner;
  }
}

__device__ inline int route_hot_find(const RouteLds& L, const Name& nm) {
  const u32 tag = (u32)(nm.h >> 48);
  for (u32 hs = route_home(nm.h);; hs = (hs + 1) & (kRouteLds - 1)) {
    const u32 v = L.slot[hs];
    if (!v) return -1;
    const u32 e = v & 0xFFFFu;
    if ((v >> 16) == tag && L.h[e - 1] == nm.h && L.w0[e - 1] == nm.w0 && L.w1[e - 1] == nm.w1)
      return (int)e - 1;
  }
}

// Inclusive wave sum scan with DPP moves (VALU only; the row_shr /
// row_bcast pattern of wave_incl_max).  All 64 lanes must be active.
template <int Ctrl, int RowMask = 0xF>
__device__ inline u32 dpp_u32(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, Ctrl, RowMask, 0xF, true);
}
__device__ inline u32 wave_incl_sum(u32 x) {
  x += dpp_u32<0x111>(x);
  x += dpp_u32<0x112>(x);
  x += dpp_u32<0x114>(x);
  x += dpp_u32<0x118>(x);
  x += dpp_u32<0x142, 0xA>(x);
  x += dpp_u32<0x143, 0xC>(x);
  return x;
}

constexpr u32 kRoutePlain = 0, kRouteCombine = 1, kRouteRecount = 2;   // k_route_count modes

template <class Src>
__global__ __launch_bounds__(kRouteBlock) void k_route_count(
    Src src, const uint64_t* __restrict__ a, const uint64_t* __restrict__ t,
    const int64_t* __restrict__ e, u32 n, u32 span, u32 world, u32 ntile,
    const HotHdr* __restrict__ hot, const RouteHot* __restrict__ dir, u32* __restrict__ ctr,
    u16* __restrict__ code, u32* __restrict__ cnt, u32* __restrict__ bytes, u32 mode) {
  __shared__ RouteLds L;
  __shared__ u32 wc[kRouteWaves][kRouteMaxWorld], wb[kRouteWaves][kRouteMaxWorld];
  __shared__ u32 hit[kRouteHotMax];
  // mode kRouteCombine: combine hot names and classify the batch on the way
  // (the replica fields are read here: no k_route_classify pass); mode
  // kRouteRecount: count again without combining if that found a dirty
  // message (nothing to do on a clean batch); mode kRoutePlain: no combine.
  if (mode == kRouteRecount && ctr[kCtrDirty] == ~0u) return;
  const bool comb = mode == kRouteCombine;
  const u32 nh = comb ? route_hot_n(hot, ctr) : 0u;
  for (u32 j = threadIdx.x; j < kRouteWaves * kRouteMaxWorld; j += kRouteBlock) {
    (&wc[0][0])[j] = 0; (&wb[0][0])[j] = 0;
  }
  for (u32 j = threadIdx.x; j < kRouteHotMax; j += kRouteBlock) hit[j] = 0;
  route_lds_load(L, dir, nh);
  __syncthreads();
  const u32 wave = threadIdx.x / 64, lane = threadIdx.x & 63;
  const u32 tile = blockIdx.x;
  const u64 t0 = (u64)tile * span, t1 = min((u64)n, t0 + span);
  // kRUC chunks of 64 per wave step, their loads issued together (the loads
  // of one message depend on each other; those of different chunks do not);
  // the waves of the workgroup interleave over its tile
  u32 acc_c = 0, acc_b = 0;   // world <= 8: lane o's totals for owner o
#if PHIP_ROUTE_COUNT_CONTIG
  // every wave a contiguous eighth of the tile (the tile is whole steps)
  const u64 wspan = ((u64)span / kRouteWaves + 63) & ~63ull;
  const u64 w0b = t0 + wave * wspan, wend = min(t1, w0b + wspan);
  for (u64 b0 = w0b; b0 < wend; b0 += 64 * kRUC) {
#else
  const u64 wend = t1;
  for (u64 b0 = t0 + (u64)wave * 64 * kRUC; b0 < t1; b0 += (u64)kRouteWaves * 64 * kRUC) {
#endif
    u32 o[kRUC], len[kRUC];
    int hidx[kRUC];
    bool valid[kRUC];
    u64 off[kRUC], w0[kRUC], w1[kRUC], w2[kRUC];
    u64 ra[kRUC], rt[kRUC];
#pragma unroll
    for (u32 u = 0; u < kRUC; ++u) {
      const u64 i = b0 + u * 64 + lane;
      valid[u] = i < wend;   // (the last step of a wave's range may reach past it)
      const u32 ic = (u32)(valid[u] ? i : t0);
      src.template get<true>(ic, off[u], len[u]);
      if (comb) { ra[u] = ld<true>(a + ic); rt[u] = ld<true>(t + ic); }
    }
#pragma unroll
    for (u32 u = 0; u < kRUC; ++u) load_words3<true>(src.blob, off[u], len[u], w0[u], w1[u], w2[u]);
#pragma unroll
    for (u32 u = 0; u < kRUC; ++u) {
      const u64 i = b0 + u * 64 + lane;
      Name nm;
      if (len[u] <= kShortName) short_name(w0[u], w1[u], w2[u], off[u], len[u], nm);
      else load_name_wide<true>(src.blob, off[u], len[u], nm);
      o[u] = owner_of_hash(nm.h, world);
      hidx[u] = -1;
      bool ok = true;   // combinable: some field > 0 (elapsed read only when neither float is)
      if (comb) {
        const bool fpos = as_f64(ra[u]) > 0.0 || as_f64(rt[u]) > 0.0;
        bool dirty = ra[u] == kSign || rt[u] == kSign;
        if (valid[u] && !fpos) {
          const i64 ev = e[i];
          ok = ev > 0;
          dirty |= replica_dirty(ra[u], rt[u], ev);
        }
        note_dirty(valid[u] && dirty, (u32)i, ctr);
      }
      if (valid[u] && nh && ok && len[u] <= kShortName) hidx[u] = route_hot_find(L, nm);
      if (valid[u]) code[i] = hidx[u] >= 0 ? (u16)(kRouteHot | (u32)hidx[u]) : (u16)o[u];
      if (hidx[u] >= 0) hit[hidx[u]] = 1;
    }
    bool small = PHIP_ROUTE_COUNT_PACKED && world <= 8;
#pragma unroll
    for (u32 u = 0; u < kRUC; ++u) small &= !__ballot(valid[u] && hidx[u] < 0 && len[u] > 255);
    if (small) {
      // up to 8 owners: the chunks' counts and name bytes as packed wave
      // sums (8-bit counts, four owners a register; 16-bit byte sums, two a
      // register), lane o keeping owner o's totals: no LDS atomics (8
      // owners' same-address atomics were half the LDS cycles)
      u32 pc[2] = {0, 0}, pb[4] = {0, 0, 0, 0};
#pragma unroll
      for (u32 u = 0; u < kRUC; ++u) {
        const bool take = valid[u] && hidx[u] < 0;
#pragma unroll
        for (u32 r = 0; r < 2; ++r) pc[r] += (take && (o[u] >> 2) == r) ? 1u << (8 * (o[u] & 3)) : 0u;
#pragma unroll
        for (u32 r = 0; r < 4; ++r) pb[r] += (take && (o[u] >> 1) == r) ? len[u] << (16 * (o[u] & 1)) : 0u;
      }
      const u32 ol = lane & 7;
      u32 mc = 0, mb = 0;
#pragma unroll
      for (u32 r = 0; r < 2; ++r) {
        const u32 tot = (u32)__builtin_amdgcn_readlane((int)wave_incl_sum(pc[r]), 63);
        if ((ol >> 2) == r) mc = (tot >> (8 * (ol & 3))) & 0xFFu;
      }
#pragma unroll
      for (u32 r = 0; r < 4; ++r) {
        const u32 tot = (u32)__builtin_amdgcn_readlane((int)wave_incl_sum(pb[r]), 63);
        if ((ol >> 1) == r) mb = (tot >> (16 * (ol & 1))) & 0xFFFFu;
      }
      acc_c += mc;
      acc_b += mb;
    } else {
#pragma unroll
      for (u32 u = 0; u < kRUC; ++u) {   // the wave's own row: LDS atomics, no cross-lane loop
        if (valid[u] && hidx[u] < 0) {
          atomicAdd(&wc[wave][o[u]], 1u);
          atomicAdd(&wb[wave][o[u]], len[u]);
        }
      }
    }
  }
  if (lane < world && lane < 8) {   // the packed sums' lane totals
    wc[wave][lane] += acc_c;
    wb[wave][lane] += acc_b;
  }
  __syncthreads();
  if (wave == kRouteWaves - 1) {   // the workgroup's combined messages
    for (u32 j = lane; j < nh; j += 64) {
      if (!hit[j]) continue;
      atomicAdd(&wc[wave][L.owner[j]], 1u);
      atomicAdd(&wb[wave][L.owner[j]], (u32)(L.w0[j] & 0xFFu));
    }
  }
  __syncthreads();
  if (wave == 0) {   // the workgroup's cells
    for (u32 o = lane; o < world; o += 64) {
      u32 c = 0, b = 0;
#pragma unroll
      for (u32 w = 0; w < kRouteWaves; ++w) { c += wc[w][o]; b += wb[w][o]; }
      cnt[(u64)o * ntile + tile] = c;
      bytes[(u64)o * ntile + tile] = b;
    }
  }
}

// Inclusive wave scan (64 lanes).
__device__ inline u32 wave_incl_scan(u32 v) {
  const u32 lane = __lane_id();
#pragma unroll
  for (u32 d = 1; d < 64; d <<= 1) {
    const u32 o = __shfl_up(v, d);
    if (lane >= d) v += o;
  }
  return v;
}

// Place the lanes of `take` by owner `o`, in lane order, after each owner's
// running place run[o] / runb[o] (messages / name bytes), which advance.
__device__ inline void route_place(bool take, u32 o, u32 len, u32* run, u32* runb, u32& dst,
                                   u32& dby) {
  const u32 lane = __lane_id();
  u64 rest = __ballot(take);
  while (rest) {
    const u32 leader = __ffsll((long long)rest) - 1;
    const u32 ob = __shfl(o, leader);
    const bool mine = take && o == ob;
    const u64 m = __ballot(mine);
    const u32 sc = wave_incl_scan(mine ? len : 0u);
    const u32 base = run[ob], bbase = runb[ob];
    if (mine) {
      dst = base + __popcll(m & ((1ull << lane) - 1));
      dby = bbase + sc - len;
    }
    const u32 tot = __shfl(sc, 63);
    if (lane == leader) { run[ob] = base + __popcll(m); runb[ob] = bbase + tot; }
    rest &= ~m;
  }
}

// route_place for world <= 4 * NC (and 2 * NB == 4 * NC) and names of <= 255
// bytes: every owner's running count and byte total packed in fields of a
// few registers (8-bit counts, four owners a register; 16-bit byte sums, two
// a register: a wave's 64 names fit), one DPP scan per register instead of
// a ballot round and an LDS shuffle scan per owner present.  A lane's place
// is its owner's base plus its inclusive field minus itself; the owner's
// last lane advances the base.  Same result as route_place.
template <u32 NC, u32 NB>
__device__ inline void route_place_packed(bool take, u32 o, u32 len, u32* run, u32* runb, u32& dst,
                                          u32& dby) {
  u32 c[NC], b[NB];
#pragma unroll
  for (u32 r = 0; r < NC; ++r) c[r] = (take && (o >> 2) == r) ? 1u << (8 * (o & 3)) : 0u;
#pragma unroll
  for (u32 r = 0; r < NB; ++r) b[r] = (take && (o >> 1) == r) ? len << (16 * (o & 1)) : 0u;
#pragma unroll
  for (u32 r = 0; r < NC; ++r) c[r] = wave_incl_sum(c[r]);
#pragma unroll
  for (u32 r = 0; r < NB; ++r) b[r] = wave_incl_sum(b[r]);
  u32 ci = 0, ct = 0, bi = 0, bt = 0;
#pragma unroll
  for (u32 r = 0; r < NC; ++r) {
    const u32 tot = (u32)__builtin_amdgcn_readlane((int)c[r], 63);
    if ((o >> 2) == r) { ci = c[r]; ct = tot; }
  }
#pragma unroll
  for (u32 r = 0; r < NB; ++r) {
    const u32 tot = (u32)__builtin_amdgcn_readlane((int)b[r], 63);
    if ((o >> 1) == r) { bi = b[r]; bt = tot; }
  }
  ci = (ci >> (8 * (o & 3))) & 0xFFu;
  ct = (ct >> (8 * (o & 3))) & 0xFFu;
  bi = (bi >> (16 * (o & 1))) & 0xFFFFu;
  bt = (bt >> (16 * (o & 1))) & 0xFFFFu;
  if (take) {
    const u32 base = run[o], bbase = runb[o];
    dst = base + ci - 1;
    dby = bbase + bi - len;
    if (ci == ct) { run[o] = base + ct; runb[o] = bbase + bt; }
  }
}

// Short names (<= 16 bytes) reach out_names as whole dwords.  A chunk's
// names are staged by owner in the wave's LDS buffer at the byte alignment
// they have in out_names, and the dwords the chunk completes are stored with
// one dword store each (byte stores of 64 lanes scattered over 8 owners made
// the scatter L2-request bound).  Per owner (lane o < world):
//   t0   the first byte this call may store whole dwords from (bytes before
//        it in its first dword belong to another run: stored one by one)
//   pend the dword holding the run's end, not yet complete, returned to the
//        caller, who stores its bytes (route_flush_pend)
// k_route_scatter passes t0 = the run's start and flushes pend after every
// chunk: a run's first and last dwords are shared with the runs of other
// waves and steps.  A chunk with a longer name stores every name byte by
// byte instead.
constexpr u32 kStageWords = (64 * 16) / 4 + 2 * kRouteMaxWorld;

__device__ inline void route_store_bytes(u8* out, u32 from, u32 to, u32 word_start, u32 word) {
  for (u32 x = from; x < to; ++x) out[x] = (u8)(word >> (8 * (x - word_start)));
}

// Flush of the carried partial dwords (lane o: owner o's run ends at `be`).
__device__ inline void route_flush_pend(u8* out, u32 world, u32 be, u32 t0, u32 pend) {
  const u32 lane = __lane_id();
  if (lane < world && (be & 3)) {
    const u32 ws = be & ~3u;
    route_store_bytes(out, max(ws, t0), be, ws, pend);
  }
}

// The staged path for one chunk.  All 64 lanes active.  bo / be: lane o's
// owner run [bo, be) in out_names for this chunk; plain lanes carry a name of
// len <= 16 bytes (n0, n1) for owner o at byte dby.
__device__ inline void route_names_staged(u8* __restrict__ out, u32* stg, u32 world, bool plain, u32 o,
                                          u32 len, u32 dby, u64 n0, u64 n1, u32 bo, u32 be, u32 t0,
                                          u32& pend) {
  const u32 lane = __lane_id();
  const u32 so = be - bo, lead = bo & 3u;
  const u32 dcnt = (lane < world && so) ? (lead + so + 3) >> 2 : 0u;
  const u32 pstart = wave_incl_sum(dcnt) - dcnt;   // dwords, exclusive over owners
  if (dcnt && lead) stg[pstart] = pend;   // the run's first dword: bytes before bo
  const u32 oo = o & 63u;
  const u32 ps_o = (u32)__shfl((int)pstart, (int)oo), bo_o = (u32)__shfl((int)bo, (int)oo);
  if (plain) {
    u8* sb = reinterpret_cast<u8*>(stg);
    const u32 p = ps_o * 4 + (bo_o & 3u) + (dby - bo_o);
#pragma unroll
    for (u32 k = 0; k < 16; ++k)
      if (k < len) sb[p + k] = (u8)((k < 8 ? n0 >> (8 * k) : n1 >> (8 * (k - 8))) & 0xFFu);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // The stores: lanes in groups of G per owner (G = 64 / world rounded up to
  // a power of two), group g storing owner g's staged dwords G at a time, so
  // a lane's owner and run are fixed for the whole chunk (a search of the
  // owners per staged dword cost a third of the name stores).
  u32* outw = reinterpret_cast<u32*>(out);
  const u32 lg = 6u - (world <= 1 ? 0u : 32u - (u32)__builtin_clz(world - 1));
  const u32 og = min(lane >> lg, 63u), k0 = lane & ((1u << lg) - 1u);
  const u32 ps_g = (u32)__shfl((int)pstart, (int)og), dc_g = og < world ? (u32)__shfl((int)dcnt, (int)og) : 0u;
  const u32 bw = (u32)__shfl((int)bo, (int)og), ew = (u32)__shfl((int)be, (int)og);
  const u32 tw = (u32)__shfl((int)t0, (int)og);
  for (u32 k = k0; __ballot(k < dc_g); k += 1u << lg) {
    if (k < dc_g) {
      const u32 gdw = (bw >> 2) + k;
      const u32 word = stg[ps_g + k];
      if (4 * gdw + 4 <= ew) {   // complete
        if (4 * gdw >= tw) outw[gdw] = word;
        else route_store_bytes(out, tw, 4 * gdw + 4, 4 * gdw, word);   // the tile's first dword
      }
    }
  }
  // the carried dword: lane o keeps the one holding its run's end
  if (dcnt && (be & 3u)) pend = stg[pstart + dcnt - 1];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();   // stg is rewritten by the next chunk
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class Src>
__global__ __launch_bounds__(kRouteBlock) __attribute__((amdgpu_waves_per_eu(6, 6))) void k_route_scatter(
    Src src, const uint64_t* __restrict__ a, const uint64_t* __restrict__ t,
    const int64_t* __restrict__ e, u32 n, u32 span, u32 world, u32 ntile,
    const HotHdr* __restrict__ hot, const RouteHot* __restrict__ dir, const u32* __restrict__ ctr,
    const u16* __restrict__ code, const u32* __restrict__ cbase, const u32* __restrict__ bbase,
    u8* __restrict__ out_names, u32* __restrict__ out_lens, uint64_t* __restrict__ out_a,
    uint64_t* __restrict__ out_t, int64_t* __restrict__ out_e) {
  __shared__ RouteNames L;
  // per step (two parities, so one barrier a step suffices): each wave's own
  // running place per owner, and the workgroup's place before the step
  __shared__ u32 lrun[2][kRouteWaves][kRouteMaxWorld], lrunb[2][kRouteWaves][kRouteMaxWorld];
  __shared__ u32 run[2][kRouteMaxWorld], runb[2][kRouteMaxWorld];
  __shared__ u64 hmax[3][kRouteHotMax];
  __shared__ u32 hit[kRouteHotMax];
  __shared__ u32 nstage[kRouteWaves][kStageWords];
  const u32 nh = route_hot_n(hot, ctr);
  const u32 wave = threadIdx.x / 64, lane = threadIdx.x & 63;
  const u32 tile = blockIdx.x;
  for (u32 j = threadIdx.x; j < kRouteHotMax; j += kRouteBlock) {
    hit[j] = 0; hmax[0][j] = 0; hmax[1][j] = 0; hmax[2][j] = 0;
  }
  if (wave == 0)
    for (u32 o = lane; o < world; o += 64) {
      run[0][o] = cbase[(u64)o * ntile + tile];
      runb[0][o] = bbase[(u64)o * ntile + tile];
    }
  route_names_load(L, dir, nh);
  __syncthreads();
  const u64 t0 = (u64)tile * span, t1 = min((u64)n, t0 + span);
  u32* stg = nstage[wave];
  u32 p = 0;
  for (u64 s0 = t0; s0 < t1; s0 += kRouteStep, p ^= 1) {
    u32* lr = lrun[p][wave];
    u32* lrb = lrunb[p][wave];
    for (u32 o = lane; o < world; o += 64) { lr[o] = 0; lrb[o] = 0; }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    u32 c[kRU], len[kRU], dst[kRU], dby[kRU], bo_l[kRU], be_l[kRU];
    u64 off[kRU], va[kRU], vt[kRU], w0[kRU], w1[kRU], w2[kRU];
    i64 ve[kRU];
    bool valid[kRU];
    // (issuing the next step's loads before this step's barrier measured the
    // same, 1.70 ms per 100M: the step is not bound by these loads' latency)
#pragma unroll
    for (u32 u = 0; u < kRU; ++u) {   // every load unconditional (index clamped into the tile)
      const u64 i = s0 + (u64)(wave * kRU + u) * 64 + lane;
      valid[u] = i < t1;
      const u32 ic = (u32)(valid[u] ? i : t0);
      c[u] = code[ic];
      src.get(ic, off[u], len[u]);
      va[u] = a[ic]; vt[u] = t[ic]; ve[u] = e[ic];
    }
    // the name as three aligned words (all of a name of <= 16 bytes)
#pragma unroll
    for (u32 u = 0; u < kRU; ++u) load_words3<false>(src.blob, off[u], len[u], w0[u], w1[u], w2[u]);
    // 1. this wave's ranks per owner, chunk after chunk (lane o keeps owner
    //    o's byte run of every chunk for the name staging)
#pragma unroll
    for (u32 u = 0; u < kRU; ++u) {
      const bool comb = valid[u] && (c[u] & kRouteHot);
      const bool plain = valid[u] && !(c[u] & kRouteHot);
      if (comb) {   // clean domain: replica fields hold no -0.0
        const u32 j = c[u] & (kRouteHot - 1);
        const u64 ea = enc_replica_nz(va[u]), et = enc_replica_nz(vt[u]);
        const u64 ee = (u64)ve[u] ^ kSign;
        if (ea > hmax[0][j]) atomicMax(&hmax[0][j], ea);
        if (et > hmax[1][j]) atomicMax(&hmax[1][j], et);
        if (ee > hmax[2][j]) atomicMax(&hmax[2][j], ee);
        hit[j] = 1;
      }
      bo_l[u] = lane < world ? lrb[lane] : 0u;
      const u32 pl = plain ? len[u] : 0u;
      dst[u] = 0; dby[u] = 0;
      if (world <= 8 && !__ballot(pl > 255))
        route_place_packed<2, 4>(plain, c[u], pl, lr, lrb, dst[u], dby[u]);
      else if (world <= 16 && !__ballot(pl > 255))
        route_place_packed<4, 8>(plain, c[u], pl, lr, lrb, dst[u], dby[u]);
      else
        route_place(plain, c[u], pl, lr, lrb, dst[u], dby[u]);
      be_l[u] = lane < world ? lrb[lane] : 0u;
      c[u] = plain ? c[u] : 0xFFFFu;   // plain lanes keep their owner
    }
    __syncthreads();   // every wave's totals for this step are in LDS
    // 2. this wave's base per owner: the workgroup's place before the step
    //    plus the waves before this one (lane o: owner o); wave 0 also moves
    //    the workgroup's place past the step (the other parity)
    u32 pc = 0, pb = 0;
    if (lane < world) {
      pc = run[p][lane];
      pb = runb[p][lane];
      u32 tc = 0, tb = 0;
#pragma unroll
      for (u32 w = 0; w < kRouteWaves; ++w) {
        const u32 xc = lrun[p][w][lane], xb = lrunb[p][w][lane];
        if (w < wave) { pc += xc; pb += xb; }
        tc += xc; tb += xb;
      }
      if (wave == 0) {
        run[p ^ 1][lane] = run[p][lane] + tc;
        runb[p ^ 1][lane] = runb[p][lane] + tb;
      }
    }
    // 3. the columns and the names
#pragma unroll
    for (u32 u = 0; u < kRU; ++u) {
      const bool plain = c[u] != 0xFFFFu;
      const u32 oo = plain ? c[u] : 0u;
      const u32 d = (u32)__shfl((int)pc, (int)oo) + dst[u];
      const u32 db = (u32)__shfl((int)pb, (int)oo) + dby[u];
      if (plain) {
        out_lens[d] = len[u];
        out_a[d] = va[u];
        out_t[d] = vt[u];
        out_e[d] = ve[u];
      }
      // owner runs of this chunk [bo, be) (lane o), in the send buffer
      const u32 bo = pb + bo_l[u], be = pb + be_l[u];
      const u32 sh = (u32)(off[u] & 7) * 8;
      const u64 n0 = sh ? (w0[u] >> sh) | (w1[u] << (64 - sh)) : w0[u];
      const u64 n1 = sh ? (w1[u] >> sh) | (w2[u] << (64 - sh)) : w1[u];
      if (!__ballot(plain && len[u] > 16)) {
        // a run's first and last dwords are shared with the runs of other
        // waves or steps: stored byte by byte (t0 = bo, pend flushed)
        u32 pend = 0;
        route_names_staged(out_names, stg, world, plain, oo, plain ? len[u] : 0u, db, n0, n1, bo,
                           be, bo, pend);
        route_flush_pend(out_names, world, be, bo, pend);
      } else if (plain) {   // a longer name in the chunk: every name byte by byte
        if (len[u] <= 16) {
#pragma unroll
          for (u32 k = 0; k < 16; ++k)
            if (k < len[u]) out_names[db + k] = (u8)((k < 8 ? n0 >> (8 * k) : n1 >> (8 * (k - 8))) & 0xFFu);
        } else {
          for (u32 k = 0; k < len[u]; ++k) out_names[db + k] = src.blob[off[u] + k];
        }
      }
    }
  }
  __syncthreads();
  if (wave != kRouteWaves - 1 || !nh) return;
  // The workgroup's combined messages, in directory order, after its tile
  // (run[p] / runb[p]: its place after the last step).
  constexpr u64 kNaN = 0x7FF8000000000000ull;   // "no value": a merge never adopts NaN
  for (u32 j0 = 0; j0 < nh; j0 += 64) {
    const u32 j = j0 + lane;
    const bool on = j < nh && hit[j];
    const u32 o = on ? L.owner[j] : 0u;
    const u32 ln = on ? (u32)(L.w0[j] & 0xFFu) : 0u;
    u32 d = 0, db = 0;
    route_place(on, o, ln, run[p], runb[p], d, db);
    if (!on) continue;
    const u64 ma = hmax[0][j], mt = hmax[1][j];
    out_lens[d] = ln;
    out_a[d] = ma ? dec_f64(ma) : kNaN;
    out_t[d] = mt ? dec_f64(mt) : kNaN;
    out_e[d] = (i64)(hmax[2][j] ^ kSign);
    for (u32 k = 0; k < ln; ++k) {   // name byte k is canonical byte k + 2
      const u32 cb = k + 2;
      out_names[db + k] = (u8)((cb < 8 ? L.w0[j] >> (8 * cb) : L.w1[j] >> (8 * (cb - 8))) & 0xFFu);
    }
  }
}

// Per-owner totals from the scanned (exclusive) bases.
__global__ void k_route_totals(const u32* __restrict__ cnt, const u32* __restrict__ bytes,
                               const u32* __restrict__ cbase, const u32* __restrict__ bbase,
                               u32 nblk, u32 world, uint64_t* __restrict__ counts,
                               uint64_t* __restrict__ nbytes) {
  const u32 o = threadIdx.x;
  if (o >= world) return;
  const u64 last = (u64)world * nblk - 1;
  const u32 c0 = cbase[(u64)o * nblk], b0 = bbase[(u64)o * nblk];
  const u32 c1 = o + 1 < world ? cbase[(u64)(o + 1) * nblk] : cbase[last] + cnt[last];
  const u32 b1 = o + 1 < world ? bbase[(u64)(o + 1) * nblk] : bbase[last] + bytes[last];
  counts[o] = c1 - c0;
  nbytes[o] = b1 - b0;
}

// ------------------------------------------------------------ shard layer --
// Anti-entropy over simulated cluster replicas (BASELINE configs[4], SURVEY
// §8e).  Replica r of a GPU is three planes of B int64 for the same B buckets:
//   [r][0][i], [r][1][i]  E codes of added and taken (phip_device.hpp enc_f64)
//   [r][2][i]             elapsed ns
// The CvRDT join of any set of replicas is then a field-wise max, with Go's
// `if b.x < o.x { b.x = o.x }` rule (bucket.go:250-256) for NaN: a NaN replica
// value is never adopted (E'(NaN) = 0), a replica's own NaN sticks.  RCCL
// reduces signed int64, so the float planes cross the wire as E ^ 2^63.
//
// k_ae_local_max: m[f][i] = max over the R local replicas, in the signed
// form RCCL's all-reduce(MAX) takes; k_ae_apply: every local replica becomes
// max(own, m) after the all-reduce (one read per replica, and a write only
// where the join differs: a round that changed a few buckets rewrites those,
// not every replica plane).
__global__ __launch_bounds__(kBlock) void k_ae_local_max(const int64_t* __restrict__ rep, u32 R,
                                                         u64 B, int64_t* __restrict__ m) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  const u32 f = blockIdx.y;
  if (i >= B) return;
  const int64_t* p = rep + (u64)f * B + i;
  const u64 stride = 3 * B;
  if (f < 2) {
    u64 best = 0;   // E'(NaN) = 0 = E(-Inf): never wins
    for (u32 r = 0; r < R; ++r) {
      u64 e = (u64)__builtin_nontemporal_load(p + r * stride);
      if (e >= kNanBase) e = 0;
      best = e > best ? e : best;
    }
    m[(u64)f * B + i] = (int64_t)(best ^ kSign);
  } else {
    int64_t best = INT64_MIN;
    for (u32 r = 0; r < R; ++r) {
      const int64_t e = __builtin_nontemporal_load(p + r * stride);
      best = e > best ? e : best;
    }
    m[(u64)f * B + i] = best;
  }
}

__global__ __launch_bounds__(kBlock) void k_ae_apply(int64_t* __restrict__ rep, u32 R, u64 B,
                                                     const int64_t* __restrict__ m) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  const u32 f = blockIdx.y;
  if (i >= B) return;
  const int64_t mv = m[(u64)f * B + i];
  int64_t* p = rep + (u64)f * B + i;
  const u64 stride = 3 * B;
  for (u32 r = 0; r < R; ++r) {
    const int64_t own = p[r * stride];
    if (f < 2) {
      const u64 theirs = (u64)mv ^ kSign;   // already NaN-free
      if (theirs > (u64)own) p[r * stride] = (int64_t)theirs;
    } else {
      if (mv > own) p[r * stride] = mv;
    }
  }
}

// k_ae_join: the one-GPU join (phip_ae_join; the group's world-1 round).
// local_max and apply fused: each lane reads its two buckets' R values once,
// keeps them in registers (R <= kAeRegs; a larger R re-reads them), and
// writes back only those below the join, so a round costs one read of the planes plus
// the changed fields instead of two reads and the [3, B] join's round trip.
constexpr u32 kAeRegs = 16;
// One field of one bucket pair (buckets 2q, 2q+1) of every replica: 16-byte
// loads, the values kept in registers for the write-back test.
template <bool kPair>
__device__ inline void ae_join_pair(int64_t* __restrict__ p, u32 R, u64 stride, u64 bias,
                                    bool nanf) {
  u64x2 v[kAeRegs];
  u64x2 best = {0, 0};
  auto ld2 = [&](u32 r) -> u64x2 {
    // plain loads: the lines stay in L2 for the write-back of a changed
    // field (non-temporal loads: 1.10 vs 0.75-0.84 ms at 8 x 2^24)
    const int64_t* q = p + r * stride;
    if constexpr (kPair) return *reinterpret_cast<const u64x2*>(q);
    else return u64x2{(u64)*q, 0};
  };
  auto acc = [&](u64x2 e) {
    e ^= bias;
    u64x2 c = e;
    if (nanf) {
      c.x = c.x >= kNanBase ? 0 : c.x;
      c.y = c.y >= kNanBase ? 0 : c.y;
    }
    best.x = c.x > best.x ? c.x : best.x;
    best.y = c.y > best.y ? c.y : best.y;
    return e;
  };
#pragma unroll
  for (u32 r = 0; r < kAeRegs; ++r)
    if (r < R) v[r] = acc(ld2(r));
  for (u32 r = kAeRegs; r < R; ++r) (void)acc(ld2(r));
  auto put = [&](u32 r, u64x2 own) {
    int64_t* q = p + r * stride;
    if (best.x > own.x) q[0] = (int64_t)(best.x ^ bias);
    if (kPair && best.y > own.y) q[1] = (int64_t)(best.y ^ bias);
  };
#pragma unroll
  for (u32 r = 0; r < kAeRegs; ++r)
    if (r < R) put(r, v[r]);
  for (u32 r = kAeRegs; r < R; ++r) {
    const int64_t* q = p + r * stride;
    put(r, u64x2{(u64)q[0] ^ bias, kPair ? (u64)q[1] ^ bias : 0});
  }
}

__global__ __launch_bounds__(kBlock) void k_ae_join(int64_t* __restrict__ rep, u32 R, u64 B) {
  const u64 i = 2 * ((u64)blockIdx.x * kBlock + threadIdx.x);
  const u32 f = blockIdx.y;
  if (i >= B) return;
  // the join in the unsigned E order (float planes: NaN never wins; elapsed
  // is signed, so it is biased by 2^63 into the same order)
  const u64 bias = f < 2 ? 0 : kSign;
  int64_t* p = rep + (u64)f * B + i;
  // pairs need 16-byte alignment: rep aligned, B even (every plane start
  // aligned) and i even
  if (i + 1 < B && !(B & 1) && !(reinterpret_cast<uintptr_t>(rep) & 15)) {
    ae_join_pair<true>(p, R, 3 * B, bias, f < 2);
  } else {
    ae_join_pair<false>(p, R, 3 * B, bias, f < 2);
    if (i + 1 < B) ae_join_pair<false>(p + 1, R, 3 * B, bias, f < 2);
  }
}

__global__ void k_hash_names(NamesOffs src, u32 n, uint64_t* out) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u64 off; u32 len;
  src.get(i, off, len);
  Name nm;
  load_name_wide<false>(src.blob, off, len, nm);
  out[i] = nm.h;
}

// Egress batching (phip_export_datagrams; SURVEY §8f, repo.go:129-169): the
// current state of bucket names[i] as its MarshalBinary datagram
// (bucket.go:51-68: added, taken, elapsed big-endian, one length byte, the
// name) at out[25 * i + name_offs[i] - name_offs[0]].  An absent bucket
// gets zero bytes and found[i] = 0.
__global__ void k_export(NamesOffs src, u32 n, Table T, u8* __restrict__ out,
                         u8* __restrict__ found) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u64 off; u32 len;
  src.get(i, off, len);
  Name nm;
  load_name_wide<false>(src.blob, off, len, nm);
  u32 s;
  Rec r;
  const bool hit = probe(T, nm, src.blob, &s, &r) == kFound;
  u64 w[3] = {0, 0, 0};
  if (hit) {
    r = load_rec(&T.recs[s]);   // probe's copy may be the 48-byte view
    w[0] = dec_f64(r.added);
    w[1] = dec_f64(r.taken);
    w[2] = (u64)r.elapsed;
  }
  u8* d = out + (u64)PHIP_BUCKET_FIXED_SIZE * i + (off - src.offs[0]);
  for (u32 k = 0; k < 24; ++k) d[k] = hit ? (u8)(w[k >> 3] >> (56 - 8 * (k & 7))) : 0;
  d[24] = hit ? (u8)len : 0;
  for (u32 k = 0; k < len; ++k) d[PHIP_BUCKET_FIXED_SIZE + k] = hit ? src.blob[off + k] : 0;
  found[i] = hit;
}

// Single lookup (phip_get).
__global__ void k_get_one(const u8* name, u32 len, Table T, Rec* out, int* found) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Name nm;
  load_name_wide<false>(name, 0, len, nm);
  u32 s;
  Rec r;
  int pr = probe(T, nm, name, &s, &r);
  *found = pr == kFound;
  if (pr == kFound) *out = load_rec(&T.recs[s]);   // probe's copy may be the 48-byte view
}

}  // namespace phip
