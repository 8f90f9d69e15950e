// libpatrolhip host orchestration: the C ABI of include/patrolhip.h.
//
// Pipelines:
//   fast receive  classify -> hot directory -> k_receive_fast
//                 -> [insert rounds -> k_receive_list(miss list)]
//   ordered       resolve -> [insert rounds -> resolve(miss)] -> sort(slot, seq)
//                 (ops packed to 32-byte records, kind in the sort value)
//                 -> run-length segments
//                 -> k_fold_thread / k_fold_wave / k_fold_block (stream2)
// Everything runs on the handle's own HIP stream; host synchronisation only
// reads back small counters (miss count, segment count) between stages.
#include <sys/random.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "patrolhip.h"
#include "phip_kernels.hpp"
#include "phip_host.hpp"

using namespace phip;

namespace {

// The ordered path's (slot, seq) sort: slots have L <= 31 bits (25 for the
// C2/C3 tables), so 8-bit places spend a whole fourth pass on one bit; wider
// places (PHIP_SORT_BITS) cover 25 bits in three.
#ifndef PHIP_SORT_BITS
#define PHIP_SORT_BITS 9
#endif
#ifndef PHIP_SORT_BLOCK
#define PHIP_SORT_BLOCK 1024
#endif
#ifndef PHIP_SORT_ITEMS
#define PHIP_SORT_ITEMS 8
#endif
using SlotSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<
        rocprim::kernel_config<PHIP_SORT_BLOCK, PHIP_SORT_ITEMS>,
        rocprim::kernel_config<PHIP_SORT_BLOCK, PHIP_SORT_ITEMS>, PHIP_SORT_BITS,
        rocprim::block_radix_rank_algorithm::match>>;

enum BufId {
  B_NAMES, B_OFFS, B_A, B_T, B_E, B_KIND, B_NOW, B_FREQ, B_PER, B_COUNT,
  B_STATUS, B_REM, B_HAVE, B_REPLY,
  B_BYTES, B_DOFFS, B_NOFF, B_NLEN, B_DA, B_DT, B_DE,
  B_MISS, B_MISS2, B_RETRY, B_CSLOT, B_CMSG,
  B_SLOT, B_IDX, B_SSLOT, B_SIDX, B_USLOT, B_SCNT, B_SSTART, B_LONG, B_HUGE, B_TEMP, B_DUMP,
  B_OPS, B_HOFF, B_HOP, B_HVAL, B_RPOS, B_RST, B_RUNN, B_SEGEX, B_WOFF, B_SUMS, B_WRUN,
  B_WING, B_SEGXF, B_FOLDDBG, B_SMALL, B_HUGE2, B_LONG2,
  B_STATES, B_NAME1, B_HOT, B_ROUTE, B_EXPORT, B_MSHARD, B_MSCNT, B_FSCNT, B_DEDUP, B_DSET, B_TSTATS, B_SEGT, B_RHOT,
  B_DLIST, B_DTAB, B_DMARK, B_SMAP, B_SOFF, B_SLEN, B_SA, B_ST, B_SE, B_SSTAT, B_SREP,
  B_COUNT_
};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

struct Timing {
  const char* name;
  hipEvent_t a, b;
};

}  // namespace

struct phip_handle {
  int device = 0;
  int ncu = 256;             // compute units (persistent grid size)
  u32 ndef = 0;   // the last fast pass's ordered sub-batch (dirty buckets), entries
  // Dirty-bucket isolation (phip_kernels.hpp "Dirty buckets"): always
  // (PHIP_CFG_ISOLATE), or while iso_left > 0 -- kIsoKeep fast passes after
  // the last one that met a dirty message.  coll_iso: whether the pass whose
  // counters were collected last ran with it (its nested pass must too).
  bool iso_always = false;
  u32 iso_left = 0;
  bool coll_iso = false;
  uint64_t stats[4] = {0, 0, 0, 0};   // last fast batch: hot entries, hot hits, misses,
                                      // messages it sent through the ordered path
  hipStream_t stream = nullptr;      // the stream every call runs on (own_stream or the caller's)
  hipStream_t own_stream = nullptr;  // created by phip_open
  hipStream_t stream2 = nullptr;   // second stream: the hot-bucket fold overlaps the others
  hipStream_t stream3 = nullptr;   // third stream: the other huge segments beside the largest
  // fourth stream: the thread folds beside the wave folds, created by the
  // first ordered batch that folds (a stream created at open would shift how
  // a process's later streams, e.g. a group's pack and exchange streams, map
  // onto its hardware queues: the bench's c4 leg took 8.3 instead of 6.9 ms)
  hipStream_t stream4 = nullptr;
  hipEvent_t ev_t4a = nullptr, ev_t4b = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_fork3 = nullptr, ev_join3 = nullptr;
  hipEvent_t ev_gather = nullptr, ev_gather3 = nullptr;   // huge-segment gathers done
  hipEvent_t ev_pack = nullptr;   // ordered path: op records packed (stream2)
  std::mutex mu;
  std::string err;
  u32 L = 0;
  u64 cap = 0;
  u64 max_load = 0;
  u32 load_pct = 90;
  bool grow = true;          // !PHIP_CFG_NO_GROW
  bool small = true;         // !PHIP_CFG_NO_SMALL
  u64 grows = 0;             // table rehashes so far
  u64 long_need = 0;         // arena bytes the last reserve() counted
  Rec* recs = nullptr;
  u32* aux = nullptr;
  u8* arena = nullptr;
  u64 arena_cap = 0;
  u64* arena_cursor = nullptr;
  u32* ctr = nullptr;        // device counters: kCtrWords general, then two fast-pass sets (fctr)
  u32* ctr_host = nullptr;   // pinned mirror
  u32* ctr_map = nullptr;    // ctr_host as the device sees it (k_shard_scan stores there)
  u32 fpar = 0;              // parity of the last fast batch (its shard counters in B_FSCNT)
  u64 nfast = 0;             // fast passes begun (a queued front is redone after a nested one)
  u64 n_buckets = 0;
  u64 tag_mask = ~0ull;
  u64 seed = 0;              // placement seed (Table::home, seeded_mix)
  DevBuf buf[B_COUNT_];
  bool timing = false;
  bool timing_accumulate = false;   // phip_set_timing(h, 2): keep every call's timings
  std::vector<Timing> timings;
  std::vector<Timing> event_pool;
  size_t pool_used = 0;
  u8* small_pin = nullptr;   // pinned staging of small ordered batches (both ways)
  size_t small_pin_cap = 0;
  // PHIP_RECV_ASYNC: a decoded batch whose fast pass is queued; its counters
  // are read, and its misses / dirty buckets finished, at the handle's next
  // call (or phip_flush)
  struct Pending {
    bool active = false;
    NamesOffs src{};
    const uint64_t *a = nullptr, *t = nullptr;
    const int64_t* e = nullptr;
    u32 n = 0;
    u32 par = 0;
    bool iso = false;
    i64 now = 0;
    OutView ow{};
  } pend;
  hipEvent_t ev_ctr = nullptr;   // a queued batch's counters reached ctr_host
  int deferred_rc = 0;   // a queued batch's error met by a call that returns no status
};

namespace {

int set_err(phip_handle* h, int code, const char* fmt, ...) {
  char tmp[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(tmp, sizeof tmp, fmt, ap);
  va_end(ap);
  if (h) h->err = tmp;
  return code;
}

#define HIPCHK(h, x)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      return set_err((h), PHIP_ERR_HIP, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), \
                     __FILE__, __LINE__);                                                 \
  } while (0)

template <class T>
int ensure(phip_handle* h, BufId id, size_t count, T** out) {
  size_t bytes = std::max<size_t>(count * sizeof(T), 64) + 64;  // +64: 8-byte over-read slack
  DevBuf& b = h->buf[id];
  if (b.cap < bytes) {
    size_t want = std::max(bytes, b.cap * 3 / 2);
    if (b.p) HIPCHK(h, hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    HIPCHK(h, hipMalloc(&b.p, want));
    b.cap = want;
  }
  *out = (T*)b.p;
  return PHIP_OK;
}

inline Table table(phip_handle* h) {
  Table t;
  t.recs = h->recs;
  t.aux = h->aux;
  t.arena = h->arena;
  t.L = h->L;
  t.tag_mask = h->tag_mask;
  t.seed = h->seed;
  return t;
}

inline unsigned grid_for(u64 n, unsigned block = kBlock) {
  return (unsigned)std::max<u64>(1, (n + block - 1) / block);
}

// Event-timed launch helper (the pool entry is held by index: a nested
// Launch may grow the pool).
struct Launch {
  phip_handle* h;
  const char* name;
  size_t idx = ~size_t(0);
  hipStream_t s;
  Launch(phip_handle* h_, const char* n, hipStream_t st = nullptr)
      : h(h_), name(n), s(st ? st : h_->stream) {
    if (!h->timing) return;
    if (h->pool_used == h->event_pool.size()) {
      Timing tm{n, nullptr, nullptr};
      if (hipEventCreate(&tm.a) != hipSuccess) return;
      if (hipEventCreate(&tm.b) != hipSuccess) {
        (void)hipEventDestroy(tm.a);
        return;
      }
      h->event_pool.push_back(tm);
    }
    idx = h->pool_used++;
    h->event_pool[idx].name = n;
    if (hipEventRecord(h->event_pool[idx].a, s) != hipSuccess) idx = ~size_t(0);
  }
  ~Launch() {
    if (idx < h->event_pool.size()) {
      Timing& t = h->event_pool[idx];
      if (hipEventRecord(t.b, s) == hipSuccess) h->timings.push_back(t);
    }
  }
};

// Device counters: ctr[0..15] u32 per batch (k_batch_reset), ctr[16..17] one
// u64 scratch sum (k_list_long_bytes).
constexpr u32 kCtrWords = 32;
constexpr u32 kCtrLongBytes = 16;

int read_ctr(phip_handle* h) {
  HIPCHK(h, hipMemcpyAsync(h->ctr_host, h->ctr, kCtrWords * sizeof(u32), hipMemcpyDeviceToHost,
                           h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int reset_ctr(phip_handle* h) {
  // ctr[5] = first short datagram, ctr[kCtrDirty] = first dirty message
  // (phip_kernels.hpp): both start at "none", the rest at zero.
  static_assert(kCtrDirty == 12, "k_batch_reset");
  k_batch_reset<<<1, kShards, 0, h->stream>>>(h->ctr, nullptr);
  HIPCHK(h, hipGetLastError());
  return PHIP_OK;
}

int check_flags(phip_handle* h) {
  if (h->ctr_host[kCtrBadName])
    return set_err(h, PHIP_ERR_INVALID, "malformed name offsets (names_len check): nothing applied");
  if (h->ctr_host[8]) return set_err(h, PHIP_ERR_FULL, "hash table full (probe wrapped)");
  if (h->ctr_host[7]) return set_err(h, PHIP_ERR_ARENA, "long-name arena exhausted");
  return PHIP_OK;
}

// Every entry point binds the handle's device first: Go goroutines migrate
// across OS threads, and the HIP current device is per thread.
int finish_pending(phip_handle* h, bool* worked = nullptr);
int after_error(phip_handle* h, int rc);

// (finish_queued: a batch PHIP_RECV_ASYNC queued is finished first, and its
// error is this call's)
int begin_call(phip_handle* h, bool finish_queued = true) {
  if (h->deferred_rc) {   // (phip_len / phip_capacity finished a queued batch that failed)
    const int rc = h->deferred_rc;
    h->deferred_rc = 0;
    return rc;
  }
  h->err.clear();
  if (h->timing && !h->timing_accumulate) {
    h->timings.clear();
    h->pool_used = 0;
  }
  HIPCHK(h, hipSetDevice(h->device));
  if (finish_queued && h->pend.active) {
    int rc = finish_pending(h);
    if (rc) return after_error(h, rc);
  }
  return PHIP_OK;
}

// Copy a host array into a device staging buffer (or pass device pointers).
template <class T>
int stage(phip_handle* h, BufId id, const T* src, size_t count, bool dev, const T** out) {
  if (!src) { *out = nullptr; return PHIP_OK; }
  if (dev) { *out = src; return PHIP_OK; }
  T* d;
  int rc = ensure(h, id, count, &d);
  if (rc) return rc;
  if (count) HIPCHK(h, hipMemcpyAsync(d, src, count * sizeof(T), hipMemcpyHostToDevice, h->stream));
  *out = d;
  return PHIP_OK;
}

template <class T>
int out_buf(phip_handle* h, BufId id, T* user, size_t count, bool dev, T** out) {
  if (!user) { *out = nullptr; return PHIP_OK; }
  if (dev) { *out = user; return PHIP_OK; }
  return ensure(h, id, count, out);
}

template <class T>
int copy_back(phip_handle* h, T* user, const T* dev_buf, size_t count, bool dev) {
  if (!user || dev || !count) return PHIP_OK;
  HIPCHK(h, hipMemcpyAsync(user, dev_buf, count * sizeof(T), hipMemcpyDeviceToHost, h->stream));
  return PHIP_OK;
}

// ----------------------------------------------------------- inserts -----
inline u64 load_limit(u64 cap, u32 pct) { return cap * pct / 100; }

// Rehash the table into 2^newL slots (k_rehash).  Both tables are resident
// while records move; the old one is freed after.
int grow_table(phip_handle* h, u32 newL) {
  const u64 ncap = 1ull << newL;
  Rec* nrecs = nullptr;
  u32* naux = nullptr;
  if (hipMalloc(&nrecs, ncap * sizeof(Rec)) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(h, PHIP_ERR_FULL, "table growth to 2^%u slots: device memory", newL);
  }
  if (hipMalloc(&naux, ncap * sizeof(u32)) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(nrecs);
    return set_err(h, PHIP_ERR_FULL, "table growth to 2^%u slots: device memory", newL);
  }
  // from here on an error frees the new table (the old one stays live)
  auto drop_new = [&](int rc) {
    (void)hipStreamSynchronize(h->stream);
    (void)hipFree(nrecs);
    (void)hipFree(naux);
    return rc;
  };
  if (hipMemsetAsync(nrecs, 0, ncap * sizeof(Rec), h->stream) != hipSuccess ||
      hipMemsetAsync(naux, 0, ncap * sizeof(u32), h->stream) != hipSuccess ||
      hipMemsetAsync(h->ctr + 8, 0, sizeof(u32), h->stream) != hipSuccess)
    return drop_new(set_err(h, PHIP_ERR_HIP, "table growth: clearing the new table failed"));
  Table nt = table(h);
  nt.recs = nrecs;
  nt.aux = naux;
  nt.L = newL;
  {
    Launch l(h, "k_rehash");
    k_rehash<<<grid_for(h->cap), kBlock, 0, h->stream>>>(h->recs, h->aux, h->cap, nt, h->ctr);
  }
  if (hipGetLastError() != hipSuccess)
    return drop_new(set_err(h, PHIP_ERR_HIP, "k_rehash launch failed"));
  int rc;
  if ((rc = read_ctr(h))) return drop_new(rc);   // synchronises: the old table is no longer read
  if (h->ctr_host[8]) return drop_new(set_err(h, PHIP_ERR_INVALID, "internal: rehash probe wrapped"));
  HIPCHK(h, hipFree(h->recs));
  HIPCHK(h, hipFree(h->aux));
  h->recs = nrecs;
  h->aux = naux;
  h->L = newL;
  h->cap = ncap;
  h->max_load = load_limit(ncap, h->load_pct);
  ++h->grows;
  return PHIP_OK;
}

int grow_arena(phip_handle* h, u64 used, u64 want) {
  u64 ncap = std::max<u64>(h->arena_cap * 2, want);
  u8* na = nullptr;
  if (hipMalloc(&na, ncap + 64) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(h, PHIP_ERR_ARENA, "arena growth to %llu bytes: device memory",
                   (unsigned long long)ncap);
  }
  if (used) HIPCHK(h, hipMemcpyAsync(na, h->arena, used, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipFree(h->arena));
  h->arena = na;
  h->arena_cap = ncap;
  return PHIP_OK;
}

// Room for `bound` more buckets and the long names of list[0..nlist), before
// any of them is claimed: grow the table / arena, or refuse with nothing
// claimed.  *grew is set when the table was rehashed (slot numbers changed).
template <class Src>
int reserve(phip_handle* h, Src src, const u32* list, u32 nlist, u64 bound, bool* grew) {
  u64* lb = (u64*)(h->ctr + kCtrLongBytes);
  HIPCHK(h, hipMemsetAsync(lb, 0, sizeof(u64), h->stream));
  k_list_long_bytes<Src><<<grid_for(nlist), kBlock, 0, h->stream>>>(src, nlist, list, lb);
  HIPCHK(h, hipGetLastError());
  u64 used = 0;
  HIPCHK(h, hipMemcpyAsync(&used, h->arena_cursor, sizeof(u64), hipMemcpyDeviceToHost, h->stream));
  int rc;
  if ((rc = read_ctr(h))) return rc;
  u64 need;
  std::memcpy(&need, h->ctr_host + kCtrLongBytes, sizeof need);
  h->long_need = need;
  if (used + need > h->arena_cap) {
    if (!h->grow)
      return set_err(h, PHIP_ERR_ARENA, "long-name arena: %llu of %llu bytes used, %llu more needed",
                     (unsigned long long)used, (unsigned long long)h->arena_cap,
                     (unsigned long long)need);
    if ((rc = grow_arena(h, used, used + need))) return rc;
  }
  if (h->n_buckets + bound > h->max_load) {
    u32 L = h->L;
    while (L < 31 && h->n_buckets + bound > load_limit(1ull << L, h->load_pct)) ++L;
    if (!h->grow || h->n_buckets + bound > load_limit(1ull << L, h->load_pct))
      return set_err(h, PHIP_ERR_FULL,
                     "table load limit: %llu buckets + up to %llu new > %llu allowed in 2^%u slots",
                     (unsigned long long)h->n_buckets, (unsigned long long)bound,
                     (unsigned long long)(h->grow ? load_limit(1ull << L, h->load_pct) : h->max_load),
                     h->grow ? L : h->L);
    if ((rc = grow_table(h, L))) return rc;
    *grew = true;
  }
  return PHIP_OK;
}

// Insert every name of `list` (all known to be absent) into the table, after
// reserve() made room for all of them.  Claimed slots are accumulated in
// B_CSLOT/B_CMSG; *n_claimed returns their count (callers clear the NEW flag
// once done).  Every claimed slot is published before an error returns, so a
// failing round leaves no claimed-but-unnamed slot behind.
template <class Src>
int dedupe_names(phip_handle* h, Src src, const u32* list, u32 n, u32** out, u32* nout);

// `distinct`: the list holds each name once (a k_dedupe output); otherwise a
// name may be listed many times (a fast batch's misses), and a list whose
// length alone would pass the load limit is bounded by its distinct names
// first, so that one new hot name does not grow (or, without growth, fill)
// the table for the thousands of messages naming it.
template <class Src>
int insert_names(phip_handle* h, Src src, u32* list, u32 nlist, const int64_t* now_arr, i64 now0,
                 u32* n_claimed, bool* grew = nullptr, bool distinct = false) {
  u32 *cslot, *cmsg, *retry, *cur = list;
  int rc;
  *n_claimed = 0;
  bool g = false;
  u64 bound = nlist;
  // the names whose long-name arena bytes reserve() counts: the list, or its
  // distinct names once they are known (one new long hot name listed by
  // 65535 misses needs its bytes once)
  const u32* blist = list;
  u32 nb = nlist;
  if (!distinct && nlist > 1 && h->n_buckets + nlist > h->max_load) {
    u32 *dd, nd = 0;
    if ((rc = dedupe_names(h, src, list, nlist, &dd, &nd))) return rc;
    // names that share a 64-bit tag count once there: with full tags that is
    // a birthday rarity; narrowed test tags keep the list's length (and the
    // bytes of every listed name)
    if (h->tag_mask == ~0ull) {
      bound = nd;
      blist = dd;
      nb = nd;
    }
  }
  if ((rc = reserve(h, src, blist, nb, bound, &g))) return rc;
  if (grew) *grew = g;
  if ((rc = ensure(h, B_CSLOT, nlist, &cslot)) || (rc = ensure(h, B_CMSG, nlist, &cmsg)) ||
      (rc = ensure(h, B_RETRY, nlist, &retry)))
    return rc;
  u32 total = 0, ncur = nlist;
  // ctr[3] counts this call's claims (B_CSLOT/B_CMSG positions): a batch can
  // run the pipeline twice (finish_many_misses, resolve_all), so it starts
  // from zero here, not at the batch's reset_ctr.
  HIPCHK(h, hipMemsetAsync(h->ctr + 3, 0, sizeof(u32), h->stream));
  // Swap buffers between rounds: round k reads `cur`, writes retries to `nxt`.
  u32* nxt = retry;
  u32* spare = nullptr;
  if ((rc = ensure(h, B_MISS2, nlist, &spare))) return rc;
  // Every round claims at least one slot while names are pending (a pending
  // name met a slot claimed in that same round), so this terminates; with a
  // 64-bit tag a second round is already rare.
  while (ncur > 0) {
    // ctr[3] is the running claimed count (cumulative), ctr[4] the retry count.
    HIPCHK(h, hipMemsetAsync(h->ctr + 4, 0, sizeof(u32), h->stream));
    {
      Launch l(h, "k_claim");
      k_claim<Src><<<grid_for(ncur), kBlock, 0, h->stream>>>(src, ncur, cur, table(h), cslot, cmsg,
                                                              nxt, h->ctr);
    }
    HIPCHK(h, hipGetLastError());
    if ((rc = read_ctr(h))) return rc;
    u32 claimed_total = h->ctr_host[3];
    u32 fresh = claimed_total - total;
    // The round's claims are published before any error is reported.
    if (fresh) {
      Launch l(h, "k_publish");
      k_publish<Src><<<grid_for(fresh), kBlock, 0, h->stream>>>(
          src, total, fresh, cslot, cmsg, table(h), h->arena, h->arena_cap, h->arena_cursor, now_arr,
          now0, h->ctr);
    }
    HIPCHK(h, hipGetLastError());
    h->n_buckets += fresh;
    total = claimed_total;
    *n_claimed = total;
    ncur = h->ctr_host[4];
    if ((rc = check_flags(h))) return rc;
    if (fresh == 0 && ncur != 0)
      return set_err(h, PHIP_ERR_INVALID, "internal: insert round made no progress");
    // next round reads the retries
    cur = nxt;
    nxt = (nxt == retry) ? spare : retry;
  }
  *n_claimed = total;
  // An arena overflow would show only in the last publish's flags (it cannot
  // happen after reserve(); checked all the same when long names were inserted).
  if (h->long_need) {
    if ((rc = read_ctr(h)) || (rc = check_flags(h))) return rc;
  }
  return PHIP_OK;
}

int clear_new(phip_handle* h, u32 n_claimed) {
  if (!n_claimed) return PHIP_OK;
  u32* cslot = (u32*)h->buf[B_CSLOT].p;
  Launch l(h, "k_clear_new");
  k_clear_new<<<grid_for(n_claimed), kBlock, 0, h->stream>>>(cslot, n_claimed, table(h));
  HIPCHK(h, hipGetLastError());
  return PHIP_OK;
}

// After a failed batch: no slot may keep the NEW flag (the ordered fold reads
// it as "GetBucket is creating this bucket", phip_kernels.hpp load_state),
// whichever insert call of the batch claimed it.  Returns rc.
int after_error(phip_handle* h, int rc) {
  if (rc == PHIP_OK) return rc;
  // Nothing of the failed call may still run when it returns: the side
  // streams (the hot-directory chain of a batch whose front was queued, the
  // ordered path's folds) may still read the caller's inputs.
  if (h->stream2) (void)hipStreamSynchronize(h->stream2);
  if (h->stream3) (void)hipStreamSynchronize(h->stream3);
  if (h->stream4) (void)hipStreamSynchronize(h->stream4);
  if (rc == PHIP_ERR_HIP) return rc;
  std::string keep = h->err;
  k_clear_new_all<<<grid_for(h->cap), kBlock, 0, h->stream>>>(table(h), h->cap);
  if (hipGetLastError() == hipSuccess) (void)hipStreamSynchronize(h->stream);
  h->err = keep;
  return rc;
}

// ------------------------------------------------------- fast receive ----
// Hot directory of a fast batch (phip_kernels.hpp): sample -> count ->
// threshold -> directory, all on the stream (no host round trip).  Returns
// the header/directory to hand to k_receive_fast (nullptr: none).
template <class Src>
int build_hot(phip_handle* h, Src src, u32 n, hipStream_t st, const HotHdr** hdr_out,
              const HotEntry** dir_out) {
  *hdr_out = nullptr;
  *dir_out = nullptr;
  if (n < kHotMinBatch) return PHIP_OK;
  constexpr size_t kCnt = size_t(1) << kHotCntBits;
  const size_t zero_bytes = 2 * kCnt * sizeof(u32) + kHotHist * sizeof(u32) + sizeof(HotHdr);
  u8* base;
  int rc;
  if ((rc = ensure(h, B_HOT, zero_bytes + kHotMax * sizeof(HotEntry), &base))) return rc;
  u32* ckeys = (u32*)base;
  u32* ccnt = ckeys + kCnt;
  u32* hist = ccnt + kCnt;
  HotHdr* hdr = (HotHdr*)(hist + kHotHist);
  HotEntry* dir = (HotEntry*)(hdr + 1);
  HIPCHK(h, hipMemsetAsync(base, 0, zero_bytes, st));
  const u32 stride = std::max<u32>(64, (n + kHotSampleMax - 1) / kHotSampleMax);
  const u32 nsample = (n + stride - 1) / stride;
  {
    Launch l(h, "k_hot_sample", st);
    k_hot_sample<Src><<<grid_for(nsample, kHotSamplePerBlock), 256, 0, st>>>(
        src, n, stride, nsample, table(h), ckeys, ccnt);
  }
  {
    Launch l(h, "k_hot_select", st);
    k_hot_hist<<<grid_for(kCnt), kBlock, 0, st>>>(ccnt, hist);
    k_hot_select<<<1, 256, 0, st>>>(hist, hdr, kHotMax);
    k_hot_build<<<grid_for(kCnt), kBlock, 0, st>>>(ckeys, ccnt, hdr, table(h), dir);
  }
  HIPCHK(h, hipGetLastError());
  *hdr_out = hdr;
  *dir_out = dir;
  return PHIP_OK;
}

inline unsigned fast_grid(phip_handle* h, u32 n) {
  const u64 tiles = (n + kFastBlock - 1) / kFastBlock;
  return (unsigned)std::max<u64>(1, std::min<u64>(tiles, (u64)h->ncu * kFastPerCU));
}

int join_hot(phip_handle* h, const HotHdr* hot);

// The fast path over a batch input (SoaIn or WireIn; hsrc: its names for the
// hot-directory sample).  Resets the batch's counters, classifies, builds the
// hot directory on stream2 and applies the batch's clean prefix: the messages
// before the first dirty one (*first_dirty; n if none) and before the first
// malformed datagram (ctr[5]).  The prefix's misses (*nmiss of them) are
// listed in B_MISS.
// A sharded append list over `units` units of up to `per_unit` entries
// (counters zeroed on the stream).
int sharded(phip_handle* h, BufId base_id, u32 units, u32 per_unit, Sharded* out,
            bool zero = true) {
  int rc;
  out->cap = shard_cap(units, per_unit);
  if ((rc = ensure(h, base_id, (size_t)kShards * out->cap, &out->base)) ||
      (rc = ensure(h, B_MSCNT, 2 * kShards, &out->cnt)))
    return rc;
  if (zero) HIPCHK(h, hipMemsetAsync(out->cnt, 0, kShards * sizeof(u32), h->stream));
  return PHIP_OK;
}

// Pack a sharded list into `out`: the total lands in ctr[total_slot] and is
// returned in *total (one counter read-back).
int pack_sharded(phip_handle* h, const Sharded& sh, u32 total_slot, u32* out, u32* total) {
  k_shard_scan<<<1, kShards, 0, h->stream>>>(sh.cnt, h->ctr, total_slot, nullptr, 0, nullptr,
                                             nullptr);
  HIPCHK(h, hipGetLastError());
  int rc;
  if ((rc = read_ctr(h))) return rc;
  *total = h->ctr_host[total_slot];
  if (*total) {
    Launch l(h, "k_shard_compact");
    dim3 grid(grid_for(h->ctr_host[13]), kShards);
    k_shard_compact<<<grid, 256, 0, h->stream>>>(sh.base, sh.cap, sh.cnt, out);
    HIPCHK(h, hipGetLastError());
  }
  return PHIP_OK;
}

template <class Src>
int fork_hot(phip_handle* h, Src src, u32 n, const HotHdr** hot, const HotEntry** hot_dir);

// A fast batch in three parts, so that a queued batch (PHIP_RECV_ASYNC) can
// put the next batch's front in front of its own read-back:
//   front    counter reset, hot directory (stream2), k_classify (which also
//            fills the status column);
//   back     k_receive_fast (after the directory), then one k_shard_scan
//            that packs the miss shards' offsets and stores the counters in
//            the host's mapped mirror (queued: and resets them for the next
//            batch), ev_ctr behind it;
//   collect  the miss list packed from the host's counters, flags, stats.
// The miss list's shard counters alternate between two sets by batch parity
// (B_FSCNT): the next batch's front resets its own set while the batch
// before still has to pack its list from the other.
struct FastFront {
  const HotHdr* hot = nullptr;
  const HotEntry* dir = nullptr;
  u32 par = 0;
  bool iso = false;     // this pass sets its dirty buckets apart (the isolation kernels run)
  u32* c = nullptr;     // the pass's counter set (fctr)
  u8* mark = nullptr;   // decoded batches: the status column, or a cleared one (k_dirty_pass)
};

// A fast pass's device counters: one of two sets by batch parity, apart
// from the general set every other path uses (ordered batches, inserts, the
// miss path), so that a queued batch's front -- its classification's
// counters -- survives the previous batch's leftover work, and is queued
// again only when that work ran a nested fast pass or grew the table.
inline u32* fctr(phip_handle* h, u32 par) { return h->ctr + kCtrWords * (1 + par); }

inline u32* fast_counts(phip_handle* h, u32 par) {
  return (u32*)h->buf[B_FSCNT].p + par * 2 * kShards;
}

// The dirty-bucket set and list (phip_kernels.hpp "Dirty buckets").
int dirty_set(phip_handle* h, DirtySet* d, u32** dlist) {
  int rc;
  u64* b;
  if ((rc = ensure(h, B_DTAB, DirtySet::kWords, &b)) || (rc = ensure(h, B_DLIST, kDirtyCap, dlist)))
    return rc;
  *d = DirtySet::at(b);
  return PHIP_OK;
}
// The ordered sub-batch dirty_finish builds (at most 3 entries per dirty
// message).
struct SubBatch {
  uint64_t *off, *a, *t;
  int64_t* e;
  u8* len;
  u32* map;
};
int sub_batch(phip_handle* h, SubBatch* b) {
  constexpr size_t m = 3 * (size_t)kDirtyCap;
  int rc;
  if ((rc = ensure(h, B_SOFF, m, &b->off)) || (rc = ensure(h, B_SLEN, m, &b->len)) ||
      (rc = ensure(h, B_SA, m, &b->a)) || (rc = ensure(h, B_ST, m, &b->t)) ||
      (rc = ensure(h, B_SE, m, &b->e)) || (rc = ensure(h, B_SMAP, m, &b->map)))
    return rc;
  return PHIP_OK;
}

int fast_shards(phip_handle* h, u32 n, u32 par, Sharded* out) {
  int rc;
  u32* c;
  out->cap = shard_cap((n + 63) / 64, 64);
  if ((rc = ensure(h, B_MSHARD, (size_t)kShards * out->cap, &out->base)) ||
      (rc = ensure(h, B_FSCNT, 4 * kShards, &c)))
    return rc;
  out->cnt = fast_counts(h, par);
  return PHIP_OK;
}

// Enqueue order matters at this size (2 ms per 100M messages): the counter
// reset and the classification go first, so the GPU starts reading the batch
// while the host still enqueues the hot-directory chain on stream2 (about
// 0.1 ms of API calls that used to sit in front of k_classify).
// reset = false: the batch queued just before (nothing since) reset the
// counters in its last launch.
// iso: whether the pass sets its dirty buckets apart (-1: the handle's
// policy, phip_handle::iso_left).
template <class In, class HotSrc>
int fast_front(phip_handle* h, In in, HotSrc hsrc, u32 n, u8* status, FastFront* ff,
               bool reset = true, int iso = -1) {
  int rc;
  *ff = FastFront{};
  ff->iso = iso >= 0 ? iso != 0 : (h->iso_always || h->iso_left > 0);
  u32 *c, *dlist = nullptr;
  DirtySet dset;
  if ((rc = ensure(h, B_FSCNT, 4 * kShards, &c))) return rc;
  // (the classification lists the dirty messages either way: the policy
  // learns of them, and an isolating pass builds its set from the list)
  if ((rc = dirty_set(h, &dset, &dlist))) return rc;
  if (ff->iso) {
    ff->mark = status;
    if (!status) {   // (marks need a column: a cleared one)
      if ((rc = ensure(h, B_DMARK, n, &ff->mark))) return rc;
      HIPCHK(h, hipMemsetAsync(ff->mark, 0, n, h->stream));
    }
  }
  ff->par = h->fpar ^= 1u;
  ff->c = fctr(h, ff->par);
  ++h->nfast;
  if (reset) {
    k_batch_reset<<<1, kShards, 0, h->stream>>>(ff->c, fast_counts(h, ff->par));
    HIPCHK(h, hipGetLastError());
  }
  const bool with_hot = n >= kHotMinBatch;
  // A small batch classifies in a few µs, less than the directory chain
  // takes: that chain goes first then.
  const bool hot_first = n < (1u << 23);
  // Statuses: the fast kernel merges most of the batch and writes none; the
  // column is filled with PHIP_ST_MERGED up front (by k_classify_soa2 as it
  // streams the batch, else a fill on the main stream), and every message
  // the kernel leaves is written again after it (k_receive_list and
  // k_mark_created for misses, the ordered path for dirty buckets).  Byte
  // stores from the fast kernel's lanes cost it 2%; a fill on stream2 beside
  // the classification slowed the classification more than it cost here
  // (DESIGN.md §4).
  if (with_hot) HIPCHK(h, hipEventRecord(h->ev_fork, h->stream));
  if (with_hot && hot_first && (rc = fork_hot(h, hsrc, n, &ff->hot, &ff->dir))) return rc;
  {
    bool done = false;
    if constexpr (In::kSoa) {
      if ((((uintptr_t)in.ma | (uintptr_t)in.mt) & 15) == 0) {
        Launch l(h, "k_classify");
        // checked names (names_len): their offsets too (0.1 ms per 100M
        // messages; on stream2 beside this pass it cost 0.12)
        NamesOffs chk{};
        if constexpr (In::kOffs) chk = in.src;
        k_classify_soa2<<<grid_for((n + 1) / 2), kBlock, 0, h->stream>>>(in.ma, in.mt, in.me, n,
                                                                          ff->c, status, chk,
                                                                          dlist);
        done = true;
      }
    }
    if (!done) {
      if (status) HIPCHK(h, hipMemsetAsync(status, PHIP_ST_MERGED, n, h->stream));
      Launch l(h, "k_classify");
      k_classify<In><<<grid_for(n), kBlock, 0, h->stream>>>(in, n, ff->c, dlist);
    }
  }
  HIPCHK(h, hipGetLastError());
  if (with_hot && !hot_first && (rc = fork_hot(h, hsrc, n, &ff->hot, &ff->dir))) return rc;
  return PHIP_OK;
}

// The fast kernel is enqueued behind the classification without a host
// round trip; it reads the counters itself.
template <class In>
int fast_back(phip_handle* h, In in, u32 n, const FastFront& ff, bool queued) {
  u32* miss;
  int rc;
  Sharded msh;
  DirtySet dset{};
  SubBatch sb{};
  u32* dlist = nullptr;
  if ((rc = ensure(h, B_MISS, n, &miss)) || (rc = fast_shards(h, n, ff.par, &msh))) return rc;
  if (ff.iso) {
    // the dirty set behind the classification (a batch without a dirty
    // message returns at once: one launch of ~3 us)
    if ((rc = dirty_set(h, &dset, &dlist)) || (rc = sub_batch(h, &sb))) return rc;
    Launch l(h, "k_dirty_build");
    k_dirty_build<In><<<1, 1024, 0, h->stream>>>(in, n, ff.c, dlist, dset, table(h));
    HIPCHK(h, hipGetLastError());
  }
  if ((rc = join_hot(h, ff.hot))) return rc;
  {
    Launch l(h, "k_receive_fast");
    k_receive_fast<In><<<fast_grid(h, n), kFastBlock, 0, h->stream>>>(
        in, 0, n, table(h), msh, ff.c, ff.hot, ff.dir, ff.iso ? dset.key : nullptr, ff.mark);
  }
  HIPCHK(h, hipGetLastError());
  if (ff.iso) {
    // the messages the fast kernel marked (an isolated batch's only: others
    // return at once), then the dirty buckets' records unmarked and their
    // ordered sub-batch built in the launch that ends the batch
    {
      Launch l(h, "k_dirty_pass");
      const unsigned g = (unsigned)std::max<u64>(
          1, std::min<u64>(((u64)n + 1023) / 1024, (u64)h->ncu * 2));
      k_dirty_pass<In><<<g, 1024, 0, h->stream>>>(in, n, ff.c, ff.mark, dset.key, table(h), msh);
      HIPCHK(h, hipGetLastError());
    }
    k_batch_end<In><<<1, kShards, 0, h->stream>>>(
        in, ff.c, dset.key, table(h), SubOut{sb.off, sb.len, sb.a, sb.t, sb.e, sb.map}, msh.cnt,
        h->ctr_map, kCtrWords, queued ? fast_counts(h, ff.par ^ 1u) : nullptr,
        fctr(h, ff.par ^ 1u));
  } else {
    k_shard_scan<<<1, kShards, 0, h->stream>>>(msh.cnt, ff.c, 2, h->ctr_map, kCtrWords,
                                               queued ? fast_counts(h, ff.par ^ 1u) : nullptr,
                                               fctr(h, ff.par ^ 1u));
  }
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev_ctr, h->stream));
  if (!queued) HIPCHK(h, hipEventSynchronize(h->ev_ctr));
  return PHIP_OK;
}

// *first_dirty: n when the batch's dirty buckets were set apart (iso ran and
// at most kDirtyCap dirty messages, short names), else its first dirty
// message (the prefix rule).  Updates the isolation policy: kIsoKeep passes
// after one that met a dirty message.
constexpr u32 kIsoKeep = 256;
int fast_collect(phip_handle* h, u32 n, u32 par, u32* first_dirty, u32* nmiss, bool iso_ran) {
  int rc;
  if ((rc = check_flags(h))) return rc;
  *nmiss = h->ctr_host[2];
  if (*nmiss) {
    Sharded msh;
    if ((rc = fast_shards(h, n, par, &msh))) return rc;
    Launch l(h, "k_shard_compact");
    dim3 grid(grid_for(h->ctr_host[13]), kShards);
    k_shard_compact<<<grid, 256, 0, h->stream>>>(msh.base, msh.cap, msh.cnt,
                                                 (u32*)h->buf[B_MISS].p);
    HIPCHK(h, hipGetLastError());
  }
  const u32 nd = h->ctr_host[kCtrNDirty];
  const bool iso = iso_ran && nd != 0 && nd <= kDirtyCap;
  *first_dirty = iso ? n : std::min<u32>(h->ctr_host[kCtrDirty], n);
  if (h->ctr_host[kCtrDirty] < n) h->iso_left = kIsoKeep;
  else if (h->iso_left) --h->iso_left;
  h->coll_iso = iso_ran;
  h->ndef = iso ? h->ctr_host[kCtrNDefer] : 0;   // (the ordered sub-batch, run_deferred)
  h->stats[3] = 0;   // (finish_receive: the messages it sends through the ordered path)
  h->stats[0] = h->ctr_host[11];
  h->stats[1] = h->ctr_host[10];
  h->stats[2] = *nmiss;
  return PHIP_OK;
}

// The whole fast path of a batch (SoaIn or WireIn; hsrc: its names for the
// hot-directory sample), synchronously: resets the batch's counters,
// classifies, builds the hot directory on stream2 and applies the batch's
// clean prefix: the messages before the first dirty one (*first_dirty; n if
// none) and before the first malformed datagram (ctr[5]).  The prefix's
// misses (*nmiss of them) are listed in B_MISS.
template <class In, class HotSrc>
int fast_apply(phip_handle* h, In in, HotSrc hsrc, u32 n, u8* status, u32* first_dirty,
               u32* nmiss, int iso = -1) {
  int rc;
  FastFront ff;
  if ((rc = fast_front(h, in, hsrc, n, status, &ff, true, iso)) ||
      (rc = fast_back(h, in, n, ff, false)))
    return rc;
  return fast_collect(h, n, ff.par, first_dirty, nmiss, ff.iso);
}

template <class Src>
int fork_hot(phip_handle* h, Src src, u32 n, const HotHdr** hot, const HotEntry** hot_dir);

// One message per distinct name of list[0..n) (k_dedupe) into B_DEDUP.
template <class Src>
int dedupe_names(phip_handle* h, Src src, const u32* list, u32 n, u32** out, u32* nout) {
  int rc;
  u32 setbits = 1;
  while ((1ull << setbits) < 2ull * n) ++setbits;
  u64* set;
  Sharded dsh;
  if ((rc = ensure(h, B_DSET, size_t(1) << setbits, &set)) ||
      (rc = ensure(h, B_DEDUP, n, out)) ||
      (rc = sharded(h, B_MSHARD, grid_for(n), kBlock, &dsh)))
    return rc;
  HIPCHK(h, hipMemsetAsync(set, 0, (size_t(1) << setbits) * sizeof(u64), h->stream));
  {
    Launch l(h, "k_dedupe");
    k_dedupe<Src><<<grid_for(n), kBlock, 0, h->stream>>>(src, n, list, table(h), set, setbits, dsh);
    HIPCHK(h, hipGetLastError());
  }
  return pack_sharded(h, dsh, 14, *out, nout);
}

// Many misses (an insert-heavy batch: a node starting empty, a fresh key
// range): create each distinct missing name once (k_dedupe, then the insert
// pipeline over one message per name), then merge by running the fast pass
// again over the whole clean prefix [0, prefix).  In that prefix every merge
// is an order-free max, so the messages the first pass already merged are
// merged again to no effect, and the hot directory now covers the new hot
// buckets: their messages fold in LDS instead of each sending a
// device-scope atomic to one record (134 ms per 100M-message batch through
// k_receive_list).  Returns the misses of the second pass
// (names dropped by k_dedupe for a shared tag) in *nmiss2, listed in B_MISS.
template <class Src>
int finish_many_misses(phip_handle* h, Src src, const uint64_t* a, const uint64_t* t,
                       const int64_t* e, u32 nmiss, u32 prefix, i64 now, u8* status, u32* nmiss2) {
  u32* miss = (u32*)h->buf[B_MISS].p;
  int rc;
  // 1. distinct names
  u32 *dedup, nd = 0;
  if ((rc = dedupe_names(h, src, miss, nmiss, &dedup, &nd))) return rc;
  // 2. create them (aux = ~0 and the NEW flag on every claimed slot)
  u32 n_claimed = 0;
  if ((rc = insert_names(h, src, dedup, nd, nullptr, now, &n_claimed, nullptr, true))) return rc;
  // 3. creator tracking over the first pass's misses (every message of a new
  //    bucket is among them), before the second pass reuses B_MISS
  if (status) {
    Launch l(h, "k_first_seen");
    k_first_seen<Src><<<grid_for(nmiss), kBlock, 0, h->stream>>>(src, nmiss, miss, table(h));
    HIPCHK(h, hipGetLastError());
  }
  // 4. the fast pass again
  u32 fd = prefix;
  // (as the pass being finished did: its dirty buckets stay apart)
  if ((rc = fast_apply(h, SoaIn<Src>{src, a, t, e}, src, prefix, status, &fd, nmiss2,
                       h->coll_iso ? 1 : 0)))
    return rc;
  // 5. PHIP_ST_CREATED after the second pass wrote its statuses
  if (status && n_claimed) {
    Launch l(h, "k_mark_created");
    k_mark_created_slots<<<grid_for(n_claimed), kBlock, 0, h->stream>>>(
        (const u32*)h->buf[B_CSLOT].p, n_claimed, table(h), status);
    HIPCHK(h, hipGetLastError());
  }
  return clear_new(h, n_claimed);
}

// The messages fast_apply missed: create their buckets, merge them with
// creator tracking (PHIP_ST_CREATED on the first message of a new bucket).
template <class Src>
int finish_misses(phip_handle* h, Src src, const uint64_t* a, const uint64_t* t, const int64_t* e,
                  u32 nmiss, u32 prefix, i64 now, u8* status) {
  if (nmiss == 0) return PHIP_OK;
  int rc;
  if (nmiss >= kManyMisses &&
      (rc = finish_many_misses(h, src, a, t, e, nmiss, prefix, now, status, &nmiss)))
    return rc;
  if (nmiss == 0) return PHIP_OK;
  u32* miss = (u32*)h->buf[B_MISS].p;
  u32 n_claimed = 0;
  if ((rc = insert_names(h, src, miss, nmiss, nullptr, now, &n_claimed))) return rc;
  HIPCHK(h, hipMemsetAsync(h->ctr + 2, 0, sizeof(u32), h->stream));
  u32* miss2;
  if ((rc = ensure(h, B_MISS2, nmiss, &miss2))) return rc;
  {
    Launch l(h, "k_receive_list");
    k_receive_list<Src><<<grid_for(nmiss), kBlock, 0, h->stream>>>(
        src, a, t, e, nmiss, miss, table(h), status, miss2, h->ctr);
  }
  HIPCHK(h, hipGetLastError());
  {
    Launch l(h, "k_mark_created");
    k_mark_created<Src><<<grid_for(nmiss), kBlock, 0, h->stream>>>(src, nmiss, miss, table(h),
                                                                    status);
  }
  HIPCHK(h, hipGetLastError());
  if ((rc = read_ctr(h))) return rc;
  if (h->ctr_host[2]) return set_err(h, PHIP_ERR_INVALID, "internal: %u names missing after insert", h->ctr_host[2]);
  return clear_new(h, n_claimed);
}

// Start the hot directory of a fast batch on stream2 (joined by join_hot).
template <class Src>
int fork_hot(phip_handle* h, Src src, u32 n, const HotHdr** hot, const HotEntry** hot_dir) {
  *hot = nullptr;
  *hot_dir = nullptr;
  if (n < kHotMinBatch) return PHIP_OK;
  // ev_fork: recorded by fast_apply before the classification (stream2 waits
  // only for the batch's producers, not for k_classify)
  HIPCHK(h, hipStreamWaitEvent(h->stream2, h->ev_fork, 0));
  int rc;
  if ((rc = build_hot(h, src, n, h->stream2, hot, hot_dir))) return rc;
  HIPCHK(h, hipEventRecord(h->ev_join, h->stream2));
  return PHIP_OK;
}

int join_hot(phip_handle* h, const HotHdr* hot) {
  if (hot) HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_join, 0));
  return PHIP_OK;
}

// ------------------------------------------------------------ ordered ----

// A launch for the run-time output mask (out_mask): CALL(M) with M a
// compile-time constant.
#define PHIP_OUT_DISPATCH(mask, CALL) \
  switch (mask) {                     \
    case 0: CALL(0); break;           \
    case 1: CALL(1); break;           \
    case 2: CALL(2); break;           \
    case 3: CALL(3); break;           \
    case 4: CALL(4); break;           \
    case 5: CALL(5); break;           \
    case 6: CALL(6); break;           \
    case 7: CALL(7); break;           \
    case 8: CALL(8); break;           \
    case 9: CALL(9); break;           \
    case 10: CALL(10); break;         \
    case 11: CALL(11); break;         \
    case 12: CALL(12); break;         \
    case 13: CALL(13); break;         \
    case 14: CALL(14); break;         \
    default: CALL(15); break;         \
  }

template <class Src>
int resolve_all(phip_handle* h, Src src, u32 n, const int64_t* now_arr, i64 now0, u32** slot_out,
                u32* n_claimed, SortVals sv = SortVals{nullptr, 0, nullptr}) {
  u32 *slot, *miss;
  int rc;
  Sharded rsh;
  if ((rc = ensure(h, B_SLOT, n, &slot)) || (rc = ensure(h, B_MISS, n, &miss)) ||
      (rc = sharded(h, B_MSHARD, grid_for(n), kBlock, &rsh)))
    return rc;
  if ((rc = reset_ctr(h))) return rc;
  {
    // (kResPer ops per thread; a persistent version that took the hot names'
    // slots from C2's directory in LDS first lost: 1.85 against 1.49 ms on
    // C3 with one op per thread)
    Launch l(h, "k_resolve");
    k_resolve_batch<Src><<<grid_for(n, kBlock * kResPer), kBlock, 0, h->stream>>>(
        src, n, table(h), slot, rsh, h->ctr, sv);
  }
  HIPCHK(h, hipGetLastError());
  u32 nmiss = 0;
  if ((rc = pack_sharded(h, rsh, 2, miss, &nmiss))) return rc;
  if ((rc = check_flags(h))) return rc;
  *n_claimed = 0;
  bool grew = false;
  if (nmiss >= kManyMisses) {
    // Many new names (an ordered batch on a fresh key range, a large seed):
    // create each once, then resolve the misses again; names k_dedupe
    // dropped for a shared tag miss again and take the general rounds below.
    u32 *dedup, nd = 0;
    if ((rc = dedupe_names(h, src, miss, nmiss, &dedup, &nd)) ||
        (rc = insert_names(h, src, dedup, nd, now_arr, now0, n_claimed, &grew, true)))
      return rc;
    Sharded r2;
    if ((rc = sharded(h, B_MSHARD, grid_for(nmiss), kBlock, &r2))) return rc;
    {
      Launch l(h, "k_resolve_miss");
      k_resolve<Src><<<grid_for(nmiss), kBlock, 0, h->stream>>>(src, nmiss, miss, table(h), slot,
                                                                 r2, h->ctr, SortVals{});
    }
    HIPCHK(h, hipGetLastError());
    if ((rc = pack_sharded(h, r2, 2, miss, &nmiss))) return rc;
  }
  if (nmiss) {
    u32 more = 0;
    bool g2 = false;
    if ((rc = insert_names(h, src, miss, nmiss, now_arr, now0, &more, &g2))) return rc;
    grew |= g2;
    *n_claimed += more;
    if (!grew) {
      Launch l(h, "k_resolve_miss");
      k_resolve<Src><<<grid_for(nmiss), kBlock, 0, h->stream>>>(src, nmiss, miss, table(h), slot,
                                                                 Sharded{}, h->ctr, SortVals{});
      HIPCHK(h, hipGetLastError());
    }
  }
  if (grew) {
    // The table was rehashed: every op's slot is looked up again.
    Launch l(h, "k_resolve");
    k_resolve<Src><<<grid_for(n), kBlock, 0, h->stream>>>(src, n, nullptr, table(h), slot,
                                                           Sharded{}, h->ctr, SortVals{});
    HIPCHK(h, hipGetLastError());
  }
  *slot_out = slot;
  return PHIP_OK;
}

// Apply a mixed op stream in seq order.  The NEW flag of created buckets is
// consumed (cleared) by the fold itself.
template <class Src>
int ordered(phip_handle* h, Src src, u32 n, const OpView& ov, const OutView& ow) {
  if (n == 0) return PHIP_OK;
  if (n > kMaxOrderedOps)
    return set_err(h, PHIP_ERR_INVALID, "ordered batch of %u ops exceeds 2^30", n);
  int rc;
  u32 *idx, *sslot, *sidx, *uslot, *scnt, *sstart, *lng, *huge;
  if ((rc = ensure(h, B_IDX, n, &idx)) || (rc = ensure(h, B_SSLOT, n, &sslot)) ||
      (rc = ensure(h, B_SIDX, n, &sidx)) || (rc = ensure(h, B_USLOT, n, &uslot)) ||
      (rc = ensure(h, B_SCNT, n, &scnt)) || (rc = ensure(h, B_SSTART, n, &sstart)) ||
      (rc = ensure(h, B_LONG, n, &lng)) || (rc = ensure(h, B_HUGE, n, &huge)))
    return rc;
  OpRec* opr;
  if ((rc = ensure(h, B_OPS, n, &opr))) return rc;
  // The op records are read by the folds only: k_pack_ops runs on stream2
  // beside the resolve, the sort and the segmentation (independent streams of
  // the batch's columns; the resolve is bound by probe latency), and the main
  // stream joins it before the first fold, or on any error return (PackJoin).
  struct PackJoin {
    phip_handle* h;
    bool armed = true;
    int join() {
      armed = false;
      return hipStreamWaitEvent(h->stream, h->ev_pack, 0) == hipSuccess
                 ? PHIP_OK
                 : set_err(h, PHIP_ERR_HIP, "hipStreamWaitEvent (op records)");
    }
    ~PackJoin() { if (armed) (void)hipStreamWaitEvent(h->stream, h->ev_pack, 0); }
  } pack_join{h};
  auto fork_pack = [&]() -> int {
    HIPCHK(h, hipEventRecord(h->ev_fork, h->stream));
    HIPCHK(h, hipStreamWaitEvent(h->stream2, h->ev_fork, 0));
    {
      Launch l(h, "k_pack_ops", h->stream2);
      k_pack_ops<<<grid_for(n, kBlock * kPackPer), kBlock, 0, h->stream2>>>(ov, n, opr);
    }
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->ev_pack, h->stream2));
    return PHIP_OK;
  };
  if ((rc = fork_pack())) return rc;
  u32* slot;
  u32 n_claimed = 0;
  if ((rc = resolve_all(h, src, n, ov.now, ov.now0, &slot, &n_claimed,
                        SortVals{ov.kind, ov.kind0, idx})))
    return rc;
  // Stable radix sort of (slot, seq) pairs: per-bucket arrival order kept.
  // (A hot split, the hot buckets' ops partitioned by name before the sort
  // and the sort ordering only the rest, was built and measured in round 6:
  // slower)
  size_t tb = 0;
  HIPCHK(h, rocprim::radix_sort_pairs<SlotSortConfig>(nullptr, tb, slot, sslot, idx, sidx, n, 0u, h->L,
                                                       h->stream));
  // segmentation buffers and scan temp sized before the sort is enqueued (a
  // larger B_TEMP must not replace the one the sort is using)
  const u32 ntiles = (u32)(((u64)n + kSegTile - 1) / kSegTile);
  u32 *segt = nullptr, *segb = nullptr;
  size_t tbs = 0;
  if ((rc = ensure(h, B_SEGT, 2 * ((size_t)ntiles + 1), &segt))) return rc;
  segb = segt + ntiles + 1;
  HIPCHK(h, rocprim::exclusive_scan(nullptr, tbs, segt, segb, 0u, (size_t)ntiles + 1,
                                    rocprim::plus<u32>(), h->stream));
  u8* temp;
  if ((rc = ensure(h, B_TEMP, std::max(tb, tbs), &temp))) return rc;
  {
    Launch l(h, "radix_sort_pairs");
    HIPCHK(h, rocprim::radix_sort_pairs<SlotSortConfig>(temp, tb, slot, sslot, idx, sidx, n, 0u,
                                                         h->L, h->stream));
  }
  u32 nseg = 0;
  {
    Launch l(h, "segments");
    k_seg_count<<<ntiles, 256, 0, h->stream>>>(sslot, n, segt, h->ctr);
    HIPCHK(h, rocprim::exclusive_scan(temp, tbs, segt, segb, 0u, (size_t)ntiles + 1,
                                      rocprim::plus<u32>(), h->stream));
    k_seg_write<<<ntiles, 256, 0, h->stream>>>(sslot, n, segb, uslot, sstart);
    k_seg_finish<<<std::max(1u, std::min<u32>(ntiles, (u32)h->ncu * 4)), 256, 0, h->stream>>>(
        segb, ntiles, sstart, n, scnt, lng, huge, h->ctr);
    HIPCHK(h, hipGetLastError());
    if ((rc = read_ctr(h))) return rc;
    nseg = h->ctr_host[kCtrSegs];
  }
  u32 nlong = h->ctr_host[6], nhuge = h->ctr_host[9];
  if ((rc = pack_join.join())) return rc;
  // Different segments touch different slots, so the folds may overlap: the
  // hot-bucket workgroups run on stream2 beside the wave and thread folds.
  if (nhuge) {
    // k_huge_outputs stores only results that differ from the defaults
    // (write_out_nd): the defaults go in first, as streams
    if (ow.status) HIPCHK(h, hipMemsetAsync(ow.status, PHIP_ST_MERGED, n, h->stream));
    if (ow.remaining) HIPCHK(h, hipMemsetAsync(ow.remaining, 0, (size_t)n * 8, h->stream));
    if (ow.have) HIPCHK(h, hipMemsetAsync(ow.have, 0, (size_t)n * 8, h->stream));
    u64 *hoff, *woff;
    OpRec* hop;
    u32 *hval, *rpos, *runn, *wrun;
    RunState* rst;
    u8* segex;
    WinSum* sums;
    GMax* wing;
    u32* segxf;
    const size_t nwin_max = (size_t)n / kFoldWin + nhuge + 1;
    if ((rc = ensure(h, B_WOFF, (size_t)nhuge + 1, &woff)) ||
        (rc = ensure(h, B_SUMS, nwin_max, &sums)) || (rc = ensure(h, B_WRUN, nwin_max, &wrun)) ||
        (rc = ensure(h, B_HOFF, nhuge, &hoff)) || (rc = ensure(h, B_HOP, n, &hop)) ||
        (rc = ensure(h, B_HVAL, n, &hval)) || (rc = ensure(h, B_RPOS, (size_t)n + nhuge, &rpos)) ||
        (rc = ensure(h, B_RST, (size_t)n + nhuge, &rst)) || (rc = ensure(h, B_RUNN, nhuge, &runn)) ||
        (rc = ensure(h, B_SEGEX, nhuge, &segex)) || (rc = ensure(h, B_WING, nwin_max, &wing)) ||
        (rc = ensure(h, B_SEGXF, nhuge, &segxf)))
      return rc;
    // The largest huge segments (kFirst of them, moved to the front of the
    // list) run gather -> fold -> outputs on stream2, the other huge segments
    // the same chain on stream3, beside the wave and thread folds on the
    // main stream: the largest segments' folds are the longest sequential
    // chains, so they start as soon as their own (smaller) gather is done.
    const u32 kFirst = std::min<u32>(PHIP_HUGE_FIRST, kHugeFirstMax);
    const bool split = kFirst > 0 && nhuge > kFirst;
    const u32 hsplit = split ? kFirst : nhuge;
    u32* hl = huge;
    if (split && (rc = ensure(h, B_HUGE2, nhuge, &hl))) return rc;
    HIPCHK(h, hipEventRecord(h->ev_fork, h->stream));
    HIPCHK(h, hipStreamWaitEvent(h->stream2, h->ev_fork, 0));
    if (split) {
      k_huge_order<<<1, 1024, 0, h->stream2>>>(huge, nhuge, scnt, kFirst, hl);
      HIPCHK(h, hipGetLastError());
    }
    k_huge_offsets<<<1, 1024, 0, h->stream2>>>(hl, nhuge, scnt, hoff, woff);
    HIPCHK(h, hipGetLastError());
    if (split) {
      HIPCHK(h, hipEventRecord(h->ev_fork3, h->stream2));
      HIPCHK(h, hipStreamWaitEvent(h->stream3, h->ev_fork3, 0));
    }
    // A diagnostics build (tools/build_variants.sh "stats:-DPHIP_FOLD_STATS")
    // prints per hot segment ops / windows / windows folded / rounds / bursts
    // / ops walked / runs / cycles to stderr.
    u64* fold_dbg = nullptr;
#ifdef PHIP_FOLD_STATS
    if ((rc = ensure(h, B_FOLDDBG, (size_t)nhuge * 16, &fold_dbg))) return rc;
#endif
    // gather / outputs: window-striding grids of 8 workgroups per CU (the
    // window count is known on the device only)
    const unsigned hgrid = (unsigned)std::min<size_t>(nwin_max, (size_t)h->ncu * 8);
    // one chain per group: segments [h0, h1) of the list on stream st; the
    // main stream's wave and thread folds wait for the gathers (ev): the
    // gathers alone, then the latency-bound block folds beside those
    // bandwidth-bound folds, is the shorter schedule.
    auto chain = [&](u32 h0, u32 h1, hipStream_t st, hipEvent_t ev, const char* ng,
                     const char* nf, const char* no) -> int {
      {
        Launch l(h, ng, st);
        k_gather_huge<<<hgrid, kBlock, 0, st>>>(hl, h1, hoff, woff, sstart, scnt, sidx, opr, hop,
                                                 hval, sums, h0);
      }
      HIPCHK(h, hipGetLastError());
      HIPCHK(h, hipEventRecord(ev, st));
      HIPCHK(h, hipStreamWaitEvent(h->stream, ev, 0));
      {
        Launch l(h, nf, st);
        k_fold_block<<<h1 - h0, kFoldThreads, 0, st>>>(hl, h1, uslot, hoff, scnt, hval, hop,
                                                       h->recs, rpos, rst, runn, segex, segxf,
                                                       woff, sums, wrun, wing, fold_dbg, h0);
      }
      HIPCHK(h, hipGetLastError());
      {
        Launch l(h, no, st);
#define PHIP_HUGE_OUT(M)                                                                      \
  k_huge_outputs<M><<<hgrid, kBlock, 0, st>>>(hl, h1, hoff, woff, scnt, hval, hop, rpos, rst, \
                                              runn, segex, segxf, wrun, wing, ow, h0)
        PHIP_OUT_DISPATCH(out_mask(ow), PHIP_HUGE_OUT);
#undef PHIP_HUGE_OUT
      }
      HIPCHK(h, hipGetLastError());
      return PHIP_OK;
    };
    if ((rc = chain(0, hsplit, h->stream2, h->ev_gather, "k_gather_huge", "k_fold_block",
                    "k_huge_outputs")))
      return rc;
    if (split) {
      if ((rc = chain(hsplit, nhuge, h->stream3, h->ev_gather3, "k_gather_huge2", "k_fold_block2",
                      "k_huge_outputs2")))
        return rc;
      HIPCHK(h, hipEventRecord(h->ev_join3, h->stream3));
      HIPCHK(h, hipStreamWaitEvent(h->stream2, h->ev_join3, 0));
    }
    if (fold_dbg) {
      std::vector<u64> d((size_t)nhuge * 16);
      HIPCHK(h, hipMemcpyAsync(d.data(), fold_dbg, d.size() * 8, hipMemcpyDeviceToHost, h->stream2));
      HIPCHK(h, hipStreamSynchronize(h->stream2));
      std::vector<u32> ord(nhuge);
      for (u32 k = 0; k < nhuge; ++k) ord[k] = k;
      std::sort(ord.begin(), ord.end(), [&](u32 x, u32 y) { return d[16 * x + 7] > d[16 * y + 7]; });
      fprintf(stderr, "fold: %u huge segments\n", nhuge);
      for (u32 i = 0; i < nhuge && i < 6; ++i) {
        const u32 k = ord[i];
        const u64* e = &d[16 * k];
        fprintf(stderr, "fold[%u] ops %llu windows %llu folded %llu rounds %llu bursts %llu walked "
                "%llu runs %llu us %.1f | scan %.1f stage %.1f prefix %.1f round %.1f burst %.1f "
                "| burst iterations %llu (stopped at a merge %llu)\n",
                k, e[0], e[1], e[2], e[3], e[4], e[5], e[6], e[7] / 100.0, e[8] / 100.0,
                e[9] / 100.0, e[10] / 100.0, e[11] / 100.0, e[12] / 100.0, e[13], e[14]);
      }
    }
  }
  // The thread folds (short segments, one thread each) run on stream4 beside
  // the wave folds: different segments, different slots.  6.37-6.38 against
  // 6.45-6.50 ms per C3 step.  The main stream joins them
  // before returning, or on any error return (ThreadJoin).
  struct ThreadJoin {
    phip_handle* h;
    bool armed = false;
    ~ThreadJoin() { if (armed) (void)hipStreamWaitEvent(h->stream, h->ev_t4b, 0); }
  } thread_join{h};
  if (!h->ev_t4a) HIPCHK(h, hipEventCreateWithFlags(&h->ev_t4a, hipEventDisableTiming));
  if (!h->ev_t4b) HIPCHK(h, hipEventCreateWithFlags(&h->ev_t4b, hipEventDisableTiming));
  if (!h->stream4) HIPCHK(h, hipStreamCreateWithFlags(&h->stream4, hipStreamNonBlocking));
  hipStream_t ts = h->stream4;
  HIPCHK(h, hipEventRecord(h->ev_t4a, h->stream));
  HIPCHK(h, hipStreamWaitEvent(ts, h->ev_t4a, 0));
  {
    Launch l(h, "k_fold_thread", ts);
#define PHIP_FOLD_THREAD(M)                                                            \
  k_fold_thread<M><<<grid_for(nseg), kBlock, 0, ts>>>(uslot, sstart, scnt, nseg, sidx, \
                                                      opr, h->recs, ow)
    PHIP_OUT_DISPATCH(out_mask(ow), PHIP_FOLD_THREAD);
#undef PHIP_FOLD_THREAD
    HIPCHK(h, hipGetLastError());
  }
  HIPCHK(h, hipEventRecord(h->ev_t4b, ts));
  thread_join.armed = true;
  if (nlong) {
    // the long segments over kBigLongSeg ops first (their sequential chains
    // are the longest), then the rest
    if (nlong > 1) {
      u32* lng2;
      if ((rc = ensure(h, B_LONG2, nlong, &lng2))) return rc;
      size_t tb7 = 0;
      HIPCHK(h, rocprim::partition(nullptr, tb7, lng, lng2, h->ctr + 14, (size_t)nlong,
                                   BigLongSeg{scnt}, h->stream));
      if ((rc = ensure(h, B_TEMP, tb7, &temp))) return rc;
      HIPCHK(h, rocprim::partition(temp, tb7, lng, lng2, h->ctr + 14, (size_t)nlong,
                                   BigLongSeg{scnt}, h->stream));
      lng = lng2;
    }
    Launch l(h, "k_fold_wave");
#define PHIP_FOLD_WAVE(M)                                                                  \
  k_fold_wave<M><<<nlong, 64, 0, h->stream>>>(lng, nlong, uslot, sstart, scnt, sidx, opr, \
                                              h->recs, ow)
    PHIP_OUT_DISPATCH(out_mask(ow), PHIP_FOLD_WAVE);
#undef PHIP_FOLD_WAVE
    HIPCHK(h, hipGetLastError());
  }
  thread_join.armed = false;
  HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_t4b, 0));
  if (nhuge) {
    HIPCHK(h, hipEventRecord(h->ev_join, h->stream2));
    HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_join, 0));
  }
  (void)n_claimed;  // NEW flags cleared by store_state in the folds
  return PHIP_OK;
}

int stage_names(phip_handle* h, const uint8_t* names, const uint32_t* offs, u32 n, bool dev,
                NamesOffs* src, u32 names_len = 0) {
  const u32* d_offs;
  int rc;
  if ((rc = stage(h, B_OFFS, offs, (size_t)n + 1, dev, &d_offs))) return rc;
  const u8* d_names;
  size_t nb = 0;
  if (!dev) nb = offs[n];
  if ((rc = stage(h, B_NAMES, names, nb, dev, &d_names))) return rc;
  if (!dev && nb == 0) {
    u8* p;
    if ((rc = ensure(h, B_NAMES, 1, &p))) return rc;
    d_names = p;
  }
  src->blob = d_names;
  src->offs = d_offs;
  // (a device batch's offsets are checked on the device when the caller gave
  // the blob's length; a host batch's were checked on the host)
  src->lim = dev ? names_len : 0;
  return PHIP_OK;
}

// Datagram offsets from the host: non-decreasing, so every datagram the
// kernels read lies inside the bytes[offs[0] .. offs[n]) that were copied.
bool datagrams_ok(const uint64_t* offs, u32 n) {
  for (u32 i = 0; i < n; ++i)
    if (offs[i + 1] < offs[i]) return false;
  return true;
}

bool names_ok(const uint32_t* offs, u32 n) {
  for (u32 i = 0; i < n; ++i) {
    if (offs[i + 1] < offs[i]) return false;
    if (offs[i + 1] - offs[i] > PHIP_MAX_NAME_LEN) return false;
  }
  return true;
}

int outputs(phip_handle* h, const phip_results* res, u32 n, bool dev, OutView* ow) {
  int rc;
  phip_results r{};
  if (res) r = *res;
  if ((rc = out_buf(h, B_STATUS, r.status, n, dev, &ow->status)) ||
      (rc = out_buf(h, B_REM, r.remaining, n, dev, &ow->remaining)) ||
      (rc = out_buf(h, B_HAVE, r.have, n, dev, &ow->have)) ||
      (rc = out_buf(h, B_REPLY, r.reply, n, dev, &ow->reply)))
    return rc;
  // an entry with no reply state (a merged replica) reads as zeros, on every
  // path (the staged buffer would otherwise hand back an earlier call's data)
  if (ow->reply) HIPCHK(h, hipMemsetAsync(ow->reply, 0, (size_t)n * sizeof(phip_state), h->stream));
  return PHIP_OK;
}

int copy_outputs(phip_handle* h, const phip_results* res, u32 n, bool dev, const OutView& ow) {
  if (!res || dev) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return PHIP_OK;
  }
  int rc;
  if ((rc = copy_back(h, res->status, ow.status, n, dev)) ||
      (rc = copy_back(h, res->remaining, ow.remaining, n, dev)) ||
      (rc = copy_back(h, res->have, ow.have, n, dev)) ||
      (rc = copy_back(h, res->reply, ow.reply, n, dev)))
    return rc;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

// A batch from message k on.
inline NamesOffs shifted(NamesOffs s, u32 k) {
  s.offs += k;
  return s;
}
inline NamesPairs shifted(NamesPairs s, u32 k) {
  s.off += k;
  s.len += k;
  return s;
}
inline OutView shifted(OutView o, u32 k) {
  if (o.status) o.status += k;
  if (o.remaining) o.remaining += k;
  if (o.have) o.have += k;
  if (o.reply) o.reply += k;
  return o;
}

// The last fast pass's ordered sub-batch (its dirty buckets' dirty messages
// and the merges of their cells, dirty_finish) through the ordered path,
// its statuses and replies scattered back.  The dirty buckets' other
// messages were merged by the fast pass (before each bucket's first dirty
// message) or folded into the cells (after it); no other bucket is touched,
// and Receive is per bucket (repo.go:77-106), so applying the sub-batch
// after the rest of the batch gives each dirty bucket the Go loop's states.
template <class Src>
int run_deferred(phip_handle* h, Src src, i64 now, const OutView& ow) {
  const u32 nd = h->ndef;   // (the last fast pass's: a second pass rebuilt it)
  h->stats[3] = nd;
  if (nd == 0) return PHIP_OK;
  if (nd > 3 * kDirtyCap) return set_err(h, PHIP_ERR_HIP, "ordered sub-batch of %u entries", nd);
  int rc;
  SubBatch sb;
  u8* st2 = nullptr;
  phip_state* rep2 = nullptr;
  if ((rc = sub_batch(h, &sb)) || (ow.status && (rc = ensure(h, B_SSTAT, nd, &st2))) ||
      (ow.reply && (rc = ensure(h, B_SREP, nd, &rep2))))
    return rc;
  if (rep2) HIPCHK(h, hipMemsetAsync(rep2, 0, (size_t)nd * sizeof(phip_state), h->stream));
  OpView ov{};
  ov.kind = nullptr; ov.kind0 = PHIP_OP_RECEIVE;
  ov.now = nullptr; ov.now0 = now;
  ov.a = sb.a; ov.t = sb.t; ov.e = sb.e;
  if ((rc = ordered(h, NamesPairs{src.blob, sb.off, sb.len}, nd, ov,
                    OutView{st2, nullptr, nullptr, rep2})))
    return rc;
  if (st2 || rep2) {
    k_defer_scatter<<<grid_for(nd), kBlock, 0, h->stream>>>(sb.map, nd, st2, rep2, ow);
    HIPCHK(h, hipGetLastError());
  }
  return PHIP_OK;
}

// After the fast path: the clean prefix's new buckets (finish_misses), then
// the ordered path over messages [first_dirty, stop), which starts from the
// state the prefix left (the Go loop's state at that message) -- or, when the
// fast pass deferred the dirty buckets (first_dirty == n), over their
// messages (run_deferred).
template <class Src>
int finish_receive(phip_handle* h, Src src, const uint64_t* a, const uint64_t* t,
                   const int64_t* e, u32 stop, u32 first_dirty, u32 nmiss, i64 now,
                   const OutView& ow, u32 n, bool deferred) {
  int rc;
  if ((rc = finish_misses(h, src, a, t, e, nmiss, std::min(stop, first_dirty), now, ow.status)))
    return rc;
  if (deferred) return run_deferred(h, src, now, ow);
  h->stats[3] = first_dirty < stop ? stop - first_dirty : 0;
  if (first_dirty >= stop) return PHIP_OK;
  const u32 k = first_dirty;
  OpView ov{};
  ov.kind = nullptr; ov.kind0 = PHIP_OP_RECEIVE;
  ov.now = nullptr; ov.now0 = now;
  ov.a = a + k; ov.t = t + k; ov.e = e + k;
  return ordered(h, shifted(src, k), stop - k, ov, shifted(ow, k));
}

// A checked batch (names_len) whose first malformed name entry is message
// `stop` < n (k_classify_soa2, ctr[5]) stopped there, as the Go loop stops at
// a short datagram (repo.go:70-74): that message reads PHIP_ST_SHORT, every
// later one PHIP_ST_NOT_PROCESSED, and the call returns PHIP_ERR_INVALID.
int stopped_at_bad_name(phip_handle* h, const OutView& ow, u32 n, u32 stop) {
  if (stop >= n) return PHIP_OK;
  if (ow.status) {
    HIPCHK(h, hipMemsetAsync(ow.status + stop, PHIP_ST_NOT_PROCESSED, n - stop, h->stream));
    HIPCHK(h, hipMemsetAsync(ow.status + stop, PHIP_ST_SHORT, 1, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  return set_err(h, PHIP_ERR_INVALID,
                 "malformed name offsets at message %u (names_len check): the batch stopped there",
                 stop);
}

// Receive-mode batch (decoded): the fast path over its clean prefix, the
// ordered path from its first incast or -0.0 on.
template <class Src>
int receive_decoded(phip_handle* h, Src src, const uint64_t* a, const uint64_t* t,
                    const int64_t* e, u32 n, i64 now, const OutView& ow) {
  int rc;
  // The hot directory (read-only on the table and the batch) is built on
  // stream2 while the batch is classified.
  u32 fd = n, nmiss = 0;
  if ((rc = fast_apply(h, SoaIn<Src>{src, a, t, e}, src, n, ow.status, &fd, &nmiss))) return rc;
  const u32 stop = std::min<u32>(h->ctr_host[5], n);   // (a checked batch's malformed entry)
  if ((rc = finish_receive(h, src, a, t, e, stop, fd, nmiss, now, ow, n, h->ndef != 0)))
    return rc;
  return stopped_at_bad_name(h, ow, n, stop);
}

// PHIP_RECV_ASYNC: the queued batch's counters, then what its fast pass left
// (misses, dirty buckets).  *worked: whether anything was left (its work
// has used the counters and maybe moved the table).
int finish_pending(phip_handle* h, bool* worked) {
  if (worked) *worked = false;
  if (!h->pend.active) return PHIP_OK;
  const phip_handle::Pending p = h->pend;
  h->pend.active = false;
  HIPCHK(h, hipEventSynchronize(h->ev_ctr));
  u32 fd = p.n, nmiss = 0;
  int rc;
  if ((rc = fast_collect(h, p.n, p.par, &fd, &nmiss, p.iso))) return rc;
  const u32 stop = std::min<u32>(h->ctr_host[5], p.n);   // (a checked batch's malformed entry)
  const bool deferred = h->ndef != 0;
  if (nmiss == 0 && fd >= stop && !deferred) return stopped_at_bad_name(h, p.ow, p.n, stop);
  if (worked) *worked = true;
  if ((rc = finish_receive(h, p.src, p.a, p.t, p.e, stop, fd, nmiss, p.now, p.ow, p.n,
                           deferred)) ||
      (rc = stopped_at_bad_name(h, p.ow, p.n, stop)))
    return rc;
  // The leftover work (the miss merges, the ordered path's folds, which also
  // join stream2/stream4 into the handle's stream) writes this batch's
  // statuses and replies: they are final when the call that finished the
  // batch returns (patrolhip.h PHIP_RECV_ASYNC), and the caller may then
  // free or reuse them.  Only batches that left work pay this wait.
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

// Whether an op's phip_results.reply entry is written (step_sop): Takes,
// Upserts and incast requests carry the bucket's state right after the op.
inline bool has_reply_state(u8 status, u8 kind) {
  const u8 st = status & 0x7F;
  return kind == PHIP_OP_TAKE || kind == PHIP_OP_UPSERT || st == PHIP_ST_INCAST_REPLY ||
         st == PHIP_ST_INCAST_NOREPLY;
}

// A host-pointer batch of at most kSmallMax ops through k_small_mixed: one
// pinned copy in, one launch, one pinned copy out (the large path takes a
// dozen launches and several host round trips, ~0.2 ms whatever the size).
// *done = false leaves the batch to the large path with nothing changed: too
// many ops or name bytes, a bucket bound past the load limit (the large path
// grows the table), or a long-name arena the kernel found too small.
int small_mixed(phip_handle* h, const phip_ops* ops, const phip_results* res, bool* done) {
  *done = false;
  const u32 n = ops->n;
  if (n > kSmallMax || h->n_buckets + n > h->max_load) return PHIP_OK;
  const u64 nbytes = ops->name_offs[n];
  if (nbytes > (u64)kSmallMax * PHIP_MAX_NAME_LEN) return PHIP_OK;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const bool take = ops->freq != nullptr, state = ops->added != nullptr;
  // inputs: offsets | kind | now | freq per count | added taken elapsed | names
  const size_t o_kind = al(4 * ((size_t)n + 1)), o_now = o_kind + al(n), o_freq = o_now + 8 * n;
  const size_t o_per = o_freq + 8 * n, o_count = o_per + 8 * n, o_a = o_count + 8 * n;
  const size_t o_t = o_a + 8 * n, o_e = o_t + 8 * n, o_names = o_e + 8 * n;
  const size_t in_bytes = al(o_names + nbytes + 8);
  // outputs: header | status | remaining | have | reply
  const size_t o_st = sizeof(SmallHdr), o_rem = al(o_st + n), o_have = o_rem + 8 * n;
  const size_t o_reply = o_have + 8 * n, out_bytes = o_reply + sizeof(phip_state) * n;
  const size_t total = in_bytes + out_bytes;
  if (h->small_pin_cap < total) {
    if (h->small_pin) HIPCHK(h, hipHostFree(h->small_pin));
    h->small_pin = nullptr;
    h->small_pin_cap = 0;
    const size_t want = std::max<size_t>(total, 1 << 20);
    HIPCHK(h, hipHostMalloc(&h->small_pin, want, 0));
    h->small_pin_cap = want;
  }
  u8 *d = nullptr, *pin = h->small_pin;
  int rc;
  if ((rc = ensure(h, B_SMALL, total, &d))) return rc;
  std::memcpy(pin, ops->name_offs, 4 * ((size_t)n + 1));
  std::memcpy(pin + o_kind, ops->kind, n);
  std::memcpy(pin + o_now, ops->now, 8 * n);
  if (take) {
    std::memcpy(pin + o_freq, ops->freq, 8 * n);
    std::memcpy(pin + o_per, ops->per, 8 * n);
    std::memcpy(pin + o_count, ops->count, 8 * n);
  }
  if (state) {
    std::memcpy(pin + o_a, ops->added, 8 * n);
    std::memcpy(pin + o_t, ops->taken, 8 * n);
    std::memcpy(pin + o_e, ops->elapsed, 8 * n);
  }
  std::memcpy(pin + o_names, ops->names, nbytes);
  std::memset(pin + o_names + nbytes, 0, 8);
  std::memset(pin + in_bytes, 0, sizeof(SmallHdr));
  HIPCHK(h, hipMemcpyAsync(d, pin, in_bytes + sizeof(SmallHdr), hipMemcpyHostToDevice, h->stream));
  NamesOffs src{d + o_names, (const u32*)d};
  OpView ov{};
  ov.kind = d + o_kind;
  ov.now = (const int64_t*)(d + o_now);
  if (take) {
    ov.freq = (const int64_t*)(d + o_freq);
    ov.per = (const int64_t*)(d + o_per);
    ov.count = (const uint64_t*)(d + o_count);
  }
  if (state) {
    ov.a = (const uint64_t*)(d + o_a);
    ov.t = (const uint64_t*)(d + o_t);
    ov.e = (const int64_t*)(d + o_e);
  }
  u8* dout = d + in_bytes;
  phip_results r{};
  if (res) r = *res;
  OutView ow{};
  ow.status = r.status ? dout + o_st : nullptr;
  ow.remaining = r.remaining ? (uint64_t*)(dout + o_rem) : nullptr;
  ow.have = r.have ? (uint64_t*)(dout + o_have) : nullptr;
  ow.reply = r.reply ? (phip_state*)(dout + o_reply) : nullptr;
  {
    Launch l(h, "k_small_mixed");
    k_small_mixed<<<1, kSmallMax, 0, h->stream>>>(src, ov, n, table(h), h->arena, h->arena_cap,
                                                  h->arena_cursor, ow, (SmallHdr*)dout);
  }
  HIPCHK(h, hipGetLastError());
  // the header and the columns the caller asked for, in one copy
  const size_t back = r.reply ? out_bytes : r.have ? o_reply : r.remaining ? o_have : o_rem;
  u8* pout = pin + in_bytes;
  HIPCHK(h, hipMemcpyAsync(pout, dout, back, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  SmallHdr hd;
  std::memcpy(&hd, pout, sizeof hd);
  h->n_buckets += hd.created;
  if (hd.fallback) return PHIP_OK;
  if (hd.full) return set_err(h, PHIP_ERR_FULL, "internal: small batch probe wrapped the table");
  if (r.status) std::memcpy(r.status, pout + o_st, n);
  if (r.remaining) std::memcpy(r.remaining, pout + o_rem, 8 * n);
  if (r.have) std::memcpy(r.have, pout + o_have, 8 * n);
  if (r.reply) {
    // reply states are defined for Takes, Upserts and incasts (step_sop);
    // the other entries read as zeros, as on the large path (outputs())
    const phip_state* src_r = (const phip_state*)(pout + o_reply);
    std::vector<u8> st;
    const u8* stp = r.status;
    if (!stp) {
      st.assign(n, 0);
      HIPCHK(h, hipMemcpy(st.data(), dout + o_st, n, hipMemcpyDeviceToHost));
      stp = st.data();
    }
    for (u32 i = 0; i < n; ++i)
      r.reply[i] = has_reply_state(stp[i], ops->kind ? ops->kind[i] : (u8)PHIP_OP_RECEIVE)
                       ? src_r[i] : phip_state{};
  }
  *done = true;
  return PHIP_OK;
}


// A uniform-kind host batch (Receive or Upsert of decoded states, all at one
// clock reading) through small_mixed: the ordered code is the same Go loop
// (repo.go:78-90, :215-235), so statuses, replies and states are those of
// the large paths.
int small_uniform(phip_handle* h, const phip_msgs* m, u8 kind, int64_t now, const phip_results* res,
                  bool* done) {
  *done = false;
  if (!h->small || m->n > kSmallMax) return PHIP_OK;
  std::vector<u8> kinds(m->n, kind);
  std::vector<int64_t> nows(m->n, now);
  phip_ops ops{};
  ops.n = m->n;
  ops.kind = kinds.data();
  ops.names = m->names;
  ops.name_offs = m->name_offs;
  ops.now = nows.data();
  ops.added = m->added;
  ops.taken = m->taken;
  ops.elapsed = m->elapsed;
  return small_mixed(h, &ops, res, done);
}

// ReplicatedRepo.Receive over at most kSmallMax host datagrams: decoded on
// the host (UnmarshalBinary, bucket.go:71-91: a datagram under 25 bytes or
// shorter than its name is io.ErrShortBuffer, where the Go loop stops), the
// prefix before the first short one through small_mixed.
int small_datagrams(phip_handle* h, const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                    int64_t now, const phip_results* res, uint32_t* stop_index, bool* done) {
  *done = false;
  if (!h->small || n > kSmallMax) return PHIP_OK;
  std::vector<uint64_t> a(n), t(n);
  std::vector<int64_t> e(n);
  std::vector<uint32_t> no(n + 1);
  std::vector<uint8_t> names;
  names.reserve((size_t)n * 16 + 8);
  auto be64 = [](const uint8_t* p) {
    uint64_t v = 0;
    for (int k = 0; k < 8; ++k) v = (v << 8) | p[k];
    return v;
  };
  u32 stop = n;
  for (u32 i = 0; i < n; ++i) {
    const uint8_t* d = bytes + offs[i];
    const uint64_t sz = offs[i + 1] - offs[i];
    if (sz < PHIP_BUCKET_FIXED_SIZE || sz - PHIP_BUCKET_FIXED_SIZE < d[24]) { stop = i; break; }
    a[i] = be64(d);
    t[i] = be64(d + 8);
    e[i] = (int64_t)be64(d + 16);
    no[i] = (uint32_t)names.size();
    names.insert(names.end(), d + PHIP_BUCKET_FIXED_SIZE, d + PHIP_BUCKET_FIXED_SIZE + d[24]);
  }
  no[stop] = (uint32_t)names.size();
  names.resize(names.size() + 8, 0);
  if (stop) {
    phip_msgs m{};
    m.n = stop;
    m.names = names.data();
    m.name_offs = no.data();
    m.added = a.data();
    m.taken = t.data();
    m.elapsed = e.data();
    bool ok = false;
    int rc;
    if ((rc = small_uniform(h, &m, PHIP_OP_RECEIVE, now, res, &ok))) return rc;
    if (!ok) return PHIP_OK;   // the large path takes the whole batch
  }
  if (res && res->status && stop < n) {   // the short datagram and everything after it
    std::memset(res->status + stop, PHIP_ST_NOT_PROCESSED, n - stop);
    res->status[stop] = PHIP_ST_SHORT;
  }
  if (stop_index) *stop_index = stop;
  *done = true;
  if (stop < n) return set_err(h, PHIP_ERR_SHORT_BUFFER, "short buffer at datagram %u", stop);
  return PHIP_OK;
}
}  // namespace

// ------------------------------------------------------- owner routing ----
// The pack of phip_route_pack (and of phip_group_receive's chunks), queued on
// stream `st` without a host synchronisation.
// One workgroup per tile of `span` messages.  12 workgroups
// per CU: k_route_count holds 4 per CU, k_route_scatter 3, so both grids run
// in whole rounds (no tail round of a quarter of the chip).
// (tiles per CU: 12 = whole rounds of both grids; fewer, longer tiles also
// mean fewer combined messages, one per hot name a workgroup saw)
#ifndef PHIP_ROUTE_WG_PER_CU
#define PHIP_ROUTE_WG_PER_CU 12
#endif
struct RoutePlan {
  u32 nblk, ntile, span;
  size_t cells;
};
static RoutePlan route_plan(const phip_handle* h, u32 n, u32 world) {
  RoutePlan p;
  p.nblk = (u32)std::max<u64>(1, std::min<u64>((n + kRouteStep - 1) / kRouteStep,
                                                (u64)h->ncu * PHIP_ROUTE_WG_PER_CU));
  p.ntile = p.nblk;   // one tile per workgroup, a whole number of scatter steps
  p.span = (u32)((((u64)n + p.ntile - 1) / p.ntile + kRouteStep - 1) / kRouteStep * kRouteStep);
  p.cells = (size_t)world * p.ntile;
  return p;
}

// Scratch of a pack of up to n messages, all in B_ROUTE: the per-(owner,
// tile) cells, the route codes, its own counter block and the scans'
// temporary storage.  Sized before anything is queued: the packs of a
// pipelined exchange reuse it in stream order, and the owner's merges that
// run beside them (phip_group_receive) touch none of it.
static int route_scratch(phip_handle* h, u32 n, u32 world, u8** base, u32** pctr, size_t* scan_bytes,
                         u8** temp) {
  const RoutePlan p = route_plan(h, n, world);
  size_t tb = 0;
  HIPCHK(h, rocprim::exclusive_scan(nullptr, tb, (u32*)nullptr, (u32*)nullptr, 0u, p.cells,
                                    rocprim::plus<u32>(), h->stream));
  // cells | codes | counter block | scan temp (16-byte aligned parts)
  const size_t ctr_off = (4 * p.cells * sizeof(u32) + 2 * (size_t)n + 15) & ~(size_t)15;
  const size_t tmp_off = (ctr_off + kCtrWords * sizeof(u32) + 255) & ~(size_t)255;
  int rc;
  if ((rc = ensure(h, B_ROUTE, tmp_off + tb, base))) return rc;
  *pctr = (u32*)(*base + ctr_off);
  *scan_bytes = tb;
  *temp = *base + tmp_off;
  return PHIP_OK;
}

// Sender-side combine: the hot names of a strided sample of the
// whole batch, counted by name hash (the buckets live on other ranks, so
// there is no slot to count), as a directory for every pack of the batch.
static int route_dir_on(phip_handle* h, hipStream_t st, const phip_msgs& m, u32 world, const void** out) {
  *out = nullptr;
  const u32 n = m.n;
  if (n < kRouteMinBatch) return PHIP_OK;
  constexpr size_t kCnt = size_t(1) << kHotCntBits;
  const size_t zero_bytes = 3 * kCnt * sizeof(u32) + kHotHist * sizeof(u32) + sizeof(HotHdr);
  u8* hb;
  int rc;
  if ((rc = ensure(h, B_RHOT, zero_bytes + kRouteHotMax * sizeof(RouteHot), &hb))) return rc;
  u32* ckeys = (u32*)hb;
  u32* ccnt = ckeys + kCnt;
  u32* cidx = ccnt + kCnt;
  u32* hist = cidx + kCnt;
  HotHdr* hdr = (HotHdr*)(hist + kHotHist);
  RouteHot* d = (RouteHot*)(hdr + 1);
  HIPCHK(h, hipMemsetAsync(hb, 0, zero_bytes, st));
  const u32 stride = std::max<u32>(64, (n + kHotSampleMax - 1) / kHotSampleMax);
  const u32 nsample = (n + stride - 1) / stride;
  NamesOffs src{m.names, m.name_offs, m.names_len};
  {
    Launch l(h, "k_route_sample", st);
    k_route_sample<NamesOffs><<<grid_for(nsample, kHotSamplePerBlock), 256, 0, st>>>(
        src, n, stride, nsample, ckeys, ccnt, cidx);
    k_hot_hist<<<grid_for(kCnt), kBlock, 0, st>>>(ccnt, hist);
    k_hot_select<<<1, 256, 0, st>>>(hist, hdr, kRouteHotMax);
    k_route_dir_build<NamesOffs><<<grid_for(kCnt), kBlock, 0, st>>>(ckeys, ccnt, cidx, hdr, src,
                                                                     world, d);
  }
  HIPCHK(h, hipGetLastError());
  *out = hdr;
  return PHIP_OK;
}

// Stable owner partition of m's messages into owner-major send buffers, the
// per-owner totals into counts / nbytes (device).  With a directory (dir) a
// clean batch's hot names are max-combined (k_route_count classifies the
// batch on the way; a dirty one is counted again without combining).
static int route_pack_on(phip_handle* h, hipStream_t st, const phip_msgs& m, u32 world, const void* dir,
                  uint8_t* send_names, uint32_t* send_lens, uint64_t* send_added,
                  uint64_t* send_taken, int64_t* send_elapsed, uint64_t* counts,
                  uint64_t* nbytes) {
  const u32 n = m.n;
  if (n == 0) {
    HIPCHK(h, hipMemsetAsync(counts, 0, world * sizeof(uint64_t), st));
    HIPCHK(h, hipMemsetAsync(nbytes, 0, world * sizeof(uint64_t), st));
    return PHIP_OK;
  }
  const RoutePlan p = route_plan(h, n, world);
  u8 *base, *temp;
  u32* pctr;
  size_t tb;
  int rc;
  if ((rc = route_scratch(h, n, world, &base, &pctr, &tb, &temp))) return rc;
  u32* cnt = (u32*)base;
  u32* bytes = cnt + p.cells;
  u32* cbase = bytes + p.cells;
  u32* bbase = cbase + p.cells;
  u16* code = (u16*)(bbase + p.cells);
  const HotHdr* hot = (const HotHdr*)dir;
  const RouteHot* rdir = hot ? (const RouteHot*)(hot + 1) : nullptr;
  NamesOffs src{m.names, m.name_offs, m.names_len};
  k_batch_reset<<<1, kShards, 0, st>>>(pctr, nullptr);
  {
    Launch l(h, "k_route_count", st);
    k_route_count<NamesOffs><<<p.nblk, kRouteBlock, 0, st>>>(
        src, m.added, m.taken, m.elapsed, n, p.span, world, p.ntile, hot, rdir, pctr, code, cnt,
        bytes, hot ? kRouteCombine : kRoutePlain);
    if (hot)
      k_route_count<NamesOffs><<<p.nblk, kRouteBlock, 0, st>>>(
          src, m.added, m.taken, m.elapsed, n, p.span, world, p.ntile, hot, rdir, pctr, code, cnt,
          bytes, kRouteRecount);
  }
  HIPCHK(h, hipGetLastError());
  {
    Launch l(h, "route_scan", st);
    HIPCHK(h, rocprim::exclusive_scan(temp, tb, cnt, cbase, 0u, p.cells, rocprim::plus<u32>(), st));
    HIPCHK(h, rocprim::exclusive_scan(temp, tb, bytes, bbase, 0u, p.cells, rocprim::plus<u32>(), st));
  }
  {
    Launch l(h, "k_route_scatter", st);
    k_route_scatter<NamesOffs><<<p.nblk, kRouteBlock, 0, st>>>(
        src, m.added, m.taken, m.elapsed, n, p.span, world, p.ntile, hot, rdir, pctr, code, cbase,
        bbase, send_names, send_lens, send_added, send_taken, send_elapsed);
  }
  k_route_totals<<<1, kRouteMaxWorld, 0, st>>>(cnt, bytes, cbase, bbase, p.ntile, world, counts,
                                               nbytes);
  HIPCHK(h, hipGetLastError());
  return PHIP_OK;
}

// ===================================================================== ABI
extern "C" {

int phip_abi_version(void) { return PHIP_ABI_VERSION; }

// phip_build_id: patrol_amd/Makefile links it from build/build_id.o (a hash
// of every source and the flags); single-command builds of the sources
// (tools/build_variants.sh) name theirs with -DPHIP_BUILD_ID.
#ifdef PHIP_BUILD_ID
const char* phip_build_id(void) { return PHIP_BUILD_ID; }
#endif

int phip_open(const phip_config* cfg, phip_handle** out) {
  if (!cfg || !out) return PHIP_ERR_INVALID;
  *out = nullptr;
  if (cfg->log2_slots < 4 || cfg->log2_slots > 31) return PHIP_ERR_INVALID;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PHIP_ERR_NO_DEVICE;
  if (cfg->device < 0 || cfg->device >= ndev) return PHIP_ERR_NO_DEVICE;
  phip_handle* h = new phip_handle;
  h->device = cfg->device;
  h->L = cfg->log2_slots;
  h->cap = 1ull << h->L;
  h->load_pct = cfg->max_load_pct ? std::min<u32>(cfg->max_load_pct, 95) : 90;
  h->max_load = load_limit(h->cap, h->load_pct);
  h->grow = !(cfg->flags & PHIP_CFG_NO_GROW);
  h->iso_always = cfg->flags & PHIP_CFG_ISOLATE;
  h->small = !(cfg->flags & PHIP_CFG_NO_SMALL);
  h->arena_cap = cfg->arena_bytes ? cfg->arena_bytes : (1ull << 20);
  if (cfg->debug_tag_bits && cfg->debug_tag_bits < 64) h->tag_mask = (1ull << cfg->debug_tag_bits) - 1;
  if (cfg->flags & PHIP_CFG_FIXED_SEED) {
    h->seed = cfg->hash_seed;
  } else if (getrandom(&h->seed, sizeof h->seed, 0) != (ssize_t)sizeof h->seed) {
    // no entropy source: a seed from the clock and the handle's address
    h->seed = seeded_mix((u64)std::chrono::steady_clock::now().time_since_epoch().count(),
                         (u64)(uintptr_t)h);
  }
  auto fail = [&](hipError_t e) {
    phip_close(h);
    (void)e;
    return PHIP_ERR_HIP;
  };
  hipError_t e;
  if ((e = hipSetDevice(h->device)) != hipSuccess) return fail(e);
  if ((e = hipDeviceGetAttribute(&h->ncu, hipDeviceAttributeMultiprocessorCount, h->device)) !=
      hipSuccess)
    return fail(e);
  if ((e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(e);
  h->stream = h->own_stream;
  if ((e = hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking)) != hipSuccess) return fail(e);
  if ((e = hipStreamCreateWithFlags(&h->stream3, hipStreamNonBlocking)) != hipSuccess) return fail(e);
  if ((e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming)) != hipSuccess) return fail(e);
  if ((e = hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming)) != hipSuccess) return fail(e);
  if ((e = hipEventCreateWithFlags(&h->ev_fork3, hipEventDisableTiming)) != hipSuccess) return fail(e);
  if ((e = hipEventCreateWithFlags(&h->ev_join3, hipEventDisableTiming)) != hipSuccess) return fail(e);
  if ((e = hipEventCreateWithFlags(&h->ev_gather, hipEventDisableTiming)) != hipSuccess) return fail(e);
  if ((e = hipEventCreateWithFlags(&h->ev_gather3, hipEventDisableTiming)) != hipSuccess)
    return fail(e);
  if ((e = hipEventCreateWithFlags(&h->ev_pack, hipEventDisableTiming)) != hipSuccess) return fail(e);
  if ((e = hipEventCreateWithFlags(&h->ev_ctr, hipEventDisableTiming)) != hipSuccess) return fail(e);
  if ((e = hipMalloc(&h->recs, h->cap * sizeof(Rec))) != hipSuccess) return fail(e);
  if ((e = hipMalloc(&h->aux, h->cap * sizeof(u32))) != hipSuccess) return fail(e);
  if ((e = hipMalloc(&h->arena, h->arena_cap + 64)) != hipSuccess) return fail(e);
  if ((e = hipMalloc(&h->arena_cursor, 64)) != hipSuccess) return fail(e);
  if ((e = hipMalloc(&h->ctr, 3 * kCtrWords * sizeof(u32))) != hipSuccess) return fail(e);
  if ((e = hipHostMalloc(&h->ctr_host, kCtrWords * sizeof(u32),
                         hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
      (e = hipHostGetDevicePointer((void**)&h->ctr_map, h->ctr_host, 0)) != hipSuccess)
    return fail(e);
  if ((e = hipMemsetAsync(h->recs, 0, h->cap * sizeof(Rec), h->stream)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(h->aux, 0, h->cap * sizeof(u32), h->stream)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(h->arena_cursor, 0, 64, h->stream)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(h->ctr, 0, 3 * kCtrWords * sizeof(u32), h->stream)) != hipSuccess)
    return fail(e);
  if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return fail(e);
  *out = h;
  return PHIP_OK;
}

void phip_close(phip_handle* h) {
  // Teardown is best effort: every resource is released whatever the
  // earlier calls return.
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->pend.active) (void)after_error(h, finish_pending(h));   // a queued PHIP_RECV_ASYNC batch
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->stream2) (void)hipStreamSynchronize(h->stream2);
  if (h->stream3) (void)hipStreamSynchronize(h->stream3);
  if (h->stream4) (void)hipStreamSynchronize(h->stream4);
  for (auto& b : h->buf)
    if (b.p) (void)hipFree(b.p);
  for (auto& t : h->event_pool) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  if (h->recs) (void)hipFree(h->recs);
  if (h->aux) (void)hipFree(h->aux);
  if (h->arena) (void)hipFree(h->arena);
  if (h->arena_cursor) (void)hipFree(h->arena_cursor);
  if (h->ctr) (void)hipFree(h->ctr);
  if (h->ctr_host) (void)hipHostFree(h->ctr_host);
  if (h->small_pin) (void)hipHostFree(h->small_pin);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->ev_fork3) (void)hipEventDestroy(h->ev_fork3);
  if (h->ev_join3) (void)hipEventDestroy(h->ev_join3);
  if (h->ev_gather) (void)hipEventDestroy(h->ev_gather);
  if (h->ev_gather3) (void)hipEventDestroy(h->ev_gather3);
  if (h->ev_pack) (void)hipEventDestroy(h->ev_pack);
  if (h->ev_ctr) (void)hipEventDestroy(h->ev_ctr);
  if (h->stream2) (void)hipStreamDestroy(h->stream2);
  if (h->stream3) (void)hipStreamDestroy(h->stream3);
  if (h->stream4) (void)hipStreamDestroy(h->stream4);
  if (h->ev_t4a) (void)hipEventDestroy(h->ev_t4a);
  if (h->ev_t4b) (void)hipEventDestroy(h->ev_t4b);
  if (h->own_stream) {
    (void)hipStreamSynchronize(h->own_stream);
    (void)hipStreamDestroy(h->own_stream);
  }
  delete h;
}

const char* phip_last_error(const phip_handle* h) { return h ? h->err.c_str() : "null handle"; }

int phip_flush(phip_handle* h) {
  if (!h) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;   // (finishes a queued PHIP_RECV_ASYNC batch)
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

// (a queued PHIP_RECV_ASYNC batch is finished first: its new buckets count)
// (their own result carries no status: a queued batch's error is kept for the
// handle's next call that returns one)
uint64_t phip_len(phip_handle* h) {
  if (!h) return 0;
  std::lock_guard<std::mutex> g(h->mu);
  if (!h->deferred_rc) h->deferred_rc = begin_call(h);
  return h->n_buckets;
}
uint64_t phip_capacity(phip_handle* h) {
  if (!h) return 0;
  std::lock_guard<std::mutex> g(h->mu);
  if (!h->deferred_rc) h->deferred_rc = begin_call(h);
  return h->cap;
}

int phip_seed(phip_handle* h, const uint8_t* names, const uint32_t* name_offs, uint32_t n,
              const phip_state* states, uint32_t flags) {
  if (!h || (n && (!names || !name_offs || !states))) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  if (n == 0) return PHIP_OK;
  bool dev = flags & PHIP_DEVICE_PTRS;
  if (!dev && !names_ok(name_offs, n)) return set_err(h, PHIP_ERR_NAME_TOO_LARGE, "name > 231 bytes");
  int rc;
  NamesOffs src;
  if ((rc = stage_names(h, names, name_offs, n, dev, &src))) return rc;
  const phip_state* d_st;
  if ((rc = stage(h, B_STATES, states, n, dev, &d_st))) return rc;
  u32* slot;
  u32 n_claimed = 0;
  if ((rc = resolve_all(h, src, n, nullptr, 0, &slot, &n_claimed))) return after_error(h, rc);
  // aux is the per-slot "last writer" scratch: clear, pick the last entry of
  // each name, apply it, clear again.
  k_seed_finish<<<grid_for(n), kBlock, 0, h->stream>>>(slot, n, table(h));
  k_seed_pick<<<grid_for(n), kBlock, 0, h->stream>>>(slot, n, table(h));
  k_seed_apply<<<grid_for(n), kBlock, 0, h->stream>>>(slot, n, d_st, table(h));
  k_seed_finish<<<grid_for(n), kBlock, 0, h->stream>>>(slot, n, table(h));
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int phip_get(phip_handle* h, const uint8_t* name, uint32_t len, phip_state* out) {
  if (!h || (!name && len) || !out) return PHIP_ERR_INVALID;
  if (len > PHIP_MAX_NAME_LEN) return 0;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  u8* d_name;
  Rec* d_rec;
  int rc;
  if ((rc = ensure(h, B_NAME1, 256 + sizeof(Rec) + 16, &d_name))) return rc;
  d_rec = (Rec*)(d_name + 256);
  int* d_found = (int*)(d_name + 256 + sizeof(Rec));
  if (len) HIPCHK(h, hipMemcpyAsync(d_name, name, len, hipMemcpyHostToDevice, h->stream));
  k_get_one<<<1, 64, 0, h->stream>>>(d_name, len, table(h), d_rec, d_found);
  HIPCHK(h, hipGetLastError());
  Rec r;
  int found = 0;
  HIPCHK(h, hipMemcpyAsync(&r, d_rec, sizeof(Rec), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipMemcpyAsync(&found, d_found, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (!found) return 0;
  out->added = dec_f64(r.added);
  out->taken = dec_f64(r.taken);
  out->elapsed = r.elapsed;
  out->created = r.created;
  return 1;
}

// Snapshot image: header, the 2^L slot records as they lie in HBM, then the
// used part of the long-name arena.  Restoring it into a handle of the same
// table size reproduces the table exactly (slots, probe chains, arena
// offsets), with no rehash.
struct SnapHeader {
  char magic[8];
  u32 abi, log2_slots;
  u64 n_buckets, arena_used, rec_bytes, reserved[3];
};
static_assert(sizeof(SnapHeader) == 64, "snapshot header");
constexpr char kSnapMagic[8] = {'P', 'H', 'I', 'P', 'S', 'N', 'P', '1'};

static u64 arena_used(phip_handle* h) {
  u64 used = 0;
  if (hipMemcpyAsync(&used, h->arena_cursor, sizeof(u64), hipMemcpyDeviceToHost, h->stream) !=
          hipSuccess ||
      hipStreamSynchronize(h->stream) != hipSuccess)
    return ~0ull;
  return std::min<u64>(used, h->arena_cap);
}

uint64_t phip_snapshot_bytes(phip_handle* h) {
  if (!h) return 0;
  std::lock_guard<std::mutex> g(h->mu);
  if (begin_call(h)) return 0;
  const u64 used = arena_used(h);
  if (used == ~0ull) return 0;
  return sizeof(SnapHeader) + h->cap * sizeof(Rec) + used;
}

int phip_snapshot(phip_handle* h, uint8_t* out, uint64_t cap) {
  if (!h || !out) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  const u64 used = arena_used(h);
  if (used == ~0ull) return set_err(h, PHIP_ERR_HIP, "snapshot: arena cursor read failed");
  const u64 need = sizeof(SnapHeader) + h->cap * sizeof(Rec) + used;
  if (cap < need) return set_err(h, PHIP_ERR_INVALID, "snapshot needs %llu bytes", (unsigned long long)need);
  SnapHeader hd{};
  std::memcpy(hd.magic, kSnapMagic, 8);
  hd.abi = PHIP_ABI_VERSION;
  hd.log2_slots = h->L;
  hd.n_buckets = h->n_buckets;
  hd.arena_used = used;
  hd.rec_bytes = sizeof(Rec);
  hd.reserved[0] = h->seed;   // the records lie where this seed placed them
  std::memcpy(out, &hd, sizeof hd);
  u8* p = out + sizeof hd;
  HIPCHK(h, hipMemcpyAsync(p, h->recs, h->cap * sizeof(Rec), hipMemcpyDeviceToHost, h->stream));
  if (used) HIPCHK(h, hipMemcpyAsync(p + h->cap * sizeof(Rec), h->arena, used, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int phip_restore(phip_handle* h, const uint8_t* in, uint64_t len) {
  if (!h || !in || len < sizeof(SnapHeader)) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  SnapHeader hd;
  std::memcpy(&hd, in, sizeof hd);
  if (std::memcmp(hd.magic, kSnapMagic, 8) || hd.abi != PHIP_ABI_VERSION || hd.rec_bytes != sizeof(Rec))
    return set_err(h, PHIP_ERR_INVALID, "not a snapshot of this ABI");
  if (hd.log2_slots < 4 || hd.log2_slots > 31)
    return set_err(h, PHIP_ERR_INVALID, "snapshot of 2^%u slots", hd.log2_slots);
  const u64 scap = 1ull << hd.log2_slots;
  if (len != sizeof hd + scap * sizeof(Rec) + hd.arena_used)
    return set_err(h, PHIP_ERR_INVALID, "snapshot truncated");
  if (hd.n_buckets > load_limit(scap, h->load_pct))
    return set_err(h, PHIP_ERR_FULL, "snapshot above the handle's load limit");
  if (hd.arena_used > h->arena_cap) {
    if (!h->grow) return set_err(h, PHIP_ERR_ARENA, "snapshot arena larger than the handle's");
    if (int rc = grow_arena(h, 0, hd.arena_used)) return rc;
  }
  if (hd.log2_slots != h->L) {
    // The image's table size wins (the table may have grown since it was
    // opened): the handle's table is replaced by one of that size.
    Rec* nrecs = nullptr;
    u32* naux = nullptr;
    if (hipMalloc(&nrecs, scap * sizeof(Rec)) != hipSuccess ||
        hipMalloc(&naux, scap * sizeof(u32)) != hipSuccess) {
      (void)hipGetLastError();
      if (nrecs) (void)hipFree(nrecs);
      return set_err(h, PHIP_ERR_FULL, "restore: no device memory for 2^%u slots", hd.log2_slots);
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipFree(h->recs));
    HIPCHK(h, hipFree(h->aux));
    h->recs = nrecs;
    h->aux = naux;
    h->L = hd.log2_slots;
    h->cap = scap;
    h->max_load = load_limit(scap, h->load_pct);
  }
  const u8* p = in + sizeof hd;
  HIPCHK(h, hipMemcpyAsync(h->recs, p, h->cap * sizeof(Rec), hipMemcpyHostToDevice, h->stream));
  if (hd.arena_used)
    HIPCHK(h, hipMemcpyAsync(h->arena, p + h->cap * sizeof(Rec), hd.arena_used, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemsetAsync(h->aux, 0, h->cap * sizeof(u32), h->stream));
  HIPCHK(h, hipMemcpyAsync(h->arena_cursor, &hd.arena_used, sizeof(u64), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->n_buckets = hd.n_buckets;
  h->seed = hd.reserved[0];   // the image's placement
  return PHIP_OK;
}

int phip_export_datagrams(phip_handle* h, const uint8_t* names, const uint32_t* name_offs,
                          uint32_t n, uint8_t* out, uint8_t* found, uint32_t flags) {
  if (!h || (n && (!names || !name_offs || !out || !found))) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  if (n == 0) return PHIP_OK;
  const bool dev = flags & PHIP_DEVICE_PTRS;
  if (!dev && !names_ok(name_offs, n)) return set_err(h, PHIP_ERR_NAME_TOO_LARGE, "name > 231 bytes");
  int rc;
  NamesOffs src;
  if ((rc = stage_names(h, names, name_offs, n, dev, &src))) return rc;
  const size_t nbytes = dev ? 0 : (size_t)PHIP_BUCKET_FIXED_SIZE * n + (name_offs[n] - name_offs[0]);
  u8 *d_out, *d_found;
  if ((rc = out_buf(h, B_EXPORT, out, nbytes, dev, &d_out)) ||
      (rc = out_buf(h, B_STATUS, found, n, dev, &d_found)))
    return rc;
  {
    Launch l(h, "k_export");
    k_export<<<grid_for(n), kBlock, 0, h->stream>>>(src, n, table(h), d_out, d_found);
  }
  HIPCHK(h, hipGetLastError());
  if ((rc = copy_back(h, out, d_out, nbytes, dev)) || (rc = copy_back(h, found, d_found, n, dev)))
    return rc;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int phip_dump(phip_handle* h, uint8_t* names, uint64_t names_cap, uint64_t* name_offs,
              phip_state* states, uint64_t max_n, uint64_t* n_out, uint64_t* names_bytes_out) {
  if (!h) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  int rc;
  u32* list;
  // count the occupied slots first, then size the list by that count
  if ((rc = reset_ctr(h))) return rc;
  k_dump_collect<<<grid_for(h->cap), kBlock, 0, h->stream>>>(h->recs, h->cap, nullptr, h->ctr);
  HIPCHK(h, hipGetLastError());
  if ((rc = read_ctr(h))) return rc;
  const u32 occupied = h->ctr_host[2];
  if ((rc = ensure(h, B_DUMP, (size_t)occupied + 1, &list))) return rc;
  if ((rc = reset_ctr(h))) return rc;
  k_dump_collect<<<grid_for(h->cap), kBlock, 0, h->stream>>>(h->recs, h->cap, list, h->ctr);
  HIPCHK(h, hipGetLastError());
  if ((rc = read_ctr(h))) return rc;
  u32 n = h->ctr_host[2];
  if (n != occupied) return set_err(h, PHIP_ERR_INVALID, "internal: table changed during dump");
  Rec* d_out;
  if ((rc = ensure(h, B_TEMP, (size_t)n * sizeof(Rec), (u8**)&d_out))) return rc;
  k_dump_gather<<<grid_for(n), kBlock, 0, h->stream>>>(list, n, h->recs, d_out);
  HIPCHK(h, hipGetLastError());
  std::vector<Rec> recs(n);
  if (n) HIPCHK(h, hipMemcpyAsync(recs.data(), d_out, n * sizeof(Rec), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  // Long names come from the arena.
  std::vector<u8> arena;
  u64 cursor = 0;
  HIPCHK(h, hipMemcpy(&cursor, h->arena_cursor, 8, hipMemcpyDeviceToHost));
  cursor = std::min(cursor, h->arena_cap);
  if (cursor) {
    arena.resize(cursor);
    HIPCHK(h, hipMemcpy(arena.data(), h->arena, cursor, hipMemcpyDeviceToHost));
  }
  u64 total = 0;
  for (auto& r : recs) total += r.name0 & 0xFF;   // byte 0 = length
  if (n_out) *n_out = n;
  if (names_bytes_out) *names_bytes_out = total;
  if (!names) return PHIP_OK;
  if (total > names_cap || n > max_n || !name_offs || !states)
    return set_err(h, PHIP_ERR_INVALID, "dump buffers too small");
  u64 o = 0;
  for (u32 k = 0; k < n; ++k) {
    const Rec& r = recs[k];
    u32 len = r.name0 & 0xFF;
    name_offs[k] = o;
    if (len <= kInlineName) {
      const u64 w[3] = {r.name0, r.name1, r.name2};
      for (u32 j = 0; j < len; ++j) names[o + j] = (u8)(w[(j + 2) >> 3] >> (((j + 2) & 7) * 8));
    } else {
      u64 aoff = r.name0 >> 32;
      if (aoff + len <= arena.size()) std::memcpy(names + o, arena.data() + aoff, len);
    }
    o += len;
    states[k].added = dec_f64(r.added);
    states[k].taken = dec_f64(r.taken);
    states[k].elapsed = r.elapsed;
    states[k].created = r.created;
  }
  name_offs[n] = o;
  return PHIP_OK;
}

int phip_receive_soa(phip_handle* h, const phip_msgs* m, int64_t now, const phip_results* res,
                     uint32_t flags) {
  if (!h || !m) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  bool dev = flags & PHIP_DEVICE_PTRS;
  u32 n = m->n;
  if ((flags & PHIP_RECV_ASYNC) && dev && n >= kHotMinBatch && m->names && m->name_offs &&
      m->added && m->taken && m->elapsed) {
    // Queue this batch's front (reset, directory, status fill,
    // classification) behind the batch queued before, read that batch's
    // counters meanwhile and finish it, then queue this batch's fast pass
    // and return.  The front's counters are a fast-pass set of their own
    // (fctr), so the previous batch's leftover work leaves it standing
    // unless that work ran a fast pass itself or grew the table (below).
    if (int rc0 = begin_call(h, false)) return rc0;
    NamesOffs src{m->names, m->name_offs, m->names_len};
    SoaIn<NamesOffs> in{src, m->added, m->taken, m->elapsed};
    OutView ow{};
    FastFront ff;
    int rc;
    bool worked = false;
    if ((rc = outputs(h, res, n, true, &ow))) return rc;
    const bool prev = h->pend.active;
    if ((rc = fast_front(h, in, src, n, ow.status, &ff, !prev))) return after_error(h, rc);
    const u64 nfast = h->nfast, grows = h->grows;
    if (prev && (rc = finish_pending(h, &worked))) return after_error(h, rc);
    // The leftover work of the batch before (its misses, its dirty buckets)
    // runs on the general counters and leaves this front standing, unless it
    // ran a fast pass of its own (the directory and dirty list buffers) or
    // grew the table (the directory's slots).
    if (worked && (h->nfast != nfast || h->grows != grows) &&
        (rc = fast_front(h, in, src, n, ow.status, &ff)))
      return after_error(h, rc);
    if ((rc = fast_back(h, in, n, ff, true))) return after_error(h, rc);
    h->pend.active = true;
    h->pend.src = src;
    h->pend.a = m->added;
    h->pend.t = m->taken;
    h->pend.e = m->elapsed;
    h->pend.n = n;
    h->pend.par = ff.par;
    h->pend.iso = ff.iso;
    h->pend.now = now;
    h->pend.ow = ow;
    return PHIP_OK;
  }
  if (int rc0 = begin_call(h)) return rc0;
  if (n == 0) return PHIP_OK;
  if (!m->names || !m->name_offs || !m->added || !m->taken || !m->elapsed) return PHIP_ERR_INVALID;
  if (!dev && !names_ok(m->name_offs, n)) return set_err(h, PHIP_ERR_NAME_TOO_LARGE, "name > 231 bytes");
  int rc;
  if (!dev) {
    bool done = false;
    if ((rc = small_uniform(h, m, PHIP_OP_RECEIVE, now, res, &done))) return after_error(h, rc);
    if (done) return PHIP_OK;
  }
  NamesOffs src;
  const uint64_t *a, *t;
  const int64_t* e;
  OutView ow{};
  if ((rc = stage_names(h, m->names, m->name_offs, n, dev, &src, m->names_len)) ||
      (rc = stage(h, B_A, m->added, n, dev, &a)) || (rc = stage(h, B_T, m->taken, n, dev, &t)) ||
      (rc = stage(h, B_E, m->elapsed, n, dev, &e)) || (rc = outputs(h, res, n, dev, &ow)))
    return rc;
  if ((rc = receive_decoded(h, src, a, t, e, n, now, ow))) return after_error(h, rc);
  return copy_outputs(h, res, n, dev, ow);
}

}  // extern "C"

namespace {
// ReplicatedRepo.Receive over datagrams already in device memory (the
// caller's, the staging buffers, or a ring slot's copy); results go to
// device (dev) or host buffers.  Called with the handle's mutex held.
int receive_datagrams_dev(phip_handle* h, const u8* d_bytes, const uint64_t* d_offs, u32 n,
                          int64_t now, const phip_results* res, uint32_t* stop_index, bool dev) {
  int rc;
  OutView ow{};
  if ((rc = outputs(h, res, n, dev, &ow))) return rc;
  // Fast path straight from the wire bytes: k_classify reads the headers
  // (and finds the first malformed datagram), k_receive_fast reads every
  // datagram in place; no decoded copy is written.
  // Only a clean prefix with new buckets, or an incast / -0.0 past the dirty
  // set's reach, has the datagrams decoded to the SoA form, for the paths
  // that need it; a batch's dirty buckets (at most kDirtyCap dirty messages)
  // go through the ordered path as a sub-batch dirty_finish
  // reads from the wire.
  u32 fd = n, nmiss = 0;
  if ((rc = fast_apply(h, WireIn{d_bytes, d_offs}, Datagrams{d_bytes, d_offs}, n, ow.status, &fd,
                       &nmiss)))
    return after_error(h, rc);
  const u32 stop = std::min<u32>(h->ctr_host[5], n);
  // Statuses of the short datagram and everything after it (the Go loop exits).
  if (ow.status && stop < n) {
    HIPCHK(h, hipMemsetAsync(ow.status + stop, PHIP_ST_NOT_PROCESSED, n - stop, h->stream));
    HIPCHK(h, hipMemsetAsync(ow.status + stop, PHIP_ST_SHORT, 1, h->stream));
  }
  if (fd < stop || nmiss || h->ndef) {
    uint64_t *a, *t, *no;
    int64_t* e;
    u8* nl;
    if ((rc = ensure(h, B_DA, n, &a)) || (rc = ensure(h, B_DT, n, &t)) ||
        (rc = ensure(h, B_DE, n, &e)) || (rc = ensure(h, B_NOFF, n, &no)) ||
        (rc = ensure(h, B_NLEN, n, &nl)))
      return rc;
    if (fd < stop || nmiss) {   // (a batch whose dirty buckets alone are left reads no decode)
      Launch l(h, "k_decode");
      k_decode<<<grid_for(stop), kBlock, 0, h->stream>>>(d_bytes, d_offs, stop, a, t, e, no, nl,
                                                          h->ctr);
      HIPCHK(h, hipGetLastError());
    }
    if ((rc = finish_receive(h, NamesPairs{d_bytes, no, nl}, a, t, e, stop, fd, nmiss, now, ow, n,
                             h->ndef != 0)))
      return after_error(h, rc);
  }
  if ((rc = copy_outputs(h, res, n, dev, ow))) return rc;
  if (dev) HIPCHK(h, hipStreamSynchronize(h->stream));
  if (stop_index) *stop_index = stop;
  if (stop < n) return set_err(h, PHIP_ERR_SHORT_BUFFER, "short buffer at datagram %u", stop);
  return PHIP_OK;
}
}  // namespace

extern "C" {

int phip_receive_datagrams(phip_handle* h, const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                           int64_t now, const phip_results* res, uint32_t* stop_index,
                           uint32_t flags) {
  if (!h || (n && (!bytes || !offs))) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  if (stop_index) *stop_index = n;
  if (n == 0) return PHIP_OK;
  bool dev = flags & PHIP_DEVICE_PTRS;
  int rc;
  const uint64_t* d_offs;
  const u8* d_bytes;
  if (!dev && !datagrams_ok(offs, n))
    return set_err(h, PHIP_ERR_INVALID, "datagram offsets decrease");
  if (!dev) {
    bool done = false;
    rc = small_datagrams(h, bytes, offs, n, now, res, stop_index, &done);
    if (done || (rc && rc != PHIP_ERR_SHORT_BUFFER)) return rc == PHIP_ERR_SHORT_BUFFER ? rc : after_error(h, rc);
  }
  if ((rc = stage(h, B_DOFFS, offs, (size_t)n + 1, dev, &d_offs))) return rc;
  size_t nb = dev ? 0 : offs[n];
  if ((rc = stage(h, B_BYTES, bytes, nb, dev, &d_bytes))) return rc;
  return receive_datagrams_dev(h, d_bytes, d_offs, n, now, res, stop_index, dev);
}

// ------------------------------------------------------------ ingest ring --
// Pinned host slots, each with its own device copy; the copies run on the
// ring's stream, so filling and copying slot k+1 overlaps merging slot k.
struct phip_ring {
  phip_handle* h = nullptr;
  hipStream_t copy = nullptr;
  std::mutex mu;
  u32 max_msgs = 0;
  u64 max_bytes = 0;
  enum State { kFree, kAcquired, kSubmitted };
  struct Slot {
    u8* hbytes = nullptr;
    uint64_t* hoffs = nullptr;
    u8* dbytes = nullptr;
    uint64_t* doffs = nullptr;
    hipEvent_t copied = nullptr;
    u32 n = 0;
    State state = kFree;
  };
  std::vector<Slot> slots;
  u32 next_acquire = 0, next_receive = 0;
  std::string err;
};

void phip_ring_close(phip_ring* r) {
  if (!r) return;
  (void)hipSetDevice(r->h->device);
  if (r->copy) (void)hipStreamSynchronize(r->copy);
  for (auto& s : r->slots) {
    if (s.hbytes) (void)hipHostFree(s.hbytes);
    if (s.hoffs) (void)hipHostFree(s.hoffs);
    if (s.dbytes) (void)hipFree(s.dbytes);
    if (s.doffs) (void)hipFree(s.doffs);
    if (s.copied) (void)hipEventDestroy(s.copied);
  }
  if (r->copy) (void)hipStreamDestroy(r->copy);
  delete r;
}

int phip_ring_open(phip_handle* h, uint32_t nslots, uint32_t max_msgs, uint64_t max_bytes,
                   phip_ring** out) {
  if (!out) return PHIP_ERR_INVALID;
  *out = nullptr;
  if (!h || nslots < 1 || nslots > 64 || max_msgs < 1 || max_bytes < 1) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  phip_ring* r = new phip_ring;
  r->h = h;
  r->max_msgs = max_msgs;
  r->max_bytes = max_bytes;
  r->slots.resize(nslots);
  auto fail = [&](hipError_t e, const char* what) {
    set_err(h, PHIP_ERR_HIP, "phip_ring_open: %s failed: %s", what, hipGetErrorString(e));
    phip_ring_close(r);
    return PHIP_ERR_HIP;
  };
  hipError_t e;
  if ((e = hipStreamCreateWithFlags(&r->copy, hipStreamNonBlocking)) != hipSuccess)
    return fail(e, "hipStreamCreate");
  // +64: the fast path's 8-byte over-read slack past the last datagram.
  const size_t nbytes = max_bytes + 64, noffs = ((size_t)max_msgs + 1) * sizeof(uint64_t);
  for (auto& s : r->slots) {
    if ((e = hipHostMalloc(&s.hbytes, nbytes, 0)) != hipSuccess) return fail(e, "hipHostMalloc");
    if ((e = hipHostMalloc(&s.hoffs, noffs, 0)) != hipSuccess) return fail(e, "hipHostMalloc");
    if ((e = hipMalloc(&s.dbytes, nbytes)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&s.doffs, noffs)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipEventCreateWithFlags(&s.copied, hipEventDisableTiming)) != hipSuccess)
      return fail(e, "hipEventCreate");
    s.hoffs[0] = 0;
  }
  *out = r;
  return PHIP_OK;
}

int phip_ring_acquire(phip_ring* r, uint32_t* slot, uint8_t** bytes, uint64_t** offs) {
  if (!r || !slot || !bytes || !offs) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(r->mu);
  phip_ring::Slot& s = r->slots[r->next_acquire];
  if (s.state != phip_ring::kFree) return PHIP_ERR_BUSY;
  s.state = phip_ring::kAcquired;
  *slot = r->next_acquire;
  *bytes = s.hbytes;
  *offs = s.hoffs;
  s.hoffs[0] = 0;
  r->next_acquire = (r->next_acquire + 1) % (u32)r->slots.size();
  return PHIP_OK;
}

int phip_ring_submit(phip_ring* r, uint32_t slot, uint32_t n) {
  if (!r || slot >= r->slots.size() || n > r->max_msgs) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(r->mu);
  phip_ring::Slot& s = r->slots[slot];
  if (s.state != phip_ring::kAcquired) return PHIP_ERR_BUSY;
  const u64 nb = s.hoffs[n];
  if (s.hoffs[0] != 0 || nb > r->max_bytes || !datagrams_ok(s.hoffs, n)) return PHIP_ERR_INVALID;
  hipError_t e = hipSetDevice(r->h->device);
  if (e != hipSuccess) {
    r->err = hipGetErrorString(e);
    return PHIP_ERR_HIP;
  }
  if ((e = hipMemcpyAsync(s.doffs, s.hoffs, ((size_t)n + 1) * sizeof(uint64_t),
                          hipMemcpyHostToDevice, r->copy)) != hipSuccess ||
      (nb && (e = hipMemcpyAsync(s.dbytes, s.hbytes, nb, hipMemcpyHostToDevice, r->copy)) !=
                 hipSuccess) ||
      (e = hipEventRecord(s.copied, r->copy)) != hipSuccess) {
    r->err = hipGetErrorString(e);
    return PHIP_ERR_HIP;
  }
  s.n = n;
  s.state = phip_ring::kSubmitted;
  return PHIP_OK;
}

int phip_ring_receive(phip_ring* r, uint32_t slot, int64_t now, const phip_results* res,
                      uint32_t* stop_index) {
  if (!r || slot >= r->slots.size()) return PHIP_ERR_INVALID;
  phip_ring::Slot* s;
  {
    std::lock_guard<std::mutex> g(r->mu);
    s = &r->slots[slot];
    if (s->state != phip_ring::kSubmitted || slot != r->next_receive) return PHIP_ERR_BUSY;
  }
  phip_handle* h = r->h;
  int rc;
  {
    std::lock_guard<std::mutex> g(h->mu);
    if ((rc = begin_call(h))) return rc;
    if (stop_index) *stop_index = s->n;
    // A small slot is merged from its pinned host bytes in one launch (the
    // device copy is not waited for; the slot is freed only after it
    // finished, below); a larger one from the device copy.
    bool done = false;
    if (s->n && s->n <= kSmallMax) {
      rc = small_datagrams(h, s->hbytes, s->hoffs, s->n, now, res, stop_index, &done);
      if (done || (rc && rc != PHIP_ERR_SHORT_BUFFER)) {
        if (rc && rc != PHIP_ERR_SHORT_BUFFER) rc = after_error(h, rc);
        done = true;
        const hipError_t ce = hipEventSynchronize(s->copied);
        if (ce != hipSuccess && rc == PHIP_OK)
          rc = set_err(h, PHIP_ERR_HIP, "hipEventSynchronize: %s", hipGetErrorString(ce));
      }
    }
    if (!done) {
      hipError_t e = hipStreamWaitEvent(h->stream, s->copied, 0);
      if (e != hipSuccess)
        rc = set_err(h, PHIP_ERR_HIP, "hipStreamWaitEvent: %s", hipGetErrorString(e));
      else if (s->n == 0)
        rc = PHIP_OK;
      else
        rc = receive_datagrams_dev(h, s->dbytes, s->doffs, s->n, now, res, stop_index, false);
    }
    // On success the stream has drained (results copied back), so the slot's
    // host and device buffers are free; after an error wait for them first.
    if (rc) (void)hipStreamSynchronize(h->stream);  // drain; rc already set
  }
  std::lock_guard<std::mutex> g(r->mu);
  s->state = phip_ring::kFree;
  r->next_receive = (r->next_receive + 1) % (u32)r->slots.size();
  return rc;
}

int phip_upsert_soa(phip_handle* h, const phip_msgs* m, int64_t now, const phip_results* res,
                    uint32_t flags) {
  if (!h || !m) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  u32 n = m->n;
  if (n == 0) return PHIP_OK;
  if (!m->names || !m->name_offs || !m->added || !m->taken || !m->elapsed) return PHIP_ERR_INVALID;
  bool dev = flags & PHIP_DEVICE_PTRS;
  if (!dev && !names_ok(m->name_offs, n)) return set_err(h, PHIP_ERR_NAME_TOO_LARGE, "name > 231 bytes");
  int rc;
  if (!dev) {
    bool done = false;
    if ((rc = small_uniform(h, m, PHIP_OP_UPSERT, now, res, &done))) return after_error(h, rc);
    if (done) return PHIP_OK;
  }
  NamesOffs src;
  const uint64_t *a, *t;
  const int64_t* e;
  OutView ow{};
  if ((rc = stage_names(h, m->names, m->name_offs, n, dev, &src, m->names_len)) ||
      (rc = stage(h, B_A, m->added, n, dev, &a)) || (rc = stage(h, B_T, m->taken, n, dev, &t)) ||
      (rc = stage(h, B_E, m->elapsed, n, dev, &e)) || (rc = outputs(h, res, n, dev, &ow)))
    return rc;
  OpView ov{};
  ov.kind0 = PHIP_OP_UPSERT;
  ov.now0 = now;
  ov.a = a; ov.t = t; ov.e = e;
  if ((rc = ordered(h, src, n, ov, ow))) return after_error(h, rc);
  return copy_outputs(h, res, n, dev, ow);
}

int phip_apply_mixed(phip_handle* h, const phip_ops* ops, const phip_results* res, uint32_t flags) {
  if (!h || !ops) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  u32 n = ops->n;
  if (n == 0) return PHIP_OK;
  if (!ops->kind || !ops->names || !ops->name_offs || !ops->now) return PHIP_ERR_INVALID;
  bool dev = flags & PHIP_DEVICE_PTRS;
  if (!dev && !names_ok(ops->name_offs, n)) return set_err(h, PHIP_ERR_NAME_TOO_LARGE, "name > 231 bytes");
  if (!dev) {
    bool need_take = false, need_state = false;
    for (u32 i = 0; i < n; ++i) {
      if (ops->kind[i] > PHIP_OP_UPSERT) return set_err(h, PHIP_ERR_INVALID, "bad op kind at %u", i);
      if (ops->kind[i] == PHIP_OP_TAKE) need_take = true; else need_state = true;
    }
    if (need_take && (!ops->freq || !ops->per || !ops->count)) return PHIP_ERR_INVALID;
    if (need_state && (!ops->added || !ops->taken || !ops->elapsed)) return PHIP_ERR_INVALID;
  }
  int rc;
  if (!dev && h->small) {
    bool done = false;
    if ((rc = small_mixed(h, ops, res, &done))) return after_error(h, rc);
    if (done) return PHIP_OK;
  }
  NamesOffs src;
  OpView ov{};
  const u8* kind;
  OutView ow{};
  if ((rc = stage_names(h, ops->names, ops->name_offs, n, dev, &src, ops->names_len)) ||
      (rc = stage(h, B_KIND, ops->kind, n, dev, &kind)) ||
      (rc = stage(h, B_NOW, ops->now, n, dev, &ov.now)) ||
      (rc = stage(h, B_FREQ, ops->freq, n, dev, &ov.freq)) ||
      (rc = stage(h, B_PER, ops->per, n, dev, &ov.per)) ||
      (rc = stage(h, B_COUNT, ops->count, n, dev, &ov.count)) ||
      (rc = stage(h, B_A, ops->added, n, dev, &ov.a)) ||
      (rc = stage(h, B_T, ops->taken, n, dev, &ov.t)) ||
      (rc = stage(h, B_E, ops->elapsed, n, dev, &ov.e)) || (rc = outputs(h, res, n, dev, &ow)))
    return rc;
  ov.kind = kind;
  if ((rc = ordered(h, src, n, ov, ow))) return after_error(h, rc);
  return copy_outputs(h, res, n, dev, ow);
}

int phip_take(phip_handle* h, const uint8_t* names, const uint32_t* name_offs, uint32_t n,
              const int64_t* now, const int64_t* freq, const int64_t* per, const uint64_t* count,
              uint64_t* remaining_out, uint8_t* ok_out, uint32_t flags) {
  if (!h) return PHIP_ERR_INVALID;
  if (n == 0) return PHIP_OK;
  if (flags & PHIP_DEVICE_PTRS) return set_err(h, PHIP_ERR_INVALID, "phip_take: use phip_apply_mixed for device pointers");
  std::vector<u8> kind(n, PHIP_OP_TAKE), st(n);
  phip_ops ops{};
  ops.n = n;
  ops.kind = kind.data();
  ops.names = names;
  ops.name_offs = name_offs;
  ops.now = now;
  ops.freq = freq;
  ops.per = per;
  ops.count = count;
  phip_results res{};
  res.status = st.data();
  res.remaining = remaining_out;
  int rc = phip_apply_mixed(h, &ops, &res, flags);
  if (rc) return rc;
  if (ok_out)
    for (u32 i = 0; i < n; ++i) ok_out[i] = (st[i] & 0x7F) == PHIP_ST_TAKE_OK;
  return PHIP_OK;
}

int phip_hash_names(phip_handle* h, const uint8_t* names, const uint32_t* name_offs, uint32_t n,
                    uint64_t* out, uint32_t flags) {
  if ((n && (!names || !name_offs)) || (n && !out)) return PHIP_ERR_INVALID;
  if (!(flags & PHIP_DEVICE_PTRS)) {
    for (u32 i = 0; i < n; ++i) {
      u64 hh = kFnvOffset;
      for (u32 k = name_offs[i]; k < name_offs[i + 1]; ++k) hh = fnv_step(hh, names[k]);
      out[i] = hh;
    }
    return PHIP_OK;
  }
  if (!h) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  if (n == 0) return PHIP_OK;
  k_hash_names<<<grid_for(n), kBlock, 0, h->stream>>>(NamesOffs{names, name_offs}, n, out);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int phip_route_pack(phip_handle* h, const phip_msgs* m, uint32_t world, uint8_t* send_names,
                    uint32_t* send_lens, uint64_t* send_added, uint64_t* send_taken,
                    int64_t* send_elapsed, uint64_t* counts, uint64_t* name_bytes,
                    uint32_t flags) {
  if (!h || !m || !(flags & PHIP_DEVICE_PTRS) || world == 0 || world > kRouteMaxWorld)
    return PHIP_ERR_INVALID;
  const u32 n = m->n;
  if (n && (!m->names || !m->name_offs || !m->added || !m->taken || !m->elapsed || !send_names ||
            !send_lens || !send_added || !send_taken || !send_elapsed || !counts || !name_bytes))
    return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  int rc;
  const void* dir = nullptr;
  if ((flags & PHIP_ROUTE_COMBINE) && (rc = route_dir_on(h, h->stream, *m, world, &dir))) return rc;
  if ((rc = route_pack_on(h, h->stream, *m, world, dir, send_names, send_lens, send_added,
                          send_taken, send_elapsed, counts, name_bytes)))
    return rc;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int phip_ae_local_max(phip_handle* h, const int64_t* replicas, uint32_t nrep, uint64_t nbuckets,
                      int64_t* out, uint32_t flags) {
  if (!h || !(flags & PHIP_DEVICE_PTRS) || (nbuckets && (!replicas || !out)) || nrep == 0)
    return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  if (nbuckets == 0) return PHIP_OK;
  {
    Launch l(h, "k_ae_local_max");
    k_ae_local_max<<<dim3(grid_for(nbuckets), 3), kBlock, 0, h->stream>>>(replicas, nrep, nbuckets,
                                                                         out);
  }
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int phip_ae_apply(phip_handle* h, int64_t* replicas, uint32_t nrep, uint64_t nbuckets,
                  const int64_t* joined, uint32_t flags) {
  if (!h || !(flags & PHIP_DEVICE_PTRS) || (nbuckets && (!replicas || !joined)) || nrep == 0)
    return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  if (nbuckets == 0) return PHIP_OK;
  {
    Launch l(h, "k_ae_apply");
    k_ae_apply<<<dim3(grid_for(nbuckets), 3), kBlock, 0, h->stream>>>(replicas, nrep, nbuckets,
                                                                     joined);
  }
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int phip_ae_join(phip_handle* h, int64_t* replicas, uint32_t nrep, uint64_t nbuckets,
                 uint32_t flags) {
  if (!h || !(flags & PHIP_DEVICE_PTRS) || (nbuckets && !replicas) || nrep == 0)
    return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  if (nbuckets == 0) return PHIP_OK;
  {
    Launch l(h, "k_ae_join");
    k_ae_join<<<dim3(grid_for((nbuckets + 1) / 2), 3), kBlock, 0, h->stream>>>(replicas, nrep,
                                                                                nbuckets);
  }
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PHIP_OK;
}

int phip_last_timings(phip_handle* h, const char** names, float* ms, int max) {
  if (!h) return 0;
  std::lock_guard<std::mutex> g(h->mu);
  if (hipSetDevice(h->device) != hipSuccess || hipStreamSynchronize(h->stream) != hipSuccess) return 0;
  int k = 0;
  for (auto& t : h->timings) {
    if (k >= max) break;
    float v = 0;
    if (hipEventElapsedTime(&v, t.a, t.b) != hipSuccess) v = -1.0f;
    if (names) names[k] = t.name;
    if (ms) ms[k] = v;
    ++k;
  }
  return k;
}

void phip_set_timing(phip_handle* h, int on) {
  if (!h) return;
  std::lock_guard<std::mutex> g(h->mu);
  h->timing = on != 0;
  h->timing_accumulate = on == 2;
  h->timings.clear();
  h->pool_used = 0;
  // events for a timed loop made up front, not inside it
  while (on == 2 && h->event_pool.size() < 1024) {
    Timing tm{"", nullptr, nullptr};
    if (hipEventCreate(&tm.a) != hipSuccess) break;
    if (hipEventCreate(&tm.b) != hipSuccess) {
      (void)hipEventDestroy(tm.a);
      break;
    }
    h->event_pool.push_back(tm);
  }
}

int phip_set_stream(phip_handle* h, void* stream) {
  if (!h) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  // work already queued on the previous stream comes first
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->stream = stream ? (hipStream_t)stream : h->own_stream;
  return PHIP_OK;
}

int phip_table_stats(phip_handle* h, uint64_t* out, int max) {
  if (!h || !out) return PHIP_ERR_INVALID;
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = begin_call(h)) return rc0;
  u64* d;
  int rc;
  if ((rc = ensure(h, B_TSTATS, 2, &d))) return rc;
  HIPCHK(h, hipMemsetAsync(d, 0, 2 * sizeof(u64), h->stream));
  k_table_stats<<<grid_for(h->cap), kBlock, 0, h->stream>>>(table(h), h->cap, d);
  HIPCHK(h, hipGetLastError());
  u64 r[2] = {0, 0};
  HIPCHK(h, hipMemcpyAsync(r, d, sizeof r, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const u64 v[4] = {h->n_buckets, h->cap, r[0], r[1]};
  int k = 0;
  for (; k < max && k < 4; ++k) out[k] = v[k];
  return k;
}

int phip_last_stats(phip_handle* h, uint64_t* out, int max) {
  if (!h || !out) return 0;
  std::lock_guard<std::mutex> g(h->mu);
  // a queued PHIP_RECV_ASYNC batch is finished first, so the stats are its
  // own (its error, if any, is kept for the next call that returns one)
  if (h->pend.active && !h->deferred_rc) h->deferred_rc = begin_call(h);
  const uint64_t v[5] = {h->stats[0], h->stats[1], h->stats[2], h->grows, h->stats[3]};
  int k = 0;
  for (; k < max && k < 5; ++k) out[k] = v[k];
  return k;
}

}  // extern "C"

namespace phip_host {
void* handle_stream(phip_handle* h) { return h ? (void*)h->stream : nullptr; }
// (route_dir / route_pack use the handle's counters on the group's stream: a
// batch PHIP_RECV_ASYNC queued on the handle is finished first, so its
// kernels never race them)
int finish_queued(phip_handle* h) {
  HIPCHK(h, hipSetDevice(h->device));
  if (!h->pend.active) return PHIP_OK;
  const int rc = finish_pending(h);
  return rc ? after_error(h, rc) : PHIP_OK;
}
int route_dir(phip_handle* h, void* stream, const phip_msgs* m, uint32_t world, const void** dir) {
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = finish_queued(h)) return rc0;
  return route_dir_on(h, (hipStream_t)stream, *m, world, dir);
}
int route_pack(phip_handle* h, void* stream, const phip_msgs* m, uint32_t world, const void* dir,
               uint8_t* names, uint32_t* lens, uint64_t* a, uint64_t* t, int64_t* e,
               uint64_t* counts, uint64_t* nbytes) {
  std::lock_guard<std::mutex> g(h->mu);
  if (int rc0 = finish_queued(h)) return rc0;
  return route_pack_on(h, (hipStream_t)stream, *m, world, dir, names, lens, a, t, e, counts, nbytes);
}
const char* last_error(phip_handle* h) { return h ? h->err.c_str() : ""; }
int handle_device(const phip_handle* h) { return h ? h->device : -1; }
}  // namespace phip_host
