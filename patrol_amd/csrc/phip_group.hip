// Shard group: the buckets of one node hash-sharded by name over
// its GPUs, one phip_handle and one RCCL rank per GPU.  The reference has a
// single map behind one mutex (repo.go:171-235) fed by one Receive goroutine
// (repo.go:54-92); here every GPU owns the buckets whose name hashes to it,
// messages that arrive anywhere are routed to their owner, and simulated
// replicas converge by an all-reduce(max).
//
// Per member and call, one host thread: it binds its GPU and queues the
// member's work on three streams, synchronising only to read the split sizes
// of each chunk's exchange.  With one process per GPU the calling thread is
// the member's thread.
//
// Owner-routed Receive is pipelined by chunks of kChunk messages, over two
// send sets and two receive sets: while chunk k travels (exchange stream: the
// split sizes, then the grouped per-peer send/recv), the pack of chunk k+1
// (pack stream) and the owner's merge of chunk k-1 (the handle's stream) run
// beside it.
//
// Members sharing one GPU (phip_group_open_all with a device listed more
// than once: several shards' tables on one device, e.g. to rehearse an
// N-GPU group on one) exchange without RCCL, which refuses two ranks on one
// device: the member threads meet at a barrier once every member's packed
// send buffers and split sizes are ready, and each copies its segments from
// its peers' buffers with device copies; the all-reduce is an element-wise
// max over the members' joins.  The packing, segment offsets, source order
// and merge are the same code as the RCCL path.
#include <dlfcn.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "patrolhip.h"
#include "phip_host.hpp"

namespace {

typedef uint64_t u64;
typedef unsigned int u32;

// A device buffer that only grows.
struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (cap >= bytes) return hipSuccess;
    if (p) {
      hipError_t e = hipFree(p);
      if (e != hipSuccess) return e;
    }
    const size_t want = std::max(bytes, cap * 3 / 2) + 64;   // +64: 8-byte over-read slack
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Messages per pipelined chunk.  The send sets' name space is sized from the
// chunks' real name bytes (the batch's offsets at the chunk boundaries, one
// small read per call), so a name of any length fits and a set holds no more
// than its largest chunk needs.
constexpr uint32_t kChunk = 1u << 24;
constexpr uint32_t kSmallChunk = 1u << 12;   // PHIP_GROUP_SMALL_CHUNKS

// One chunk's send buffers (owner-major, phip_route_pack's layout) and its
// split sizes.  sizes (device) and host (pinned) hold [6 * world] u64:
//   send counts | send name bytes | send chunk totals | recv counts | recv name bytes | recv chunk totals
// (the chunk totals: every member's chunk count K, so that all members run
// the same number of exchange rounds).
struct SendSet {
  Buf names, lens, a, t, e, sizes;
  uint64_t* host = nullptr;
  hipEvent_t ev_pack = nullptr, ev_sz = nullptr, ev_x = nullptr;
  bool x_pending = false;   // ev_x recorded for an exchange reading this set
};

// One chunk's received segments (sources in rank order), merged while the
// next chunk travels.
struct RecvSet {
  Buf names, lens, offs, a, t, e;
  u64 n = 0;                      // messages received into it
  hipEvent_t ev_recv = nullptr;   // its exchange (exchange stream)
  hipEvent_t ev_merged = nullptr; // its merge (handle stream)
  bool merge_pending = false;     // ev_merged recorded for a merge reading it
};

// Busy spans of one group call per stage (0 pack, 1 exchange, 2 merge):
// event pairs recorded around each chunk's work on the stream it runs on,
// summed after the call (phip_group_stage_ms).
struct StageTimer {
  std::vector<hipEvent_t> ev[3];   // pairs per stage: [2k] start, [2k+1] end
  size_t used[3] = {0, 0, 0};
  bool on = false;
  void reset() { used[0] = used[1] = used[2] = 0; }
  hipError_t mark(int s, hipStream_t st) {
    if (!on) return hipSuccess;
    if (used[s] == ev[s].size()) {
      hipEvent_t e;
      hipError_t r = hipEventCreate(&e);
      if (r != hipSuccess) return r;
      ev[s].push_back(e);
    }
    return hipEventRecord(ev[s][used[s]++], st);
  }
  hipError_t sum(int s, float* ms) {
    *ms = 0;
    for (size_t k = 0; k + 1 < used[s]; k += 2) {
      float x = 0;
      hipError_t r = hipEventSynchronize(ev[s][k + 1]);
      if (r == hipSuccess) r = hipEventElapsedTime(&x, ev[s][k], ev[s][k + 1]);
      if (r != hipSuccess) return r;
      *ms += x;
    }
    return hipSuccess;
  }
  void release() {
    for (auto& v : ev)
      for (hipEvent_t e : v) (void)hipEventDestroy(e);
    for (auto& v : ev) v.clear();
  }
};

struct Member {
  phip_handle* h = nullptr;
  bool own = false;            // opened by the group (phip_group_open_all)
  int device = 0;
  u32 rank = 0;
  ncclComm_t comm = nullptr;
  hipStream_t sp = nullptr, sx = nullptr;   // pack stream, exchange stream
  hipEvent_t ev_done = nullptr;             // the call's last exchange
  SendSet set[2];
  RecvSet rset[2];             // chunk k is received into rset[k & 1]
  Buf scan_tmp, ae, bounds;
  u64* host_k = nullptr;       // pinned [world]: this member's chunk count, to every peer
  u64 k_local = 0;             // (shared-device groups read each other's)
  StageTimer tm;
  std::string err;
};

}  // namespace

// A reusable barrier of the member threads of one call (shared-device
// exchange).  abort() releases every waiter with false: a member that fails
// before a barrier must not leave the others waiting.
struct Barrier {
  std::mutex mu;
  std::condition_variable cv;
  u32 n = 0, count = 0, gen = 0;
  bool aborted = false;
  bool wait() {
    std::unique_lock<std::mutex> l(mu);
    if (aborted) return false;
    const u32 g0 = gen;
    if (++count == n) {
      count = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    cv.wait(l, [&] { return gen != g0 || aborted; });
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> l(mu);
    aborted = true;
    cv.notify_all();
  }
  void reset(u32 members) {
    std::lock_guard<std::mutex> l(mu);
    n = members;
    count = 0;
    aborted = false;
  }
};

struct phip_group {
  u32 world = 0;
  std::vector<Member> m;
  std::string err;
  bool shared = false;   // every member on one device: exchange by device copies (no RCCL)
  Barrier bar;
};

namespace {

int fail(Member& mb, int code, const char* fmt, ...) {
  char tmp[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(tmp, sizeof tmp, fmt, ap);
  va_end(ap);
  mb.err = tmp;
  return code;
}

#define GHIP(mb, x)                                                                        \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess)                                                                  \
      return fail((mb), PHIP_ERR_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                               \
  } while (0)

#define GNCCL(mb, x)                                                                        \
  do {                                                                                      \
    ncclResult_t r_ = (x);                                                                  \
    if (r_ != ncclSuccess)                                                                  \
      return fail((mb), PHIP_ERR_RCCL, "%s: %s (%s:%d)", #x, ncclGetErrorString(r_), __FILE__, \
                  __LINE__);                                                                \
  } while (0)

#define GPHIP(mb, x)                                                                   \
  do {                                                                                 \
    int rc_ = (x);                                                                     \
    if (rc_ != PHIP_OK)                                                                \
      return fail((mb), rc_, "%s: %s", #x, phip_last_error((mb).h));                    \
  } while (0)

// Run f(member index) on one host thread per local member (the calling
// thread when there is one); returns the first member's error.  A member
// that fails releases the others from the call's barriers.
template <class F>
int for_members(phip_group* g, F f) {
  const size_t n = g->m.size();
  std::vector<int> rc(n, PHIP_OK);
  g->bar.reset((u32)n);
  if (n == 1) {
    rc[0] = f(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(n);
    for (size_t i = 0; i < n; ++i)
      th.emplace_back([&, i] {
        rc[i] = f(i);
        if (rc[i] != PHIP_OK) g->bar.abort();
      });
    for (auto& t : th) t.join();
  }
  for (size_t i = 0; i < n; ++i)
    if (rc[i] != PHIP_OK) {
      g->err = "member " + std::to_string(i) + ": " + g->m[i].err;
      return rc[i];
    }
  g->err.clear();
  return PHIP_OK;
}

// The exchange plan of one chunk of one member, shared by the RCCL and the
// shared-device paths: with hs = the chunk's split sizes (SendSet::host),
// peer p's entry gives
//   send side: where the member's packed segment for owner p lies in its
//              owner-major send buffers (so messages / sb name bytes in) and
//              its size (sc, sbytes);
//   recv side: where the segment source p sends this member lands in the
//              chunk's part of the receive buffers (ro / rb: sources in rank
//              order) and its size (rc, rbytes).
struct Seg {
  u64 so, sb, sc, sbytes;
  u64 ro, rb, rc, rbytes;
};
void segment_plan(const u64* hs, u32 W, std::vector<Seg>* plan) {
  plan->resize(W);
  u64 so = 0, sb = 0, ro = 0, rb = 0;
  for (u32 p = 0; p < W; ++p) {
    Seg& g = (*plan)[p];
    g.so = so; g.sb = sb; g.sc = hs[p]; g.sbytes = hs[W + p];
    g.ro = ro; g.rb = rb; g.rc = hs[3 * W + p]; g.rbytes = hs[4 * W + p];
    so += g.sc; sb += g.sbytes; ro += g.rc; rb += g.rbytes;
  }
}

// The send side of one segment only (where a source's segment for owner p
// lies in its send set): what a shared-device peer reads of another
// member's sizes (their receive side is that member's own to write).
Seg send_seg(const u64* hs, u32 W, u32 p) {
  Seg g{};
  for (u32 q = 0; q < p; ++q) {
    g.so += hs[q];
    g.sb += hs[W + q];
  }
  g.sc = hs[p];
  g.sbytes = hs[W + p];
  return g;
}

// The owner's merge of one received chunk (lengths, packed names, states):
// name offsets by an inclusive scan of the lengths, then phip_receive_soa
// (sources in rank order, each in its order), on the handle's stream behind
// the chunk's exchange.
int merge_chunk(Member& mb, RecvSet& rs, hipStream_t st, int64_t now) {
  if (rs.n) {
    const u64 n = rs.n;
    GHIP(mb, hipStreamWaitEvent(st, rs.ev_recv, 0));
    GHIP(mb, mb.tm.mark(2, st));
    GHIP(mb, rs.offs.ensure(n * 4 + 8));
    u32* offs = (u32*)rs.offs.p;
    const u32* lens = (const u32*)rs.lens.p;
    GHIP(mb, hipMemsetAsync(offs, 0, sizeof(u32), st));
    size_t tb = 0;
    GHIP(mb, rocprim::inclusive_scan(nullptr, tb, lens, offs + 1, (size_t)n, rocprim::plus<u32>(), st));
    GHIP(mb, mb.scan_tmp.ensure(tb));
    GHIP(mb, rocprim::inclusive_scan(mb.scan_tmp.p, tb, lens, offs + 1, (size_t)n,
                                     rocprim::plus<u32>(), st));
    phip_msgs rm{};
    rm.n = (u32)n;
    rm.names = (const uint8_t*)rs.names.p;
    rm.name_offs = offs;
    rm.added = (const u64*)rs.a.p;
    rm.taken = (const u64*)rs.t.p;
    rm.elapsed = (const int64_t*)rs.e.p;
    GPHIP(mb, phip_receive_soa(mb.h, &rm, now, nullptr, PHIP_DEVICE_PTRS));
    GHIP(mb, mb.tm.mark(2, st));
  }
  GHIP(mb, hipEventRecord(rs.ev_merged, st));
  rs.merge_pending = true;
  return PHIP_OK;
}

// Chunk k of a batch: messages [k * chunk, ...) (empty past the batch).
phip_msgs chunk_of(const phip_msgs& in, u64 chunk, u64 k) {
  phip_msgs c = in;
  const u64 lo = k * chunk;
  c.n = lo < in.n ? (u32)std::min<u64>(chunk, in.n - lo) : 0u;
  if (c.n) {
    c.name_offs = in.name_offs + lo;   // absolute offsets into the same blob
    c.added = in.added + lo;
    c.taken = in.taken + lo;
    c.elapsed = in.elapsed + lo;
  }
  return c;
}

// Room in a receive set for n messages and nb name bytes, once the merge
// of the chunk it held before is done.
int recv_room(Member& mb, RecvSet& rs, u64 n, u64 nb) {
  if (rs.merge_pending) GHIP(mb, hipEventSynchronize(rs.ev_merged));
  rs.merge_pending = false;
  GHIP(mb, rs.lens.ensure(n * 4 + 4));
  GHIP(mb, rs.a.ensure(n * 8 + 8));
  GHIP(mb, rs.t.ensure(n * 8 + 8));
  GHIP(mb, rs.e.ensure(n * 8 + 8));
  GHIP(mb, rs.names.ensure(nb + 64));
  return PHIP_OK;
}

// One segment from a source's send set (src) into receive set rs, on
// stream st.
int copy_seg(Member& mb, const SendSet& src, const Seg& s_, const Seg& d_, RecvSet& rs,
             hipStream_t st) {
  if (!d_.rc) return PHIP_OK;
  GHIP(mb, hipMemcpyAsync((u32*)rs.lens.p + d_.ro, (const u32*)src.lens.p + s_.so, d_.rc * 4,
                          hipMemcpyDeviceToDevice, st));
  if (d_.rbytes)
    GHIP(mb, hipMemcpyAsync((uint8_t*)rs.names.p + d_.rb, (const uint8_t*)src.names.p + s_.sb,
                            d_.rbytes, hipMemcpyDeviceToDevice, st));
  GHIP(mb, hipMemcpyAsync((u64*)rs.a.p + d_.ro, (const u64*)src.a.p + s_.so, d_.rc * 8,
                          hipMemcpyDeviceToDevice, st));
  GHIP(mb, hipMemcpyAsync((u64*)rs.t.p + d_.ro, (const u64*)src.t.p + s_.so, d_.rc * 8,
                          hipMemcpyDeviceToDevice, st));
  GHIP(mb, hipMemcpyAsync((int64_t*)rs.e.p + d_.ro, (const int64_t*)src.e.p + s_.so, d_.rc * 8,
                          hipMemcpyDeviceToDevice, st));
  return PHIP_OK;
}

// name_offs at the chunk boundaries: out[k] = offs[min(k * chunk, n)].
__global__ void k_chunk_bounds(const uint32_t* __restrict__ offs, u32 n, u64 chunk, u64 kc,
                               u32* __restrict__ out) {
  const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (k <= kc) out[k] = offs[k * chunk < n ? k * chunk : n];
}

int member_receive(phip_group* g, Member& mb, const phip_msgs& in, int64_t now, uint64_t* sent,
                   uint64_t* merged, uint32_t flags) {
  const u32 W = g->world;
  const u32 n = in.n;
  GHIP(mb, hipSetDevice(mb.device));
  hipStream_t st = (hipStream_t)phip_host::handle_stream(mb.h);
  // PHIP_GROUP_RCCL_SELF: the member's own segment goes through RCCL too (a
  // send/recv pair to itself), so that the per-peer exchange below runs at
  // world 1, on one GPU, with the plan the multi-GPU group uses
  const bool rccl_self = (flags & PHIP_GROUP_RCCL_SELF) && !g->shared;
  mb.tm.reset();
  if (W == 1 && !rccl_self) {
    // One owner: every message is this member's, so there is nothing to
    // pack or exchange; the batch is merged as it came (the sender-side
    // combine is subsumed by the fast path's hot directory).
    if (sent) *sent = n;
    if (merged) *merged = n;
    if (n == 0) return PHIP_OK;
    GHIP(mb, mb.tm.mark(2, st));
    GPHIP(mb, phip_receive_soa(mb.h, &in, now, nullptr, PHIP_DEVICE_PTRS));
    GHIP(mb, mb.tm.mark(2, st));
    return PHIP_OK;
  }
  // The batch's producers are on the handle's stream: both pipeline streams
  // start behind it.
  GHIP(mb, hipEventRecord(mb.ev_done, st));
  GHIP(mb, hipStreamWaitEvent(mb.sp, mb.ev_done, 0));
  GHIP(mb, hipStreamWaitEvent(mb.sx, mb.ev_done, 0));
  // (PHIP_GROUP_SMALL_CHUNKS, testing: many rounds on small batches)
  const u64 chunk = (flags & PHIP_GROUP_SMALL_CHUNKS) ? kSmallChunk : kChunk;
  const u64 k_local = ((u64)n + chunk - 1) / chunk;
  mb.k_local = k_local;
  for (u32 p = 0; p < W; ++p) mb.host_k[p] = k_local;
  const u64 cmax = std::max<u64>(1, std::min<u64>(n, chunk));
  // name bytes per chunk: the offsets at the chunk boundaries
  u64 set_bytes[2] = {0, 0};
  if (n) {
    std::vector<u32> bnd(k_local + 1);
    GHIP(mb, mb.bounds.ensure((k_local + 1) * 4));
    k_chunk_bounds<<<(unsigned)((k_local + 1 + 255) / 256), 256, 0, st>>>(
        in.name_offs, n, chunk, k_local, (u32*)mb.bounds.p);
    GHIP(mb, hipGetLastError());
    GHIP(mb, hipMemcpyAsync(bnd.data(), mb.bounds.p, (k_local + 1) * 4, hipMemcpyDeviceToHost, st));
    GHIP(mb, hipStreamSynchronize(st));
    for (u64 k = 0; k < k_local; ++k)
      set_bytes[k & 1] = std::max<u64>(set_bytes[k & 1], (u64)(bnd[k + 1] - bnd[k]));
  }
  for (u32 si = 0; si < 2; ++si) {
    SendSet& ss = mb.set[si];
    GHIP(mb, ss.names.ensure(set_bytes[si] + 64));
    GHIP(mb, ss.lens.ensure(cmax * 4 + 4));
    GHIP(mb, ss.a.ensure(cmax * 8 + 8));
    GHIP(mb, ss.t.ensure(cmax * 8 + 8));
    GHIP(mb, ss.e.ensure(cmax * 8 + 8));
    GHIP(mb, ss.sizes.ensure((size_t)6 * W * 8));
    ss.x_pending = false;
  }
  // 1. the combine's directory, from a sample of the whole batch
  const void* dir = nullptr;
  if ((flags & PHIP_ROUTE_COMBINE) && n &&
      phip_host::route_dir(mb.h, mb.sp, &in, W, &dir) != PHIP_OK)
    return fail(mb, PHIP_ERR_HIP, "route directory: %s", phip_host::last_error(mb.h));
  // 2. pack chunk k into set k & 1 (pack stream), once no exchange reads it
  auto pack = [&](u64 k) -> int {
    SendSet& ss = mb.set[k & 1];
    if (ss.x_pending) GHIP(mb, hipStreamWaitEvent(mb.sp, ss.ev_x, 0));
    const phip_msgs c = chunk_of(in, chunk, k);
    u64* sz = (u64*)ss.sizes.p;
    GHIP(mb, mb.tm.mark(0, mb.sp));
    if (phip_host::route_pack(mb.h, mb.sp, &c, W, dir, (uint8_t*)ss.names.p, (uint32_t*)ss.lens.p,
                              (uint64_t*)ss.a.p, (uint64_t*)ss.t.p, (int64_t*)ss.e.p, sz, sz + W) !=
        PHIP_OK)
      return fail(mb, PHIP_ERR_HIP, "route pack: %s", phip_host::last_error(mb.h));
    GHIP(mb, hipMemcpyAsync(sz + 2 * W, mb.host_k, W * 8, hipMemcpyHostToDevice, mb.sp));
    GHIP(mb, mb.tm.mark(0, mb.sp));
    GHIP(mb, hipEventRecord(ss.ev_pack, mb.sp));
    return PHIP_OK;
  };
  // 3. chunk k's split sizes: every member learns what each source sends it
  //    (RCCL; shared-device groups read each other's after a barrier)
  auto sizes = [&](u64 k) -> int {
    SendSet& ss = mb.set[k & 1];
    u64* sz = (u64*)ss.sizes.p;
    GHIP(mb, hipStreamWaitEvent(mb.sx, ss.ev_pack, 0));
    GHIP(mb, mb.tm.mark(1, mb.sx));
    if (!g->shared) {
      GNCCL(mb, ncclGroupStart());
      GNCCL(mb, ncclAllToAll(sz, sz + 3 * W, 1, ncclUint64, mb.comm, mb.sx));
      GNCCL(mb, ncclAllToAll(sz + W, sz + 4 * W, 1, ncclUint64, mb.comm, mb.sx));
      GNCCL(mb, ncclAllToAll(sz + 2 * W, sz + 5 * W, 1, ncclUint64, mb.comm, mb.sx));
      GNCCL(mb, ncclGroupEnd());
    }
    GHIP(mb, hipMemcpyAsync(ss.host, sz, 6 * W * sizeof(u64), hipMemcpyDeviceToHost, mb.sx));
    GHIP(mb, mb.tm.mark(1, mb.sx));
    GHIP(mb, hipEventRecord(ss.ev_sz, mb.sx));
    return PHIP_OK;
  };
  int rc;
  if ((rc = pack(0)) || (rc = sizes(0))) return rc;
  if (k_local > 1 && (rc = pack(1))) return rc;
  u64 K = 1, n_send = 0, recv_msgs = 0;
  u64 packed = k_local > 1 ? 2 : 1;   // chunks whose pack is queued
  std::vector<Seg> plan;
  for (u64 k = 0; k < K; ++k) {
    SendSet& ss = mb.set[k & 1];
    GHIP(mb, hipEventSynchronize(ss.ev_sz));
    u64* hs = ss.host;
    if (g->shared) {   // what member p packed for this one, after every member packed chunk k
      if (!g->bar.wait()) return fail(mb, PHIP_ERR_INVALID, "another member failed");
      for (u32 p = 0; p < W; ++p) {
        const SendSet& ps = g->m[p].set[k & 1];
        hs[3 * W + p] = ps.host[mb.rank];
        hs[4 * W + p] = ps.host[W + mb.rank];
        hs[5 * W + p] = g->m[p].k_local;
      }
    }
    if (k == 0) {   // every member runs max(K) rounds (a shorter batch sends empty chunks)
      for (u32 p = 0; p < W; ++p) K = std::max<u64>(K, hs[5 * W + p]);
      K = std::max<u64>(K, 1);
    }
    segment_plan(hs, W, &plan);
    u64 c_send = 0, c_recv = 0, b_recv = 0;
    for (u32 p = 0; p < W; ++p) {
      c_send += plan[p].sc;
      c_recv += plan[p].rc;
      b_recv += plan[p].rbytes;
    }
    if (c_recv > 0xFFFFFFFFull || b_recv > 0xFFFFFFFFull)
      return fail(mb, PHIP_ERR_INVALID, "routed chunk of %llu messages / %llu name bytes exceeds 2^32",
                  (unsigned long long)c_recv, (unsigned long long)b_recv);
    RecvSet& rs = mb.rset[k & 1];
    if ((rc = recv_room(mb, rs, c_recv, b_recv))) return rc;
    // 4. the segments: one send and one receive per peer and column; this
    //    member's own segment is a device copy unless rccl_self
    GHIP(mb, mb.tm.mark(1, mb.sx));
    if (g->shared) {
      for (u32 p = 0; p < W; ++p) {
        const Member& src = g->m[p];
        const Seg s_ = send_seg(src.set[k & 1].host, W, mb.rank);   // the source's send side
        if (s_.sc != plan[p].rc || s_.sbytes != plan[p].rbytes)
          return fail(mb, PHIP_ERR_INVALID, "internal: member %u sends %llu/%llu, %u expects %llu/%llu",
                      p, (unsigned long long)s_.sc, (unsigned long long)s_.sbytes, mb.rank,
                      (unsigned long long)plan[p].rc, (unsigned long long)plan[p].rbytes);
        if ((rc = copy_seg(mb, src.set[k & 1], s_, plan[p], rs, mb.sx))) return rc;
      }
    } else {
      const Seg& own = plan[mb.rank];
      if (own.sc != own.rc || own.sbytes != own.rbytes)
        return fail(mb, PHIP_ERR_INVALID, "internal: own segment %llu/%llu vs %llu/%llu",
                    (unsigned long long)own.sc, (unsigned long long)own.sbytes,
                    (unsigned long long)own.rc, (unsigned long long)own.rbytes);
      if (!rccl_self && (rc = copy_seg(mb, ss, own, own, rs, mb.sx))) return rc;
      GNCCL(mb, ncclGroupStart());
      for (u32 p = 0; p < W; ++p) {
        if (p == mb.rank && !rccl_self) continue;
        const Seg& x = plan[p];
        GNCCL(mb, ncclSend((u32*)ss.lens.p + x.so, x.sc, ncclUint32, p, mb.comm, mb.sx));
        GNCCL(mb, ncclRecv((u32*)rs.lens.p + x.ro, x.rc, ncclUint32, p, mb.comm, mb.sx));
        GNCCL(mb, ncclSend((uint8_t*)ss.names.p + x.sb, x.sbytes, ncclUint8, p, mb.comm, mb.sx));
        GNCCL(mb, ncclRecv((uint8_t*)rs.names.p + x.rb, x.rbytes, ncclUint8, p, mb.comm, mb.sx));
        GNCCL(mb, ncclSend((u64*)ss.a.p + x.so, x.sc, ncclUint64, p, mb.comm, mb.sx));
        GNCCL(mb, ncclRecv((u64*)rs.a.p + x.ro, x.rc, ncclUint64, p, mb.comm, mb.sx));
        GNCCL(mb, ncclSend((u64*)ss.t.p + x.so, x.sc, ncclUint64, p, mb.comm, mb.sx));
        GNCCL(mb, ncclRecv((u64*)rs.t.p + x.ro, x.rc, ncclUint64, p, mb.comm, mb.sx));
        GNCCL(mb, ncclSend((u64*)ss.e.p + x.so, x.sc, ncclUint64, p, mb.comm, mb.sx));
        GNCCL(mb, ncclRecv((int64_t*)rs.e.p + x.ro, x.rc, ncclUint64, p, mb.comm, mb.sx));
      }
      GNCCL(mb, ncclGroupEnd());
    }
    GHIP(mb, mb.tm.mark(1, mb.sx));
    GHIP(mb, hipEventRecord(ss.ev_x, mb.sx));
    GHIP(mb, hipEventRecord(rs.ev_recv, mb.sx));
    ss.x_pending = true;
    rs.n = c_recv;
    n_send += c_send;
    recv_msgs += c_recv;
    // 6. the owner's merge of chunk k-1 beside chunk k's exchange (chunk
    //    order: the merges queue on the handle's stream; a shared-device
    //    member merges before it waits for its copies)
    const bool merge_prev = k >= 1;
    if (g->shared) {
      if (merge_prev && (rc = merge_chunk(mb, mb.rset[(k - 1) & 1], st, now))) return rc;
      // every member has copied chunk k out of every set k & 1 before any
      // packs chunk k + 2 into it
      GHIP(mb, hipEventSynchronize(ss.ev_x));
      if (!g->bar.wait()) return fail(mb, PHIP_ERR_INVALID, "another member failed");
    }
    // 5. next: chunk k+1's sizes behind chunk k's exchange (RCCL keeps one
    //    order per communicator), chunk k+2's pack into the set just sent
    if (k + 1 < K) {
      if (packed < k + 2) {   // a chunk past this member's batch: an empty pack
        if ((rc = pack(k + 1))) return rc;
        packed = k + 2;
      }
      if ((rc = sizes(k + 1))) return rc;
      if (k + 2 < K && packed < k + 3) {
        if ((rc = pack(k + 2))) return rc;
        packed = k + 3;
      }
    }
    if (!g->shared && merge_prev && (rc = merge_chunk(mb, mb.rset[(k - 1) & 1], st, now)))
      return rc;
  }
  if (sent) *sent = n_send;
  if (merged) *merged = recv_msgs;
  // the last chunk's merge; the handle's stream ends behind every exchange
  // (the next call's packs reuse the send sets)
  if ((rc = merge_chunk(mb, mb.rset[(K - 1) & 1], st, now))) return rc;
  GHIP(mb, hipEventRecord(mb.ev_done, mb.sx));
  GHIP(mb, hipStreamWaitEvent(st, mb.ev_done, 0));
  return PHIP_OK;
}

__global__ void k_max_into(int64_t* __restrict__ dst, const int64_t* __restrict__ src, u64 n) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && src[i] > dst[i]) dst[i] = src[i];
}

int member_anti_entropy(phip_group* g, Member& mb, int64_t* reps, uint32_t nrep, uint64_t B) {
  GHIP(mb, hipSetDevice(mb.device));
  mb.tm.reset();
  hipStream_t st = (hipStream_t)phip_host::handle_stream(mb.h);
  if (g->world == 1) {   // nothing to exchange: the fused local join
    GHIP(mb, mb.tm.mark(0, st));
    GPHIP(mb, phip_ae_join(mb.h, reps, nrep, B, PHIP_DEVICE_PTRS));
    GHIP(mb, mb.tm.mark(0, st));
    return PHIP_OK;
  }
  GHIP(mb, mb.ae.ensure((size_t)3 * B * 8 * (g->shared ? 2 : 1)));
  int64_t* j = (int64_t*)mb.ae.p;
  GHIP(mb, mb.tm.mark(0, st));
  GPHIP(mb, phip_ae_local_max(mb.h, reps, nrep, B, j, PHIP_DEVICE_PTRS));
  GHIP(mb, mb.tm.mark(0, st));
  if (g->shared) {   // the all-reduce: every member's join, max'd element-wise
    if (!g->bar.wait()) return fail(mb, PHIP_ERR_INVALID, "another member failed");
    int64_t* jm = j + 3 * B;
    GHIP(mb, hipMemcpyAsync(jm, j, 3 * B * 8, hipMemcpyDeviceToDevice, st));
    for (const Member& p : g->m) {
      if (&p == &mb) continue;
      k_max_into<<<(unsigned)((3 * B + 255) / 256), 256, 0, st>>>(jm, (const int64_t*)p.ae.p, 3 * B);
      GHIP(mb, hipGetLastError());
    }
    GHIP(mb, hipStreamSynchronize(st));
    if (!g->bar.wait()) return fail(mb, PHIP_ERR_INVALID, "another member failed");
    GHIP(mb, mb.tm.mark(2, st));
    GPHIP(mb, phip_ae_apply(mb.h, reps, nrep, B, jm, PHIP_DEVICE_PTRS));
    GHIP(mb, mb.tm.mark(2, st));
    return PHIP_OK;
  }
  GHIP(mb, mb.tm.mark(1, st));
  GNCCL(mb, ncclAllReduce(j, j, 3 * B, ncclInt64, ncclMax, mb.comm, st));
  GHIP(mb, mb.tm.mark(1, st));
  GHIP(mb, mb.tm.mark(2, st));
  GPHIP(mb, phip_ae_apply(mb.h, reps, nrep, B, j, PHIP_DEVICE_PTRS));
  GHIP(mb, mb.tm.mark(2, st));
  return PHIP_OK;
}

void destroy(phip_group* g) {
  for (auto& mb : g->m) {
    (void)hipSetDevice(mb.device);
    if (mb.h) (void)phip_flush(mb.h);
    if (mb.sp) (void)hipStreamSynchronize(mb.sp);
    if (mb.sx) (void)hipStreamSynchronize(mb.sx);
    if (mb.comm) (void)ncclCommDestroy(mb.comm);
    for (SendSet& ss : mb.set) {
      for (Buf* b : {&ss.names, &ss.lens, &ss.a, &ss.t, &ss.e, &ss.sizes}) b->release();
      if (ss.host) (void)hipHostFree(ss.host);
      for (hipEvent_t ev : {ss.ev_pack, ss.ev_sz, ss.ev_x})
        if (ev) (void)hipEventDestroy(ev);
    }
    for (RecvSet& rs : mb.rset) {
      for (Buf* b : {&rs.names, &rs.lens, &rs.offs, &rs.a, &rs.t, &rs.e}) b->release();
      for (hipEvent_t ev : {rs.ev_recv, rs.ev_merged})
        if (ev) (void)hipEventDestroy(ev);
    }
    for (Buf* b : {&mb.scan_tmp, &mb.ae, &mb.bounds}) b->release();
    mb.tm.release();
    if (mb.host_k) (void)hipHostFree(mb.host_k);
    if (mb.ev_done) (void)hipEventDestroy(mb.ev_done);
    if (mb.sp) (void)hipStreamDestroy(mb.sp);
    if (mb.sx) (void)hipStreamDestroy(mb.sx);
    if (mb.own && mb.h) phip_close(mb.h);
  }
  delete g;
}

// Per member: the pipeline's two streams, the send sets' pinned size mirrors
// and events.
int alloc_member_state(phip_group* g) {
  for (auto& mb : g->m) {
    if (hipSetDevice(mb.device) != hipSuccess ||
        hipStreamCreateWithFlags(&mb.sp, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&mb.sx, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&mb.ev_done, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(&mb.host_k, (size_t)g->world * sizeof(u64), 0) != hipSuccess)
      return PHIP_ERR_HIP;
    for (SendSet& ss : mb.set)
      if (hipHostMalloc(&ss.host, 6 * (size_t)g->world * sizeof(u64), 0) != hipSuccess ||
          hipEventCreateWithFlags(&ss.ev_pack, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&ss.ev_sz, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&ss.ev_x, hipEventDisableTiming) != hipSuccess)
        return PHIP_ERR_HIP;
    for (RecvSet& rs : mb.rset) {
      rs.merge_pending = false;
      if (hipEventCreateWithFlags(&rs.ev_recv, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&rs.ev_merged, hipEventDisableTiming) != hipSuccess)
        return PHIP_ERR_HIP;
    }
  }
  return PHIP_OK;
}

}  // namespace

extern "C" {

int phip_group_unique_id(uint8_t* id) {
  if (!id) return PHIP_ERR_INVALID;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return PHIP_ERR_RCCL;
  std::memcpy(id, u.internal, PHIP_GROUP_ID_BYTES);
  return PHIP_OK;
}

int phip_group_open_all(const phip_config* cfg, const int32_t* devices, uint32_t n,
                        phip_group** out) {
  if (!cfg || !devices || !out || n == 0 || n > 64) return PHIP_ERR_INVALID;
  *out = nullptr;
  phip_group* g = new phip_group;
  g->world = n;
  g->m.resize(n);
  std::vector<int> devs(devices, devices + n);
  for (u32 i = 0; i < n; ++i) {
    phip_config c = *cfg;
    c.device = devices[i];
    g->m[i].device = devices[i];
    g->m[i].rank = i;
    g->m[i].own = true;
    int rc = phip_open(&c, &g->m[i].h);
    if (rc) {
      destroy(g);
      return rc;
    }
  }
  // one device listed more than once: RCCL takes one rank per device, so the
  // members exchange by device copies (all of them on that one device)
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool repeated = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
  if (repeated) {
    if (sorted.front() != sorted.back()) {   // mixed: some devices shared, some not
      destroy(g);
      return PHIP_ERR_INVALID;
    }
    g->shared = n > 1;
  } else {
    std::vector<ncclComm_t> comms(n);
    if (ncclCommInitAll(comms.data(), (int)n, devs.data()) != ncclSuccess) {
      destroy(g);
      return PHIP_ERR_RCCL;
    }
    for (u32 i = 0; i < n; ++i) g->m[i].comm = comms[i];
  }
  if (int rc = alloc_member_state(g)) {
    destroy(g);
    return rc;
  }
  *out = g;
  return PHIP_OK;
}

int phip_group_open_rank(phip_handle* h, const uint8_t* id, uint32_t nranks, uint32_t rank,
                         phip_group** out) {
  if (!h || !id || !out || nranks == 0 || nranks > 64 || rank >= nranks) return PHIP_ERR_INVALID;
  *out = nullptr;
  phip_group* g = new phip_group;
  g->world = nranks;
  g->m.resize(1);
  Member& mb = g->m[0];
  mb.h = h;
  mb.device = phip_host::handle_device(h);
  mb.rank = rank;
  ncclUniqueId u;
  std::memcpy(u.internal, id, PHIP_GROUP_ID_BYTES);
  if (hipSetDevice(mb.device) != hipSuccess ||
      ncclCommInitRank(&mb.comm, (int)nranks, u, (int)rank) != ncclSuccess) {
    mb.comm = nullptr;
    destroy(g);
    return PHIP_ERR_RCCL;
  }
  if (int rc = alloc_member_state(g)) {
    destroy(g);
    return rc;
  }
  *out = g;
  return PHIP_OK;
}

void phip_group_close(phip_group* g) {
  if (g) destroy(g);
}

const char* phip_group_last_error(const phip_group* g) { return g ? g->err.c_str() : "null group"; }
uint32_t phip_group_world(const phip_group* g) { return g ? g->world : 0; }
uint32_t phip_group_local(const phip_group* g) { return g ? (uint32_t)g->m.size() : 0; }
phip_handle* phip_group_handle(phip_group* g, uint32_t i) {
  return (g && i < g->m.size()) ? g->m[i].h : nullptr;
}

int phip_group_receive(phip_group* g, const phip_msgs* batches, int64_t now, uint64_t* sent,
                       uint64_t* merged, uint32_t flags) {
  if (!g || !batches || !(flags & PHIP_DEVICE_PTRS)) return PHIP_ERR_INVALID;
  return for_members(g, [&](size_t i) {
    return member_receive(g, g->m[i], batches[i], now, sent ? sent + i : nullptr,
                          merged ? merged + i : nullptr, flags);
  });
}

int phip_group_set_timing(phip_group* g, int on) {
  if (!g) return PHIP_ERR_INVALID;
  for (Member& mb : g->m) mb.tm.on = on != 0;
  return PHIP_OK;
}

int phip_group_stage_ms(phip_group* g, uint32_t i, float* ms) {
  if (!g || !ms || i >= g->m.size()) return PHIP_ERR_INVALID;
  Member& mb = g->m[i];
  if (hipSetDevice(mb.device) != hipSuccess) return PHIP_ERR_HIP;
  for (int s = 0; s < 3; ++s)
    if (mb.tm.sum(s, &ms[s]) != hipSuccess) return PHIP_ERR_HIP;
  return PHIP_OK;
}

int phip_group_rccl_info(phip_group* g, uint32_t i, int32_t* version, int32_t* comm_count,
                         char* lib_path, uint32_t path_cap) {
  if (!g || i >= g->m.size()) return PHIP_ERR_INVALID;
  const Member& mb = g->m[i];
  int v = 0;
  if (ncclGetVersion(&v) != ncclSuccess) return PHIP_ERR_RCCL;
  if (version) *version = v;
  int c = 0;
  if (mb.comm && ncclCommCount(mb.comm, &c) != ncclSuccess) return PHIP_ERR_RCCL;
  if (comm_count) *comm_count = c;
  if (lib_path && path_cap) {
    Dl_info di{};
    const char* p = dladdr((const void*)&ncclGetVersion, &di) && di.dli_fname ? di.dli_fname : "";
    std::snprintf(lib_path, path_cap, "%s", p);
  }
  return PHIP_OK;
}

int phip_group_anti_entropy(phip_group* g, int64_t* const* replicas, uint32_t nrep,
                            uint64_t nbuckets, uint32_t flags) {
  if (!g || !replicas || nrep == 0 || !(flags & PHIP_DEVICE_PTRS)) return PHIP_ERR_INVALID;
  if (nbuckets == 0) return PHIP_OK;
  return for_members(g, [&](size_t i) {
    return member_anti_entropy(g, g->m[i], replicas[i], nrep, nbuckets);
  });
}

}  // extern "C"
