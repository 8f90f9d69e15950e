// Shard group: the buckets of one node hash-sharded by name over
// its GPUs, one phip_handle and one RCCL rank per GPU.  The reference has a
// single map behind one mutex (repo.go:171-235) fed by one Receive goroutine
// (repo.go:54-92); here every GPU owns the buckets whose name hashes to it,
// messages that arrive anywhere are routed to their owner, and simulated
// replicas converge by an all-reduce(max).
//
// Per member and call, one host thread: it binds its GPU, queues the member's
// kernels and RCCL calls on the member handle's stream, and synchronises only
// to read the split sizes of the exchange.  With one process per GPU the
// calling thread is the member's thread.
//
// Members sharing one GPU (phip_group_open_all with a device listed more
// than once: several shards' tables on one device, e.g. to rehearse an
// N-GPU group on one) exchange without RCCL, which refuses two ranks on one
// device: the member threads meet at a barrier once every member's packed
// send buffers and split sizes are ready, and each copies its segments from
// its peers' buffers with device copies; the all-reduce is an element-wise
// max over the members' joins.  The packing, segment offsets, source order
// and merge are the same code as the RCCL path.
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

struct Member {
  phip_handle* h = nullptr;
  bool own = false;            // opened by the group (phip_group_open_all)
  int device = 0;
  u32 rank = 0;
  ncclComm_t comm = nullptr;
  // send side (phip_route_pack's owner-major buffers), receive side
  Buf s_names, s_lens, s_a, s_t, s_e, r_names, r_lens, r_offs, r_a, r_t, r_e;
  Buf sizes, scan_tmp, ae;
  u64* host_sizes = nullptr;   // pinned [4 * world]: send counts, send bytes, recv counts, recv bytes
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

// The exchange plan of one member, shared by the RCCL and the shared-device
// paths: with hs = the member's split sizes [send counts | send name bytes |
// recv counts | recv name bytes] (W entries each), peer p's entry gives
//   send side: where the member's packed segment for owner p lies in its
//              owner-major send buffers (so messages / sb name bytes in) and
//              its size (sc, sbytes);
//   recv side: where the segment source p sends this member lands in the
//              receive buffers (ro / rb: sources in rank order) and its size
//              (rc, rbytes).
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
    g.ro = ro; g.rb = rb; g.rc = hs[2 * W + p]; g.rbytes = hs[3 * W + p];
    so += g.sc; sb += g.sbytes; ro += g.rc; rb += g.rbytes;
  }
}

// One member's owner-routed Receive.
// The owner's merge of n received messages (lengths, packed names, states):
// name offsets by an inclusive scan of the lengths, then phip_receive_soa
// (sources in rank order, each in its order).
int merge_received(Member& mb, hipStream_t st, const u32* lens, const uint8_t* names, const u64* a,
                   const u64* t, const int64_t* e, u64 n, int64_t now) {
  GHIP(mb, mb.r_offs.ensure(n * 4 + 8));
  u32* offs = (u32*)mb.r_offs.p;
  GHIP(mb, hipMemsetAsync(offs, 0, sizeof(u32), st));
  size_t tb = 0;
  GHIP(mb, rocprim::inclusive_scan(nullptr, tb, lens, offs + 1, (size_t)n, rocprim::plus<u32>(), st));
  GHIP(mb, mb.scan_tmp.ensure(tb));
  GHIP(mb, rocprim::inclusive_scan(mb.scan_tmp.p, tb, lens, offs + 1, (size_t)n,
                                   rocprim::plus<u32>(), st));
  phip_msgs rm{};
  rm.n = (u32)n;
  rm.names = names;
  rm.name_offs = offs;
  rm.added = a;
  rm.taken = t;
  rm.elapsed = e;
  GPHIP(mb, phip_receive_soa(mb.h, &rm, now, nullptr, PHIP_DEVICE_PTRS));
  return PHIP_OK;
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
  if (W == 1 && !rccl_self) {
    // One owner: every message is this member's, so there is nothing to
    // pack or exchange; the batch is merged as it came (the sender-side
    // combine is subsumed by the fast path's hot directory).
    if (sent) *sent = n;
    if (merged) *merged = n;
    if (n == 0) return PHIP_OK;
    GPHIP(mb, phip_receive_soa(mb.h, &in, now, nullptr, PHIP_DEVICE_PTRS));
    return PHIP_OK;
  }
  // 1. pack by owner (device; phip_route_pack returns when the sizes are written)
  size_t in_bytes = 0;
  if (n) {
    u32 last = 0;
    GHIP(mb, hipMemcpyAsync(&last, in.name_offs + n, sizeof last, hipMemcpyDeviceToHost, st));
    GHIP(mb, hipStreamSynchronize(st));
    in_bytes = last;
  }
  GHIP(mb, mb.s_names.ensure(in_bytes + 64));
  GHIP(mb, mb.s_lens.ensure((size_t)n * 4 + 4));
  GHIP(mb, mb.s_a.ensure((size_t)n * 8 + 8));
  GHIP(mb, mb.s_t.ensure((size_t)n * 8 + 8));
  GHIP(mb, mb.s_e.ensure((size_t)n * 8 + 8));
  GHIP(mb, mb.sizes.ensure((size_t)4 * W * 8));
  u64* sz = (u64*)mb.sizes.p;   // [send counts | send bytes | recv counts | recv bytes]
  GPHIP(mb, phip_route_pack(mb.h, &in, W, (uint8_t*)mb.s_names.p, (uint32_t*)mb.s_lens.p,
                            (uint64_t*)mb.s_a.p, (uint64_t*)mb.s_t.p, (int64_t*)mb.s_e.p, sz,
                            sz + W, PHIP_DEVICE_PTRS | (flags & PHIP_ROUTE_COMBINE)));
  // 2. split sizes: every member learns what each source sends it
  if (g->shared) {
    GHIP(mb, hipMemcpyAsync(mb.host_sizes, sz, 2 * W * sizeof(u64), hipMemcpyDeviceToHost, st));
    GHIP(mb, hipStreamSynchronize(st));
    if (!g->bar.wait()) return fail(mb, PHIP_ERR_INVALID, "another member failed");
    for (u32 p = 0; p < W; ++p) {   // what member p packed for this one
      mb.host_sizes[2 * W + p] = g->m[p].host_sizes[mb.rank];
      mb.host_sizes[3 * W + p] = g->m[p].host_sizes[W + mb.rank];
    }
  } else {
    GNCCL(mb, ncclGroupStart());
    GNCCL(mb, ncclAllToAll(sz, sz + 2 * W, 1, ncclUint64, mb.comm, st));
    GNCCL(mb, ncclAllToAll(sz + W, sz + 3 * W, 1, ncclUint64, mb.comm, st));
    GNCCL(mb, ncclGroupEnd());
    GHIP(mb, hipMemcpyAsync(mb.host_sizes, sz, 4 * W * sizeof(u64), hipMemcpyDeviceToHost, st));
    GHIP(mb, hipStreamSynchronize(st));
  }
  const u64* hs = mb.host_sizes;
  u64 n_send = 0, n_recv = 0, b_recv = 0;
  for (u32 p = 0; p < W; ++p) {
    n_send += hs[p];
    n_recv += hs[2 * W + p];
    b_recv += hs[3 * W + p];
  }
  if (n_recv > 0xFFFFFFFFull || b_recv > 0xFFFFFFFFull)
    return fail(mb, PHIP_ERR_INVALID, "routed batch of %llu messages / %llu name bytes exceeds 2^32",
                (unsigned long long)n_recv, (unsigned long long)b_recv);
  if (sent) *sent = n_send;
  if (merged) *merged = n_recv;
  GHIP(mb, mb.r_names.ensure(b_recv + 64));
  GHIP(mb, mb.r_lens.ensure(n_recv * 4 + 4));
  GHIP(mb, mb.r_offs.ensure(n_recv * 4 + 8));
  GHIP(mb, mb.r_a.ensure(n_recv * 8 + 8));
  GHIP(mb, mb.r_t.ensure(n_recv * 8 + 8));
  GHIP(mb, mb.r_e.ensure(n_recv * 8 + 8));
  // 3. the segments: one send and one receive per peer and column; this
  // member's own segment is a device copy (no RCCL round trip through its
  // buffers) unless rccl_self
  std::vector<Seg> plan;
  segment_plan(hs, W, &plan);
  // one segment from a source's packed buffers (src: its send side) into
  // this member's receive buffers (dst: its receive side)
  auto copy_seg = [&](const Member& src, const Seg& s_, const Seg& d_) -> int {
    GHIP(mb, hipMemcpyAsync((u32*)mb.r_lens.p + d_.ro, (const u32*)src.s_lens.p + s_.so, d_.rc * 4,
                            hipMemcpyDeviceToDevice, st));
    GHIP(mb, hipMemcpyAsync((uint8_t*)mb.r_names.p + d_.rb, (const uint8_t*)src.s_names.p + s_.sb,
                            d_.rbytes, hipMemcpyDeviceToDevice, st));
    GHIP(mb, hipMemcpyAsync((u64*)mb.r_a.p + d_.ro, (const u64*)src.s_a.p + s_.so, d_.rc * 8,
                            hipMemcpyDeviceToDevice, st));
    GHIP(mb, hipMemcpyAsync((u64*)mb.r_t.p + d_.ro, (const u64*)src.s_t.p + s_.so, d_.rc * 8,
                            hipMemcpyDeviceToDevice, st));
    GHIP(mb, hipMemcpyAsync((int64_t*)mb.r_e.p + d_.ro, (const int64_t*)src.s_e.p + s_.so,
                            d_.rc * 8, hipMemcpyDeviceToDevice, st));
    return PHIP_OK;
  };
  if (g->shared) {   // each segment copied from its source member's packed buffers
    std::vector<Seg> splan;
    for (u32 p = 0; p < W; ++p) {
      const Member& src = g->m[p];
      segment_plan(src.host_sizes, W, &splan);   // the source's send side
      const Seg& s_ = splan[mb.rank];
      if (s_.sc != plan[p].rc || s_.sbytes != plan[p].rbytes)
        return fail(mb, PHIP_ERR_INVALID, "internal: member %u sends %llu/%llu, %u expects %llu/%llu",
                    p, (unsigned long long)s_.sc, (unsigned long long)s_.sbytes, mb.rank,
                    (unsigned long long)plan[p].rc, (unsigned long long)plan[p].rbytes);
      if (int rc = copy_seg(src, s_, plan[p])) return rc;
    }
    // every member copied what it needs before any packs again (the next
    // call's route_pack overwrites the send buffers)
    GHIP(mb, hipStreamSynchronize(st));
    if (!g->bar.wait()) return fail(mb, PHIP_ERR_INVALID, "another member failed");
    if (n_recv == 0) return PHIP_OK;
    return merge_received(mb, st, (const u32*)mb.r_lens.p, (const uint8_t*)mb.r_names.p,
                          (const u64*)mb.r_a.p, (const u64*)mb.r_t.p, (const int64_t*)mb.r_e.p,
                          n_recv, now);
  }
  void* tm = phip_host::timing_begin(mb.h, "rccl_exchange");
  // the own segment's size must be what this member packed for itself
  if (plan[mb.rank].sc != plan[mb.rank].rc || plan[mb.rank].sbytes != plan[mb.rank].rbytes)
    return fail(mb, PHIP_ERR_INVALID, "internal: own segment %llu/%llu vs %llu/%llu",
                (unsigned long long)plan[mb.rank].sc, (unsigned long long)plan[mb.rank].sbytes,
                (unsigned long long)plan[mb.rank].rc, (unsigned long long)plan[mb.rank].rbytes);
  if (!rccl_self)
    if (int rc = copy_seg(mb, plan[mb.rank], plan[mb.rank])) return rc;
  GNCCL(mb, ncclGroupStart());
  for (u32 p = 0; p < W; ++p) {
    if (p == mb.rank && !rccl_self) continue;
    const Seg& x = plan[p];
    GNCCL(mb, ncclSend((u32*)mb.s_lens.p + x.so, x.sc, ncclUint32, p, mb.comm, st));
    GNCCL(mb, ncclRecv((u32*)mb.r_lens.p + x.ro, x.rc, ncclUint32, p, mb.comm, st));
    GNCCL(mb, ncclSend((uint8_t*)mb.s_names.p + x.sb, x.sbytes, ncclUint8, p, mb.comm, st));
    GNCCL(mb, ncclRecv((uint8_t*)mb.r_names.p + x.rb, x.rbytes, ncclUint8, p, mb.comm, st));
    GNCCL(mb, ncclSend((u64*)mb.s_a.p + x.so, x.sc, ncclUint64, p, mb.comm, st));
    GNCCL(mb, ncclRecv((u64*)mb.r_a.p + x.ro, x.rc, ncclUint64, p, mb.comm, st));
    GNCCL(mb, ncclSend((u64*)mb.s_t.p + x.so, x.sc, ncclUint64, p, mb.comm, st));
    GNCCL(mb, ncclRecv((u64*)mb.r_t.p + x.ro, x.rc, ncclUint64, p, mb.comm, st));
    GNCCL(mb, ncclSend((u64*)mb.s_e.p + x.so, x.sc, ncclUint64, p, mb.comm, st));
    GNCCL(mb, ncclRecv((u64*)mb.r_e.p + x.ro, x.rc, ncclUint64, p, mb.comm, st));
  }
  GNCCL(mb, ncclGroupEnd());
  phip_host::timing_end(mb.h, tm);
  if (n_recv == 0) return PHIP_OK;
  return merge_received(mb, st, (const u32*)mb.r_lens.p, (const uint8_t*)mb.r_names.p,
                        (const u64*)mb.r_a.p, (const u64*)mb.r_t.p, (const int64_t*)mb.r_e.p, n_recv,
                        now);
}

__global__ void k_max_into(int64_t* __restrict__ dst, const int64_t* __restrict__ src, u64 n) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && src[i] > dst[i]) dst[i] = src[i];
}

int member_anti_entropy(phip_group* g, Member& mb, int64_t* reps, uint32_t nrep, uint64_t B) {
  GHIP(mb, hipSetDevice(mb.device));
  if (g->world == 1) {   // nothing to exchange: the fused local join
    GPHIP(mb, phip_ae_join(mb.h, reps, nrep, B, PHIP_DEVICE_PTRS));
    return PHIP_OK;
  }
  hipStream_t st = (hipStream_t)phip_host::handle_stream(mb.h);
  GHIP(mb, mb.ae.ensure((size_t)3 * B * 8 * (g->shared ? 2 : 1)));
  int64_t* j = (int64_t*)mb.ae.p;
  GPHIP(mb, phip_ae_local_max(mb.h, reps, nrep, B, j, PHIP_DEVICE_PTRS));
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
    GPHIP(mb, phip_ae_apply(mb.h, reps, nrep, B, jm, PHIP_DEVICE_PTRS));
    return PHIP_OK;
  }
  void* tm = phip_host::timing_begin(mb.h, "rccl_allreduce");
  GNCCL(mb, ncclAllReduce(j, j, 3 * B, ncclInt64, ncclMax, mb.comm, st));
  phip_host::timing_end(mb.h, tm);
  GPHIP(mb, phip_ae_apply(mb.h, reps, nrep, B, j, PHIP_DEVICE_PTRS));
  return PHIP_OK;
}

void destroy(phip_group* g) {
  for (auto& mb : g->m) {
    (void)hipSetDevice(mb.device);
    if (mb.h) (void)phip_flush(mb.h);
    if (mb.comm) (void)ncclCommDestroy(mb.comm);
    for (Buf* b : {&mb.s_names, &mb.s_lens, &mb.s_a, &mb.s_t, &mb.s_e, &mb.r_names, &mb.r_lens,
                   &mb.r_offs, &mb.r_a, &mb.r_t, &mb.r_e, &mb.sizes, &mb.scan_tmp, &mb.ae})
      b->release();
    if (mb.host_sizes) (void)hipHostFree(mb.host_sizes);
    if (mb.own && mb.h) phip_close(mb.h);
  }
  delete g;
}

int alloc_host_sizes(phip_group* g) {
  for (auto& mb : g->m) {
    if (hipSetDevice(mb.device) != hipSuccess ||
        hipHostMalloc(&mb.host_sizes, 4 * (size_t)g->world * sizeof(u64), 0) != hipSuccess)
      return PHIP_ERR_HIP;
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
  if (int rc = alloc_host_sizes(g)) {
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
  if (int rc = alloc_host_sizes(g)) {
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

int phip_group_anti_entropy(phip_group* g, int64_t* const* replicas, uint32_t nrep,
                            uint64_t nbuckets, uint32_t flags) {
  if (!g || !replicas || nrep == 0 || !(flags & PHIP_DEVICE_PTRS)) return PHIP_ERR_INVALID;
  if (nbuckets == 0) return PHIP_OK;
  return for_members(g, [&](size_t i) {
    return member_anti_entropy(g, g->m[i], replicas[i], nrep, nbuckets);
  });
}

}  // extern "C"
