// Ablation harness for the fast Receive kernel (not product code).
// Builds the C2 table (10M names "b<id>" in 2^24 slots) host-side with the
// same layout/hash as libpatrolhip, then times variants of the per-message
// work on 100M Zipf(1.1) messages whose states are later than the previous
// run's (every run is a first application, like bench.py).
//   V0 product kernel (k_receive_fast)
//   V1 resolve + state read, no atomics (counts would-be atomics)
//   V2 precomputed slot + state read + atomics (no name/hash/probe)
//   V3 name load + hash only
//   V4 resolve only (tag + record name compare)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../patrol_amd/csrc/phip_kernels.hpp"

using namespace phip;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

__global__ void v1_noatomic(NamesOffs src, const uint64_t* ma, const uint64_t* mt, const int64_t* me,
                            u32 n, Table T, u32* ctr) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  bool would = false;
  if (i < n) {
    u64 off; u32 len;
    src.get(i, off, len);
    Name nm;
    load_name(src.blob, off, len, nm);
    u32 s;
    Rec r;
    if (probe(T, nm, src.blob, &s, &r) == kFound) {
      would = enc_replica(ma[i]) > r.added || enc_replica(mt[i]) > r.taken ||
              (i64)me[i] > r.elapsed;
    }
  }
  u64 m = __ballot(would);
  if (__lane_id() == 0 && m) atomicAdd(&ctr[blockIdx.x & 1023], (u32)__popcll(m));
}

__global__ void v2_slot(const u32* slot, const uint64_t* ma, const uint64_t* mt, const int64_t* me,
                        u32 n, Table T, u32* ctr) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  bool did = false;
  if (i < n) {
    Rec* r = &T.recs[slot[i]];
    u64 ea = enc_replica(ma[i]), et = enc_replica(mt[i]);
    i64 eb = me[i];
    u64 ca = r->added, ct = r->taken;
    i64 ce = r->elapsed;
    if (ea > ca) { atomicMax(&r->added, ea); did = true; }
    if (et > ct) { atomicMax(&r->taken, et); did = true; }
    if (eb > ce) { atomicMax(&r->elapsed, eb); did = true; }
  }
  u64 m = __ballot(did);
  if (__lane_id() == 0 && m) atomicAdd(&ctr[blockIdx.x & 1023], (u32)__popcll(m));
}

__global__ void v3_hash(NamesOffs src, u32 n, u64* sink) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u64 off; u32 len;
  src.get(i, off, len);
  Name nm;
  load_name(src.blob, off, len, nm);
  if (nm.h == 0x1234567ull) sink[0] = nm.w0;
}

__global__ void v4_resolve(NamesOffs src, u32 n, Table T, u32* slot_out) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u64 off; u32 len;
  src.get(i, off, len);
  Name nm;
  load_name(src.blob, off, len, nm);
  u32 s = 0;
  Rec r;
  probe(T, nm, src.blob, &s, &r);
  slot_out[i] = s;
}

// V0 with a counter of atomics issued (same code path otherwise).
__global__ void v0_count(NamesOffs src, const uint64_t* ma, const uint64_t* mt, const int64_t* me,
                         u32 n, Table T, u32* ctr) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  bool did = false;
  if (i < n) {
    u64 off; u32 len;
    src.get(i, off, len);
    Name nm;
    load_name(src.blob, off, len, nm);
    u32 s;
    Rec cur;
    if (probe(T, nm, src.blob, &s, &cur) == kFound) {
      Rec* r = &T.recs[s];
      u64 ea = enc_replica(ma[i]), et = enc_replica(mt[i]);
      i64 eb = me[i];
      if (ea > cur.added) { atomicMax(&r->added, ea); did = true; }
      if (et > cur.taken) { atomicMax(&r->taken, et); did = true; }
      if (eb > cur.elapsed) { atomicMax(&r->elapsed, eb); did = true; }
    }
  }
  u64 m = __ballot(did);
  if (__lane_id() == 0 && m) atomicAdd(&ctr[blockIdx.x & 1023], (u32)__popcll(m));
}


static u64 host_fnv(const char* p, size_t n) {
  u64 h = kFnvOffset;
  for (size_t k = 0; k < n; ++k) h = fnv_step(h, (u8)p[k]);
  return h;
}

int main(int argc, char** argv) {
  const u32 K = argc > 1 ? atoi(argv[1]) : 10000000u;
  const u32 n = argc > 2 ? atoi(argv[2]) : 100000000u;
  const u32 L = 24;
  const u64 cap = 1ull << L;
  printf("K=%u n=%u slots=2^%u\n", K, n, L);
  auto t0 = std::chrono::steady_clock::now();
  // --- host table
  std::vector<Rec> recs(cap);
  memset(recs.data(), 0, cap * sizeof(Rec));
  char buf[32];
  for (u32 id = 0; id < K; ++id) {
    int len = snprintf(buf, sizeof buf, "b%u", id);
    u64 h = host_fnv(buf, len);
    u64 tag = tag_of(h);
    u32 s = (u32)((tag * 0x9E3779B97F4A7C15ull) >> (64 - L));
    while (recs[s].tag) s = (s + 1) & (cap - 1);
    Rec& r = recs[s];
    r.tag = tag;
    r.added = kEPosZero; r.taken = kEPosZero; r.elapsed = 0; r.created = 0;
    Name nm;
    load_name((const u8*)buf, 0, len, nm);
    r.name0 = with_flags(nm.w0, kRecPublished); r.name1 = nm.w1; r.name2 = nm.w2;
  }
  // --- messages
  std::vector<double> cdf(K);
  double acc = 0;
  for (u32 r = 0; r < K; ++r) { acc += std::pow((double)(r + 1), -1.1); cdf[r] = acc; }
  u64 mult = 2654435761ull % K;
  while (std::__gcd<u64>(mult, K) != 1) ++mult;
  std::mt19937_64 rng(42);
  std::vector<u32> offs(n + 1);
  std::vector<u8> blob;
  blob.reserve((size_t)n * 9 + 8);
  std::vector<u32> ids(n);
  for (u32 i = 0; i < n; ++i) {
    double u = (rng() >> 11) * (1.0 / 9007199254740992.0) * acc;
    u32 r = (u32)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
    if (r >= K) r = K - 1;
    ids[i] = (u32)(((u64)r * mult) % K);
    offs[i] = (u32)blob.size();
    int len = snprintf(buf, sizeof buf, "b%u", ids[i]);
    blob.insert(blob.end(), buf, buf + len);
  }
  offs[n] = (u32)blob.size();
  for (int k = 0; k < 8; ++k) blob.push_back(0);
  // slots for V2
  std::vector<u32> slot(n);
  {
    std::vector<u32> slot_of_id(K);
    for (u32 id = 0; id < K; ++id) {
      int len = snprintf(buf, sizeof buf, "b%u", id);
      u64 tag = tag_of(host_fnv(buf, len));
      u32 s = (u32)((tag * 0x9E3779B97F4A7C15ull) >> (64 - L));
      while (recs[s].tag != tag || ((recs[s].name0 & 0xFF) != (u64)len)) s = (s + 1) & (cap - 1);
      slot_of_id[id] = s;
    }
    for (u32 i = 0; i < n; ++i) slot[i] = slot_of_id[ids[i]];
  }
  auto t1 = std::chrono::steady_clock::now();
  printf("host gen %.1f s\n", std::chrono::duration<double>(t1 - t0).count());
  // --- device
  Table T;
  Rec* drecs; u32* daux; u8* dblob; u32* doffs; u32* dslot; u32* ctr; u64* sink;
  uint64_t *da, *dt; int64_t* de;
  CK(hipMalloc(&daux, cap * 4)); CK(hipMalloc(&drecs, cap * sizeof(Rec)));
  CK(hipMalloc(&dblob, blob.size())); CK(hipMalloc(&doffs, (n + 1) * 4ull)); CK(hipMalloc(&dslot, n * 4ull));
  CK(hipMalloc(&ctr, 4096)); CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&da, n * 8ull)); CK(hipMalloc(&dt, n * 8ull)); CK(hipMalloc(&de, n * 8ull));
  CK(hipMemcpy(drecs, recs.data(), cap * sizeof(Rec), hipMemcpyHostToDevice));
  CK(hipMemcpy(dblob, blob.data(), blob.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(doffs, offs.data(), (n + 1) * 4ull, hipMemcpyHostToDevice));
  CK(hipMemcpy(dslot, slot.data(), n * 4ull, hipMemcpyHostToDevice));
  T.aux = daux; T.recs = drecs; T.arena = nullptr; T.L = L; T.tag_mask = ~0ull;
  NamesOffs src{dblob, doffs};
  std::vector<uint64_t> ha(n), ht(n);
  std::vector<int64_t> he(n);
  int step = 0;
  auto new_states = [&]() {
    ++step;
    std::mt19937_64 g(1000 + step);
    for (u32 i = 0; i < n; ++i) {
      double taken = (double)(g() % 1000000) + step * 2e6;
      double added = taken + (g() >> 11) * (1.0 / 9007199254740992.0) * 100.0;
      memcpy(&ha[i], &added, 8); memcpy(&ht[i], &taken, 8);
      he[i] = (int64_t)(g() & ((1ull << 40) - 1)) + (int64_t)step * (1ll << 40);
    }
    CK(hipMemcpy(da, ha.data(), n * 8ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, ht.data(), n * 8ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(de, he.data(), n * 8ull, hipMemcpyHostToDevice));
  };
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const unsigned G = (n + 255) / 256;
  auto timeit = [&](const char* name, auto launch, bool fresh) {
    if (fresh) new_states();
    CK(hipMemset(ctr, 0, 4096));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    u32 cc[1024]; CK(hipMemcpy(cc, ctr, 4096, hipMemcpyDeviceToHost));
    u64 c = 0; for (int k = 0; k < 1024; ++k) c += cc[k];
    printf("%-34s %8.3f ms  %7.2f G msg/s  counter=%.4f of n\n", name, ms, n / ms / 1e6, (double)c / n);
  };
  u32* miss; CK(hipMalloc(&miss, n * 4ull));
  u32* dslot2; CK(hipMalloc(&dslot2, n * 4ull));
  for (int rep = 0; rep < 1; ++rep) {
    timeit("V0 product k_receive_fast", [&] {
      k_receive_fast<NamesOffs><<<G, 256>>>(src, da, dt, de, n, nullptr, T, nullptr, miss, ctr, 0); }, true);
    timeit("V0-old (no combine, counting)", [&] { v0_count<<<G, 256>>>(src, da, dt, de, n, T, ctr); }, true);
    timeit("V0 same batch again (all no-op)", [&] { v0_count<<<G, 256>>>(src, da, dt, de, n, T, ctr); }, false);
    timeit("V1 resolve+read, no atomics", [&] { v1_noatomic<<<G, 256>>>(src, da, dt, de, n, T, ctr); }, true);
    timeit("V2 slot given + atomics", [&] { v2_slot<<<G, 256>>>(dslot, da, dt, de, n, T, ctr); }, true);
    timeit("V3 name+hash only", [&] { v3_hash<<<G, 256>>>(src, n, sink); }, false);
    timeit("V4 resolve only", [&] { v4_resolve<<<G, 256>>>(src, n, T, miss); }, false);
#define VAR(OPT, PER, label) \
    timeit("P" #OPT "x" #PER " " label " fresh", [&] { CK(hipMemset(ctr + 512, 0, 4)); \
      k_receive_fast<NamesOffs, OPT, PER><<<(n + 256 * PER - 1) / (256 * PER), 256>>>(src, da, dt, de, n, nullptr, T, nullptr, miss, ctr + 512, 0); }, true); \
    timeit("P" #OPT "x" #PER " " label " no-op", [&] { CK(hipMemset(ctr + 512, 0, 4)); \
      k_receive_fast<NamesOffs, OPT, PER><<<(n + 256 * PER - 1) / (256 * PER), 256>>>(src, da, dt, de, n, nullptr, T, nullptr, miss, ctr + 512, 0); }, false);
    VAR(31, 1, "c+nt+wide+skip+small")
    VAR(63, 1, "c+nt+wide+skip+small+noseen")
    VAR(61, 1, "c+wide+skip+small+noseen")
    VAR(47, 1, "c+nt+wide+skip+noseen")
  }
  return 0;
}
