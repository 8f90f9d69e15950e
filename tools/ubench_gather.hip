// Random record-read rate on gfx950 (not product code): how fast can 100M
// messages each read one 64-byte slot record of a 2^25-slot (2 GiB) table?
// Index streams: uniform, and Zipf(1.1) over 10M keys at scattered slots
// (the C2 bench shape).  Variants: lane per record with 1/3/4 16-byte loads,
// quad per record (4 lanes x 16 B, one 64-B burst per quad), and a
// slot-sorted stream (locality upper bound).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned long long u64;
typedef unsigned int u32;

template <int NLD>
__global__ __launch_bounds__(256) void lane_rec(const uint4* __restrict__ recs, const u32* __restrict__ idx,
                                                u32 n, u32* __restrict__ out) {
  u32 i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  u32 s = __builtin_nontemporal_load(idx + i);
  const uint4* p = recs + (size_t)s * 4;
  uint4 a = p[0];
  u32 x = a.x ^ a.w;
  if (NLD > 1) { uint4 b = p[1]; x ^= b.x ^ b.w; }
  if (NLD > 2) { uint4 c = p[2]; x ^= c.x ^ c.w; }
  if (NLD > 3) { uint4 d = p[3]; x ^= d.x ^ d.w; }
  out[i] = x;
}

// one 16-B load per lane with explicit cache-policy bits
template <int POL>
__global__ __launch_bounds__(256) void lane_rec_pol(const uint4* __restrict__ recs, const u32* __restrict__ idx,
                                                    u32 n, u32* __restrict__ out) {
  u32 i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  u32 s = __builtin_nontemporal_load(idx + i);
  const uint4* p = recs + (size_t)s * 4;
  uint4 a;
  if (POL == 0) asm volatile("global_load_dwordx4 %0, %1, off nt\n s_waitcnt vmcnt(0)" : "=v"(a) : "v"(p));
  if (POL == 1) asm volatile("global_load_dwordx4 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(a) : "v"(p));
  if (POL == 2) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" : "=v"(a) : "v"(p));
  if (POL == 3) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt\n s_waitcnt vmcnt(0)" : "=v"(a) : "v"(p));
  if (POL == 4) asm volatile("global_load_dwordx4 %0, %1, off sc0\n s_waitcnt vmcnt(0)" : "=v"(a) : "v"(p));
  out[i] = a.x ^ a.w;
}

__global__ __launch_bounds__(256) void quad_rec(const uint4* __restrict__ recs, const u32* __restrict__ idx,
                                                u32 n, u32* __restrict__ out) {
  u32 t = blockIdx.x * 256 + threadIdx.x;
  u32 i = t >> 2, q = t & 3;
  if (i >= n) return;
  u32 s = __builtin_nontemporal_load(idx + i);
  uint4 a = recs[(size_t)s * 4 + q];
  u32 x = a.x ^ a.w;
  x ^= __shfl_xor(x, 1);
  x ^= __shfl_xor(x, 2);
  if (q == 0) out[i] = x;
}

// 8 messages per lane, loads of all 8 records issued before any use.
__global__ __launch_bounds__(256) void lane_rec_x8(const uint4* __restrict__ recs, const u32* __restrict__ idx,
                                                   u32 n, u32* __restrict__ out) {
  u32 base = blockIdx.x * 256 * 8 + threadIdx.x;
  u32 s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { u32 i = base + k * 256; s[k] = i < n ? __builtin_nontemporal_load(idx + i) : 0; }
  uint4 a[8], b[8], c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { const uint4* p = recs + (size_t)s[k] * 4; a[k] = p[0]; b[k] = p[1]; c[k] = p[2]; }
#pragma unroll
  for (int k = 0; k < 8; ++k) { u32 i = base + k * 256; if (i < n) out[i] = a[k].x ^ b[k].y ^ c[k].z; }
}

// Atomic cost: one 64-bit atomicMax per message on its record (no-return).
__global__ __launch_bounds__(256) void lane_atomic(uint4* recs, const u32* __restrict__ idx, u32 n, u64 v) {
  u32 i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  u32 s = __builtin_nontemporal_load(idx + i);
  atomicMax((unsigned long long*)(recs + (size_t)s * 4) + 1, v + i);
}

int main(int argc, char** argv) {
  const u32 L = 25, K = 10000000u, n = argc > 1 ? atoi(argv[1]) : 100000000u;
  const u64 cap = 1ull << L;
  std::vector<u32> zipf(n), unif(n), sorted;
  {
    std::vector<double> cdf(K);
    double acc = 0;
    for (u32 r = 0; r < K; ++r) { acc += std::pow((double)(r + 1), -1.1); cdf[r] = acc; }
    std::mt19937_64 rng(42);
    std::vector<u32> slot_of(K);
    for (u32 k = 0; k < K; ++k) slot_of[k] = (u32)((u64)k * 0x9E3779B97F4A7C15ull >> (64 - L));
    for (u32 i = 0; i < n; ++i) {
      double u = (rng() >> 11) * (1.0 / 9007199254740992.0) * acc;
      u32 r = (u32)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
      if (r >= K) r = K - 1;
      zipf[i] = slot_of[r];
      unif[i] = (u32)(rng() & (cap - 1));
    }
    sorted = zipf;
    std::sort(sorted.begin(), sorted.end());
  }
  uint4* recs; u32 *dz, *du, *ds, *out;
  const int mode = argc > 2 ? atoi(argv[2]) : 0;   // 0 hipMalloc, 1 uncached, 2 fine-grained
  if (mode == 0) CK(hipMalloc(&recs, cap * 64));
  else CK(hipExtMallocWithFlags((void**)&recs, cap * 64, mode == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
  CK(hipMemset(recs, 1, cap * 64));
  printf("table alloc mode %d\n", mode);
  CK(hipMalloc(&dz, n * 4ull)); CK(hipMalloc(&du, n * 4ull)); CK(hipMalloc(&ds, n * 4ull));
  CK(hipMalloc(&out, n * 4ull));
  CK(hipMemcpy(dz, zipf.data(), n * 4ull, hipMemcpyHostToDevice));
  CK(hipMemcpy(du, unif.data(), n * 4ull, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, sorted.data(), n * 4ull, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    float best = 1e9;
    for (int r = 0; r < 4; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r) best = std::min(best, ms);
    }
    printf("%-40s %8.3f ms  %7.2f G rec/s\n", name, best, n / best / 1e6);
  };
  const unsigned G = (n + 255) / 256;
  const u32* streams[3] = {dz, du, ds};
  const char* sn[3] = {"zipf", "uniform", "sorted-zipf"};
  for (int k = 0; k < 3; ++k) {
    const u32* I = streams[k];
    char b[96];
    snprintf(b, sizeof b, "%s lane 1x16B", sn[k]); timeit(b, [&] { lane_rec<1><<<G, 256>>>(recs, I, n, out); });
    snprintf(b, sizeof b, "%s lane 3x16B", sn[k]); timeit(b, [&] { lane_rec<3><<<G, 256>>>(recs, I, n, out); });
    snprintf(b, sizeof b, "%s lane 4x16B", sn[k]); timeit(b, [&] { lane_rec<4><<<G, 256>>>(recs, I, n, out); });
    snprintf(b, sizeof b, "%s lane 1x16B nt", sn[k]); timeit(b, [&] { lane_rec_pol<0><<<G, 256>>>(recs, I, n, out); });
    snprintf(b, sizeof b, "%s lane 1x16B sc1", sn[k]); timeit(b, [&] { lane_rec_pol<1><<<G, 256>>>(recs, I, n, out); });
    snprintf(b, sizeof b, "%s lane 1x16B sc0 sc1", sn[k]); timeit(b, [&] { lane_rec_pol<2><<<G, 256>>>(recs, I, n, out); });
    snprintf(b, sizeof b, "%s lane 1x16B sc0 sc1 nt", sn[k]); timeit(b, [&] { lane_rec_pol<3><<<G, 256>>>(recs, I, n, out); });
    snprintf(b, sizeof b, "%s lane 1x16B sc0", sn[k]); timeit(b, [&] { lane_rec_pol<4><<<G, 256>>>(recs, I, n, out); });
    snprintf(b, sizeof b, "%s quad 4x16B", sn[k]); timeit(b, [&] { quad_rec<<<(unsigned)((4ull * n + 255) / 256), 256>>>(recs, I, n, out); });

    static u64 v = 1ull << 40;
    if (k == 1) snprintf(b, sizeof b, "%s atomicMax u64 per msg", sn[k]), timeit(b, [&] { v += 1ull << 32; lane_atomic<<<G, 256>>>(recs, I, n, v); });
  }
  return 0;
}
