// Streaming cost of the fast Receive kernel's per-message inputs on gfx950
// (not product code): 100M messages of the C2 shape (names "b<id>", Zipf
// ids over 10M keys, u32 offsets, three 8-byte replica fields), read the way
// k_receive_fast reads them, with no table access.
//   T1 offsets          T2 + name words       T3 + replica fields
//   T4 T3 + FNV/canonical name (the product's VALU for the name)
//   T5 replica fields only
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../patrol_amd/csrc/phip_kernels.hpp"

using namespace phip;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

template <int V>
__global__ __launch_bounds__(256) void k_stream(NamesOffs src, const uint64_t* __restrict__ ma,
                                                const uint64_t* __restrict__ mt,
                                                const int64_t* __restrict__ me, u32 n, u64* sink) {
  const u32 i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  u64 acc = 0;
  u64 off = 0; u32 len = 0;
  if (V != 5) { src.get<true>(i, off, len); acc = off + len; }
  if (V >= 2 && V != 5) {
    u64 w0, w1, w2;
    load_words3<true>(src.blob, off, len, w0, w1, w2);
    if (V == 4) {
      Name nm;
      short_name(w0, w1, w2, off, len, nm);
      acc ^= nm.h ^ nm.w0 ^ nm.w1;
    } else {
      acc ^= w0 ^ w1 ^ w2;
    }
  }
  if (V >= 3) acc ^= ld<true>(ma + i) ^ ld<true>(mt + i) ^ (u64)ld<true>(me + i);
  if (acc == 0x123456789ull) sink[0] = acc;
}

int main() {
  const u32 K = 10000000u, n = 100000000u;
  std::vector<double> cdf(K);
  double acc = 0;
  for (u32 r = 0; r < K; ++r) { acc += std::pow((double)(r + 1), -1.1); cdf[r] = acc; }
  u64 mult = 2654435761ull % K;
  while (std::__gcd<u64>(mult, K) != 1) ++mult;
  std::mt19937_64 rng(42);
  std::vector<u32> offs(n + 1);
  std::vector<u8> blob;
  blob.reserve((size_t)n * 8 + 16);
  char buf[32];
  for (u32 i = 0; i < n; ++i) {
    double u = (rng() >> 11) * (1.0 / 9007199254740992.0) * acc;
    u32 r = (u32)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
    if (r >= K) r = K - 1;
    u32 id = (u32)(((u64)r * mult) % K);
    offs[i] = (u32)blob.size();
    int len = snprintf(buf, sizeof buf, "b%u", id);
    blob.insert(blob.end(), buf, buf + len);
  }
  offs[n] = (u32)blob.size();
  for (int k = 0; k < 16; ++k) blob.push_back(0);
  printf("blob %.2f GB\n", blob.size() / 1e9);
  u8* dblob; u32* doffs; uint64_t *da, *dt; int64_t* de; u64* sink;
  CK(hipMalloc(&dblob, blob.size())); CK(hipMalloc(&doffs, (n + 1) * 4ull));
  CK(hipMalloc(&da, n * 8ull)); CK(hipMalloc(&dt, n * 8ull)); CK(hipMalloc(&de, n * 8ull));
  CK(hipMalloc(&sink, 64));
  CK(hipMemcpy(dblob, blob.data(), blob.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(doffs, offs.data(), (n + 1) * 4ull, hipMemcpyHostToDevice));
  CK(hipMemset(da, 1, n * 8ull)); CK(hipMemset(dt, 2, n * 8ull)); CK(hipMemset(de, 3, n * 8ull));
  NamesOffs src{dblob, doffs};
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto launch) {
    float best = 1e9;
    for (int r = 0; r < 4; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r) best = std::min(best, ms);
    }
    printf("%-34s %8.3f ms  %7.2f G msg/s  %7.1f GB/s\n", name, best, n / best / 1e6, bytes / best / 1e6);
  };
  const unsigned G = (n + 255) / 256;
  const double ob = 4.0 * n, nb = (double)blob.size(), sb = 24.0 * n;
  timeit("T1 offsets", ob, [&] { k_stream<1><<<G, 256>>>(src, da, dt, de, n, sink); });
  timeit("T2 + name words", ob + nb, [&] { k_stream<2><<<G, 256>>>(src, da, dt, de, n, sink); });
  timeit("T3 + replica fields", ob + nb + sb, [&] { k_stream<3><<<G, 256>>>(src, da, dt, de, n, sink); });
  timeit("T4 T3 + hash/canonical", ob + nb + sb, [&] { k_stream<4><<<G, 256>>>(src, da, dt, de, n, sink); });
  timeit("T5 replica fields only", sb, [&] { k_stream<5><<<G, 256>>>(src, da, dt, de, n, sink); });
  return 0;
}
