// Would a dense "warm" record layout pay? (not product code)
// The C2 fast kernel reads a 64-B slot record for every message that misses
// the 384-entry hot directory (Zipf ranks >= 384, 41% of the batch).  Records
// sit at hash-scattered slots of a 2^25-slot table, so every 128-B L2 line
// holds one useful record and one unrelated one.  This measures the same
// 41M tail reads (3 x 16 B per lane, as load_rec48) with two layouts:
//   scattered: every rank at its hash slot (today's table);
//   dense W:   ranks 384 .. W-1 packed contiguously (two warm records per
//              128-B line, W*64 B of warm data), the rest scattered.
// Usage: ubench_warm [n_messages]
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

__global__ __launch_bounds__(256) void read48(const uint4* __restrict__ recs, const u32* __restrict__ idx,
                                              u32 n, u32* __restrict__ out) {
  u32 i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  u32 s = __builtin_nontemporal_load(idx + i);
  const uint4* p = recs + (size_t)s * 4;
  uint4 a = p[0], b = p[1], c = p[2];
  out[i] = a.x ^ b.y ^ c.z;
}

int main(int argc, char** argv) {
  const u32 L = 25, K = 10000000u, kHot = 384;
  const u32 n_all = argc > 1 ? atoi(argv[1]) : 100000000u;
  const u64 cap = 1ull << L;
  std::vector<u32> ranks;
  ranks.reserve(n_all / 2);
  {
    std::vector<double> cdf(K);
    double acc = 0;
    for (u32 r = 0; r < K; ++r) { acc += std::pow((double)(r + 1), -1.1); cdf[r] = acc; }
    std::mt19937_64 rng(42);
    for (u32 i = 0; i < n_all; ++i) {
      double u = (rng() >> 11) * (1.0 / 9007199254740992.0) * acc;
      u32 r = (u32)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
      if (r >= K) r = K - 1;
      if (r >= kHot) ranks.push_back(r);   // the directory takes the rest
    }
  }
  const u32 n = (u32)ranks.size();
  printf("tail messages: %u of %u (%.1f%%)\n", n, n_all, 100.0 * n / n_all);
  auto scattered = [&](u32 r) { return (u32)((u64)r * 0x9E3779B97F4A7C15ull >> (64 - L)); };
  uint4* recs; u32 *didx, *out;
  CK(hipMalloc(&recs, cap * 64));
  CK(hipMemset(recs, 1, cap * 64));
  CK(hipMalloc(&didx, n * 4ull));
  CK(hipMalloc(&out, n * 4ull));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<u32> idx(n);
  const u32 widths[] = {0, 16384, 32768, 65536, 131072, 262144};
  for (u32 W : widths) {
    // dense region at the top of the table: slot cap - W + r for r < W
    for (u32 i = 0; i < n; ++i) {
      const u32 r = ranks[i];
      idx[i] = (W && r < W) ? (u32)(cap - W + r) : scattered(r);
    }
    CK(hipMemcpy(didx, idx.data(), n * 4ull, hipMemcpyHostToDevice));
    float best = 1e9;
    for (int k = 0; k < 5; ++k) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      read48<<<(n + 255) / 256, 256>>>(recs, didx, n, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (k) best = std::min(best, ms);
    }
    if (W) printf("dense ranks < %-7u (%6.1f MB warm)  %7.3f ms  %6.2f G rec/s\n", W, W * 64.0 / 1e6, best, n / best / 1e6);
    else printf("scattered (today's table)            %7.3f ms  %6.2f G rec/s\n", best, n / best / 1e6);
  }
  return 0;
}
