// Microbenchmark: what does a random bucket-state update cost on gfx950?
// Used to choose between (a) device-scope 64-bit atomicMax on scattered slots
// and (b) owner-partitioned plain read-modify-write for the batched merge.
// Not part of the product; results are recorded in DESIGN.md.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>
#include <cmath>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

typedef unsigned long long u64;

// (a) 3 lanes-worth of atomics issued by one lane, AoS slot of 32 B.
__global__ void k_atomic_aos(const uint32_t* __restrict__ slot, const u64* __restrict__ va,
                             const u64* __restrict__ vt, const u64* __restrict__ ve,
                             u64* table, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u64* p = table + 4ull * slot[i];
  atomicMax(p + 0, va[i]);
  atomicMax(p + 1, vt[i]);
  atomicMax(p + 2, ve[i]);
}

// (b) 4 lanes per message, one u64 each: lanes of one message hit one 32-B chunk.
__global__ void k_atomic_aos4(const uint32_t* __restrict__ slot, const u64* __restrict__ va,
                              const u64* __restrict__ vt, const u64* __restrict__ ve,
                              u64* table, uint32_t n) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t i = (uint32_t)(t >> 2), f = (uint32_t)(t & 3);
  if (i >= n || f == 3) return;
  u64 v = f == 0 ? va[i] : (f == 1 ? vt[i] : ve[i]);
  atomicMax(table + 4ull * slot[i] + f, v);
}

// (c) plain random RMW (not correct under races; throughput only).
__global__ void k_plain_rmw(const uint32_t* __restrict__ slot, const u64* __restrict__ va,
                            const u64* __restrict__ vt, const u64* __restrict__ ve,
                            u64* table, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ulonglong2* p = reinterpret_cast<ulonglong2*>(table + 4ull * slot[i]);
  ulonglong2 a = p[0], b = p[1];
  a.x = max(a.x, va[i]); a.y = max(a.y, vt[i]); b.x = max(b.x, ve[i]);
  p[0] = a; p[1] = b;
}

// (d) streaming read of the 28 B message (slot + 3 u64) and a tiny write.
__global__ void k_stream(const uint32_t* __restrict__ slot, const u64* __restrict__ va,
                         const u64* __restrict__ vt, const u64* __restrict__ ve,
                         u64* out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u64 x = va[i] ^ vt[i] ^ ve[i] ^ slot[i];
  if (x == 0x1234567ull) out[0] = x;
}

// (e) block-local LDS combine (open addressing on slot), then global atomics
// for the survivors.  T messages per block.
template <int BLOCK, int PER>
__global__ __launch_bounds__(BLOCK) void k_lds_combine(const uint32_t* __restrict__ slot,
    const u64* __restrict__ va, const u64* __restrict__ vt, const u64* __restrict__ ve,
    u64* table, uint32_t n, u64* survivors) {
  constexpr int T = BLOCK * PER, CAP = 2 * T;
  __shared__ uint32_t key[CAP];
  __shared__ u64 A[CAP], B[CAP], C[CAP];
  for (int j = threadIdx.x; j < CAP; j += BLOCK) { key[j] = 0xFFFFFFFFu; A[j] = 0; B[j] = 0; C[j] = 0; }
  __syncthreads();
  uint64_t base = (uint64_t)blockIdx.x * T;
  for (int k = 0; k < PER; ++k) {
    uint64_t i = base + (uint64_t)k * BLOCK + threadIdx.x;
    if (i >= n) break;
    uint32_t s = slot[i];
    uint32_t h = (s * 2654435761u) & (CAP - 1);
    while (true) {
      uint32_t old = atomicCAS(&key[h], 0xFFFFFFFFu, s);
      if (old == 0xFFFFFFFFu || old == s) break;
      h = (h + 1) & (CAP - 1);
    }
    atomicMax(&A[h], va[i]); atomicMax(&B[h], vt[i]); atomicMax(&C[h], ve[i]);
  }
  __syncthreads();
  uint32_t cnt = 0;
  for (int j = threadIdx.x; j < CAP; j += BLOCK) {
    uint32_t s = key[j];
    if (s == 0xFFFFFFFFu) continue;
    ++cnt;
    u64* p = table + 4ull * s;
    atomicMax(p + 0, A[j]); atomicMax(p + 1, B[j]); atomicMax(p + 2, C[j]);
  }
  atomicAdd(survivors, (u64)cnt);
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? atoi(argv[1]) : 100000000u;
  const uint32_t K = 10000000u;          // distinct buckets
  const uint32_t L = 24;                 // 2^24 slots
  printf("n=%u K=%u slots=2^%u\n", n, K, L);
  // Zipf(1.1) ranks via inverse CDF over K, mapped to slots by a bijection.
  std::vector<double> cdf(K);
  double acc = 0;
  for (uint32_t r = 0; r < K; ++r) { acc += std::pow((double)(r + 1), -1.1); cdf[r] = acc; }
  std::vector<uint32_t> hz(n), hu(n);
  std::vector<u64> ha(n), ht(n), he(n);
  std::mt19937_64 rng(42);
  std::vector<uint32_t> slot_of(K);
  for (uint32_t r = 0; r < K; ++r) slot_of[r] = (uint32_t)(((u64)r * 0x9E3779B97F4A7C15ull) >> (64 - L));
  for (uint32_t i = 0; i < n; ++i) {
    double u = (rng() >> 11) * (1.0 / 9007199254740992.0) * acc;
    uint32_t r = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
    if (r >= K) r = K - 1;
    hz[i] = slot_of[r];
    hu[i] = slot_of[rng() % K];
    ha[i] = rng(); ht[i] = rng(); he[i] = rng();
  }
  uint32_t *dz, *du; u64 *da, *dt, *de, *tab, *surv;
  CK(hipMalloc(&dz, 4ull * n)); CK(hipMalloc(&du, 4ull * n));
  CK(hipMalloc(&da, 8ull * n)); CK(hipMalloc(&dt, 8ull * n)); CK(hipMalloc(&de, 8ull * n));
  CK(hipMalloc(&tab, 32ull << L)); CK(hipMalloc(&surv, 8));
  CK(hipMemcpy(dz, hz.data(), 4ull * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(du, hu.data(), 4ull * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(da, ha.data(), 8ull * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ht.data(), 8ull * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(de, he.data(), 8ull * n, hipMemcpyHostToDevice));
  CK(hipMemset(tab, 0, 32ull << L));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    const int reps = 5;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    printf("%-28s %8.3f ms  %7.2f G msg/s  %7.1f GB/s@88B\n", name, ms, n / ms / 1e6, 88.0 * n / ms / 1e6);
  };
  const int B = 256;
  for (int z = 0; z < 2; ++z) {
    uint32_t* ds = z ? du : dz;
    const char* tag = z ? "uniform" : "zipf1.1";
    printf("-- %s\n", tag);
    timeit("stream 28B", [&] { k_stream<<<(n + B - 1) / B, B>>>(ds, da, dt, de, surv, n); });
    timeit("plain rmw 32B", [&] { k_plain_rmw<<<(n + B - 1) / B, B>>>(ds, da, dt, de, tab, n); });
    timeit("atomic aos 1 lane", [&] { k_atomic_aos<<<(n + B - 1) / B, B>>>(ds, da, dt, de, tab, n); });
    timeit("atomic aos 4 lanes", [&] { k_atomic_aos4<<<(unsigned)((4ull * n + B - 1) / B), B>>>(ds, da, dt, de, tab, n); });
    CK(hipMemset(surv, 0, 8));
    timeit("lds combine 256x8", [&] { k_lds_combine<256, 8><<<(n + 2047) / 2048, 256>>>(ds, da, dt, de, tab, n, surv); });
    u64 sv; CK(hipMemcpy(&sv, surv, 8, hipMemcpyDeviceToHost));
    printf("   survivors/launch %.3f of n\n", sv / 6.0 / n);
    CK(hipMemset(surv, 0, 8));
    timeit("lds combine 256x4", [&] { k_lds_combine<256, 4><<<(n + 1023) / 1024, 256>>>(ds, da, dt, de, tab, n, surv); });
    CK(hipMemcpy(&sv, surv, 8, hipMemcpyDeviceToHost));
    printf("   survivors/launch %.3f of n\n", sv / 6.0 / n);
  }
  return 0;
}
