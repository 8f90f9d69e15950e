// Decoupled look-back on gfx950 (not product code): the chained per-tile
// prefix that a single-pass owner partition (phip_route_pack reading each
// message once) needs.  Every workgroup takes a tile by ticket, publishes
// its aggregate (W words, one per owner: flag and value in one 64-bit word,
// agent-scope relaxed atomic stores), looks back over its predecessors'
// descriptors in windows of 64 words (agent-scope relaxed atomic loads:
// the tiles run on all 8 XCDs, whose L2s are not coherent with each other),
// adds aggregates until it meets an inclusive prefix, and publishes its own
// inclusive prefix.  Nothing else is read or written: the time is the
// look-back chain's alone, a lower bound for the partition's look-back.
//
//   ubench_lookback [ntiles ...]      (W = 1 and W = 8 owners for each)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned long long u64;
typedef unsigned int u32;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

constexpr u64 kAgg = 1ull << 62, kInc = 2ull << 62, kVal = (1ull << 62) - 1;

__device__ inline u64 ld_agent(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_agent(u64* p, u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline u64 agg_of(u32 tile, u32 o) { return (tile * 7ull + o) % 13 + 1; }

template <int W>
__global__ __launch_bounds__(256) void k_lookback(u64* desc, u32* ticket, u32 ntiles, u64* spins) {
  __shared__ u32 tile_s;
  if (threadIdx.x == 0) tile_s = atomicAdd(ticket, 1u);
  __syncthreads();
  const u32 tile = tile_s;
  if (tile >= ntiles || threadIdx.x >= 64) return;
  const u32 lane = threadIdx.x, o = lane % W, p = lane / W;   // window position p, owner o
  constexpr u32 kTiles = 64 / W;                               // tiles per window
  const u64 mine = agg_of(tile, o);
  if (lane < W) st_agent(&desc[(u64)tile * W + o], (tile ? kAgg : kInc) | mine);
  if (tile == 0) return;
  u64 sum = 0;   // lane o < W: owner o's exclusive prefix
  u64 nspin = 0;
  for (long base = (long)tile - 1; base >= 0;) {
    const long t = base - (long)p;
    const u64 v = t >= 0 ? ld_agent(&desc[(u64)t * W + o]) : kInc;   // before tile 0: prefix 0
    const u64 f = v & ~kVal;
    // the nearest window position whose words are all inclusive
    const u64 inc = __ballot(f == kInc);
    u32 pstar = kTiles;
    for (u32 q = 0; q < kTiles; ++q) {
      const u64 m = ((W == 64) ? ~0ull : ((1ull << W) - 1)) << (q * W);
      if ((inc & m) == m) { pstar = q; break; }
    }
    const u64 ready = __ballot(f != 0);
    const u32 upto = pstar < kTiles ? pstar : kTiles - 1;
    const u64 need = (upto + 1) * W >= 64 ? ~0ull : ((1ull << ((upto + 1) * W)) - 1);
    if ((ready & need) != need) {   // a predecessor not published yet
      if (++nspin > (1ull << 22)) { sum = kVal; break; }   // bounded: a wrong result, never a hang
      continue;
    }
    u64 x = (p <= upto && t >= 0) ? (v & kVal) : 0;
    for (u32 d = W; d < 64; d <<= 1) x += __shfl_xor(x, d);   // sum over positions, per owner
    sum += x;
    if (pstar < kTiles) break;
    base -= kTiles;
  }
  if (lane < W) st_agent(&desc[(u64)tile * W + o], kInc | (sum + mine));
  if (lane == 0) atomicAdd(spins, nspin);
}

template <int W>
void run(u32 ntiles) {
  u64 *desc, *spins;
  u32* ticket;
  CK(hipMalloc(&desc, (size_t)ntiles * W * 8));
  CK(hipMalloc(&ticket, 4));
  CK(hipMalloc(&spins, 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  u64 sp = 0;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemset(desc, 0, (size_t)ntiles * W * 8));
    CK(hipMemset(ticket, 0, 4));
    CK(hipMemset(spins, 0, 8));
    CK(hipEventRecord(a));
    k_lookback<W><<<ntiles, 256>>>(desc, ticket, ntiles, spins);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
    CK(hipMemcpy(&sp, spins, 8, hipMemcpyDeviceToHost));
  }
  std::vector<u64> h((size_t)ntiles * W);
  CK(hipMemcpy(h.data(), desc, h.size() * 8, hipMemcpyDeviceToHost));
  bool ok = true;
  for (u32 o = 0; o < (u32)W; ++o) {
    u64 run = 0;
    for (u32 t = 0; t < ntiles; ++t) {
      run += (t * 7ull + o) % 13 + 1;
      if (h[(u64)t * W + o] != (kInc | run)) ok = false;
    }
  }
  printf("{\"owners\": %d, \"tiles\": %u, \"ms\": %.4f, \"us_per_tile\": %.4f, \"spins_last\": %llu, "
         "\"correct\": %s}\n", W, ntiles, best, best * 1e3 / ntiles, sp, ok ? "true" : "false");
  fflush(stdout);
  CK(hipFree(desc));
  CK(hipFree(ticket));
  CK(hipFree(spins));
}

int main(int argc, char** argv) {
  std::vector<u32> sizes;
  for (int i = 1; i < argc; ++i) sizes.push_back((u32)atoi(argv[i]));
  if (sizes.empty()) sizes = {24414, 48828, 97657};   // 100M messages in tiles of 4096 / 2048 / 1024
  for (u32 n : sizes) {
    run<1>(n);
    run<8>(n);
  }
  return 0;
}
