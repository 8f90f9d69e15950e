// Which fabric request serves a random 48-byte record read on gfx950 (not
// product code)?  k_receive_fast's cold probe reads the
// first 48 bytes of a 64-byte slot record (load_rec48, three 16-byte loads);
// every L2 miss of that kernel is a 128-byte TCC_EA0_RDREQ, so half of each
// fetched line is the neighbouring record.  This runs the same access (100M
// uniformly random records of a 2^25-slot, 2 GiB table) under every load
// form and cache policy the ISA offers for a global load, on three
// allocations (hipMalloc, uncached, fine-grained), one dispatch each, so a
// rocprofv3 --pmc pass over TCC_EA0_RDREQ_{32B,64B,128B} tells per variant
// how many bytes each record costs at the fabric.  Timing by HIP events.
//   usage: ubench_req [alloc mode 0|1|2] [n]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned long long u64;
typedef unsigned int u32;

// slot of message i: a fixed hash (uniform over the table)
__device__ inline u32 slot_of(u32 i, u32 mask) {
  u64 x = (u64)i * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 32;
  return (u32)x & mask;
}

#define LD16(POL)                                                                       \
  asm volatile("global_load_dwordx4 %0, %1, off " POL : "=v"(a) : "v"(p));             \
  asm volatile("global_load_dwordx4 %0, %1, off offset:16 " POL : "=v"(b) : "v"(p));   \
  asm volatile("global_load_dwordx4 %0, %1, off offset:32 " POL : "=v"(c) : "v"(p));   \
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

// V: 0 plain, 1 nt, 2 sc0, 3 sc1, 4 sc0 sc1, 5 sc0 sc1 nt, 6 sc1 nt
template <int V>
__global__ __launch_bounds__(256) void rec48(const char* __restrict__ recs, u32 mask, u32 n,
                                             u32* __restrict__ out) {
  const u32 i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const char* p = recs + (size_t)slot_of(i, mask) * 64;
  uint4 a, b, c;
  if (V == 0) { LD16("") }
  if (V == 1) { LD16("nt") }
  if (V == 2) { LD16("sc0") }
  if (V == 3) { LD16("sc1") }
  if (V == 4) { LD16("sc0 sc1") }
  if (V == 5) { LD16("sc0 sc1 nt") }
  if (V == 6) { LD16("sc1 nt") }
  out[i] = a.x ^ b.y ^ c.z;
}

// narrower loads: one dword / dwordx2 per lane (does a small read still
// fetch 128 bytes?), and the 48 bytes as six dwordx2
template <int W>
__global__ __launch_bounds__(256) void narrow(const char* __restrict__ recs, u32 mask, u32 n,
                                              u32* __restrict__ out) {
  const u32 i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const char* p = recs + (size_t)slot_of(i, mask) * 64;
  u32 x = 0;
  if (W == 4) x = *(const u32*)p;
  if (W == 8) { const u64 v = *(const u64*)p; x = (u32)v ^ (u32)(v >> 32); }
  if (W == 48) {
    const u64* q = (const u64*)p;
    u64 v = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) v ^= q[k];
    x = (u32)v ^ (u32)(v >> 32);
  }
  out[i] = x;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const u32 n = argc > 2 ? (u32)atoll(argv[2]) : 100000000u;
  const u32 L = 25;
  const u64 cap = 1ull << L;
  char* recs;
  if (mode == 0) CK(hipMalloc(&recs, cap * 64));
  else CK(hipExtMallocWithFlags((void**)&recs, cap * 64,
                                mode == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
  CK(hipMemset(recs, 1, cap * 64));
  u32* out;
  CK(hipMalloc(&out, n * 4ull));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned G = (n + 255) / 256;
  const u32 mask = (u32)(cap - 1);
  auto run = [&](const char* name, auto launch) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("alloc %d  %-22s %8.3f ms  %7.2f G rec/s\n", mode, name, ms, n / ms / 1e6);
  };
  run("48B plain", [&] { rec48<0><<<G, 256>>>(recs, mask, n, out); });
  run("48B nt", [&] { rec48<1><<<G, 256>>>(recs, mask, n, out); });
  run("48B sc0", [&] { rec48<2><<<G, 256>>>(recs, mask, n, out); });
  run("48B sc1", [&] { rec48<3><<<G, 256>>>(recs, mask, n, out); });
  run("48B sc0 sc1", [&] { rec48<4><<<G, 256>>>(recs, mask, n, out); });
  run("48B sc0 sc1 nt", [&] { rec48<5><<<G, 256>>>(recs, mask, n, out); });
  run("48B sc1 nt", [&] { rec48<6><<<G, 256>>>(recs, mask, n, out); });
  run("4B dword", [&] { narrow<4><<<G, 256>>>(recs, mask, n, out); });
  run("8B dwordx2", [&] { narrow<8><<<G, 256>>>(recs, mask, n, out); });
  run("48B 6x dwordx2", [&] { narrow<48><<<G, 256>>>(recs, mask, n, out); });
  CK(hipFree(recs));
  CK(hipFree(out));
  return 0;
}
