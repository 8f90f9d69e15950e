// The anti-entropy join's read pattern on gfx950 (not product code): R
// replica planes of B int64 values read together, 16 bytes per lane from
// each, the maximum kept (k_ae_join's loads, no stores).  The planes lie
// `stride` bytes apart: the bench's layout [R, 3, B] puts them 3 * 8 * B =
// 384 MiB apart (B = 2^24), a multiple of every power-of-two interleave
// below 128 MiB, so the R streams are read at the same interleave offset.
// Padding the stride by a few KiB staggers them.
//
//   ubench_ae [R] [log2 B]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef unsigned int u32;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

template <int R>
__global__ __launch_bounds__(256) void k_read(const u64* __restrict__ base, u64 stride_w, u64 B,
                                              u64* sink) {
  const u64 i = 2 * ((u64)blockIdx.x * 256 + threadIdx.x);
  if (i >= B) return;
  u64x2 best = {0, 0};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const u64x2 v = *reinterpret_cast<const u64x2*>(base + r * stride_w + i);
    best.x = v.x > best.x ? v.x : best.x;
    best.y = v.y > best.y ? v.y : best.y;
  }
  if ((best.x ^ best.y) == 0x1234567ull) sink[0] = best.x;   // keeps the loads
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 8;
  const u32 lb = argc > 2 ? (u32)atoi(argv[2]) : 24;
  const u64 B = 1ull << lb;
  const u64 pads[] = {0, 4096, 65536 + 4096, 1u << 20};
  const u64 strides_planes[] = {3, 1};   // [R, 3, B] (bench) and [R, B] (one plane per replica)
  u64* sink;
  CK(hipMalloc(&sink, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (u64 planes : strides_planes)
    for (u64 pad : pads) {
      const u64 stride_b = planes * 8 * B + pad;
      u64* base;
      CK(hipMalloc(&base, stride_b * R + 64));
      CK(hipMemset(base, 1, stride_b * R));
      const u64 sw = stride_b / 8;
      const unsigned grid = (unsigned)((B / 2 + 255) / 256);
      float best = 1e30f;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(a));
        if (R == 8) k_read<8><<<grid, 256>>>(base, sw, B, sink);
        else k_read<4><<<grid, 256>>>(base, sw, B, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep && ms < best) best = ms;
      }
      const double bytes = 8.0 * B * R;
      printf("{\"replicas\": %d, \"B\": %llu, \"plane_stride_bytes\": %llu, \"pad\": %llu, "
             "\"ms\": %.4f, \"TBps\": %.3f}\n", R, B, stride_b, pad, best, bytes / best / 1e9);
      fflush(stdout);
      CK(hipFree(base));
    }
  return 0;
}
