// Load generator for the Take batcher (phip_batcher_*): T client threads,
// each issuing M POST /take-shaped requests back to back (rate 100:1s,
// count 1, Zipf(1.1) names over K pre-created buckets), the way Go's HTTP
// server runs one goroutine per request (api.go:51-86).  Prints one JSON
// line: takes/s over the whole run, p50/p99/p999 request latency, batch
// statistics.  Links libpatrolhip through its C ABI only.
//
//   take_load [threads] [per_thread] [window_us] [buckets]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "patrolhip.h"

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 64;
  const int M = argc > 2 ? atoi(argv[2]) : 2000;
  const uint32_t window = argc > 3 ? (uint32_t)atoi(argv[3]) : 20;
  const uint32_t K = argc > 4 ? (uint32_t)atoi(argv[4]) : 100000;
  phip_config cfg{};
  cfg.device = 0;
  cfg.log2_slots = 20;
  cfg.arena_bytes = 1 << 20;
  phip_handle* h = nullptr;
  if (phip_open(&cfg, &h)) { fprintf(stderr, "phip_open failed\n"); return 1; }
  // K buckets b0..b{K-1}, created now
  const int64_t t0ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                           std::chrono::system_clock::now().time_since_epoch()).count();
  {
    std::string blob;
    std::vector<uint32_t> offs{0};
    std::vector<phip_state> st(K);
    for (uint32_t k = 0; k < K; ++k) {
      blob += "b" + std::to_string(k);
      offs.push_back((uint32_t)blob.size());
      st[k] = phip_state{0, 0, 0, t0ns};
    }
    if (phip_seed(h, (const uint8_t*)blob.data(), offs.data(), K, st.data(), 0)) return 1;
  }
  phip_batcher_config bc{window, 0};
  phip_batcher* b = nullptr;
  if (phip_batcher_open(h, &bc, &b)) return 1;
  // Zipf(1.1) ranks -> ids (a fixed scatter), per thread its own stream
  std::vector<double> cdf(K);
  double acc = 0;
  for (uint32_t k = 0; k < K; ++k) cdf[k] = (acc += std::pow((double)(k + 1), -1.1));
  for (auto& c : cdf) c /= acc;
  std::vector<std::vector<double>> lat(T);
  std::vector<uint64_t> oks(T, 0);
  auto client = [&](int tid) {
    std::mt19937_64 rng(1234 + tid);
    std::uniform_real_distribution<double> u(0, 1);
    lat[tid].reserve(M);
    std::string name;
    for (int i = 0; i < M; ++i) {
      const uint32_t r = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u(rng)) - cdf.begin());
      name = "b" + std::to_string((uint64_t)r * 2654435761ull % K);
      const auto a = std::chrono::steady_clock::now();
      const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::system_clock::now().time_since_epoch()).count();
      uint64_t rem = 0;
      uint8_t ok = 0;
      if (phip_batcher_take(b, (const uint8_t*)name.data(), (uint32_t)name.size(), now, 100,
                            1000000000, 1, &rem, &ok, nullptr)) {
        fprintf(stderr, "take failed\n");
        std::exit(1);
      }
      oks[tid] += ok;
      lat[tid].push_back(std::chrono::duration<double, std::micro>(
                             std::chrono::steady_clock::now() - a).count());
    }
  };
  std::vector<std::thread> th;
  const auto w0 = std::chrono::steady_clock::now();
  for (int t = 0; t < T; ++t) th.emplace_back(client, t);
  for (auto& x : th) x.join();
  const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
  std::vector<double> all;
  for (auto& l : lat) all.insert(all.end(), l.begin(), l.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all[std::min(all.size() - 1, (size_t)(p * all.size()))]; };
  uint64_t s[5] = {0, 0, 0, 0, 0};
  phip_batcher_stats(b, s, 5);
  uint64_t okn = 0;
  for (auto v : oks) okn += v;
  printf("{\"threads\": %d, \"requests\": %zu, \"window_us\": %u, \"buckets\": %u, "
         "\"takes_per_s\": %.1f, \"p50_us\": %.1f, \"p99_us\": %.1f, \"p999_us\": %.1f, "
         "\"batches\": %llu, \"mean_batch\": %.1f, \"max_batch\": %llu, "
         "\"gpu_call_us_per_batch\": %.1f, \"ok_fraction\": %.3f}\n",
         T, all.size(), window, K, all.size() / wall, pct(0.5), pct(0.99), pct(0.999),
         (unsigned long long)s[0], (double)s[1] / std::max<uint64_t>(1, s[0]),
         (unsigned long long)s[2], s[3] / 1e3 / std::max<uint64_t>(1, s[0]),
         (double)okn / all.size());
  phip_batcher_close(b);
  phip_close(h);
  return 0;
}
