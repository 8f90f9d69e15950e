// Load generator for the Take batcher (phip_batcher_*): T client threads,
// each issuing M POST /take-shaped requests back to back (rate 100:1s,
// count 1, Zipf(1.1) names over K pre-created buckets), the way Go's HTTP
// server runs one goroutine per request (api.go:51-86).  Prints one JSON
// line: takes/s over the whole run, p50/p99/p999 request latency, batch
// statistics.  Links libpatrolhip through its C ABI only.
//
//   take_load [threads] [per_thread] [window_us] [buckets] [peers] [new_frac]
//
// peers = 0: the bare batched Take (phip_batcher_take).
// peers > 0: the whole drop-in handler (INTEGRATION.md takeBucket): the
//   request strings go through phip_batcher_api_take_reply (ParseRate and
//   count parsing, api.go:60-65), and from the reply of the same batched
//   launch the handler replicates as the reference does: a request whose
//   GetBucket created the bucket first sends the zero-state incast
//   (repo.go:96-106), then the post-Take datagram goes to every peer
//   (UpsertBucket -> broadcast, repo.go:123-158), one sendto per peer per
//   take (a UDP sink on 127.0.0.1 stands in for the peers).  new_frac of the
//   requests name buckets that do not exist yet.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
  const int peers = argc > 5 ? atoi(argv[5]) : 0;
  const double new_frac = argc > 6 ? atof(argv[6]) : 0.01;
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
  // the peers' stand-in: one UDP sink on the loopback, drained by a thread
  int sink = -1, tx = -1;
  sockaddr_in sink_addr{};
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> got_dgrams{0};
  std::thread drain;
  if (peers > 0) {
    sink = socket(AF_INET, SOCK_DGRAM, 0);
    tx = socket(AF_INET, SOCK_DGRAM, 0);
    sink_addr.sin_family = AF_INET;
    sink_addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    sink_addr.sin_port = 0;
    socklen_t al = sizeof sink_addr;
    if (sink < 0 || tx < 0 || bind(sink, (sockaddr*)&sink_addr, sizeof sink_addr) ||
        getsockname(sink, (sockaddr*)&sink_addr, &al)) {
      perror("udp sink");
      return 1;
    }
    int big = 64 << 20;
    setsockopt(sink, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    timeval tv{0, 100000};
    setsockopt(sink, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    drain = std::thread([&] {
      uint8_t buf[512];
      while (!stop.load()) {
        if (recv(sink, buf, sizeof buf, 0) > 0) got_dgrams.fetch_add(1);
      }
    });
  }
  // Zipf(1.1) ranks -> ids (a fixed scatter), per thread its own stream
  std::vector<double> cdf(K);
  double acc = 0;
  for (uint32_t k = 0; k < K; ++k) cdf[k] = (acc += std::pow((double)(k + 1), -1.1));
  for (auto& c : cdf) c /= acc;
  std::vector<std::vector<double>> lat(T);
  std::vector<uint64_t> oks(T, 0), created(T, 0), sent(T, 0);
  auto client = [&](int tid) {
    std::mt19937_64 rng(1234 + tid);
    std::uniform_real_distribution<double> u(0, 1);
    lat[tid].reserve(M);
    std::string name;
    static const char rate[] = "100:1s", count[] = "1";
    uint8_t incast[PHIP_BUCKET_PACKET_SIZE];
    for (int i = 0; i < M; ++i) {
      const uint32_t r = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u(rng)) - cdf.begin());
      if (peers > 0 && u(rng) < new_frac)
        name = "n" + std::to_string(tid) + "-" + std::to_string(i);   // a bucket nobody holds yet
      else
        name = "b" + std::to_string((uint64_t)r * 2654435761ull % K);
      const auto a = std::chrono::steady_clock::now();
      const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::system_clock::now().time_since_epoch()).count();
      if (peers == 0) {
        uint64_t rem = 0;
        uint8_t ok = 0;
        if (phip_batcher_take(b, (const uint8_t*)name.data(), (uint32_t)name.size(), now, 100,
                              1000000000, 1, &rem, &ok, nullptr)) {
          fprintf(stderr, "take failed\n");
          std::exit(1);
        }
        oks[tid] += ok;
      } else {
        char body[64];
        uint32_t blen = 0;
        phip_take_reply rep;
        const int code = phip_batcher_api_take_reply(
            b, (const uint8_t*)name.data(), (uint32_t)name.size(), rate, sizeof rate - 1, count,
            sizeof count - 1, now, body, &blen, &rep);
        if (code < 0) {
          fprintf(stderr, "api take failed\n");
          std::exit(1);
        }
        oks[tid] += code == 200;
        if (rep.created) {   // ReplicatedRepo.GetBucket's incast (repo.go:96-106)
          ++created[tid];
          std::memset(incast, 0, 24);
          std::memcpy(incast + 24, rep.datagram + 24, rep.datagram_len - 24u);
          for (int p = 0; p < peers; ++p)
            sent[tid] += sendto(tx, incast, rep.datagram_len, 0, (sockaddr*)&sink_addr,
                                sizeof sink_addr) > 0;
        }
        for (int p = 0; p < peers; ++p)   // UpsertBucket's broadcast (repo.go:129-158)
          sent[tid] += sendto(tx, rep.datagram, rep.datagram_len, 0, (sockaddr*)&sink_addr,
                              sizeof sink_addr) > 0;
      }
      lat[tid].push_back(std::chrono::duration<double, std::micro>(
                             std::chrono::steady_clock::now() - a).count());
    }
  };
  std::vector<std::thread> th;
  const auto w0 = std::chrono::steady_clock::now();
  for (int t = 0; t < T; ++t) th.emplace_back(client, t);
  for (auto& x : th) x.join();
  const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
  if (peers > 0) {
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
    stop.store(true);
    drain.join();
    close(sink);
    close(tx);
  }
  std::vector<double> all;
  for (auto& l : lat) all.insert(all.end(), l.begin(), l.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all[std::min(all.size() - 1, (size_t)(p * all.size()))]; };
  uint64_t s[5] = {0, 0, 0, 0, 0};
  phip_batcher_stats(b, s, 5);
  uint64_t okn = 0, cr = 0, sn = 0;
  for (int t = 0; t < T; ++t) { okn += oks[t]; cr += created[t]; sn += sent[t]; }
  printf("{\"mode\": \"%s\", \"threads\": %d, \"requests\": %zu, \"window_us\": %u, \"buckets\": %u, "
         "\"peers\": %d, \"takes_per_s\": %.1f, \"p50_us\": %.1f, \"p99_us\": %.1f, \"p999_us\": %.1f, "
         "\"batches\": %llu, \"mean_batch\": %.1f, \"max_batch\": %llu, "
         "\"gpu_call_us_per_batch\": %.1f, \"ok_fraction\": %.3f, \"created\": %llu, "
         "\"datagrams_sent\": %llu, \"datagrams_received\": %llu}\n",
         peers ? "handler" : "take", T, all.size(), window, K, peers, all.size() / wall, pct(0.5),
         pct(0.99), pct(0.999), (unsigned long long)s[0], (double)s[1] / std::max<uint64_t>(1, s[0]),
         (unsigned long long)s[2], s[3] / 1e3 / std::max<uint64_t>(1, s[0]),
         (double)okn / all.size(), (unsigned long long)cr, (unsigned long long)sn,
         (unsigned long long)got_dgrams.load());
  phip_batcher_close(b);
  phip_close(h);
  return 0;
}
