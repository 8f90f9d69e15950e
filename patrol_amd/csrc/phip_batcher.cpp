// Request-coalescing Take batcher: the drop-in form of
// Patrol's POST /take handler over the batched engine.
//
// The reference answers every HTTP request on its own goroutine with
// GetBucket -> Bucket.Take -> UpsertBucket under the bucket's mutex
// (api.go:67-74, bucket.go:186-225).  A device-resident table wants batches,
// so concurrent requests are coalesced here: each caller thread enqueues its
// Take (arrival order is the batch order, which per-bucket order follows, as
// the bucket mutex serialises the reference's goroutines in lock order) and
// blocks; one dispatcher thread closes a batch `window_us` after its first
// request arrived (or at max_batch requests), runs it through
// phip_apply_mixed (GetBucket + Take per op, exact Go semantics in index
// order) and wakes the callers with their (remaining, ok).  Requests that
// arrive while a batch is on the GPU form the next batch, so under load the
// batches grow by themselves.
//
// Host code only: every device call goes through the public C ABI.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "patrolhip.h"
#include "phip_host.hpp"

namespace {

using Clock = std::chrono::steady_clock;

struct Req {
  const uint8_t* name;
  uint32_t len;
  int64_t now, freq, per;
  uint64_t count;
  uint64_t remaining = 0;
  uint64_t seq = 0;
  uint8_t status = 0;
  phip_state post{};            // the bucket right after this Take (phip_results.reply)
  int rc = 0;
  bool done = false;
  std::condition_variable cv;   // its caller waits here (woken alone, not with every waiter)
};

}  // namespace

constexpr uint32_t kSpinWindowUs = 500;   // windows up to this long are yield-waited

struct phip_batcher {
  phip_handle* h = nullptr;
  uint32_t window_us = 20;
  uint32_t max_batch = 1u << 16;
  std::mutex mu;
  std::condition_variable cv_submit;   // the dispatcher waits for requests
  std::vector<Req*> pending;
  Clock::time_point first_arrival;
  bool stop = false;
  uint32_t waiters = 0;                // callers inside submit_and_wait (under mu)
  std::condition_variable cv_idle;     // close() waits here for waiters == 0
  std::thread th;
  // stats
  uint64_t batches = 0, requests = 0, max_seen = 0, gpu_ns = 0, errors = 0;
  uint64_t arrivals = 0;   // arrival numbers handed out (under mu)
  // dispatcher scratch (host arrays of one batch)
  std::vector<uint8_t> kind, names, status;
  std::vector<uint32_t> offs;
  std::vector<int64_t> now, freq, per;
  std::vector<uint64_t> count, remaining;
  std::vector<phip_state> post;

  void run();
  void dispatch(std::vector<Req*>& batch);
};

void phip_batcher::dispatch(std::vector<Req*>& batch) {
  const uint32_t n = (uint32_t)batch.size();
  kind.assign(n, PHIP_OP_TAKE);
  offs.resize(n + 1);
  now.resize(n); freq.resize(n); per.resize(n); count.resize(n);
  status.assign(n, 0); remaining.assign(n, 0); post.assign(n, phip_state{});
  size_t nb = 0;
  for (uint32_t i = 0; i < n; ++i) nb += batch[i]->len;
  names.resize(nb + 8);
  size_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const Req* r = batch[i];
    offs[i] = (uint32_t)o;
    if (r->len) std::memcpy(names.data() + o, r->name, r->len);
    o += r->len;
    now[i] = r->now; freq[i] = r->freq; per[i] = r->per; count[i] = r->count;
  }
  offs[n] = (uint32_t)o;
  phip_ops ops{};
  ops.n = n;
  ops.kind = kind.data();
  ops.names = names.data();
  ops.name_offs = offs.data();
  ops.now = now.data();
  ops.freq = freq.data();
  ops.per = per.data();
  ops.count = count.data();
  phip_results res{};
  res.status = status.data();
  res.remaining = remaining.data();
  res.reply = post.data();   // each Take's post state: its broadcast, in the same launch
  const auto t0 = Clock::now();
  const int rc = phip_apply_mixed(h, &ops, &res, 0);
  gpu_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
  for (uint32_t i = 0; i < n; ++i) {
    batch[i]->rc = rc;
    batch[i]->status = status[i];
    batch[i]->remaining = remaining[i];
    batch[i]->post = post[i];
  }
  if (rc) ++errors;
}

void phip_batcher::run() {
  std::vector<Req*> batch;
  std::unique_lock<std::mutex> l(mu);
  for (;;) {
    cv_submit.wait(l, [&] { return stop || !pending.empty(); });
    if (pending.empty()) break;   // stop, nothing left
    const auto deadline = first_arrival + std::chrono::microseconds(window_us);
    // A short window is waited out by yielding, not by a timed sleep: the
    // kernel's timer slack (50 us by default) would stretch a 20 us window
    // to ~70 us.
    while (!stop && pending.size() < max_batch && Clock::now() < deadline) {
      if (deadline - Clock::now() > std::chrono::microseconds(kSpinWindowUs)) {
        cv_submit.wait_until(l, deadline);
      } else {
        l.unlock();
        std::this_thread::yield();
        l.lock();
      }
    }
    const size_t take = std::min<size_t>(pending.size(), max_batch);
    batch.assign(pending.begin(), pending.begin() + take);
    pending.erase(pending.begin(), pending.begin() + take);
    if (!pending.empty()) first_arrival = Clock::now();
    l.unlock();
    dispatch(batch);
    l.lock();
    ++batches;
    requests += batch.size();
    max_seen = std::max<uint64_t>(max_seen, batch.size());
    // each caller is woken on its own (notified under the lock: a caller
    // cannot see `done` and return, destroying its Req, before this loop
    // let go of it)
    for (Req* r : batch) {
      r->done = true;
      r->cv.notify_one();
    }
  }
}

namespace {

// The caller counts itself in `waiters` for as long as it touches the
// batcher: close() deletes the batcher only once every woken caller has left
// (a caller woken by the last batch may not yet have re-acquired mu when the
// dispatcher exits).
int submit_and_wait(phip_batcher* b, Req* r) {
  std::unique_lock<std::mutex> l(b->mu);
  if (b->stop) return PHIP_ERR_INVALID;
  ++b->waiters;
  if (b->pending.empty()) b->first_arrival = Clock::now();
  r->seq = b->arrivals++;
  b->pending.push_back(r);
  if (b->pending.size() == 1 || b->pending.size() >= b->max_batch) b->cv_submit.notify_one();
  r->cv.wait(l, [&] { return r->done; });
  if (--b->waiters == 0 && b->stop) b->cv_idle.notify_all();
  return r->rc;
}

// Take request -> its Req, the fields of phip_take_reply filled from it.
int run_take(phip_batcher* b, const uint8_t* name, uint32_t len, int64_t now, int64_t freq,
             int64_t per, uint64_t count, Req* r) {
  if (!b || (!name && len)) return PHIP_ERR_INVALID;
  if (len > PHIP_MAX_NAME_LEN) return PHIP_ERR_NAME_TOO_LARGE;
  r->name = name;
  r->len = len;
  r->now = now;
  r->freq = freq;
  r->per = per;
  r->count = count;
  return submit_and_wait(b, r);
}

void fill_reply(const Req& r, phip_take_reply* out) {
  out->remaining = r.remaining;
  out->ok = (r.status & 0x7F) == PHIP_ST_TAKE_OK;
  out->created = (r.status & PHIP_ST_CREATED) != 0;
  out->reserved = 0;
  out->seq = r.seq;
  out->state = r.post;
  const int sz = phip_marshal(r.len ? r.name : (const uint8_t*)"", r.len, &r.post, out->datagram);
  out->datagram_len = sz > 0 ? (uint16_t)sz : 0;
}

}  // namespace

extern "C" {

int phip_batcher_open(phip_handle* h, const phip_batcher_config* cfg, phip_batcher** out) {
  if (!h || !out) return PHIP_ERR_INVALID;
  *out = nullptr;
  phip_batcher* b = new phip_batcher;
  b->h = h;
  if (cfg) {
    b->window_us = cfg->window_us;
    if (cfg->max_batch) b->max_batch = cfg->max_batch;
  }
  try {
    b->th = std::thread([b] { b->run(); });
  } catch (...) {
    delete b;
    return PHIP_ERR_INVALID;
  }
  *out = b;
  return PHIP_OK;
}

void phip_batcher_close(phip_batcher* b) {
  if (!b) return;
  {
    std::lock_guard<std::mutex> l(b->mu);
    b->stop = true;
  }
  b->cv_submit.notify_all();
  if (b->th.joinable()) b->th.join();
  {
    std::unique_lock<std::mutex> l(b->mu);
    b->cv_idle.wait(l, [&] { return b->waiters == 0; });
  }
  delete b;
}

int phip_batcher_take(phip_batcher* b, const uint8_t* name, uint32_t len, int64_t now,
                      int64_t freq, int64_t per, uint64_t count, uint64_t* remaining,
                      uint8_t* ok, uint64_t* seq) {
  Req r;
  const int rc = run_take(b, name, len, now, freq, per, count, &r);
  if (rc) return rc;
  if (remaining) *remaining = r.remaining;
  if (ok) *ok = (r.status & 0x7F) == PHIP_ST_TAKE_OK;
  if (seq) *seq = r.seq;
  return PHIP_OK;
}

int phip_batcher_api_take(phip_batcher* b, const uint8_t* name, uint32_t len, const char* rate,
                          uint32_t rate_len, const char* count, uint32_t count_len, int64_t now,
                          char* body, uint32_t* body_len) {
  if (!b || !body || !body_len) return PHIP_ERR_INVALID;
  int64_t freq, per;
  uint64_t n;
  const int pre = phip_host::api_prepare(name, len, rate, rate_len, count, count_len, &freq,
                                         &per, &n, body, body_len);
  if (pre) return pre;                                    // 400: name too large
  uint64_t rem = 0;
  uint8_t ok = 0;
  const int rc = phip_batcher_take(b, len ? name : (const uint8_t*)"", len, now, freq, per, n,
                                   &rem, &ok, nullptr);
  if (rc < 0) return rc;
  const std::string s = std::to_string(rem);              // api.go:84-85
  std::memcpy(body, s.data(), s.size());
  *body_len = (uint32_t)s.size();
  return ok ? 200 : 429;
}

int phip_batcher_take_reply(phip_batcher* b, const uint8_t* name, uint32_t len, int64_t now,
                            int64_t freq, int64_t per, uint64_t count, phip_take_reply* out) {
  if (!out) return PHIP_ERR_INVALID;
  Req r;
  const int rc = run_take(b, name, len, now, freq, per, count, &r);
  if (rc) return rc;
  fill_reply(r, out);
  return PHIP_OK;
}

int phip_batcher_api_take_reply(phip_batcher* b, const uint8_t* name, uint32_t len,
                                const char* rate, uint32_t rate_len, const char* count,
                                uint32_t count_len, int64_t now, char* body, uint32_t* body_len,
                                phip_take_reply* out) {
  if (!b || !body || !body_len || !out) return PHIP_ERR_INVALID;
  std::memset(out, 0, sizeof *out);
  int64_t freq, per;
  uint64_t n;
  const int pre = phip_host::api_prepare(name, len, rate, rate_len, count, count_len, &freq,
                                         &per, &n, body, body_len);
  if (pre) return pre;                                    // 400: name too large, nothing sent
  Req r;
  const int rc = run_take(b, len ? name : (const uint8_t*)"", len, now, freq, per, n, &r);
  if (rc < 0) return rc;
  fill_reply(r, out);
  const std::string s = std::to_string(r.remaining);      // api.go:84-85
  std::memcpy(body, s.data(), s.size());
  *body_len = (uint32_t)s.size();
  return out->ok ? 200 : 429;
}

int phip_batcher_stats(phip_batcher* b, uint64_t* out, int max) {
  if (!b || !out) return 0;
  std::lock_guard<std::mutex> l(b->mu);
  const uint64_t v[5] = {b->batches, b->requests, b->max_seen, b->gpu_ns, b->errors};
  int k = 0;
  for (; k < max && k < 5; ++k) out[k] = v[k];
  return k;
}

}  // extern "C"
