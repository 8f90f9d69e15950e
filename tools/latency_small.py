"""Latency of small host batches through the C ABI (one GPU): median wall
time per call of receive_soa, receive_datagrams and apply_mixed at a few
batch sizes, after warm-up.  Prints one JSON line per case."""
import json
import struct
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import patrol_amd  # noqa: E402
from tests import _gen  # noqa: E402


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6, float(np.percentile(ts, 99)) * 1e6


def main():
    rng = np.random.default_rng(1)
    g = patrol_amd.GPURepo(log2_slots=20)
    K = 100000
    names = _gen.key_names(np.arange(K))
    a, t, e = _gen.clean_states(rng, K)
    g.receive_soa(names, a, t, e, _gen.T0)
    for n in (1, 64, 1024):
        ids = rng.integers(0, K, n)
        nm = [names[i] for i in ids]
        a, t, e = _gen.clean_states(rng, n)
        dg = [struct.pack(">QQQ", int(a[i]), int(t[i]), int(e[i]) & (2**64 - 1)) + bytes([len(nm[i])]) + nm[i]
              for i in range(n)]
        kind = np.zeros(n, np.uint8)
        now = np.full(n, _gen.T0, np.int64)
        fr = np.full(n, 100, np.int64)
        pe = np.full(n, 10**9, np.int64)
        cnt = np.ones(n, np.uint64)
        cases = {
            "receive_soa": lambda: g.receive_soa(nm, a, t, e, _gen.T0),
            "receive_datagrams": lambda: g.receive_datagrams(dg, _gen.T0),
            "apply_mixed_take": lambda: g.apply_mixed(kind, nm, now, fr, pe, cnt, a, t, e),
        }
        for k, fn in cases.items():
            p50, p99 = timeit(fn)
            print(json.dumps({"call": k, "n": n, "p50_us": round(p50, 1), "p99_us": round(p99, 1)}))


if __name__ == "__main__":
    main()
