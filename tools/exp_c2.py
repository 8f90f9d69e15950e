#!/usr/bin/env python3
"""C2 experiment (not the bench): time k_receive_fast on fresh batches vs
replays of an already-applied batch (no field grows, so no atomics), to
split the kernel's time between reads and atomics."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    import patrol_amd
    dev = torch.device("cuda", 0)
    K, n = 10_000_000, 100_000_000
    gen = torch.Generator(device=dev).manual_seed(1234)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    repo = patrol_amd.GPURepo(device=0, log2_slots=25, arena_bytes=1 << 20)
    repo.use_torch_stream()
    keys = torch.arange(K, dtype=torch.int64, device=dev)
    kb, ko = bench.names_for_ids(torch, keys)
    st = torch.zeros((K, 4), dtype=torch.int64, device=dev)
    st[:, 3] = bench.T0
    repo.seed_device(kb, ko, st, K)
    del kb, ko, st, keys
    ids = bench.zipf_ids(torch, gen, n, K, 1.1, dev)
    blob, offs = bench.names_for_ids(torch, ids)
    batches = [bench.replica_states(torch, gen, n, j, dev) for j in range(4)]
    repo.set_timing(True)

    def run(j, label):
        a, t, e = batches[j]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        repo.receive_soa(blob, a, t, e, bench.T0 + j, name_offs=offs, n=n, device=True)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        ks = repo.timings()
        print("%-28s wall %.3f ms  %s  stats %s" % (label, wall, "  ".join("%s %.3f" % kv for kv in ks), repo.last_stats()))
    quick = "--quick" in sys.argv
    if quick:
        run(0, "warm fresh")
        run(1, "fresh")
        run(1, "replay (no-op)")
        run(2, "fresh")
        return
    run(0, "warm fresh")
    run(1, "fresh")
    run(1, "replay (no-op)")
    run(2, "fresh")
    run(2, "replay (no-op)")
    run(3, "fresh")
    # every message on one of the 256 hottest buckets: no table reads at all
    hot_ids = bench.zipf_ids(torch, gen, n, 256, 1.1, dev)
    mult = 2654435761 % K
    import numpy as np
    while np.gcd(mult, K) != 1:
        mult += 1
    blob2, offs2 = bench.names_for_ids(torch, (hot_ids * mult) % K)
    nonlocal_blob = [blob, offs]
    blob, offs = blob2, offs2

    def run2(j, label):
        a, t, e = batches[j]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        repo.receive_soa(blob2, a, t, e, bench.T0 + j, name_offs=offs2, n=n, device=True)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        ks = repo.timings()
        print("%-28s wall %.3f ms  %s  stats %s" % (label, wall, "  ".join("%s %.3f" % kv for kv in ks), repo.last_stats()))
    run2(3, "all-hot replay")
    run2(2, "all-hot replay")


if __name__ == "__main__":
    main()
