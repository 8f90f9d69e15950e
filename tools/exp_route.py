#!/usr/bin/env python3
"""phip_route_pack on the C4 batch shape (bench.py's generators), with and
without PHIP_ROUTE_COMBINE: per-kernel times and how many messages leave.
Usage (GPU box): python tools/exp_route.py [--world W] [--messages N]"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import patrol_amd  # noqa: E402
from patrol_amd import _lib  # noqa: E402
from patrol_amd.engine import phip_msgs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--messages", type=int, default=100_000_000)
    ap.add_argument("--keys", type=int, default=80_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    n = args.messages
    ids = bench.zipf_ids(torch, gen, n, args.keys, 1.1, dev)
    blob, offs = bench.names_for_ids(torch, ids)
    a, t, e = bench.replica_states(torch, gen, n, 0, dev)
    repo = patrol_amd.GPURepo(device=0, log2_slots=10)
    repo.set_timing(True)
    s_names = torch.empty(blob.numel() + 64, dtype=torch.uint8, device=dev)
    s_lens = torch.empty(n, dtype=torch.int32, device=dev)
    s_a, s_t, s_e = (torch.empty(n, dtype=torch.int64, device=dev) for _ in range(3))
    cnt = torch.zeros(args.world, dtype=torch.int64, device=dev)
    nb = torch.zeros(args.world, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    m = phip_msgs(n, 0, blob.data_ptr(), offs.data_ptr(), a.data_ptr(), t.data_ptr(), e.data_ptr())
    L = _lib.load()
    for flags in (0, _lib.ROUTE_COMBINE):
        for r in range(args.reps):
            rc = L.phip_route_pack(repo.h, C.byref(m), args.world, s_names.data_ptr(),
                                   s_lens.data_ptr(), s_a.data_ptr(), s_t.data_ptr(), s_e.data_ptr(),
                                   cnt.data_ptr(), nb.data_ptr(), _lib.DEVICE_PTRS | flags)
            assert rc == 0, rc
            tm = repo.timings()
        c = cnt.cpu().tolist()
        print(f"combine={bool(flags)} sent={sum(c)} ({sum(c) / n:.3f}) max_owner={max(c) / max(1, sum(c)):.3f}",
              {k: round(v, 3) for k, v in tm}, flush=True)


if __name__ == "__main__":
    main()
