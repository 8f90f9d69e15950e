#!/usr/bin/env python3
"""Debug aid (not a test): the many-new-buckets ordered stream with 14-bit
tags, repeated; on a mismatch print the bucket count vs the oracle's and the
records of every bad name (duplicates show as two dump entries)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import patrol_amd as pa  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests import test_gpu_parity as T  # noqa: E402


def main():
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
        rng = np.random.default_rng(91 + 14)
        n, K = 400_000, 150_000
        args = T._mixed_stream(rng, n, K)
        g = pa.GPURepo(log2_slots=19, debug_tag_bits=14)
        o = O.Repo()
        out = g.apply_mixed(*args)
        ref = o.apply_mixed(*args)
        st_ok = np.array_equal(out["status"], ref["status"])
        od = o.dump()
        raw = g.dump()
        gd = {k: (v.added, v.taken, v.elapsed, v.created) for k, v in raw.items()}
        bad = [k for k in od if gd.get(k) != od[k]]
        print(f"rep {rep}: len gpu {len(g)} dump {len(raw)} oracle {len(od)} status_ok {st_ok} bad {len(bad)}",
              flush=True)
        names = args[1]
        for k in bad[:3]:
            idx = [i for i, nm in enumerate(names) if nm == k]
            print("  bad", k, "gpu", gd.get(k), "oracle", od[k], "ops", idx[:8], "kinds",
                  [int(args[0][i]) for i in idx[:8]], "status", [int(out["status"][i]) for i in idx[:8]],
                  flush=True)
        g.close()


if __name__ == "__main__":
    main()
