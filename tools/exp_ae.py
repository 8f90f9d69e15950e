#!/usr/bin/env python3
"""C5 experiment (not the bench): k_ae_join at 8 x 2^24 with the bench's
round (1% of every replica's buckets written first, so the join raises the
other replicas' copies) against a round with nothing to raise (replicas
already equal: the join only reads), to split the kernel's time between
the plane reads and the scattered write-back.  Prints the kernel times by
HIP events (phip_last_timings)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import patrol_amd
    from patrol_amd import shard
    dev = torch.device("cuda", 0)
    R, B = 8, 1 << 24
    gen = torch.Generator(device=dev).manual_seed(5)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    repo = patrol_amd.GPURepo(device=0, log2_slots=10)
    repo.use_torch_stream()
    taken = torch.randint(0, 10**6, (R, B), device=dev, generator=gen).to(torch.float64)
    added = taken + torch.rand((R, B), dtype=torch.float64, device=dev, generator=gen) * 100.0
    reps = torch.empty((R, 3, B), dtype=torch.int64, device=dev)
    reps[:, 0] = shard.e_encode(added.view(torch.int64))
    reps[:, 1] = shard.e_encode(taken.view(torch.int64))
    reps[:, 2] = torch.randint(0, 1 << 40, (R, B), device=dev, generator=gen, dtype=torch.int64)
    del taken, added
    flat = reps.view(-1)
    nw = B // 100
    repo.set_timing(True)

    from patrol_amd import _lib
    L = _lib.load()

    def join(label):
        torch.cuda.synchronize()
        rc = L.phip_ae_join(repo.h, reps.data_ptr(), R, B, _lib.DEVICE_PTRS)
        assert rc == 0, rc
        torch.cuda.synchronize()
        print("%-34s %s" % (label, "  ".join("%s %.3f ms" % kv for kv in repo.timings())),
              flush=True)

    join("first join (every field raised)")
    for k in range(3):
        join("converged (reads only)")
    for k in range(3):
        idx = torch.randint(0, B, (R, nw), device=dev, generator=gen) + \
            torch.arange(R, device=dev).unsqueeze(1) * (3 * B)
        flat.index_add_(0, idx.flatten() + B, torch.randint(1, 8, (R * nw,), device=dev, generator=gen))
        flat.index_add_(0, idx.flatten() + 2 * B,
                        torch.randint(1, 10**6, (R * nw,), device=dev, generator=gen))
        join("bench round (1% written per replica)")


if __name__ == "__main__":
    main()
