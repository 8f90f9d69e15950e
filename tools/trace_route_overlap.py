#!/usr/bin/env python3
"""Kernel-trace evidence of the pipelined owner-routed exchange
(phip_group_receive).

    run:      python3 tools/trace_route_overlap.py run  [--world 2] [--n 40000000]
    analyse:  python3 tools/trace_route_overlap.py show TRACE_DIR [OUT.json]

`run` (under rocprofv3 --kernel-trace) opens a shared-device group of
--world members on GPU 0 (phip_group_open_all with the device listed
--world times: the multi-member exchange by device copies; at --world 1
the RCCL send/recv to itself, PHIP_GROUP_RCCL_SELF), gives every
member a Zipf(1.1) batch of --n messages (three 2^24-message chunks at the
default), and runs two warmup and three timed phip_group_receive calls.

`show` reads the trace and reports, for the last call, every pack kernel
(k_route_*) and every exchange copy (__amd_rocclr_copyBuffer, or the RCCL kernels of an
RCCL group) by stream,
and the time during which a pack and a copy ran at the same moment (the
pack of chunk k+1 beside the copies of chunk k), and a merge and a copy
(the owner's merge of chunk k-1 beside them).
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
    import torch
    import bench
    import patrol_amd
    dev = torch.device("cuda", 0)
    g = patrol_amd.GPUGroup.open_all([0] * args.world, log2_slots=26)
    gen = torch.Generator(device=dev).manual_seed(5)
    K = 10_000_000
    batches = []
    for _ in range(args.world):
        ids = bench.zipf_ids(torch, gen, args.n, K, 1.1, dev)
        blob, offs = bench.names_for_ids(torch, ids)
        a, t, e = bench.replica_states(torch, gen, args.n, 0, dev)
        batches.append((blob, offs, a, t, e))
    torch.cuda.synchronize()
    import time
    for j in range(5):
        t0 = time.perf_counter()
        sent, merged = g.receive(batches, bench.T0 + j, combine=True,
                                 rccl_self=args.world == 1)
        torch.cuda.synchronize()
        print(f"call {j}: {1e3 * (time.perf_counter() - t0):.2f} ms sent {sent} merged {merged}",
              flush=True)
    g.close()


def show(args):
    rows = []
    for f in glob.glob(os.path.join(args.trace, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def short(r):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("phip::", "")
        return n.split("<")[0]
    # the last call: from the last k_route_sample (the directory, once per member per call)
    starts = [i for i, r in enumerate(rows) if short(r) == "k_route_sample"]
    if not starts:
        sys.exit("no k_route_sample in the trace")
    i0 = starts[-args.world] if len(starts) >= args.world else starts[0]
    call = rows[i0:]
    t0 = int(call[0]["Start_Timestamp"])
    pack = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in call
            if short(r).startswith("k_route_")]
    copy = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in call
            if "copyBuffer" in r["Kernel_Name"] or "nccl" in r["Kernel_Name"].lower()]
    merge = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in call
             if short(r) == "k_receive_fast"]

    def union(iv):
        out = []
        for s, e in sorted(iv):
            if out and s <= out[-1][1]:
                out[-1][1] = max(out[-1][1], e)
            else:
                out.append([s, e])
        return out

    def total(iv):
        return sum(e - s for s, e in iv)

    def inter(a, b):
        i = j = 0
        out = 0
        while i < len(a) and j < len(b):
            s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
            if s < e:
                out += e - s
            if a[i][1] < b[j][1]:
                i += 1
            else:
                j += 1
        return out
    P, X, M = union(pack), union(copy), union(merge)
    end = max(int(r["End_Timestamp"]) for r in call)
    res = {
        "world": args.world, "call_us": (end - t0) / 1e3,
        "pack_busy_us": total(P) / 1e3, "copy_busy_us": total(X) / 1e3,
        "merge_busy_us": total(M) / 1e3,
        "pack_and_copy_overlap_us": inter(P, X) / 1e3,
        "merge_and_copy_overlap_us": inter(M, X) / 1e3,
        "timeline": [dict(kernel=short(r)[:40], queue=r.get("Queue_Id", r.get("Stream_Id")),
                          start_us=(int(r["Start_Timestamp"]) - t0) / 1e3,
                          end_us=(int(r["End_Timestamp"]) - t0) / 1e3) for r in call],
    }
    print(json.dumps({k: v for k, v in res.items() if k != "timeline"}, indent=1))
    for r in res["timeline"]:
        print("%-40s q%-4s %9.1f %9.1f" % (r["kernel"], r["queue"], r["start_us"], r["end_us"]))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("mode", choices=["run", "show"])
    p.add_argument("trace", nargs="?")
    p.add_argument("out", nargs="?")
    p.add_argument("--world", type=int, default=2)
    p.add_argument("--n", type=int, default=40_000_000)
    args = p.parse_args()
    run(args) if args.mode == "run" else show(args)


if __name__ == "__main__":
    main()
