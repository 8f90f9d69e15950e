#!/usr/bin/env python3
"""Headline benchmark: batched replica-state merges into a device bucket table.

Workload (BASELINE.json configs[1], SURVEY.md §8d "C2"): a table pre-populated
with K = 10M buckets (2^25 slots), and per step one batch of n = 100M decoded
replica messages (name + added/taken/elapsed), Zipf(1.1) over the keys, run
through the Receive loop semantics (repo.go:54-92: GetBucket by full name,
then Bucket.Merge) by phip_receive_soa with inputs resident in HBM.  Every
step uses a fresh batch whose states are later than the previous step's
(values shifted up by the step index), so every step is a first application
of its messages to the table; the batches are generated before the timed
region.

Multi-GPU (one process per GPU; `--gpus N` without WORLD_SIZE in the
environment starts the N ranks itself through torch.distributed.run):
buckets are sharded by owner; each rank holds its own K-bucket shard and
merges its own pre-routed n-message stream (weak scaling, no data-path
collective).  value = all merges of all ranks / max-over-ranks time.

Beside it, the same JSON line carries `owner_routed`: C2's fixed total
(K buckets, n messages per step) hash-sharded by name over the N GPUs, every
rank drawing n/N messages over ALL buckets as they arrive from peers, packed
by owner on the GPU (phip_route_pack, sender-side combine), moved by RCCL
all-to-alls and merged by their owners (strong scaling).

Prints ONE JSON line (rank 0).  See DESIGN.md §4 for the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "bucket-state merges/sec + achieved HBM GB/s at 1/2/4/8 MI355X"
T0 = 1_700_000_000_000_000_000
BYTES_PER_MERGE = 88     # msg 32 + slot key 8 + state read 24 + state write 24
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md chip-level parameters (spec)
DOMINANT = "k_receive_fast"
CPU_REPS = 5                 # median of 5 runs per thread count
CPU_SLOW_SAMPLE = 2_000_000  # messages per run at 1 and nproc (> 16) threads


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--keys", type=int, default=10_000_000)
    p.add_argument("--messages", type=int, default=100_000_000)
    p.add_argument("--log2-slots", type=int, default=25)
    p.add_argument("--zipf", type=float, default=1.1)
    p.add_argument("--cpu-sample", type=int, default=10_000_000)
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--no-combine", action="store_true",
                   help="c4: no sender-side combine of hot names (PHIP_ROUTE_COMBINE)")
    p.add_argument("--route-world", type=int, default=8,
                   help="route: the number of owners phip_route_pack packs for (the per-rank "
                        "pack of an N-GPU group, timed on this one GPU)")
    p.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "route"],
                   help="c2: batched Receive merges (headline); c1: the reference's CPU case "
                        "(1M messages into 100k buckets, the whole of it timed on the CPU "
                        "restatement beside the GPU); c3: mixed Take+Merge stream")
    p.add_argument("--ops", type=int, default=50_000_000, help="c3: ops per step")
    p.add_argument("--wire", action="store_true",
                   help="c2: feed raw datagrams (bucket.go:59-64 wire format) through "
                        "phip_receive_datagrams instead of the decoded SoA")
    p.add_argument("--insert", action="store_true",
                   help="c2: insert-on-miss variant (fresh key range every step; 2^27 slots)")
    p.add_argument("--ring", action="store_true",
                   help="c2: datagrams from pinned host ring slots (phip_ring_*), PCIe-inclusive; "
                        "not the headline (inputs are not resident in HBM)")
    p.add_argument("--replicas", type=int, default=8, help="c5: simulated replicas per GPU")
    p.add_argument("--buckets", type=int, default=1 << 24, help="c5: buckets per replica")
    p.add_argument("--writes", type=float, default=0.01,
                   help="c5: fraction of buckets each replica writes between rounds")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL on ROCm) for real runs; gloo to rehearse several ranks on one GPU")
    p.add_argument("--c3-clock", default="below", choices=["below", "ahead"],
                   help="c3: replica elapsed drawn below the local clock (U[0, now - created): "
                        "Takes refill, succeed and deny) or ahead of it (round 1's input: every "
                        "Take clamps last to now, dt = 0)")
    p.add_argument("--sync-receive", action="store_true",
                   help="A/B only: c2 calls phip_receive_soa synchronously instead of queueing "
                        "each batch (PHIP_RECV_ASYNC) and flushing at the end of the timed steps")
    p.add_argument("--check-names", action="store_true",
                   help="c2: pass the names blob's length (phip_msgs.names_len) so the device "
                        "checks every name offset (the binding's default); the headline passes 0")
    p.add_argument("--no-status", action="store_true",
                   help="A/B only: the C2 step does not write the per-message status column")
    p.add_argument("--name-len", type=int, default=0,
                   help="c2: pad every bucket name to this many bytes (e.g. 32: the arena path)")
    p.add_argument("--no-routed", action="store_true",
                   help="c2: skip the owner_routed (strong-scaling) object")
    p.add_argument("--no-c3", action="store_true", help="c2: skip the c3 object")
    p.add_argument("--no-variants", action="store_true",
                   help="c2: skip the c2_variants object (uniform keys, 32-byte names)")
    p.add_argument("--no-c4", action="store_true", help="c2: skip the c4 object")
    p.add_argument("--no-ae", action="store_true", help="c2: skip the anti_entropy object")
    p.add_argument("--c4-keys", type=int, default=125_000_000,
                   help="c4 object: buckets per GPU (SURVEY C4: 1B over 8 GPUs)")
    p.add_argument("--c4-messages", type=int, default=100_000_000,
                   help="c4 object: messages per GPU per step")
    p.add_argument("--c4-log2-slots", type=int, default=28)
    p.add_argument("--route-path", default="c", choices=["c", "torch"],
                   help="owner routing / anti-entropy through the C shard group (phip_group_*, "
                        "RCCL inside libpatrolhip) or the torch.distributed glue; the gloo "
                        "rehearsal backend always takes the glue")
    return p.parse_args()


def launch_ranks(args):
    """--gpus N is authoritative.  Without WORLD_SIZE in the environment and
    N > 1, start the N ranks (torch.distributed.run, one process per GPU)
    before anything touches a GPU and exit with their status; under a
    launcher, its WORLD_SIZE must equal N."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus > 1:
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
            s.close()
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
                   f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
            sys.exit(subprocess.call(cmd))
        return
    if int(ws) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}")


# ------------------------------------------------------------ synthetic ----
def names_for_ids(torch, ids, pad_to=0):
    """ids (int64 tensor) -> (blob uint8, offs int32[n+1]) with name = b"b%d"
    (pad_to > 0: b"b" + "x" * k + "%d", k making the name pad_to bytes)."""
    if pad_to:
        return padded_names(torch, ids, pad_to)
    dev = ids.device
    nd = torch.ones_like(ids)
    p = torch.full_like(ids, 10)
    for _ in range(18):
        nd += (ids >= p).to(torch.int64)
        p = p * 10
        if bool((ids < p).all()):
            break
    lens = 1 + nd
    offs = torch.zeros(ids.numel() + 1, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)
    total = int(offs[-1])
    blob = torch.zeros(total + 8, dtype=torch.uint8, device=dev)
    start = offs[:-1]
    blob[start] = ord("b")
    maxd = int(nd.max())
    for d in range(maxd):
        m = nd > d
        pw = torch.pow(torch.tensor(10, dtype=torch.int64, device=dev), (nd[m] - 1 - d))
        digit = (ids[m] // pw) % 10
        blob[start[m] + 1 + d] = (48 + digit).to(torch.uint8)
    assert total < 2**32
    return blob, offs.to(torch.int32)


def padded_names(torch, ids, width):
    """Names of exactly `width` bytes: "b", then "x" padding, then the decimal id."""
    dev = ids.device
    n = ids.numel()
    assert width >= 12
    offs = torch.arange(n + 1, dtype=torch.int64, device=dev) * width
    blob = torch.full((n * width + 8,), ord("x"), dtype=torch.uint8, device=dev)
    blob[offs[:-1]] = ord("b")
    v = ids.clone()
    for d in range(11):   # ids < 10^11, right-aligned digits
        blob[offs[:-1] + width - 1 - d] = (48 + v % 10).to(torch.uint8)
        v //= 10
    blob[n * width:] = 0
    assert n * width < 2**32
    return blob, offs.to(torch.int32)


def zipf_ids(torch, gen, n, K, s, dev):
    ranks = torch.arange(1, K + 1, dtype=torch.float64, device=dev)
    cdf = torch.cumsum(ranks.pow(-s), 0)
    cdf /= cdf[-1].clone()
    u = torch.rand(n, dtype=torch.float64, device=dev, generator=gen)
    r = torch.searchsorted(cdf, u).clamp_(max=K - 1)
    del cdf, ranks, u
    mult = 2654435761 % K or 1
    while np.gcd(mult, K) != 1:
        mult += 1
    return (r * mult) % K


def replica_states(torch, gen, n, step, dev):
    """SURVEY §8d clean domain, shifted by `step` so each batch is later."""
    taken = torch.randint(0, 10**6, (n,), device=dev, generator=gen).to(torch.float64) + step * 2e6
    added = taken + torch.rand(n, dtype=torch.float64, device=dev, generator=gen) * 100.0
    elapsed = torch.randint(0, 1 << 40, (n,), device=dev, generator=gen, dtype=torch.int64) + step * (1 << 40)
    return added.view(torch.int64), taken.view(torch.int64), elapsed


# ---------------------------------------------------------- CPU baseline ---
def cpu_thread_counts(args):
    """1, the box's CPU share (16) and nproc threads (1 and nproc)."""
    nproc = os.cpu_count() or 1
    if args.cpu_threads:
        return [args.cpu_threads]
    return sorted({1, min(16, nproc), nproc})


def cpu_baseline(args, K, ids_host):
    """The Go-structured C++ restatement (global RWMutex + map + per-bucket
    RWMutex, repo.go:171-235 / bucket.go:240-263) timed on this host on a
    bounded sample of the same workload, at 1, 16 and nproc threads (each on
    a freshly seeded map); `value` is the nproc figure."""
    import torch
    from oracle import oracle as O
    L = O.lib()
    keys = torch.arange(K, dtype=torch.int64)
    kb, ko = names_for_ids(torch, keys, args.name_len)
    kb_np, ko_np = kb.numpy(), ko.numpy().astype(np.uint32)
    del kb, ko, keys
    z = np.zeros(K, np.uint64)

    def seeded():
        repo = O.Repo()
        L.orc_repo_seed(repo.h, kb_np, ko_np, K, z, z, np.zeros(K, np.int64), np.full(K, T0, np.int64))
        return repo
    n = min(args.cpu_sample, ids_host.numel())
    ids = ids_host[:n]
    blob, offs = names_for_ids(torch, ids, args.name_len)
    g = torch.Generator().manual_seed(args.seed + 99)
    blob_np, offs_np = blob.numpy(), offs.numpy().astype(np.uint32)
    counts = cpu_thread_counts(args)
    repo = seeded()
    runs = {}
    shift = 0
    for th in counts:
        # a bounded sample per run: 16 threads merge ~5-8 M/s, but one
        # goroutine (the reference's Receive loop, repo.go:54) and the
        # lock-bound nproc case ~0.5-3 M/s
        m = n if 1 < th <= 16 else min(n, CPU_SLOW_SAMPLE)
        vals = []
        for _ in range(CPU_REPS):
            # every run applies states above the previous run's, so each is a
            # first application (every touched bucket grows), as on the GPU
            a, t, e = replica_states(torch, g, m, shift, "cpu")
            shift += 1
            secs = L.orc_bench_receive(repo.h, blob_np, offs_np, m, a.numpy().view(np.uint64),
                                       t.numpy().view(np.uint64), e.numpy(), T0, th)
            vals.append(m / secs)
        runs[th] = dict(median=float(np.median(vals)), min=float(min(vals)),
                        max=float(max(vals)), runs=CPU_REPS, messages=m)
    del repo
    top, one = max(runs), min(runs)
    best = max(runs, key=lambda k: runs[k]["median"])
    return dict(value=runs[top]["median"], unit="merges/s", cores=top, kind="port", **host_cpu(),
                best=dict(threads=best, value=runs[best]["median"],
                          note="the thread count with the highest median; `value` is the nproc "
                               "figure SURVEY §8d asks for (lock collapse on LocalRepo's RWMutex)"),
                what="Go-semantics C++ restatement (oracle/patrol_oracle.cc: LocalRepo's "
                     "RWMutex map + per-bucket mutex, ReplicatedRepo.Receive's loop body)",
                sample=f"the first {runs[top]['messages']} step-0 messages (Zipf {args.zipf} over "
                       f"{K} buckets) into a {K}-bucket map, {top} threads (nproc); median of "
                       f"{CPU_REPS} runs, each run's states above the last",
                by_threads={str(k): v for k, v in sorted(runs.items())},
                single_thread=dict(value=runs[one]["median"], min=runs[one]["min"],
                                   max=runs[one]["max"],
                                   sample=f"{runs[one]['messages']} messages, 1 thread (the "
                                          f"reference's single Receive goroutine), median of "
                                          f"{CPU_REPS}"))


def host_cpu():
    """Provenance of the CPU baseline: the host's logical CPUs and model."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"host_nproc": os.cpu_count(), "host_affinity_cpus": affinity, "host_cpu_model": model}


def pmc_traffic(key, workload, kernel, build):
    """HBM bytes per launch of the dominant kernel from the committed PMC
    summary (profiles/pmc_summary.json, produced by tools/pmc_workloads.py):
    one entry per workload key (c1..c5), used only when it was measured on
    the same workload description, the same dominant kernel(s) and the same
    library build (phip_build_id, a hash of the sources) as this run.
    Returns (bytes or None, the entry's source or why it was not used)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f).get(key)
    except (OSError, ValueError, AttributeError):
        return None, "no profiles/pmc_summary.json"
    if not d:
        return None, f"no PMC entry for {key}"
    if d.get("workload") != workload or d.get("kernel") != kernel:
        return None, f"PMC entry for {key} measured another workload or kernel"
    if d.get("build_id") != build:
        return None, (f"PMC entry for {key} is from build {d.get('build_id')}, this run is "
                      f"build {build}")
    return d.get("hbm_bytes_per_step"), d.get("source")


def datagrams(torch, blob, offs, a, t, e):
    """MarshalBinary (bucket.go:51-68) of every message, back to back:
    added, taken, elapsed as big-endian 8-byte words, one length byte, the
    name.  Returns (bytes uint8 with 8 bytes of slack, offs int64[n+1])."""
    dev = blob.device
    n = offs.numel() - 1
    lens = (offs[1:] - offs[:-1]).to(torch.int64)
    doffs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    doffs[1:] = torch.cumsum(lens + 25, 0)
    out = torch.zeros(int(doffs[-1]) + 8, dtype=torch.uint8, device=dev)
    hdr = torch.stack([a, t, e], 1).contiguous().view(torch.uint8).view(n, 3, 8).flip(2)
    pos = doffs[:-1].unsqueeze(1) + torch.arange(24, device=dev).unsqueeze(0)
    out[pos.flatten()] = hdr.reshape(n, 24).flatten()
    out[doffs[:-1] + 24] = lens.to(torch.uint8)
    seg = torch.repeat_interleave(torch.arange(n, device=dev), lens)
    within = torch.arange(int(lens.sum()), device=dev) - offs[:-1].to(torch.int64)[seg] + \
        offs[0].to(torch.int64)
    out[doffs[:-1][seg] + 25 + within] = blob[offs[:-1].to(torch.int64)[seg] + within]
    return out, doffs


def c3_inputs(args, torch, dev, K, base, gen):
    """n ops, 50% Take(rate=100:1s, count=1) / 50% received
    replica states, interleaved by seq, Zipf over the K buckets; now = t0 +
    seq*20ns (+1 s per step).  Per-bucket order is the op order.  One op
    stream (names, kinds, rates); per step its clock and replica states."""
    n = args.ops
    ids = zipf_ids(torch, gen, n, K, args.zipf, dev)
    blob, offs = names_for_ids(torch, ids + base)
    kind = (torch.rand(n, device=dev, generator=gen) < 0.5).to(torch.uint8)   # 0 take, 1 receive
    freq = torch.full((n,), 100, dtype=torch.int64, device=dev)
    per = torch.full((n,), 10**9, dtype=torch.int64, device=dev)
    cnt = torch.ones(n, dtype=torch.int64, device=dev)
    seq_now = torch.arange(n, dtype=torch.int64, device=dev) * 20
    steps = []
    for j in range(args.warmup + args.steps):
        a, t, e = replica_states(torch, gen, n, j, dev)
        now = T0 + j * 10**9 + seq_now
        if args.c3_clock == "below":
            # replica elapsed below the local clock: created + elapsed < now,
            # so Takes refill (dt > 0, bucket.go:198-212), succeed and deny
            e = (torch.rand(n, dtype=torch.float64, device=dev, generator=gen) *
                 (now - T0).to(torch.float64)).to(torch.int64)
        steps.append((now, a, t, e))
    return dict(n=n, ids=ids, blob=blob, offs=offs, kind=kind, freq=freq, per=per, cnt=cnt,
                steps=steps)


def c3_cpu(args, torch, c, K, base, step_idx, threads=None, reps=CPU_REPS):
    """C3's stream through the Go-structured restatement (oracle) on a
    bounded prefix of step `step_idx`, on a freshly seeded map: one thread
    in stream order (orc_bench_mixed), and 16 / nproc threads
    (orc_bench_mixed_mt: each bucket's ops on one worker in stream order,
    the global map lock and the bucket mutex per op, as concurrent Go
    handlers take them).  The first run (1 thread, the step's own clock)
    starts from the state the GPU's step started from when that step ran on
    a fresh table: its statuses and `remaining` are returned beside the
    timing dict for the in-run parity check (a prefix's results depend only
    on the ops before it)."""
    from oracle import oracle as O
    L = O.lib()
    n, ids, steps = c["n"], c["ids"], c["steps"]
    kind, freq, per, cnt = c["kind"], c["freq"], c["per"], c["cnt"]
    keys = torch.arange(base, base + K, dtype=torch.int64)
    kb, ko = names_for_ids(torch, keys)
    kb_np, ko_np = kb.numpy(), ko.numpy().astype(np.uint32)
    del kb, ko, keys
    z = np.zeros(K, np.uint64)
    m = min(args.cpu_sample // 2, n)
    sb, so = names_for_ids(torch, ids[:m].cpu() + base)
    sb_np, so_np = sb.numpy(), so.numpy().astype(np.uint32)
    now, a, t, e = steps[step_idx]
    cols = [x[:m].cpu().numpy() for x in (kind, now, freq, per, cnt, a, t, e)]
    orepo = O.Repo()
    L.orc_repo_seed(orepo.h, kb_np, ko_np, K, z, z, np.zeros(K, np.int64), np.full(K, T0, np.int64))
    runs = {}
    rep = 0
    first = None
    for th in (threads or cpu_thread_counts(args)):
        mm = m if 1 < th <= 16 else min(m, CPU_SLOW_SAMPLE // 2)
        f = L.orc_bench_mixed if th == 1 else L.orc_bench_mixed_mt
        extra = () if th == 1 else (th,)
        vals = []
        for _ in range(reps):
            st = np.zeros(mm, np.uint8)
            rm = np.zeros(mm, np.uint64)
            # each run one second of clock later than the last (Takes refill)
            nw = cols[1][:mm] + rep * 10**9
            rep += 1
            secs = f(orepo.h, cols[0], sb_np, so_np, mm, nw, cols[2], cols[3],
                     cols[4].view(np.uint64), cols[5].view(np.uint64), cols[6].view(np.uint64),
                     cols[7], st, rm, *extra)
            if first is None:
                first = (st, rm)
            vals.append(mm / secs)
        runs[th] = dict(median=float(np.median(vals)), min=float(min(vals)),
                        max=float(max(vals)), runs=reps, ops=mm)
    del orepo
    top, one = max(runs), min(runs)
    best = max(runs, key=lambda k: runs[k]["median"])
    out = dict(value=runs[top]["median"], unit="ops/s", cores=top, kind="port", **host_cpu(),
               what="Go-semantics C++ restatement (oracle/patrol_oracle.cc)",
               sample=f"first {runs[top]['ops']} ops of a timed-stream step (Zipf {args.zipf} "
                      f"over {K} buckets), {top} threads (nproc; each bucket's ops on one "
                      f"worker, in stream order); median of {reps} runs, each run's "
                      "clock 1 s after the last",
               best=dict(threads=best, value=runs[best]["median"]),
               by_threads={str(k): v for k, v in sorted(runs.items())},
               single_thread=dict(value=runs[one]["median"], min=runs[one]["min"],
                                  max=runs[one]["max"],
                                  sample=f"{runs[one]['ops']} ops, 1 thread, median of {reps}"))
    return out, first


def run_c3(args, torch, dev, repo, rank, K, base, gen):
    """The C3 bench step over c3_inputs(): phip_apply_mixed with statuses and
    `remaining` written, every array resident in HBM."""
    c = c3_inputs(args, torch, dev, K, base, gen)
    n, blob, offs, steps = c["n"], c["blob"], c["offs"], c["steps"]
    kind, freq, per, cnt = c["kind"], c["freq"], c["per"], c["cnt"]
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    rem = torch.empty(n, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    def step(j):
        now, a, t, e = steps[j]
        repo.apply_mixed_device(n, kind, blob, offs, now, freq, per, cnt, a, t, e,
                                status=status, remaining=rem)

    def cpu():
        return c3_cpu(args, torch, c, K, base, args.warmup)[0]
    return n, step, cpu


def c3_workload(args, n, K, L):
    return (f"C3 mixed: {n} ops (50% Take 100:1s n=1, 50% Merge), Zipf({args.zipf}) over "
            f"{K} buckets (2^{L} slots), per-bucket order kept, replica "
            f"elapsed {args.c3_clock} the local clock")


def run_c3_leg(args, torch, dist, dev, local, rank, world):
    """The `c3` object (BASELINE configs[2]): 50M mixed ops
    per step, 50% Take(100:1s, n=1) and 50% replica merges, Zipf(1.1) over a
    10M-bucket table (2^25 slots), per-bucket order kept, replica clocks
    below the local clock, through phip_apply_mixed with statuses and
    `remaining` written (bucket.go:186-225 driven by api.go:67-74, and
    repo.go:54-92).  Every rank runs its own table (weak scaling, no
    exchange).

    `verified` (in-run parity): the untimed first step runs on the freshly
    seeded table; the restatement (oracle) replays that step's first ops on
    a freshly seeded map inside the CPU-baseline leg, and their statuses and
    `remaining` must equal the GPU's bit for bit (a prefix's results depend
    only on the ops before it)."""
    import argparse as _ap
    import patrol_amd
    K, L = args.keys, args.log2_slots
    ca = _ap.Namespace(**vars(args))
    ca.warmup, ca.steps = 1, max(1, min(args.steps, 5))
    ca.c3_clock = "below"
    gen = torch.Generator(device=dev).manual_seed(args.seed + 303 + 7919 * rank)
    base = rank * K
    repo = patrol_amd.GPURepo(device=local, log2_slots=L, arena_bytes=1 << 20)
    repo.use_torch_stream()
    keys = torch.arange(base, base + K, dtype=torch.int64, device=dev)
    kb, ko = names_for_ids(torch, keys)
    st = torch.zeros((K, 4), dtype=torch.int64, device=dev)
    st[:, 3] = T0
    torch.cuda.synchronize()
    repo.seed_device(kb, ko, st, K)
    del kb, ko, st, keys
    c = c3_inputs(ca, torch, dev, K, base, gen)
    n, blob, offs, steps = c["n"], c["blob"], c["offs"], c["steps"]
    kind, freq, per, cnt = c["kind"], c["freq"], c["per"], c["cnt"]
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    rem = torch.empty(n, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    first = {}

    def step(j):
        now, a, t, e = steps[j]
        repo.apply_mixed_device(n, kind, blob, offs, now, freq, per, cnt, a, t, e,
                                status=status, remaining=rem)
        if j == 0:   # the verification step (untimed warmup, fresh table)
            torch.cuda.synchronize()
            first["st"] = status[:CPU_SLOW_SAMPLE].cpu().numpy()
            first["rm"] = rem[:CPU_SLOW_SAMPLE].cpu().numpy().view(np.uint64)
    el = _timed_steps(dist, torch, dev, args, ca.warmup, ca.steps, step)
    repo.close()
    del status, rem
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu, ref = c3_cpu(ca, torch, c, K, base, 0)
    else:   # parity only (one thread, one run)
        _, ref = c3_cpu(ca, torch, c, K, base, 0, threads=[1], reps=1)
    mm = ref[0].size
    bad_st = int((first["st"][:mm] != ref[0]).sum())
    bad_rm = int((first["rm"][:mm] != ref[1]).sum())
    ok = torch.tensor([int(bad_st == 0 and bad_rm == 0)], dtype=torch.int64, device=dev)
    verified = int(_coll(dist, args, torch, ok, "sum").item()) == world
    del c
    step_s = el / ca.steps
    bpo = 88.5   # Take 89 B, Merge 88 B
    achieved = bpo * n / step_s / 1e9
    workload = c3_workload(ca, n, K, L)
    build = patrol_amd.build_id()
    traffic, traffic_src = pmc_traffic("c3", workload, "whole step", build)
    out = {
        "metric": "mixed Take+Merge ops/sec (C3: per-bucket ordered)",
        "value": world * n * ca.steps / el, "unit": "ops/s", "scaling": "weak", "n_gpus": world,
        "steps": ca.steps, "warmup": ca.warmup, "ms_per_step": step_s * 1e3,
        "workload": workload,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src, "kernel": "whole step",
                     "algorithmic_bytes_per_step": bpo * n},
        "verified": verified,
        "verify": {"ops_checked": mm, "status_mismatches": bad_st, "remaining_mismatches": bad_rm,
                   "reference": "oracle/patrol_oracle.cc (orc_bench_mixed) replaying the first "
                                f"{mm} ops of the untimed first step on a freshly seeded map"},
    }
    if cpu is not None:
        out["cpu_baseline"] = cpu
    return out


def run_c4(args, torch, dev, repo, rank, world, K, gen):
    """K*world buckets hash-sharded by name over the ranks
    (owner = top bits of FNV-1a, patrol_amd.shard.owner_of).  Every rank
    draws its messages over ALL buckets (Zipf, as they would arrive from
    peers), so each step packs them by owner on the GPU (phip_route_pack),
    moves them with one all-to-all per column over RCCL and merges the
    received ones (shard.route_messages_native, then phip_receive_soa)."""
    from patrol_amd import shard
    n = args.messages
    KT = K * world
    keys = torch.arange(KT, dtype=torch.int64, device=dev)
    kb, ko = names_for_ids(torch, keys)
    hk = shard.hash_names(kb, ko, repo)
    mine = torch.nonzero(shard.owner_of(hk, world) == rank).flatten()
    sb, _, so = shard._gather_names(kb, ko, mine)
    st = torch.zeros((mine.numel(), 4), dtype=torch.int64, device=dev)
    st[:, 3] = T0
    repo.seed_device(sb, so.to(torch.int32), st, mine.numel())
    owned = mine.numel()
    del keys, kb, ko, hk, sb, so, st, mine
    ids = zipf_ids(torch, gen, n, KT, args.zipf, dev)
    blob, offs = names_for_ids(torch, ids)
    batches = [replica_states(torch, gen, n, j, dev) for j in range(args.warmup + args.steps)]
    torch.cuda.synchronize()

    merged = []
    group = repo._group = open_group(args, dist_module(), repo, rank, world)
    if group is not None:
        group.set_timing(True)

    def step(j):
        a, t, e = batches[j]
        if group is not None:
            _, got = group.receive([(blob, offs, a, t, e)], T0 + j, combine=not args.no_combine)
            m = got[0]
        else:
            rb, ro, ra, rt, re = shard.route_messages_native(blob, offs, a, t, e, repo,
                                                             combine=not args.no_combine)
            m = ro.numel() - 1
            if m:
                repo.receive_soa(rb, ra, rt, re, T0 + j, name_offs=ro, n=m, device=True)
        if j >= args.warmup:
            merged.append(m)
    return n, step, owned, merged


def run_route(args, torch, dev, repo, K, gen):
    """The sender's half of C4 at N GPUs, on one: every step packs this
    rank's batch by owner for --route-world owners (phip_route_pack with the
    sender-side combine: owner hash, combine of the sampled hot names, stable
    owner-major pack), into preallocated send buffers.  No exchange: the
    step is the pack kernels only (bench c4 at N GPUs adds the RCCL
    exchange and the owner's merge)."""
    import ctypes as C
    from patrol_amd import _lib
    from patrol_amd.engine import phip_msgs
    n, W = args.messages, args.route_world
    ids = zipf_ids(torch, gen, n, K, args.zipf, dev)
    blob, offs = names_for_ids(torch, ids)
    del ids
    batches = [replica_states(torch, gen, n, j, dev) for j in range(args.warmup + args.steps)]
    s_names = torch.empty(blob.numel(), dtype=torch.uint8, device=dev)
    s_lens = torch.empty(n, dtype=torch.int32, device=dev)
    s_a, s_t, s_e = (torch.empty(n, dtype=torch.int64, device=dev) for _ in range(3))
    cnt = torch.zeros(W, dtype=torch.int64, device=dev)
    nb = torch.zeros(W, dtype=torch.int64, device=dev)
    L = _lib.load()
    sent = []
    torch.cuda.synchronize()

    def step(j):
        a, t, e = batches[j]
        m = phip_msgs(n, 0, blob.data_ptr(), offs.data_ptr(), a.data_ptr(), t.data_ptr(),
                      e.data_ptr())
        rc = L.phip_route_pack(repo.h, C.byref(m), W, s_names.data_ptr(), s_lens.data_ptr(),
                               s_a.data_ptr(), s_t.data_ptr(), s_e.data_ptr(), cnt.data_ptr(),
                               nb.data_ptr(), _lib.DEVICE_PTRS | _lib.ROUTE_COMBINE)
        if rc != 0:
            raise RuntimeError(f"phip_route_pack: {rc}")
        if j == 0:   # a warmup step (its read-back synchronises; keep it out of the timing)
            sent.append(int(cnt.sum()))
    return n, step, sent


def dist_module():
    import torch.distributed as dist
    return dist


def open_group(args, dist, repo, rank, world):
    """The shard group of the C library (phip_group_open_rank: RCCL owner
    routing and all-reduce with no torch on the data path), its id handed
    out over torch.distributed (bootstrap only).  None under the gloo
    rehearsal backend, where ranks may share one GPU (RCCL refuses that):
    the torch.distributed glue (patrol_amd.shard) stands in."""
    if args.dist_backend != "nccl" or args.route_path != "c":
        return None
    import patrol_amd
    obj = [patrol_amd.GPUGroup.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return patrol_amd.GPUGroup.open_rank(repo, obj[0], world, rank)


def group_diag(group, world, stages, names):
    """What a multi-GPU record needs to explain itself: the RCCL the
    group's communicator runs on (version, ncclCommCount, the librccl its
    symbols resolved to, every librccl mapped in this process) and rank 0's
    per-stage busy ms per step (HIP events around each chunk's work on its
    own stream: the stages overlap, phip_group_stage_ms)."""
    if group is None:
        return {}
    out = {"rccl": dict(group.rccl_info(), world=world)}
    if stages:
        out["stage_busy_ms"] = {nm: float(np.mean([s[k] for s in stages]))
                                for nm, k in zip(names, ("pack", "exchange", "merge"))}
    return out


XGMI_GBPS = 7 * 153.0   # MI355X: 7 xGMI links x ~153 GB/s per GPU (one direction)


def c4_stage_roofline(diag, n, name_bytes, sent, merged, world):
    """Rank 0's stages of one routed C4 step against their bounds (busy ms
    from HIP events on each stage's own stream, phip_group_stage_ms; the
    stages overlap, so each rate is the stage's own):
      pack      reads each message (offset 4 + name + 24 B of state) and
                writes it owner-major (length 4 + name + 24): 2 x (28 +
                name) B per message (SURVEY §8d's ~7 GB per 100M), HBM-bound;
      exchange  the segments sent after the combine, (4 + name + 24) B each:
                at N > 1 the (N-1)/N that leave go over xGMI (7 links x 153
                GB/s per GPU); at N = 1 the RCCL send/recv to itself is a
                device copy (read + write in HBM);
      merge     88 B per merged message, HBM-bound."""
    sb = (diag or {}).get("stage_busy_ms")
    if not sb or sent is None:
        return {}
    msg = 28.0 + name_bytes
    pack_b = 2.0 * msg * n
    xfer_b = msg * sent * ((world - 1) / world if world > 1 else 1.0)
    merge_b = BYTES_PER_MERGE * merged
    out = {"algorithmic_bytes_per_step": {"pack": pack_b, "exchange": xfer_b, "merge": merge_b},
           "stage_roofline": {}}
    for nm, b in (("pack", pack_b), ("merge", merge_b)):
        ms = sb.get(nm)
        if ms:
            gbs = b / (ms / 1e3) / 1e9
            out["stage_roofline"][nm] = {"bound": "hbm", "achieved_GBps": gbs,
                                         "peak_GBps": HBM_PEAK_GBS, "frac": gbs / HBM_PEAK_GBS}
    ms = sb.get("exchange")
    if ms:
        gbs = xfer_b / (ms / 1e3) / 1e9
        if world > 1:
            out["stage_roofline"]["exchange"] = {"bound": "xgmi", "achieved_GBps": gbs,
                                                 "peak_GBps": XGMI_GBPS, "frac": gbs / XGMI_GBPS}
        else:   # a copy through RCCL: the bytes are read and written in HBM
            out["stage_roofline"]["exchange"] = {
                "bound": "hbm (N = 1: RCCL send/recv to itself, a device copy)",
                "achieved_GBps": gbs, "peak_GBps": HBM_PEAK_GBS,
                "frac": 2 * gbs / HBM_PEAK_GBS}
    out["sent_after_combine_per_step_rank0"] = sent
    return out


LEG_LIMIT_S = 300   # each extra leg's watchdog (main())
LEG_TIMEOUT_EXIT = 3   # exit status when a watchdog fired
LEG_FAILED_EXIT = 4    # exit status when a leg raised or its in-run parity check failed


def run_routed(args, torch, dist, dev, local, rank, world):
    """The owner_routed object (SURVEY §8d/§8e strong scaling): C2's fixed
    total of K buckets and n messages per step, the buckets hash-sharded by
    name over the `world` GPUs.  Each rank draws n/world messages Zipf over
    ALL K buckets (as they arrive from peers), and a step is the sharded
    merge: phip_route_pack (owner partition + sender-side combine), one RCCL
    all-to-all per column, phip_receive_soa of the owned messages.  Timed
    with barriers, max over ranks; value = n * steps / time."""
    import patrol_amd
    from patrol_amd import shard
    K, n = args.keys, args.messages
    m = n // world
    gen = torch.Generator(device=dev).manual_seed(args.seed + 31 + 7919 * rank)
    # shard table sized like C2's at 1/world of the buckets (load ~0.3)
    L = max(16, args.log2_slots - (world - 1).bit_length())
    repo = patrol_amd.GPURepo(device=local, log2_slots=L, arena_bytes=1 << 20)
    repo.use_torch_stream()
    keys = torch.arange(K, dtype=torch.int64, device=dev)
    kb, ko = names_for_ids(torch, keys, args.name_len)
    hk = shard.hash_names(kb, ko, repo)
    mine = torch.nonzero(shard.owner_of(hk, world) == rank).flatten()
    sb, _, so = shard._gather_names(kb, ko, mine)
    st = torch.zeros((mine.numel(), 4), dtype=torch.int64, device=dev)
    st[:, 3] = T0
    torch.cuda.synchronize()
    repo.seed_device(sb, so.to(torch.int32), st, mine.numel())
    owned = mine.numel()
    del keys, kb, ko, hk, sb, so, st, mine
    ids = zipf_ids(torch, gen, m, K, args.zipf, dev)
    blob, offs = names_for_ids(torch, ids, args.name_len)
    del ids
    batches = [replica_states(torch, gen, m, j, dev) for j in range(args.warmup + args.steps)]
    torch.cuda.synchronize()
    merged = []
    group = open_group(args, dist, repo, rank, world)

    def step(j):
        a, t, e = batches[j]
        if group is not None:
            _, got = group.receive([(blob, offs, a, t, e)], T0 + j, combine=True)
            k = got[0]
        else:
            rb, ro, ra, rt, re = shard.route_messages_native(blob, offs, a, t, e, repo,
                                                             combine=True)
            k = ro.numel() - 1
            if k:
                repo.receive_soa(rb, ra, rt, re, T0 + j, name_offs=ro, n=k, device=True)
        if j >= args.warmup:
            merged.append(k)

    for j in range(args.warmup):
        step(j)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(args.warmup, args.warmup + args.steps):
        step(j)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    tt = torch.tensor([el, float(np.mean(merged)), float(owned)], dtype=torch.float64,
                      device=dev if args.dist_backend == "nccl" else "cpu")
    mx = tt.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = tt.clone()
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    if group is not None:
        group.close()
    repo.close()
    del batches, blob, offs
    el = float(mx[0])
    return {
        "metric": "bucket-state merges/sec, owner-routed (C2's fixed total sharded by name)",
        "value": n * args.steps / el, "unit": "merges/s", "scaling": "strong",
        "n_gpus": world, "ms_per_step": el / args.steps * 1e3,
        "messages_per_step_total": n, "messages_per_step_per_gpu": m, "buckets_total": K,
        "merged_per_step_total": float(sm[1]), "merged_per_step_max_gpu": float(mx[1]),
        "buckets_max_gpu": int(mx[2]), "slots_per_gpu": 1 << L, "sender_combine": True,
        "step": ("phip_group_receive (C ABI: at one GPU every message is owned locally and is "
                 "merged as it came, phip_receive_soa; at N GPUs phip_route_pack with "
                 "sender-side combine, RCCL all-to-all of the split sizes, grouped send/recv "
                 "per column, phip_receive_soa on the owner)" if group is not None else
                 "phip_route_pack + torch.distributed all-to-all per column + phip_receive_soa"),
    }


def _coll(dist, args, torch, x, op="max"):
    """all_reduce (max / sum) of a device tensor; the gloo rehearsal backend
    reduces a host copy.  Checker plumbing only (never on a timed path)."""
    red = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
    if args.dist_backend == "nccl":
        dist.all_reduce(x, op=red)
        return x
    h = x.cpu()
    dist.all_reduce(h, op=red)
    return h.to(x.device)


def _all_gather(dist, args, torch, x):
    """all_gather of equal-shaped device tensors -> [world, *x.shape]."""
    world = dist.get_world_size()
    src = x if args.dist_backend == "nccl" else x.cpu()
    out = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(out, src)
    return torch.stack(out).to(x.device)


def _timed_steps(dist, torch, dev, args, warmup, steps, step):
    """warmup untimed, then `steps` timed between barrier + synchronize on both
    sides; the max over ranks of the elapsed seconds."""
    for j in range(warmup):
        step(j)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for j in range(warmup, warmup + steps):
        step(j)
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    return float(_coll(dist, args, torch, el, "max").item())


def run_c2_variants_leg(args, torch, dist, dev, local, rank, world):
    """The `c2_variants` object: SURVEY §8d C2's other input shapes, each run
    exactly as the headline (a 10M-bucket table in 2^25 slots, 100M-message
    batches resident in HBM, queued phip_receive_soa with statuses, every
    step a first application), a few steps each:
      uniform   keys uniform over the 10M buckets (SURVEY §8d C1/C4's
                "uniform variant"): no hot bucket, every message reads a
                random record line;
      names15   15-byte names "b" + "x"... + decimal id (one byte past the
                14 a record holds inline with its 2-byte header: the inline
                form, bucket.go:36-44);
      names32   32-byte names (arena names, up to 231 B per
                bucket.go:36-44; the headline's are 2-8 B);
      dirty     the headline batch with 64 incasts and 64 -0.0 fields at
                random places (repo.go:86-90's incast, Go's asymmetric `<`
                on zeros): the messages Receive must see in order (their
                buckets through the ordered path's sub-batch, the rest
                merged: phip_kernels.hpp "Dirty buckets").
    `verified` per variant: 2^14 sampled bucket ids (plus the 256 hottest
    Zipf ranks) read back through phip_export_datagrams equal an
    independent max-reduce of every applied message naming them (torch
    scatter_reduce amax; clean-domain states on a zero-state table:
    Bucket.Merge, bucket.go:240-263, is the field-wise max)."""
    import patrol_amd
    K, n, L = args.keys, args.messages, args.log2_slots
    warm, steps = 1, max(1, min(args.steps, 3))
    out = {}
    for name, zipf, width in (("uniform", 0.0, 0), ("names15", args.zipf, 15),
                              ("names32", args.zipf, 32), ("dirty", args.zipf, 0)):
        gen = torch.Generator(device=dev).manual_seed(args.seed + 404 + 7919 * rank + width)
        base = rank * K
        arena = max(1 << 20, K * (width + 8)) if width > 22 else 1 << 20
        repo = patrol_amd.GPURepo(device=local, log2_slots=L, arena_bytes=arena)
        repo.use_torch_stream()
        keys = torch.arange(base, base + K, dtype=torch.int64, device=dev)
        kb, ko = names_for_ids(torch, keys, width)
        st = torch.zeros((K, 4), dtype=torch.int64, device=dev)
        st[:, 3] = T0
        torch.cuda.synchronize()
        repo.seed_device(kb, ko, st, K)
        del kb, ko, st, keys
        ids = zipf_ids(torch, gen, n, K, zipf, dev)
        blob, offs = names_for_ids(torch, ids + base, width)
        batches = [replica_states(torch, gen, n, j, dev) for j in range(warm + steps)]
        if name == "dirty":
            # Receive traffic as Patrol sees it: incasts (all-zero states, the
            # GetBucket of a restarted peer, repo.go:86-90) and -0.0 fields
            # among the merges, 64 of each at random places in every batch
            for a, t, e in batches:
                pos = torch.randint(0, n, (64,), device=dev, generator=gen)
                a[pos], t[pos], e[pos] = 0, 0, 0
                pos = torch.randint(0, n, (64,), device=dev, generator=gen)
                t[pos] = -(1 << 63)   # -0.0
        status = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        torch.cuda.synchronize()

        def step(j):
            a, t, e = batches[j]
            repo.receive_soa(blob, a, t, e, T0 + j, name_offs=offs, n=n, status=status[j % 2],
                             device=True, queue=True, names_len=0)   # (as the headline)
        for j in range(warm):
            step(j)
        repo.flush()
        torch.cuda.synchronize()
        dist.barrier()
        repo.set_timing(True, accumulate=True)
        t0 = time.perf_counter()
        for j in range(warm, warm + steps):
            step(j)
        repo.flush()
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        el = float(_coll(dist, args, torch, el, "max").item())
        kms = {}
        for nm, ms in repo.timings():
            kms[nm] = kms.get(nm, 0.0) + ms / steps
        repo.set_timing(False)
        # ---- sampled parity (outside the timed region)
        vg = torch.Generator(device=dev).manual_seed(args.seed + 556)
        hot = (torch.arange(256, dtype=torch.int64, device=dev) * zipf_mult(K)) % K
        samp = torch.unique(torch.cat([torch.randint(0, K, (1 << 14,), device=dev, generator=vg),
                                       hot]))
        S = samp.numel()
        pos = torch.searchsorted(samp, ids).clamp_(max=S - 1)
        hit = samp[pos] == ids
        pos = pos[hit]
        want = torch.zeros((3, S), dtype=torch.int64, device=dev)
        for a, t, e in batches:
            for f, x in enumerate((a, t, e)):
                want[f].scatter_reduce_(0, pos, x[hit], reduce="amax", include_self=True)
        sb, so = names_for_ids(torch, samp + base, width)
        ga, gt, ge, found = repo.export_states_device(sb, so, S)
        bad = int(((ga != want[0]) | (gt != want[1]) | (ge != want[2])).sum())
        ok = bool(found.all()) and bad == 0
        okt = _coll(dist, args, torch, torch.tensor([int(ok)], dtype=torch.int64, device=dev), "sum")
        st4 = repo.last_stats()
        repo.close()
        del batches, blob, offs, ids, status
        torch.cuda.empty_cache()
        step_s = el / steps
        fast = kms.get(DOMINANT)
        ach = BYTES_PER_MERGE * n / (fast / 1e3) / 1e9 if fast else None
        out[name] = {
            "value": world * n * steps / el, "unit": "merges/s", "ms_per_step": step_s * 1e3,
            "steps": steps, "warmup": warm,
            "workload": (f"C2 variant: {n} replica messages -> {K}-bucket table (2^{L} slots), " +
                         ("uniform keys" if zipf == 0 else f"Zipf({zipf})") +
                         (f", {width}-byte names" if width else ", names b<id> (2-8 B)") +
                         (", 64 incasts and 64 -0.0 fields at random places per batch"
                          if name == "dirty" else "")),
            # (kernel: k_receive_fast's share; step: the whole step's, which is
            # the figure for the dirty variant, whose deferred messages go
            # through the ordered path's kernels)
            "roofline": {"bound": "hbm", "kernel": DOMINANT, "kernel_ms_per_step": fast,
                         "achieved": ach, "peak": HBM_PEAK_GBS,
                         "frac": ach / HBM_PEAK_GBS if ach else None,
                         "step_achieved": BYTES_PER_MERGE * n / step_s / 1e9,
                         "step_frac": BYTES_PER_MERGE * n / step_s / 1e9 / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_step": BYTES_PER_MERGE * n},
            "kernels_ms": kms,
            "hot_directory": {"entries": int(st4[0]), "folded": int(st4[1])} if st4 else None,
            "ordered_messages": int(st4[4]) if st4 and len(st4) > 4 else None,
            "verified": int(okt.item()) == world,
            "verify": {"sampled_buckets": S, "mismatched": bad, "all_found": bool(found.all())},
        }
    out["verified"] = all(v["verified"] for v in out.values())
    return out


def zipf_mult(K):
    """zipf_ids' rank -> id multiplier (a unit mod K)."""
    mult = 2654435761 % K or 1
    while np.gcd(mult, K) != 1:
        mult += 1
    return mult


C4_CHUNK = 1 << 27   # seeding: bucket ids named and hashed per chunk


def run_c4_leg(args, torch, dist, dev, local, rank, world):
    """The `c4` object (BASELINE configs[3]): 125M buckets per
    GPU (2^28 slots; 1B buckets at N = 8) hash-sharded by name, every rank
    drawing 100M messages per step Zipf(1.1) over ALL buckets, and every step
    one phip_group_receive: phip_route_pack with the sender-side combine,
    the exchange of the split sizes and the grouped per-peer send/recv over
    RCCL, and the owner's phip_receive_soa (repo.go:54-92 sharded).  At one
    GPU the exchange runs as a send/recv pair to the member itself
    (PHIP_GROUP_RCCL_SELF), so the line measures the same routed pipeline at
    every N.  Weak scaling: value = all ranks' messages per step x steps /
    max-over-ranks time.

    `verified` (in-run parity): a sample of 2^16 uniform bucket ids plus the
    512 hottest Zipf ranks, identical on every rank.  The expectation is an
    independent max-reduce of every message every rank generated for those
    ids over all the steps it applied (torch scatter_reduce amax, then an
    all-reduce MAX over ranks: the states are clean-domain positive floats
    and the table starts at zero, so Bucket.Merge, bucket.go:240-263, is the
    field-wise max).  Each owner reads its sampled buckets back through the
    C ABI (phip_export_datagrams, MarshalBinary words); the reads are summed
    over ranks (exactly one owner per id) and must equal the expectation,
    every sampled id found exactly once."""
    import patrol_amd
    from patrol_amd import shard
    K, n, L = args.c4_keys, args.c4_messages, args.c4_log2_slots
    rehearsal = args.dist_backend != "nccl"
    if rehearsal:   # gloo moves every column through host memory: a smaller batch
        n = min(n, 10_000_000)
    KT = K * world
    warm, steps = max(1, min(args.warmup, 2)), max(1, min(args.steps, 10))
    gen = torch.Generator(device=dev).manual_seed(args.seed + 101 + 7919 * rank)
    repo = patrol_amd.GPURepo(device=local, log2_slots=L, arena_bytes=1 << 20)
    repo.use_torch_stream()
    t_setup = time.perf_counter()
    owned = 0
    for c0 in range(0, KT, C4_CHUNK):
        keys = torch.arange(c0, min(KT, c0 + C4_CHUNK), dtype=torch.int64, device=dev)
        if world > 1:
            kb, ko = names_for_ids(torch, keys)
            keys = keys[shard.owner_of(shard.hash_names(kb, ko, repo), world) == rank]
            del kb, ko
        kb, ko = names_for_ids(torch, keys)
        st = torch.zeros((keys.numel(), 4), dtype=torch.int64, device=dev)
        st[:, 3] = T0
        torch.cuda.synchronize()
        repo.seed_device(kb, ko, st, keys.numel())
        owned += keys.numel()
        del keys, kb, ko, st
    assert len(repo) == owned
    ids = zipf_ids(torch, gen, n, KT, args.zipf, dev)
    blob, offs = names_for_ids(torch, ids)
    batches = [replica_states(torch, gen, n, j, dev) for j in range(warm + steps)]
    torch.cuda.synchronize()
    group = open_group(args, dist, repo, rank, world)
    merged = []
    sent = []
    stages = []
    if group is not None:
        group.set_timing(True)
    name_bytes = float((offs[-1] - offs[0]).item()) / n   # mean name length of the batch

    def step(j):
        a, t, e = batches[j]
        if group is not None:
            snt, got = group.receive([(blob, offs, a, t, e)], T0 + j, combine=True,
                                     rccl_self=world == 1)
            k = got[0]
            sent.append(snt[0])
            if j >= warm:   # (the call ends host-synchronised: reading its events adds no wait)
                stages.append(group.stage_ms())
        else:
            rb, ro, ra, rt, re = shard.route_messages_native(blob, offs, a, t, e, repo,
                                                             combine=True)
            k = ro.numel() - 1
            if k:
                repo.receive_soa(rb, ra, rt, re, T0 + j, name_offs=ro, n=k, device=True)
        merged.append(k)
    t_setup = time.perf_counter() - t_setup
    el = _timed_steps(dist, torch, dev, args, warm, steps, step)

    # ---- in-run parity on a sample (outside the timed region)
    vg = torch.Generator(device=dev).manual_seed(args.seed + 555)   # the same on every rank
    hot = (torch.arange(512, dtype=torch.int64, device=dev) * zipf_mult(KT)) % KT
    samp = torch.unique(torch.cat([torch.randint(0, KT, (1 << 16,), device=dev, generator=vg),
                                   hot]))
    S = samp.numel()
    pos = torch.searchsorted(samp, ids).clamp_(max=S - 1)
    hit = samp[pos] == ids
    pos = pos[hit]
    want = torch.zeros((3, S), dtype=torch.int64, device=dev)
    for a, t, e in batches:
        for f, x in enumerate((a, t, e)):
            want[f].scatter_reduce_(0, pos, x[hit], reduce="amax", include_self=True)
    want = _coll(dist, args, torch, want, "max")
    sb, so = names_for_ids(torch, samp)
    mine = shard.owner_of(shard.hash_names(sb, so, repo), world) == rank
    idx = torch.nonzero(mine).flatten()
    got = torch.zeros((4, S), dtype=torch.int64, device=dev)
    if idx.numel():
        mb, mo = names_for_ids(torch, samp[idx])
        ga, gt, ge, found = repo.export_states_device(mb, mo, idx.numel())
        got[0, idx], got[1, idx], got[2, idx] = ga, gt, ge
        got[3, idx] = found.to(torch.int64)
    got = _coll(dist, args, torch, got, "sum")
    found_once = bool((got[3] == 1).all())
    bad = int((got[:3] != want).any(0).sum())
    verified = found_once and bad == 0
    tt = torch.tensor([float(np.mean(merged[warm:])), float(owned)], dtype=torch.float64,
                      device=dev)
    sm = _coll(dist, args, torch, tt.clone(), "sum")
    mx = _coll(dist, args, torch, tt.clone(), "max")
    diag = group_diag(group, world, stages, ("pack", "exchange", "merge"))
    roof = c4_stage_roofline(diag, n, name_bytes, float(np.mean(sent[warm:])) if sent else None,
                             float(np.mean(merged[warm:])), world)
    if group is not None:
        group.close()
    repo.close()
    del batches, blob, offs, ids
    return {
        "metric": "bucket-state merges/sec, owner-routed C4 (messages routed by owner and merged)",
        "value": world * n * steps / el, "unit": "merges/s", "scaling": "weak", "n_gpus": world,
        "steps": steps, "warmup": warm, "ms_per_step": el / steps * 1e3,
        "workload": (f"C4: {K} buckets per GPU ({KT} total, 2^{L} slots per GPU) hash-sharded by "
                     f"name; {n} messages per GPU per step Zipf({args.zipf}) over all buckets"),
        "buckets_total": int(sm[1]), "buckets_max_gpu": int(mx[1]),
        "messages_per_step_per_gpu": n, "merged_per_step_total": float(sm[0]),
        "merged_per_step_max_gpu": float(mx[0]), "sender_combine": True,
        "step": ("phip_group_receive: phip_route_pack (owner partition + sender-side combine), "
                 "RCCL all-to-all of the split sizes, grouped ncclSend/ncclRecv per peer and "
                 "column, phip_receive_soa on the owner" +
                 ("; one GPU: the segment goes to the member itself through ncclSend/ncclRecv "
                  "(PHIP_GROUP_RCCL_SELF)" if world == 1 and group is not None else "")
                 if group is not None else
                 "gloo rehearsal: phip_route_pack + torch.distributed all-to-all per column + "
                 "phip_receive_soa"),
        "rehearsal": rehearsal,
        "setup_s": t_setup,
        **diag,
        **roof,
        "verified": verified,
        "verify": {"sampled_buckets": S, "found_exactly_once": found_once, "mismatched": bad,
                   "reference": "independent per-id max-reduce of every rank's messages over all "
                                "applied steps (torch scatter_reduce amax + all-reduce MAX)"},
    }


def run_ae_leg(args, torch, dist, dev, local, rank, world):
    """The `anti_entropy` object (BASELINE configs[4]): R = 8
    simulated replicas per GPU of 2^24 buckets each (64 replicas at N = 8).
    A round = fresh local writes to 1% of every replica's buckets, then one
    phip_group_anti_entropy: the local join, RCCL all-reduce(MAX) of the
    [3, B] E-coded join over all GPUs, and the apply (one GPU: the fused
    k_ae_join, nothing to exchange).  value = replica-buckets brought to the
    cluster-wide join per second over all ranks.

    `verified`: one more round after the timed ones.  Right before its
    anti-entropy call a sample of 4096 buckets is read from every replica
    of every rank (all-gather).  Go's Bucket.Merge (bucket.go:240-263) of
    all of them, for these clean-domain states (positive floats, no NaN or
    -0.0: the merge is the float max, elapsed the int max), is computed in
    float64 by torch; afterwards every replica of every rank must hold
    exactly those bits, and every replica must equal replica 0 on every
    bucket with one checksum across ranks (converged)."""
    from patrol_amd import shard
    import patrol_amd
    R, B = args.replicas, args.buckets
    warm, steps = max(1, min(args.warmup, 2)), max(1, min(args.steps, 10))
    gen = torch.Generator(device=dev).manual_seed(args.seed + 202 + 7919 * rank)
    repo = patrol_amd.GPURepo(device=local, log2_slots=10)
    repo.use_torch_stream()
    taken = torch.randint(0, 10**6, (R, B), device=dev, generator=gen).to(torch.float64)
    added = taken + torch.rand((R, B), dtype=torch.float64, device=dev, generator=gen) * 100.0
    reps = torch.empty((R, 3, B), dtype=torch.int64, device=dev)
    reps[:, 0] = shard.e_encode(added.view(torch.int64))
    reps[:, 1] = shard.e_encode(taken.view(torch.int64))
    reps[:, 2] = torch.randint(0, 1 << 40, (R, B), device=dev, generator=gen, dtype=torch.int64)
    del taken, added
    nw = max(1, int(B * args.writes))
    rounds = []
    for j in range(warm + steps + 1):
        idx = torch.randint(0, B, (R, nw), device=dev, generator=gen) + \
            torch.arange(R, device=dev).unsqueeze(1) * (3 * B)
        rounds.append((idx.flatten(), torch.randint(1, 8, (R * nw,), device=dev, generator=gen),
                       torch.randint(1, 10**6, (R * nw,), device=dev, generator=gen)))
    flat = reps.view(-1)
    torch.cuda.synchronize()
    group = open_group(args, dist, repo, rank, world)
    stages = []
    if group is not None:
        group.set_timing(True)

    def writes(j):
        idx, dt, de = rounds[j]
        flat.index_add_(0, idx + B, dt)    # a local Take: taken grows by a few ulps
        flat.index_add_(0, idx + 2 * B, de)

    def exchange():
        if group is not None:
            group.anti_entropy([reps])
        else:
            shard.anti_entropy_native(reps, repo)

    def step(j):
        writes(j)
        exchange()
        if group is not None and j >= warm:
            stages.append(group.stage_ms())
    el = _timed_steps(dist, torch, dev, args, warm, steps, step)

    # ---- the verification round
    writes(warm + steps)
    vg = torch.Generator(device=dev).manual_seed(args.seed + 777)   # the same on every rank
    samp = torch.randint(0, B, (4096,), device=dev, generator=vg)
    before = _all_gather(dist, args, torch, reps[:, :, samp].contiguous())   # [W, R, 3, S]
    torch.cuda.synchronize()
    exchange()
    torch.cuda.synchronize()
    before = before.reshape(world * R, 3, -1)
    fa = shard.e_decode(before[:, 0]).view(torch.float64).max(0).values
    ft = shard.e_decode(before[:, 1]).view(torch.float64).max(0).values
    fe = before[:, 2].max(0).values
    after = reps[:, :, samp]
    go = (bool((shard.e_decode(after[:, 0]) == fa.view(torch.int64)).all()) and
          bool((shard.e_decode(after[:, 1]) == ft.view(torch.int64)).all()) and
          bool((after[:, 2] == fe).all()))
    conv = torch.tensor([int(bool((reps == reps[0:1]).all())), 0, 0], dtype=torch.int64,
                        device=dev)
    conv[1] = reps[0].sum(dtype=torch.int64)
    conv[2] = -conv[1]
    lo_hi = _coll(dist, args, torch, conv.clone(), "max")
    cnt = _coll(dist, args, torch, conv[:1].clone(), "sum")
    converged = int(cnt.item()) == world and int(lo_hi[1]) == -int(lo_hi[2])
    go_all = _coll(dist, args, torch, torch.tensor([int(go)], dtype=torch.int64, device=dev), "sum")
    go_ok = int(go_all.item()) == world
    diag = group_diag(group, world, stages, ("local_join", "allreduce", "apply"))
    if group is not None:
        group.close()
    repo.close()
    del reps, rounds
    # the fused one-GPU join reads 24 B per replica-bucket; at N GPUs the
    # local max reads R*24 + writes 24, the apply reads 24 + R*24 per bucket
    bpo = 24.0 if world == 1 else (2 * R + 2) * 24 / R
    step_s = el / steps
    roof = {}
    sb = diag.get("stage_busy_ms")
    if sb:
        # the local join's bytes per round (world 1: the fused k_ae_join reads
        # every replica's 24 B once; N > 1: k_ae_local_max reads R x 24 and
        # writes 24 per bucket, k_ae_apply reads 24 + R x 24) against its busy
        # time, and the all-reduce's bus bandwidth (ring: 2 (N-1)/N of the
        # [3, B] int64 join per GPU) against xGMI
        join_ms = sb.get("local_join", 0.0) + (sb.get("apply", 0.0) if world > 1 else 0.0)
        roof["stage_roofline"] = {}
        if join_ms:
            gbs = bpo * R * B / (join_ms / 1e3) / 1e9
            roof["stage_roofline"]["local_join"] = {"bound": "hbm", "achieved_GBps": gbs,
                                                    "peak_GBps": HBM_PEAK_GBS,
                                                    "frac": gbs / HBM_PEAK_GBS,
                                                    "bytes_per_round": bpo * R * B}
        ar_ms = sb.get("allreduce", 0.0)
        if world > 1 and ar_ms:
            alg = 3 * 8 * B / (ar_ms / 1e3) / 1e9
            bus = alg * 2 * (world - 1) / world
            roof["stage_roofline"]["allreduce"] = {"bound": "xgmi", "algbw_GBps": alg,
                                                   "busbw_GBps": bus, "peak_GBps": XGMI_GBPS,
                                                   "frac": bus / XGMI_GBPS}
    return {
        **roof,
        "metric": "anti-entropy replica-bucket joins/sec (C5: all-reduce(max) over xGMI)",
        "value": world * R * B * steps / el, "unit": "joins/s", "scaling": "weak",
        "n_gpus": world, "steps": steps, "warmup": warm, "ms_per_step": step_s * 1e3,
        "workload": (f"C5: {R} replicas/GPU ({R * world} total) x {B} buckets, {args.writes:g} of "
                     "the buckets written per replica per round, one anti-entropy pass per round"),
        "replicas_total": R * world, "allreduce_bytes": 3 * 8 * B,
        "local_GBps": bpo * R * B / step_s / 1e9,
        "step": ("phip_group_anti_entropy: " +
                 ("fused local join k_ae_join (one GPU: nothing to exchange)" if world == 1 else
                  "k_ae_local_max, ncclAllReduce(int64, MAX), k_ae_apply")
                 if group is not None else
                 "gloo rehearsal: phip_ae_local_max + torch all_reduce(MAX) + phip_ae_apply"),
        "rehearsal": args.dist_backend != "nccl",
        **diag,
        "verified": converged and go_ok, "converged": converged,
        "verify": {"sampled_buckets": 4096, "replicas_checked": R * world, "go_merge_equal": go_ok,
                   "reference": "float64 max of every replica's decoded added/taken and int max of "
                                "elapsed, gathered from all ranks before the round (Go Merge of "
                                "clean-domain states)"},
    }


def run_c5(args, torch, dev, repo, rank, world, gen):
    """R simulated replicas per GPU of B buckets each
    (E-encoded state planes, patrol_amd.shard).  A round = fresh local writes
    (a random fraction of each replica's buckets grows) followed by one
    anti-entropy pass: k_ae_local_max, RCCL all-reduce(MAX) of the [3, B]
    join over all GPUs, k_ae_apply (one GPU: the fused k_ae_join, nothing to
    exchange).  One round converges (max is idempotent);
    the loop models new writes between rounds.  A unit is one replica-bucket
    brought to the cluster-wide join."""
    from patrol_amd import shard
    R, B = args.replicas, args.buckets
    taken = torch.randint(0, 10**6, (R, B), device=dev, generator=gen).to(torch.float64)
    added = taken + torch.rand((R, B), dtype=torch.float64, device=dev, generator=gen) * 100.0
    reps = torch.empty((R, 3, B), dtype=torch.int64, device=dev)
    reps[:, 0] = shard.e_encode(added.view(torch.int64))
    reps[:, 1] = shard.e_encode(taken.view(torch.int64))
    reps[:, 2] = torch.randint(0, 1 << 40, (R, B), device=dev, generator=gen, dtype=torch.int64)
    del taken, added
    nw = max(1, int(B * args.writes))
    rounds = []
    for j in range(args.warmup + args.steps):
        idx = torch.randint(0, B, (R, nw), device=dev, generator=gen) + \
            torch.arange(R, device=dev).unsqueeze(1) * (3 * B)
        # a local Take: taken grows by a few ulps, elapsed by up to 1 ms
        rounds.append((idx.flatten(), torch.randint(1, 8, (R * nw,), device=dev, generator=gen),
                       torch.randint(1, 10**6, (R * nw,), device=dev, generator=gen)))
    flat = reps.view(-1)
    torch.cuda.synchronize()
    group = repo._group = open_group(args, dist_module(), repo, rank, world)
    if group is not None:
        group.set_timing(True)

    def step(j):
        idx, dt, de = rounds[j]
        flat.index_add_(0, idx + B, dt)
        flat.index_add_(0, idx + 2 * B, de)
        if group is not None:
            group.anti_entropy([reps])      # phip_group_anti_entropy: local max, RCCL max, apply
        else:
            shard.anti_entropy_native(reps, repo)

    def check():
        ok = bool((reps == reps[0:1]).all())
        if world > 1:
            import torch.distributed as dist
            s = reps[0].sum(dtype=torch.int64).view(1)
            lo, hi = s.clone(), s.clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            ok = ok and bool(lo == hi)
        return ok
    return R * B, step, check


def main():
    args = parse()
    launch_ranks(args)
    # The one JSON line goes to the real stdout; everything the libraries
    # print to fd 1 (RCCL's version banner at its first communicator) goes
    # to stderr instead.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    c1 = args.workload == "c1"
    if c1:
        # BASELINE configs[0]: 1M replica states into a 100k-bucket
        # repo; the C2 code path at that size, the CPU restatement on all of it.
        args.workload = "c2"
        args.keys, args.messages, args.log2_slots = 100_000, 1_000_000, 18
        args.cpu_sample = args.messages
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    routed = (args.workload == "c2" and not (c1 or args.no_routed or args.wire or args.insert or
                                             args.ring))
    if world > 1 or args.workload in ("c4", "c5") or routed:
        # c4/c5 and the owner-routed line exercise the collectives
        # (all-to-all, all-reduce) even on one GPU
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + (os.getpid() % 1000)))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group(args.dist_backend, init_method="env://")
    import patrol_amd

    K, n = args.keys, args.messages
    if args.insert:
        args.log2_slots = max(args.log2_slots, 27)
    gen = torch.Generator(device=dev).manual_seed(args.seed + 7919 * rank)

    # Shard: rank r owns bucket ids [r*K, (r+1)*K) (owner-routed upstream).
    base = rank * K
    # One stream for torch's input generation and the engine's kernels, so
    # device-pointer calls see torch's results without extra synchronisation.
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    repo = patrol_amd.GPURepo(device=local, log2_slots=args.log2_slots, arena_bytes=1 << 20)
    repo.use_torch_stream()
    keys = torch.arange(base, base + K, dtype=torch.int64, device=dev)
    kb, ko = names_for_ids(torch, keys, args.name_len if args.workload == "c2" else 0)
    st = torch.zeros((K, 4), dtype=torch.int64, device=dev)
    # added = taken = +0.0 bits, elapsed 0: the zero state GetBucket creates (repo.go:208)
    st[:, 3] = T0
    torch.cuda.synchronize()
    repo.seed_device(kb, ko, st, K)
    del kb, ko, st, keys
    assert len(repo) == K

    c5_check = None
    owned = K
    c3_cpu = None
    if args.workload == "c3":
        n, step, c3_cpu = run_c3(args, torch, dev, repo, rank, K, base, gen)
        ids = None
    elif args.workload == "c4":
        n, step, owned, c4_merged = run_c4(args, torch, dev, repo, rank, world, K, gen)
        ids = None
    elif args.workload == "c5":
        n, step, c5_check = run_c5(args, torch, dev, repo, rank, world, gen)
        ids = None
    elif args.workload == "route":
        n, step, route_sent = run_route(args, torch, dev, repo, K, gen)
        ids = None
    else:
        ids = zipf_ids(torch, gen, n, K, args.zipf, dev)
        blob, offs = names_for_ids(torch, ids + base, args.name_len)
        batches = [replica_states(torch, gen, n, j, dev) for j in range(args.warmup + args.steps)]
        # the per-message status column a Receive caller reads (merge vs incast);
        # two, alternating: a queued batch's outputs stay untouched until the
        # next call finishes it (PHIP_RECV_ASYNC), so batch j+1 writes the other
        c2_status = [None, None] if args.no_status else \
            [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        if args.insert:
            # SURVEY C2's insert-on-miss variant: every step names a fresh
            # key range (same Zipf shape), so each step creates the buckets it
            # touches (GetBucket's miss branch, repo.go:195-210).
            fresh = [names_for_ids(torch, ids + base + (j + 1) * world * K)
                     for j in range(args.warmup + args.steps)]
            n_new = []
        torch.cuda.synchronize()

        if args.ring:
            # PCIe-inclusive ingest: datagram batches in
            # pinned host ring slots; each step submits the next slot's
            # host->device copy and receives the current slot, so the copy of
            # batch j+1 overlaps the merge of batch j.  Results (statuses)
            # come back to host memory as a Go caller would read them.
            nslots = 3
            sizes = []
            ring = None
            for k in range(nslots):
                a, t, e = batches[k]
                db, do = datagrams(torch, blob, offs, a, t, e)
                nb = int(do[-1])
                if ring is None:
                    ring = patrol_amd.Ring(repo, nslots=nslots, max_msgs=n, max_bytes=nb + (1 << 20))
                slot, bv, ov = ring.acquire()
                bv[:nb] = db[:nb].cpu().numpy()
                ov[:n + 1] = do.cpu().numpy().astype(np.uint64)
                del db, do
                ring.submit(slot, n)
                ring.receive(slot, n, T0, want_status=False)
                sizes.append(nb)
            del batches
            torch.cuda.synchronize()
            ring_status = np.zeros(n, np.uint8)
            cur = [ring.acquire()[0]]
            ring.submit(cur[0], n)
            ring_bytes = sum(sizes) / nslots

            def step(j):
                nxt = ring.acquire()[0]
                ring.submit(nxt, n)
                ring.receive(cur[0], n, T0 + j, status=ring_status)
                cur[0] = nxt
        elif args.wire:
            wires = []
            for a, t, e in batches:
                wires.append(datagrams(torch, blob, offs, a, t, e))
            del batches
            torch.cuda.synchronize()

            def step(j):
                db, do = wires[j]
                repo.receive_datagrams_device(db, do, n, T0 + j)
        elif args.insert:
            def step(j):
                a, t, e = batches[j]
                fb, fo = fresh[j]
                before = len(repo)
                repo.receive_soa(fb, a, t, e, T0 + j, name_offs=fo, n=n, device=True)
                n_new.append(len(repo) - before)
        else:
            # names_len = 0: this caller produced the batch and holds it until
            # the call that finishes it returns, so the device does not check
            # its offsets (the binding's default checks them: ~0.1 ms per
            # 100M messages, patrolhip.h phip_msgs.names_len)
            def step(j):
                a, t, e = batches[j]
                repo.receive_soa(blob, a, t, e, T0 + j, name_offs=offs, n=n, status=c2_status[j % 2],
                                 device=True, queue=not args.sync_receive,
                                 names_len=0 if not args.check_names else None)

    extra = {}
    for j in range(args.warmup):
        step(j)
    repo.flush()   # (a queued receive batch: finished and checked here)
    # HIP events around every kernel of the timed steps, kept by the library
    # and read once after the timed region (reading them synchronises).
    # (c5's step reads its own per-call timings from the shard layer.)
    repo.set_timing(True, accumulate=True)
    kern = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    launches = {}
    step_tl = []
    for j in range(args.warmup, args.warmup + args.steps):
        tl = step(j)
        if tl is not None:
            step_tl.append(tl)
    repo.flush()   # the last queued batch finished (its misses / dirty buckets) inside the timing
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # per step: a kernel launched several times in a step (chunks) is summed
    for tl in (step_tl or [repo.timings()]):
        for name, ms in tl:
            kern[name] = kern.get(name, 0.0) + ms / (1 if step_tl else args.steps)
            launches[name] = launches.get(name, 0) + 1
    kern = {k: [v / (args.steps if step_tl else 1)] for k, v in kern.items()}
    repo.set_timing(False)
    if args.workload == "c2":
        st4 = repo.last_stats()   # the last batch: directory entries, folded through it, misses
        extra["hot_directory"] = {"entries": int(st4[0]), "folded": int(st4[1]),
                                  "misses": int(st4[2])}
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64,
                          device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())

    total = world * n * args.steps
    kms = {k: float(np.mean(v)) for k, v in kern.items()}
    if args.workload == "c5":
        # bytes of the two local passes per round (reads R*24, writes 24;
        # then reads 24 + R*24 per bucket) over their kernel time; k_ae_apply
        # writes only the fields the join changed, data-dependent and not
        # counted (profiles/r02_c5_kernels.json has the measured writes)
        R, B = args.replicas, args.buckets
        if "k_ae_join" in kms:
            # one GPU: the fused join (phip_ae_join) reads each replica's 24
            # bytes once and writes only what the join raised
            bpo = 24.0
            dom_name, dom_ms = "k_ae_join", kms["k_ae_join"]
        else:
            bpo = (2 * R + 2) * 24 / R
            dom_name = "k_ae_local_max+k_ae_apply"
            dom_ms = kms.get("k_ae_local_max", float("nan")) + kms.get("k_ae_apply", float("nan"))
        unit, metric = "merges/s", METRIC + " [C5: anti-entropy replica-bucket joins/sec]"
        workload = (f"C5 anti-entropy: {R} replicas/GPU x {B} buckets, {args.writes:g} of buckets "
                    f"written per replica per round, all-reduce(max) over {world} GPU(s)")
        extra["converged"] = c5_check()
        allreduce_bytes = 3 * 8 * B
        step_s = el / args.steps
        extra["allreduce_bytes"] = allreduce_bytes
        extra["replicas_total"] = R * world
        grp = getattr(repo, "_group", None)
        ar_ms = grp.stage_ms()["exchange"] if grp is not None and world > 1 else None
        if ar_ms:   # HIP events around the RCCL call (phip_group_anti_entropy)
            algbw = allreduce_bytes / (ar_ms / 1e3) / 1e9
            extra["allreduce_ms"] = ar_ms
            extra["allreduce_algbw_GBps"] = algbw
            extra["allreduce_busbw_GBps"] = algbw * 2 * (world - 1) / world
    elif args.workload == "c4":
        bpo = BYTES_PER_MERGE
        dom_name, dom_ms = DOMINANT, float(np.mean(kern.get(DOMINANT, [float("nan")])))
        unit, metric = "merges/s", METRIC + " [C4: owner-routed]"
        workload = (f"C4 owner-routed merge: {n} messages/GPU over {K * world} buckets hash-sharded "
                    f"by name across {world} GPU(s), all-to-all routing + merge, Zipf({args.zipf})")
        extra["buckets_owned_rank0"] = owned
        extra["sender_combine"] = not args.no_combine
        # the fast kernel merges what this rank received after routing and
        # the sender-side combine, not the n messages it sent
        extra["messages_sent_per_step_rank0"] = n
        extra["messages_merged_per_step_rank0"] = float(np.mean(c4_merged))
        grp = getattr(repo, "_group", None)
        if grp is not None:   # rank 0's stage busy time of the last step
            extra["stage_busy_ms"] = grp.stage_ms()
    elif args.workload == "route":
        # the pack's algorithmic bytes: read the message (offset 4 + name +
        # 24), write it owner-major (length 4 + name + 24); names ~7 B
        bpo = 2 * (4 + 24 + 7)
        dom_name = "k_route_count+k_route_scatter"
        dom_ms = kms.get("k_route_count", float("nan")) + kms.get("k_route_scatter", float("nan"))
        unit, metric = "messages/s", METRIC + " [owner-routing pack, messages packed/sec]"
        workload = (f"owner-routing pack: {n} messages (Zipf({args.zipf}) over {K} buckets) packed by "
                    f"owner for {args.route_world} owners with the sender-side combine")
        extra["route_world"] = args.route_world
        extra["messages_sent_after_combine"] = route_sent[0] if route_sent else None
    elif args.workload == "c3":
        # Take 89 B (op 24 + state read 32 + write 24 + result 9), Merge 88 B.
        bpo = 88.5
        dom_name, dom_ms = "whole step", el / args.steps * 1e3
        unit, metric = "ops/s", METRIC + " [C3: mixed Take+Merge ops/sec]"
        workload = c3_workload(args, n, K, args.log2_slots)
        extra["c3_clock"] = args.c3_clock
    else:
        bpo = BYTES_PER_MERGE
        dom_name, dom_ms = DOMINANT, float(np.mean(kern.get(DOMINANT, [float("nan")])))
        unit, metric = "merges/s", METRIC
        workload = f"C2 merge: {n} replica messages -> {K}-bucket table (2^{args.log2_slots} slots), Zipf({args.zipf})"
        if c1:
            workload = "C1 (the reference's CPU case) " + workload[3:]
        if args.wire:
            workload += ", raw datagrams (decode + merge)"
        if args.insert:
            workload += ", insert-on-miss (every step names a fresh key range)"
            extra["buckets_created_per_step"] = float(np.mean(n_new[args.warmup:]))
        if args.ring:
            workload = (f"C2 ingest ring (PCIe-inclusive): {n} datagrams per batch from pinned host "
                        f"slots -> {K}-bucket table, copy of batch j+1 overlapping merge of batch "
                        f"j, statuses back to host, Zipf({args.zipf}); slots cycle 3 batches")
            extra["h2d_bytes_per_step"] = ring_bytes
            extra["h2d_GBps"] = ring_bytes * args.steps / el / 1e9
    # c4: the dominant kernel merges this rank's received (routed, combined)
    # messages, so its algorithmic bytes count those
    n_roof = float(np.mean(c4_merged)) if args.workload == "c4" else n
    achieved = bpo * n_roof / (dom_ms / 1e3) / 1e9
    build = patrol_amd.build_id()
    traffic, traffic_src = pmc_traffic(args.workload if not c1 else "c1", workload, dom_name, build)
    out = {
        "metric": metric,
        "value": total / el,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded Zipf keys, SURVEY §8d replica states; batches resident in HBM)",
        "config": {"workload": workload, "keys_per_gpu": K, "messages_per_step_per_gpu": n,
                   "slots_per_gpu": 1 << args.log2_slots, "parallelism": f"shard{world}",
                   "name_bytes": args.name_len or "2-8 (b<id>)",
                   "world_size": world,
                   # the headline is C2 weak scaling: every rank merges its own
                   # pre-routed stream, no owner routing (that is owner_routed / c4)
                   "exchange": False,
                   "dist_backend": args.dist_backend if dist.is_initialized() else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": dom_name, "kernel_ms_per_step": dom_ms,
                     "launches_per_step": launches.get(dom_name, args.steps) / args.steps,
                     "algorithmic_bytes_per_step": bpo * n_roof},
        "kernels_ms": kms,
        "build_id": build,
    }
    out["config"].update(extra)
    if rank == 0 and world == 1 and not args.no_cpu and args.workload == "c2":
        try:
            out["cpu_baseline"] = cpu_baseline(args, K, ids.cpu())
        except Exception as ex:  # the baseline must never hide the GPU result
            out["cpu_baseline"] = {"error": repr(ex)}
    elif rank == 0 and world == 1 and not args.no_cpu and c3_cpu is not None:
        try:
            out["cpu_baseline"] = c3_cpu()
        except Exception as ex:
            out["cpu_baseline"] = {"error": repr(ex)}
    elif rank == 0:
        out["cpu_baseline"] = None
    if args.ring and args.workload == "c2":
        ring.close()
    if getattr(repo, "_group", None) is not None:
        repo._group.close()
    repo.close()
    if routed:
        # the C2 batches are freed first: every extra leg has its own
        del step
        if args.workload == "c2":
            del batches, blob, offs, ids
        legs = [("owner_routed", run_routed)]
        if not args.no_variants:
            legs.append(("c2_variants", run_c2_variants_leg))
        if not args.no_c3:
            legs.append(("c3", run_c3_leg))
        if not args.no_c4:
            legs.append(("c4", run_c4_leg))
        if not args.no_ae:
            legs.append(("anti_entropy", run_ae_leg))
        # Each extra leg is an object in the line: an error or a hang there
        # (one rank failing inside a collective leaves the others waiting)
        # must not cost the headline.  A watchdog on every rank prints the
        # line without it and ends the process with a non-zero status.
        import threading
        failed = False
        for key, fn in legs:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

            def give_up(key=key):
                # the line still carries the headline, but the exit status says
                # the leg hung (a driver or CI must be able to tell)
                if rank == 0:
                    out[key] = {"error": f"timed out after {LEG_LIMIT_S} s"}
                    print(json.dumps(out), file=json_out, flush=True)
                os._exit(LEG_TIMEOUT_EXIT)
            dog = threading.Timer(LEG_LIMIT_S, give_up)
            dog.daemon = True
            dog.start()
            try:
                out[key] = fn(args, torch, dist, dev, local, rank, world)
                if out[key].get("verified") is False:
                    failed = True
            except Exception as ex:
                out[key] = {"error": repr(ex)}
                failed = True
            dog.cancel()
        if failed:
            print("bench.py: an extra leg failed or did not verify", file=sys.stderr)
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    if routed and failed:
        sys.exit(LEG_FAILED_EXIT)


if __name__ == "__main__":
    main()
