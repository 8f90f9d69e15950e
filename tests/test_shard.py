"""Shard layer on CPU with the gloo backend, world_size 2.

* owner routing: after route_messages every message sits on its owner rank,
  nothing is lost or duplicated, per-source order is kept;
* anti-entropy: all_reduce(MAX) over E codes equals the sequential Go merge
  of every replica (bucket.go:240-263) -- checked against the Python
  restatement of the reference;
* the torch E-encoding mirrors the device encoding bit for bit.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import go_semantics as G
from patrol_amd import shard

S = 1 << 63
INF = 0x7FF0000000000000


def enc_ref(b):
    mag = b & ~S
    if mag > INF:
        return 0xFFE0000000000002 + mag - INF - 1 + ((1 << 52) - 1 if b & S else 0)
    if b & S:
        return INF + 1 if mag == 0 else INF - mag
    return INF if mag == 0 else INF + 1 + mag


def to_i64(u):
    return u - (1 << 64) if u >= S else u


def specials():
    return [0, S, 1, S | 1, INF, S | INF, INF + 1, S | (INF + 1), 0x7FF8000000000000,
            0xFFFFFFFFFFFFFFFF, 0x7FFFFFFFFFFFFFFF, G.f2b(1.0), G.f2b(-2.5), G.f2b(1e300)]


def test_e_encode_matches_device_encoding():
    rng = random.Random(3)
    vals = specials() + [rng.getrandbits(64) for _ in range(20000)]
    t = torch.tensor([to_i64(v) for v in vals], dtype=torch.int64)
    got = shard.e_encode(t).tolist()
    assert [g & (2**64 - 1) for g in got] == [enc_ref(v) for v in vals]
    back = shard.e_decode(shard.e_encode(t))
    assert torch.equal(back, t)


def test_owner_map_is_uniform():
    h = torch.tensor([to_i64(random.Random(i).getrandbits(64)) for i in range(20000)])
    for world in (2, 3, 8):
        own = shard.owner_of(h, world)
        assert int(own.min()) >= 0 and int(own.max()) < world
        cnt = torch.bincount(own, minlength=world).float()
        assert float(cnt.min() / cnt.max()) > 0.9


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_msgs(rank, n):
    rng = np.random.default_rng(100 + rank)
    ids = rng.integers(0, 5000, n)
    names = [b"b%d" % i for i in ids]
    lens = torch.tensor([len(x) for x in names], dtype=torch.int64)
    offs = torch.zeros(n + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(lens, 0)
    blob = torch.tensor(np.frombuffer(b"".join(names) + b"\0" * 8, np.uint8).copy())
    a = torch.tensor(rng.integers(0, 1 << 62, n), dtype=torch.int64)
    t = torch.tensor(rng.integers(0, 1 << 62, n), dtype=torch.int64)
    e = torch.tensor(rng.integers(-(1 << 40), 1 << 40, n), dtype=torch.int64)
    return names, blob, offs, a, t, e


def _route_worker(rank, world, port, n, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names, blob, offs, a, t, e = _make_msgs(rank, n)
        rb, ro, ra, rt, re = shard.route_messages(blob, offs, a, t, e)
        got = [(bytes(rb[ro[i]:ro[i + 1]].numpy()), int(ra[i]), int(rt[i]), int(re[i]))
               for i in range(ro.numel() - 1)]
        out_q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_route_messages_gloo_world2():
    world, n = 2, 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_route_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sent = []
    for r in range(world):
        names, blob, offs, a, t, e = _make_msgs(r, n)
        sent.append([(names[i], int(a[i]), int(t[i]), int(e[i])) for i in range(n)])
    for r in range(world):
        for (name, *_rest) in res[r]:
            h = torch.tensor([to_i64(G.fnv1a64(name))])
            assert int(shard.owner_of(h, world)) == r
        # per-source order kept: the slice from source s is s's owned messages in order
        want = []
        for s in range(world):
            want += [m for m in sent[s]
                     if int(shard.owner_of(torch.tensor([to_i64(G.fnv1a64(m[0]))]), world)) == r]
        assert res[r] == want
    assert sum(len(v) for v in res.values()) == world * n


def _replicas(rank, R, B):
    rng = random.Random(7 + rank)
    pool = [b for b in specials() if b != S] + [G.f2b(float(i)) for i in range(50)]
    reps = []
    for _ in range(R):
        a = [rng.choice(pool) if rng.random() < 0.3 else G.f2b(rng.random() * 100) for _ in range(B)]
        t = [rng.choice(pool) if rng.random() < 0.3 else G.f2b(rng.random() * 100) for _ in range(B)]
        e = [rng.randrange(-(1 << 62), 1 << 62) for _ in range(B)]
        reps.append((a, t, e))
    return reps


def _ae_worker(rank, world, port, R, B, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        reps = _replicas(rank, R, B)
        x = torch.zeros((R, 3, B), dtype=torch.int64)
        for k, (a, t, e) in enumerate(reps):
            x[k, 0] = shard.e_encode(torch.tensor([to_i64(v) for v in a]))
            x[k, 1] = shard.e_encode(torch.tensor([to_i64(v) for v in t]))
            x[k, 2] = torch.tensor(e)
        j = shard.anti_entropy(x)
        out_q.put((rank, [(shard.e_decode(j[k, 0]).tolist(), shard.e_decode(j[k, 1]).tolist(),
                           j[k, 2].tolist()) for k in range(R)]))
    finally:
        dist.destroy_process_group()


def test_anti_entropy_gloo_world2_equals_go_merge():
    world, R, B = 2, 3, 400
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ae_worker, args=(r, world, port, R, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allreps = _replicas(0, R, B) + _replicas(1, R, B)
    got_all = res[0] + res[1]
    for i, own in enumerate(allreps):
        got = got_all[i]
        for b in range(B):
            # Go: replica i's bucket Merge()s every other replica (no -0.0 in the pool)
            acc = G.Bucket(added=G.b2f(own[0][b]), taken=G.b2f(own[1][b]), elapsed=own[2][b])
            for j, (a, t, e) in enumerate(allreps):
                if j != i:
                    acc.merge(G.Bucket(added=G.b2f(a[b]), taken=G.b2f(t[b]), elapsed=e[b]))
            assert (got[0][b] & (2**64 - 1), got[1][b] & (2**64 - 1), got[2][b]) == \
                   (G.f2b(acc.added), G.f2b(acc.taken), acc.elapsed), (i, b)
