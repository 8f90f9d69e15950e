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


def _c4_worker(rank, world, port, n, out_q):
    """C4's per-rank step with the oracle as the receiving table: pack by
    owner (the layout phip_route_pack writes), exchange_packed (the same glue
    bench.py's C4 and owner-routed lines run), then Receive the owned
    messages into this rank's shard."""
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names, blob, offs, a, t, e = _c4_msgs(rank, n)
        packed = shard.pack_by_owner(blob, offs, a, t, e, world)
        rb, ro, ra, rt, re = shard.exchange_packed(*packed)
        m = ro.numel() - 1
        repo = O.Repo()
        st, _, _, _ = repo.receive_soa([bytes(rb[ro[i]:ro[i + 1]].numpy()) for i in range(m)],
                                       ra.numpy().view(np.uint64), rt.numpy().view(np.uint64),
                                       re.numpy(), 10**18)
        out_q.put((rank, m, repo.dump()))
    finally:
        dist.destroy_process_group()


def _c4_msgs(rank, n):
    rng = np.random.default_rng(300 + rank)
    ids = rng.zipf(1.3, n) % 4000
    names = [(b"b%d" % i) if i % 9 else (b"a-longer-bucket-name-%d" % i) for i in ids]
    lens = torch.tensor([len(x) for x in names], dtype=torch.int64)
    offs = torch.zeros(n + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(lens, 0)
    blob = torch.tensor(np.frombuffer(b"".join(names) + b"\0" * 8, np.uint8).copy())
    taken = rng.integers(0, 10**6, n).astype(np.float64)
    a = torch.from_numpy((taken + rng.random(n) * 100).view(np.int64).copy())
    t = torch.from_numpy(taken.view(np.int64).copy())
    e = torch.tensor(rng.integers(1, 1 << 40, n), dtype=torch.int64)
    return names, blob, offs, a, t, e


def test_owner_routed_receive_gloo_world2_equals_oracle():
    """The owner-routed merge over two gloo ranks: every
    rank's shard holds only buckets it owns, shards are disjoint, and their
    union equals one oracle repo that received every rank's messages
    (repo.go:54-92; merges commute in the clean domain)."""
    from oracle import oracle as O
    world, n = 2, 20000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (m, d) for r, m, d in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(m for m, _ in res.values()) == world * n
    whole = O.Repo()
    for r in range(world):
        names, blob, offs, a, t, e = _c4_msgs(r, n)
        whole.receive_soa(names, a.numpy().view(np.uint64), t.numpy().view(np.uint64), e.numpy(),
                          10**18)
    union = {}
    for r in range(world):
        d = res[r][1]
        for k in d:
            assert int(shard.owner_of(torch.tensor([to_i64(G.fnv1a64(k))]), world)) == r
        assert not (set(d) & set(union))
        union.update(d)
    assert union == whole.dump()


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


@pytest.mark.gpu
def test_anti_entropy_native_gpu_equals_go_merge_and_torch():
    """k_ae_local_max + k_ae_apply (libpatrolhip) on cuda:0, single rank: every
    replica ends as the Go merge of all replicas (bucket.go:240-263), and
    equal to the torch restatement."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import patrol_amd
    R, B = 6, 700
    reps = _replicas(0, 3, B) + _replicas(1, 3, B)
    x = torch.zeros((R, 3, B), dtype=torch.int64)
    for k, (a, t, e) in enumerate(reps):
        x[k, 0] = shard.e_encode(torch.tensor([to_i64(v) for v in a]))
        x[k, 1] = shard.e_encode(torch.tensor([to_i64(v) for v in t]))
        x[k, 2] = torch.tensor(e)
    want_t = shard.anti_entropy(x.clone())
    repo = patrol_amd.GPURepo(device=0, log2_slots=10)
    xd = x.cuda()
    torch.cuda.synchronize()
    shard.anti_entropy_native(xd, repo)
    got = xd.cpu()
    assert torch.equal(got, want_t)
    for i, own in enumerate(reps):
        for b in range(0, B, 7):
            acc = G.Bucket(added=G.b2f(own[0][b]), taken=G.b2f(own[1][b]), elapsed=own[2][b])
            for j, (a, t, e) in enumerate(reps):
                if j != i:
                    acc.merge(G.Bucket(added=G.b2f(a[b]), taken=G.b2f(t[b]), elapsed=e[b]))
            ga = int(shard.e_decode(got[i, 0, b:b + 1])[0]) & (2**64 - 1)
            gt = int(shard.e_decode(got[i, 1, b:b + 1])[0]) & (2**64 - 1)
            assert (ga, gt, int(got[i, 2, b])) == (G.f2b(acc.added), G.f2b(acc.taken), acc.elapsed)
    repo.close()


@pytest.mark.gpu
@pytest.mark.parametrize("R,B", [(1, 1031), (6, 1031), (6, 1032), (16, 1032), (21, 1031),
                                 (21, 1032)])
def test_ae_join_equals_local_max_apply(R, B):
    """phip_ae_join (k_ae_join: the one-GPU round, fused) on cuda:0 equals
    the torch restatement and the two-kernel path, for R held in registers
    and R above kAeRegs (16) that re-reads, odd B (one bucket per load) and
    even B (16-byte pairs); special floats (NaN sticking, +-Inf, -0.0),
    INT64_MIN/MAX elapsed."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import patrol_amd
    from patrol_amd import _lib
    reps = _replicas(R, R, B)
    x = torch.zeros((R, 3, B), dtype=torch.int64)
    for k, (a, t, e) in enumerate(reps):
        x[k, 0] = shard.e_encode(torch.tensor([to_i64(v) for v in a]))
        x[k, 1] = shard.e_encode(torch.tensor([to_i64(v) for v in t]))
        x[k, 2] = torch.tensor(e)
    x[:, 2, :5] = torch.tensor([-(1 << 63), (1 << 63) - 1, 0, -1, -(1 << 63)])
    x[:, 2, 5] = -(1 << 63)          # every replica at INT64_MIN: unchanged
    want = shard.anti_entropy(x.clone())
    repo = patrol_amd.GPURepo(device=0, log2_slots=10)
    xd = x.cuda()
    x2 = x.cuda()
    torch.cuda.synchronize()
    assert _lib.load().phip_ae_join(repo.h, xd.data_ptr(), R, B, _lib.DEVICE_PTRS) == 0
    shard.anti_entropy_native(x2, repo)
    assert torch.equal(xd.cpu(), want)
    assert torch.equal(x2.cpu(), want)
    assert _lib.load().phip_ae_join(repo.h, xd.data_ptr(), R, B, 0) == -1   # PHIP_ERR_INVALID
    repo.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,huge", [(1, False), (3, False), (8, False), (8, True), (16, False),
                                        (16, True), (64, False), (1, "short"), (3, "short"),
                                        (8, "short"), (64, "short"), (8, "sparse")])
def test_route_pack_is_stable_owner_partition(world, huge):
    """phip_route_pack on cuda:0: owner-major, per-owner original order,
    names/lengths/states moved intact, per-owner counts and byte totals.
    World <= 16 places by packed DPP scans, larger worlds (and waves holding
    a name over 255 bytes: `huge`) by the per-owner ballot rounds.  "short":
    every name of 1-16 bytes (all at every byte alignment), so every chunk
    takes the LDS-staged dword path; "sparse": a long name in one message of
    5000, so staged chunks and byte-path chunks alternate within a tile."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ctypes as C
    import patrol_amd
    from patrol_amd import _lib
    from patrol_amd.engine import phip_msgs, names_blob
    rng = np.random.default_rng(world)
    n = 200_003
    ids = rng.integers(0, 50_000, n)
    if huge == "short":
        names = [(b"%x" % i)[: 1 + k % 16].ljust(1 + k % 16, b"z") for k, i in enumerate(ids)]
    elif huge == "sparse":
        names = [(b"b%d" % i) if k % 5000 else (b"a-long-bucket-name-%d" % i) for k, i in enumerate(ids)]
    else:
        names = [(b"b%d" % i) if i % 7 else (b"a-long-bucket-name-%d-%s" % (i, b"x" * (i % 40)))
                 for i in ids]
    if huge is True:
        names = [nm + b"y" * 300 if k % 5003 == 0 else nm for k, nm in enumerate(names)]
    blob_np, offs_np = names_blob(names)
    a = rng.integers(0, 1 << 62, n).astype(np.int64)
    t = rng.integers(0, 1 << 62, n).astype(np.int64)
    e = rng.integers(-(1 << 62), 1 << 62, n).astype(np.int64)
    h = shard.hash_names(torch.from_numpy(blob_np), torch.from_numpy(offs_np.astype(np.int64)))
    own = shard.owner_of(h, world).numpy()
    order = np.argsort(own, kind="stable")
    repo = patrol_amd.GPURepo(device=0, log2_slots=10)
    dev = torch.device("cuda", 0)
    blob, offs = torch.from_numpy(blob_np).to(dev), torch.from_numpy(offs_np.view(np.int32)).to(dev)
    da, dt, de = (torch.from_numpy(x).to(dev) for x in (a, t, e))
    s_names = torch.empty(blob.numel(), dtype=torch.uint8, device=dev)
    s_lens = torch.empty(n, dtype=torch.int32, device=dev)
    s_a, s_t, s_e = (torch.empty(n, dtype=torch.int64, device=dev) for _ in range(3))
    cnt = torch.zeros(world, dtype=torch.int64, device=dev)
    nb = torch.zeros(world, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    m = phip_msgs(n, 0, blob.data_ptr(), offs.data_ptr(), da.data_ptr(), dt.data_ptr(), de.data_ptr())
    rc = _lib.load().phip_route_pack(repo.h, C.byref(m), world, s_names.data_ptr(), s_lens.data_ptr(),
                                     s_a.data_ptr(), s_t.data_ptr(), s_e.data_ptr(), cnt.data_ptr(),
                                     nb.data_ptr(), _lib.DEVICE_PTRS)
    assert rc == 0
    lens = np.diff(offs_np.astype(np.int64))
    assert np.array_equal(cnt.cpu().numpy(), np.bincount(own, minlength=world))
    assert np.array_equal(nb.cpu().numpy(), np.bincount(own, weights=lens, minlength=world).astype(np.int64))
    assert np.array_equal(s_lens.cpu().numpy(), lens[order])
    assert np.array_equal(s_a.cpu().numpy(), a[order])
    assert np.array_equal(s_t.cpu().numpy(), t[order])
    assert np.array_equal(s_e.cpu().numpy(), e[order])
    want = b"".join(names[k] for k in order)
    assert s_names.cpu().numpy()[:len(want)].tobytes() == want
    repo.close()


def _route_pack(repo, blob, offs, da, dt, de, world, flags):
    import ctypes as C
    from patrol_amd import _lib
    from patrol_amd.engine import phip_msgs
    dev = blob.device
    n = offs.numel() - 1
    s_names = torch.zeros(blob.numel() + 64, dtype=torch.uint8, device=dev)
    s_lens = torch.zeros(n, dtype=torch.int32, device=dev)
    s_a, s_t, s_e = (torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(3))
    cnt = torch.zeros(world, dtype=torch.int64, device=dev)
    nb = torch.zeros(world, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    m = phip_msgs(n, 0, blob.data_ptr(), offs.data_ptr(), da.data_ptr(), dt.data_ptr(), de.data_ptr())
    rc = _lib.load().phip_route_pack(repo.h, C.byref(m), world, s_names.data_ptr(), s_lens.data_ptr(),
                                     s_a.data_ptr(), s_t.data_ptr(), s_e.data_ptr(), cnt.data_ptr(),
                                     nb.data_ptr(), _lib.DEVICE_PTRS | flags)
    assert rc == 0
    return s_names, s_lens, s_a, s_t, s_e, cnt.cpu().tolist(), nb.cpu().tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 3])
def test_route_pack_combine_owner_states_equal_oracle(world):
    """PHIP_ROUTE_COMBINE on a 2^21-message clean Zipf batch (long and
    medium names, NaN fields, all-non-positive messages that must not be
    combined): every owner's segment received into its own table gives,
    together, exactly the oracle's table for the whole batch, with far fewer
    messages sent.  A dirty batch (one incast) packs exactly as without the
    flag."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import patrol_amd
    from oracle import oracle as O
    from patrol_amd import _lib
    from patrol_amd.engine import names_blob
    from tests import _gen
    rng = np.random.default_rng(77 + world)
    n, K = 1 << 21, 30000
    ids = _gen.zipf_ids(rng, n, K)
    names = [(b"a-much-longer-bucket-name-%d" % i) if i % 97 == 0 else
             (b"medium-name-%d" % i) if i % 89 == 0 else (b"b%d" % i) for i in ids]
    a, t, e = _gen.clean_states(rng, n)
    nanb = np.uint64(0x7FF8000000000000)
    sel = rng.random(n) < 0.02
    a[sel] = nanb
    sel = rng.random(n) < 0.02
    t[sel] = nanb
    neg = rng.random(n) < 0.01      # all fields <= 0: never combined
    a[neg] = np.float64(-3.0).view(np.uint64)
    t[neg] = np.float64(-1.0).view(np.uint64)
    e[neg] = -7
    now = _gen.T0 + 2 * _gen.SEC
    dev = torch.device("cuda", 0)
    blob_np, offs_np = names_blob(names)
    blob = torch.from_numpy(blob_np).to(dev)
    offs = torch.from_numpy(offs_np.view(np.int32)).to(dev)
    da, dt, de = (torch.from_numpy(x.view(np.int64)).to(dev) for x in (a, t, e))
    router = patrol_amd.GPURepo(device=0, log2_slots=10)
    s_names, s_lens, s_a, s_t, s_e, cnt, nb = _route_pack(router, blob, offs, da, dt, de, world,
                                                          _lib.ROUTE_COMBINE)
    assert sum(cnt) < 3 * n // 4      # the Zipf head went out combined
    o = O.Repo()
    o.receive_soa(names, a, t, e, now)
    want = o.dump()
    got = {}
    c0 = b0 = 0
    for r in range(world):
        m = cnt[r]
        g = patrol_amd.GPURepo(device=0, log2_slots=16)
        if m:
            lens = s_lens[c0:c0 + m]
            ro = torch.zeros(m + 1, dtype=torch.int32, device=dev)
            torch.cumsum(lens, 0, dtype=torch.int32, out=ro[1:])
            g.receive_soa(s_names[b0:], s_a[c0:c0 + m], s_t[c0:c0 + m], s_e[c0:c0 + m], now,
                          name_offs=ro, n=m, device=True)
            torch.cuda.synchronize()
        d = {k: (v.added, v.taken, v.elapsed, v.created) for k, v in g.dump().items()}
        assert not (set(d) & set(got))
        got.update(d)
        c0 += m
        b0 += nb[r]
        g.close()
    assert len(got) == len(want)
    bad = [k for k in want if got.get(k) != want[k]]
    assert not bad, [(k, got.get(k), want[k]) for k in bad[:5]]
    # a dirty batch: exactly the plain stable partition
    a2 = a.copy()
    a2[n // 3] = 0
    t2 = t.copy()
    t2[n // 3] = 0
    e2 = e.copy()
    e2[n // 3] = 0
    da2, dt2, de2 = (torch.from_numpy(x.view(np.int64)).to(dev) for x in (a2, t2, e2))
    x = _route_pack(router, blob, offs, da2, dt2, de2, world, _lib.ROUTE_COMBINE)
    y = _route_pack(router, blob, offs, da2, dt2, de2, world, 0)
    assert x[5] == y[5] and x[6] == y[6] and sum(x[5]) == n
    for u, v in zip(x[:5], y[:5]):
        assert torch.equal(u, v)
    router.close()
