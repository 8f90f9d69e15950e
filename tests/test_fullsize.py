"""Parity at the BASELINE configurations' full sizes, generated exactly as
bench.py generates them (same functions, seeds and shapes), checked against
the oracle (oracle/liboracle.so) on the same inputs:

* C2 (BASELINE configs[1]): 10M seeded buckets in 2^25 slots, one 100M-message
  Zipf(1.1) batch through phip_receive_soa (the timed step of bench.py):
  every status and the whole 10M-bucket table bit-exact;
* C3 (configs[2]): 50M mixed Take(100:1s)/Merge ops through phip_apply_mixed,
  with the replica clock below the local one (Takes refill, succeed, deny)
  and ahead of it: every status, `remaining`, `have` and the table.

The oracle runs the Go loop one message at a time (about 5M ops/s), so each
test takes tens of seconds on the host.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402

T0 = 1_700_000_000_000_000_000


@pytest.fixture(scope="module")
def env():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    import patrol_amd
    return torch, bench, patrol_amd


def _seeded(torch, bench, pa, dev, K, L, stream):
    """bench.py's table: K buckets b0..b{K-1}, zero state, created T0."""
    repo = pa.GPURepo(device=0, log2_slots=L, arena_bytes=1 << 20)
    repo.set_stream(stream)
    keys = torch.arange(K, dtype=torch.int64, device=dev)
    kb, ko = bench.names_for_ids(torch, keys)
    st = torch.zeros((K, 4), dtype=torch.int64, device=dev)
    st[:, 3] = T0
    torch.cuda.synchronize()
    repo.seed_device(kb, ko, st, K)
    assert len(repo) == K
    o = O.Repo()
    z = np.zeros(K, np.uint64)
    o.L.orc_repo_seed(o.h, kb.cpu().numpy(), ko.cpu().numpy().view(np.uint32), K, z, z,
                      np.zeros(K, np.int64), np.full(K, T0, np.int64))
    return repo, o


def _check_table(repo, o):
    names, offs, a, t, e, c = repo.dump_arrays()
    assert len(offs) - 1 == len(repo) == len(o)
    bad, first = o.check_dump(names, offs, a, t, e, c)
    assert bad == 0, (bad, first, bytes(names[offs[first]:offs[first + 1]]) if first < len(offs) - 1
                      else None)


@pytest.mark.timeout(900)
def test_c2_full_size_vs_oracle(env):
    torch, bench, pa = env
    dev = torch.device("cuda", 0)
    K, n, L = 10_000_000, 100_000_000, 25
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        gen = torch.Generator(device=dev).manual_seed(1234)     # bench.py, rank 0
        repo, o = _seeded(torch, bench, pa, dev, K, L, s)
        ids = bench.zipf_ids(torch, gen, n, K, 1.1, dev)
        blob, offs = bench.names_for_ids(torch, ids)
        del ids
        a, t, e = bench.replica_states(torch, gen, n, 0, dev)
        status = torch.empty(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        repo.receive_soa(blob, a, t, e, T0, name_offs=offs, n=n, status=status, device=True)
        torch.cuda.synchronize()
        hot, hits, misses = repo.last_stats()[:3]
        assert hot > 300 and hits > n // 2 and misses == 0     # the timed path ran
        g_st = status.cpu().numpy()
        blob_h, offs_h = blob.cpu().numpy(), offs.cpu().numpy().view(np.uint32)
        a_h, t_h, e_h = (x.cpu().numpy() for x in (a, t, e))
    del blob, offs, a, t, e, status
    torch.cuda.empty_cache()
    print("[c2] GPU batch done; oracle running", flush=True)
    o_st = np.zeros(n, np.uint8)
    o.L.orc_receive_soa(o.h, blob_h, offs_h, n, a_h.view(np.uint64), t_h.view(np.uint64), e_h, T0,
                        o_st, np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.int64))
    assert np.array_equal(g_st, o_st)
    assert (o_st == 1).all()
    del blob_h, offs_h, a_h, t_h, e_h, g_st, o_st
    print("[c2] statuses equal; comparing the table", flush=True)
    _check_table(repo, o)
    repo.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("first", [None, 3_000_000, 5_500_000, 9_000_001, 16_000_000])
def test_receive_dirty_positions_vs_oracle(env, first):
    """A 2^24-message batch whose first incast / -0.0 sits early, in the
    middle, near the end, or nowhere; more follow it.  The fast path merges
    the clean prefix before it, the ordered path runs from it on (incast
    replies, repo.go:78-90).  Statuses and the table equal the oracle's."""
    torch, bench, pa = env
    dev = torch.device("cuda", 0)
    K, n, L = 1_000_000, 1 << 24, 21
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        gen = torch.Generator(device=dev).manual_seed(77 + (first or 0))
        repo, o = _seeded(torch, bench, pa, dev, K, L, s)
        ids = bench.zipf_ids(torch, gen, n, K, 1.1, dev)
        blob, offs = bench.names_for_ids(torch, ids)
        del ids
        a, t, e = bench.replica_states(torch, gen, n, 0, dev)
        if first is not None:
            rng = np.random.default_rng(first)
            later = np.sort(rng.integers(first + 1, n, 30))
            neg0 = -(1 << 63)                                            # -0.0's bits
            if first % 2:
                a[first] = neg0
            else:
                a[first] = 0; t[first] = 0; e[first] = 0                  # incast
            for k, j in enumerate(later.tolist()):
                if k % 2:
                    t[j] = neg0
                else:
                    a[j] = 0; t[j] = 0; e[j] = 0
        status = torch.empty(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        repo.receive_soa(blob, a, t, e, T0, name_offs=offs, n=n, status=status, device=True)
        torch.cuda.synchronize()
        g_st = status.cpu().numpy()
        blob_h, offs_h = blob.cpu().numpy(), offs.cpu().numpy().view(np.uint32)
        a_h, t_h, e_h = (x.cpu().numpy() for x in (a, t, e))
    del blob, offs, a, t, e, status
    torch.cuda.empty_cache()
    o_st = np.zeros(n, np.uint8)
    o.L.orc_receive_soa(o.h, blob_h, offs_h, n, a_h.view(np.uint64), t_h.view(np.uint64), e_h, T0,
                        o_st, np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.int64))
    bad = np.flatnonzero(g_st != o_st)
    assert bad.size == 0, (bad[:5], g_st[bad[:5]], o_st[bad[:5]])
    if first is not None:
        assert (o_st[:first] == 1).all()
        if first % 2 == 0:   # an incast is not merged (a -0.0 replica is)
            assert (o_st[first] & 0x7F) != 1
    _check_table(repo, o)
    repo.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("clock", ["below", "ahead"])
def test_c3_full_size_vs_oracle(env, clock):
    """bench.py --workload c3 (--c3-clock below|ahead): the warmup batch, then
    the first timed batch, each through phip_apply_mixed and the oracle."""
    torch, bench, pa = env
    import argparse
    dev = torch.device("cuda", 0)
    K, n, L = 10_000_000, 50_000_000, 25
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        gen = torch.Generator(device=dev).manual_seed(1234)
        repo, o = _seeded(torch, bench, pa, dev, K, L, s)
        args = argparse.Namespace(ops=n, zipf=1.1, warmup=1, steps=1, c3_clock=clock)
        c = bench.c3_inputs(args, torch, dev, K, 0, gen)
        host = {k: c[k].cpu().numpy() for k in ("blob", "kind", "freq", "per", "cnt")}
        offs_h = c["offs"].cpu().numpy().view(np.uint32)
        status = torch.empty(n, dtype=torch.uint8, device=dev)
        rem = torch.empty(n, dtype=torch.int64, device=dev)
        have = torch.empty(n, dtype=torch.int64, device=dev)
        stats = []
        for j, (now, a, t, e) in enumerate(c["steps"]):
            torch.cuda.synchronize()
            repo.apply_mixed_device(n, c["kind"], c["blob"], c["offs"], now, c["freq"], c["per"],
                                    c["cnt"], a, t, e, status=status, remaining=rem, have=have)
            torch.cuda.synchronize()
            g = [x.cpu().numpy() for x in (status, rem, have)]
            now_h, a_h, t_h, e_h = (x.cpu().numpy() for x in (now, a, t, e))
            st = np.zeros(n, np.uint8)
            orem = np.zeros(n, np.uint64)
            ohave = np.zeros(n, np.uint64)
            r = [np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.int64),
                 np.empty(n, np.int64)]
            o.L.orc_apply_mixed(o.h, host["kind"], host["blob"], offs_h, n, now_h, host["freq"],
                                host["per"], host["cnt"].view(np.uint64), a_h.view(np.uint64),
                                t_h.view(np.uint64), e_h, st, orem, ohave, *r)
            assert np.array_equal(g[0], st), j
            take = host["kind"] == 0
            assert np.array_equal(g[1].view(np.uint64)[take], orem[take]), j
            assert np.array_equal(g[2].view(np.uint64)[take], ohave[take]), j
            stats.append((int((st == 6).sum()), int((st == 7).sum())))
            print(f"[c3 {clock}] batch {j} equal: {stats[-1][0]} Takes ok, {stats[-1][1]} denied",
                  flush=True)
            del g, now_h, a_h, t_h, e_h, st, orem, ohave, r
    # the input the step was meant to exercise: both outcomes of Take occur
    ok, denied = stats[-1]
    assert ok > 0 and denied > 0, stats
    if clock == "below":
        assert ok > n // 20, stats       # Takes refill and succeed
    _check_table(repo, o)
    repo.close()


def _ids_from_names(names, offs):
    """Bucket ids of names b"b<decimal id>" (a table dump), vectorised."""
    offs = offs.astype(np.int64)
    start, ln = offs[:-1], offs[1:] - offs[:-1]
    ids = np.zeros(start.size, np.int64)
    for d in range(1, int(ln.max())):
        m = ln > d
        ids[m] = ids[m] * 10 + (names[start[m] + d].astype(np.int64) - 48)
    return ids


@pytest.mark.timeout(900)
def test_c4_shard_full_size_rccl_exchange(env):
    """SURVEY C4's per-GPU shard at its real size: 125M buckets in 2^28 slots
    (1B buckets over 8 GPUs), one 100M-message Zipf(1.1) batch through
    phip_group_receive (RCCL group, sender-side combine) with the exchange
    itself through RCCL (PHIP_GROUP_RCCL_SELF: the segment goes out by
    ncclSend and back by ncclRecv, the multi-GPU code path).  The whole
    table is checked against an independent max-reduce of the messages by
    bucket id (torch scatter_reduce; states are clean-domain and the table
    starts at zero, so Merge is the field-wise max, bucket.go:240-263), and
    every bucket is listed exactly once."""
    torch, bench, pa = env
    dev = torch.device("cuda", 0)
    K, n, L = 125_000_000, 100_000_000, 28
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        gen = torch.Generator(device=dev).manual_seed(4321)
        repo = pa.GPURepo(device=0, log2_slots=L, arena_bytes=1 << 20)
        repo.set_stream(s)
        keys = torch.arange(K, dtype=torch.int64, device=dev)
        kb, ko = bench.names_for_ids(torch, keys)
        st = torch.zeros((K, 4), dtype=torch.int64, device=dev)
        st[:, 3] = T0
        torch.cuda.synchronize()
        repo.seed_device(kb, ko, st, K)
        del keys, kb, ko, st
        assert len(repo) == K
        ids = bench.zipf_ids(torch, gen, n, K, 1.1, dev)
        blob, offs = bench.names_for_ids(torch, ids)
        a, t, e = bench.replica_states(torch, gen, n, 0, dev)
        torch.cuda.synchronize()
        g = pa.GPUGroup.open_rank(repo, pa.GPUGroup.unique_id(), 1, 0)
        sent, merged = g.receive([(blob, offs, a, t, e)], T0 + 1, combine=True, rccl_self=True)
        torch.cuda.synchronize()
        assert sent == merged and 0 < merged[0] < n            # combined at the sender
        print(f"[c4] {n} messages -> {merged[0]} after the combine, exchanged over RCCL",
              flush=True)
        # the independent reference: per-id maxima (clean positive floats:
        # int64 order of the bits is the float order)
        want = torch.zeros((3, K), dtype=torch.int64, device=dev)
        for f, x in enumerate((a, t, e)):
            want[f].scatter_reduce_(0, ids, x, reduce="amax", include_self=True)
        want = want.cpu().numpy()
        del blob, offs, a, t, e, ids
        g.close()
    torch.cuda.empty_cache()
    names, doffs, da, dt, de, dc = repo.dump_arrays()
    repo.close()
    print("[c4] table dumped; comparing", flush=True)
    did = _ids_from_names(names, doffs)
    del names
    assert did.size == K and np.array_equal(np.sort(did), np.arange(K))
    assert np.array_equal(da.view(np.int64), want[0][did])
    assert np.array_equal(dt.view(np.int64), want[1][did])
    assert np.array_equal(de, want[2][did])
    assert (dc == T0).all()


@pytest.mark.timeout(900)
def test_c5_full_size_anti_entropy_vs_go_merge(env):
    """SURVEY C5's per-GPU shape: 8 replicas x 2^24 buckets through
    phip_group_anti_entropy (local join, RCCL all-reduce(MAX), apply), with
    NaN, negative and zero fields mixed in.  Every replica of every bucket
    is then identical to the one before it, and on a sample of 100k buckets
    every replica equals Go's Bucket.Merge (bucket.go:240-263) of all the
    other replicas into its pre-round state, one by one (no -0.0 fields:
    DESIGN §3.2, the one tie the all-reduce cannot order)."""
    torch, bench, pa = env
    from oracle import go_semantics as G
    from patrol_amd import shard
    dev = torch.device("cuda", 0)
    R, B = 8, 1 << 24
    gen = torch.Generator(device=dev).manual_seed(77)
    taken = torch.randint(0, 10**6, (R, B), device=dev, generator=gen).to(torch.float64)
    added = taken + torch.rand((R, B), dtype=torch.float64, device=dev, generator=gen) * 100.0
    ab, tb = added.view(torch.int64).clone(), taken.view(torch.int64).clone()
    del taken, added
    el = torch.randint(0, 1 << 40, (R, B), device=dev, generator=gen, dtype=torch.int64)
    special = torch.tensor([0, 0x7FF8000000000000, -0x0008000000000000, -0x4010000000000000,
                            0x7FF0000000000000], dtype=torch.int64, device=dev)   # 0, NaN, -NaN, -1.0, +Inf
    for x in (ab, tb):
        m = torch.rand((R, B), device=dev, generator=gen) < 0.01
        x[m] = special[torch.randint(0, special.numel(), (int(m.sum()),), device=dev, generator=gen)]
    m = torch.rand((R, B), device=dev, generator=gen) < 0.01
    el[m] = -el[m]
    reps = torch.empty((R, 3, B), dtype=torch.int64, device=dev)
    reps[:, 0] = shard.e_encode(ab)
    reps[:, 1] = shard.e_encode(tb)
    reps[:, 2] = el
    sample = torch.randint(0, B, (100_000,), device=dev, generator=gen)
    before = [x[:, sample].cpu().numpy() for x in (ab, tb, el)]
    del ab, tb, el
    repo = pa.GPURepo(device=0, log2_slots=10)
    g = pa.GPUGroup.open_rank(repo, pa.GPUGroup.unique_id(), 1, 0)
    torch.cuda.synchronize()
    g.anti_entropy([reps])
    torch.cuda.synchronize()
    # converged in one round, except where a replica's own NaN sticks (Go's
    # `<` never replaces a NaN and never adopts one, bucket.go:250-256)
    S = -(1 << 63)
    nan = (reps[:, :2] ^ S) >= (0xFFE0000000000002 - (1 << 64) ^ S)
    same = reps == reps[0:1]
    assert bool(same[:, 2].all())
    assert bool((same[:, :2] | nan.any(0, keepdim=True)).all())
    assert bool(nan.any())
    after = reps[:, :, sample].cpu().numpy()
    g.close()
    repo.close()
    del reps
    for j in range(0, 100_000, 97):                            # ~1000 buckets x 8 replicas
        for r in range(R):
            b = G.Bucket(added=G.b2f(int(before[0][r, j]) & (2**64 - 1)),
                         taken=G.b2f(int(before[1][r, j]) & (2**64 - 1)),
                         elapsed=int(before[2][r, j]))
            for q in range(R):
                if q != r:
                    b.merge(G.Bucket(added=G.b2f(int(before[0][q, j]) & (2**64 - 1)),
                                     taken=G.b2f(int(before[1][q, j]) & (2**64 - 1)),
                                     elapsed=int(before[2][q, j])))
            want = (G.f2b(b.added), G.f2b(b.taken), b.elapsed)
            got = (_e_dec(int(after[r, 0, j])), _e_dec(int(after[r, 1, j])), int(after[r, 2, j]))
            assert got == want, (j, r, [hex(x) for x in got[:2]], [hex(x) for x in want[:2]])


def _e_dec(code: int) -> int:
    """phip_device.hpp dec_f64 of an int64-held E code -> float64 bits."""
    S, INF = 1 << 63, 0x7FF0000000000000
    NAN_BASE, PER = 0xFFE0000000000002, (1 << 52) - 1
    e = code & (2**64 - 1)
    if e < INF:
        return S | (INF - e)
    if e == INF:
        return 0
    if e == INF + 1:
        return S
    if e < NAN_BASE:
        return e - INF - 1
    idx = e - NAN_BASE
    return INF + 1 + idx if idx < PER else S | (INF + 1 + idx - PER)
