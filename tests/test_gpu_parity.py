"""Parity of the HIP engine (through the C ABI) with the oracle, on cuda:0.

Bar: bit-exact.  Every float64 is compared as its bit pattern, every status,
every `remaining`, every reply and the final state of every bucket.  The
oracle is oracle/liboracle.so (pinned by tests/test_oracle.py) or the golden
fixtures themselves.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import _gen  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SEC, MS = 10**9, 10**6


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def hb(s):
    return int(s, 16)


@pytest.fixture(scope="module")
def pa():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import patrol_amd
    return patrol_amd


def gpu_dump(repo):
    d = {k: (v.added, v.taken, v.elapsed, v.created) for k, v in repo.dump().items()}
    # one record per name: the bucket count equals the distinct names dumped
    assert len(repo) == len(d), (len(repo), len(d))
    return d


def assert_same_dump(g, o):
    assert len(g) == len(o)   # distinct names (the dump is keyed by name)
    bad = [k for k in o if g.get(k) != o[k]]
    assert not bad, [(k, g.get(k), o[k]) for k in bad[:5]]


# ------------------------------------------------------------- golden ----
def test_receive_golden_batches(pa):
    for b in load("receive_batches.json")["batches"]:
        repo = pa.GPURepo(log2_slots=10)
        if b["seed"]:
            repo.seed([s["name"].encode() for s in b["seed"]], [hb(s["added"]) for s in b["seed"]],
                      [hb(s["taken"]) for s in b["seed"]], [s["elapsed"] for s in b["seed"]],
                      [s["created"] for s in b["seed"]])
        out = repo.receive_datagrams([bytes.fromhex(d) for d in b["datagrams"]], b["now"])
        assert list(out["status"]) == b["status"]
        for i, r in enumerate(b["replies"]):
            if r:
                rp = out["reply"][i]
                assert [int(rp["a"]), int(rp["t"]), int(rp["e"])] == [hb(r[0]), hb(r[1]), r[2]]
        want = {k.encode(): (hb(v[0]), hb(v[1]), v[2], v[3]) for k, v in b["final"].items()}
        assert_same_dump(gpu_dump(repo), want)
        repo.close()


def _mixed_arrays(ops):
    kind = np.array([o["kind"] for o in ops], np.uint8)
    names = [o["name"].encode() for o in ops]
    now = np.array([o["now"] for o in ops], np.int64)
    freq = np.array([o.get("freq", 0) for o in ops], np.int64)
    per = np.array([o.get("per", 0) for o in ops], np.int64)
    cnt = np.array([o.get("count", 0) for o in ops], np.uint64)
    a = np.array([hb(o.get("added", "0")) for o in ops], np.uint64)
    t = np.array([hb(o.get("taken", "0")) for o in ops], np.uint64)
    e = np.array([o.get("elapsed", 0) for o in ops], np.int64)
    return kind, names, now, freq, per, cnt, a, t, e


def test_mixed_golden_traces(pa):
    for tr in load("mixed_traces.json")["traces"]:
        repo = pa.GPURepo(log2_slots=10)
        out = repo.apply_mixed(*_mixed_arrays(tr["ops"]))
        for i, r in enumerate(tr["results"]):
            assert out["status"][i] == r["status"], (i, tr["ops"][i], out["status"][i], r)
            if "remaining" in r:
                assert int(out["remaining"][i]) == r["remaining"]
                assert int(out["have"][i]) == hb(r["have"])
            if "reply" in r:
                rp = out["reply"][i]
                assert [int(rp["a"]), int(rp["t"]), int(rp["e"])] == [hb(r["reply"][0]), hb(r["reply"][1]), r["reply"][2]]
        want = {k.encode(): (hb(v[0]), hb(v[1]), v[2], v[3]) for k, v in tr["final"].items()}
        assert_same_dump(gpu_dump(repo), want)
        repo.close()


def test_api_golden(pa):
    g = load("api_table.json")
    repo = pa.GPURepo(log2_slots=10)
    sb = g["seed_bucket"]
    repo.seed([sb["name"].encode()], [0], [0], [0], [sb["created"]])
    for r in g["requests"]:
        assert repo.api_take(r["name"].encode(), r["rate"].encode(), r["count"].encode(), r["now"]) == \
               (r["code"], r["body"]), r


def test_take_known_answer_reference_table(pa):
    """bucket_test.go:35-66 through phip_take (bucket pre-created at t0)."""
    g = load("take_known_answer.json")
    repo = pa.GPURepo(log2_slots=10)
    repo.seed([b"kat"], [0], [0], [0], [g["created"]])
    for s in g["steps"]:
        rem, ok = repo.take([b"kat"], [s["now"]], [g["freq"]], [g["per"]], [s["take"]])
        assert (bool(ok[0]), int(rem[0])) == (s["ok"], s["rem"])
        st = repo.get(b"kat")
        assert (st.added, st.taken, st.elapsed) == (hb(s["added"]), hb(s["taken"]), s["b_elapsed"])


# ------------------------------------------------------------- random ----
def _seed_both(pa, rng, K, log2_slots=16, **kw):
    ids = np.arange(K)
    names = _gen.key_names(ids)
    a, t, e = _gen.clean_states(rng, K)
    created = _gen.T0 - rng.integers(0, SEC, K)
    g = pa.GPURepo(log2_slots=log2_slots, **kw)
    g.seed(names, a, t, e, created)
    o = O.Repo()
    o.seed(names, a, t, e, created)
    return g, o


@pytest.mark.parametrize("seed", [1, 2])
def test_receive_soa_fast_path_vs_oracle(pa, seed):
    rng = np.random.default_rng(seed)
    K = 20000
    g, o = _seed_both(pa, rng, K)
    n = 200000
    ids = _gen.zipf_ids(rng, n, K + 2000)         # ~10% of keys are new: insert path
    names = _gen.key_names(ids)
    a, t, e = _gen.clean_states(rng, n)
    now = _gen.T0 + 5 * SEC
    out = g.receive_soa(names, a, t, e, now)
    st, _, _, _ = o.receive_soa(names, a, t, e, now)
    assert np.array_equal(out["status"], st)
    assert_same_dump(gpu_dump(g), o.dump())


def _fast_dirty_states(rng, n):
    """dirty_states without what routes a batch to the ordered path (-0.0
    fields, all-zero incast states): NaN, +-Inf, negatives stay."""
    a, t, e = _gen.dirty_states(rng, n)
    for arr in (a, t):
        arr[arr == np.uint64(0x8000000000000000)] = 0
    z = (a == 0) & (t == 0) & (e == 0)
    e[z] = 1
    return a, t, e


@pytest.mark.parametrize("kind", ["clean", "fastdirty"])
def test_receive_soa_hot_directory_vs_oracle(pa, kind):
    """Batches of >= 2^16 messages build the hot-bucket directory (the most
    sampled buckets fold in LDS, flushed once per workgroup).  Zipf(1.1) with
    new keys, 15-22 byte and arena-length names mixed in."""
    rng = np.random.default_rng(11 if kind == "clean" else 12)
    K = 30000
    g, o = _seed_both(pa, rng, K, log2_slots=17)
    n = 1 << 21
    ids = _gen.zipf_ids(rng, n, K + 3000)
    names = []
    for i in ids:
        i = int(i)
        if i % 101 == 0:
            names.append(b"a-much-longer-bucket-name-%d" % i)   # > 22 bytes: arena
        elif i % 103 == 0:
            names.append(b"medium-name-%d" % i)                 # 15-22 bytes
        else:
            names.append(b"b%d" % i)
    a, t, e = _gen.clean_states(rng, n) if kind == "clean" else _fast_dirty_states(rng, n)
    now = _gen.T0 + 5 * SEC
    out = g.receive_soa(names, a, t, e, now)
    st, _, _, _ = o.receive_soa(names, a, t, e, now)
    assert np.array_equal(out["status"], st)
    assert_same_dump(gpu_dump(g), o.dump())
    # A second batch over the same keys (no inserts): only the fast kernel.
    a2, t2, e2 = _gen.clean_states(rng, n)
    out = g.receive_soa(names, a2, t2, e2, now + SEC)
    st, _, _, _ = o.receive_soa(names, a2, t2, e2, now + SEC)
    assert np.array_equal(out["status"], st)
    assert_same_dump(gpu_dump(g), o.dump())


@pytest.mark.parametrize("seed", [3, 4])
def test_receive_soa_dirty_vs_oracle(pa, seed):
    """Incasts, -0.0, NaN, negatives: the ordered path, replies included."""
    rng = np.random.default_rng(seed)
    K = 3000
    g, o = _seed_both(pa, rng, K, log2_slots=14)
    n = 40000
    ids = _gen.zipf_ids(rng, n, K + 500)
    names = _gen.key_names(ids)
    a, t, e = _gen.dirty_states(rng, n)
    now = _gen.T0 + 7 * SEC
    out = g.receive_soa(names, a, t, e, now)
    st, ra, rt, re = o.receive_soa(names, a, t, e, now)
    assert np.array_equal(out["status"], st)
    rep = (st & 0x7F) == 2
    assert np.array_equal(out["reply"]["a"][rep], ra[rep])
    assert np.array_equal(out["reply"]["t"][rep], rt[rep])
    assert np.array_equal(out["reply"]["e"][rep], re[rep])
    assert_same_dump(gpu_dump(g), o.dump())


def test_upsert_vs_oracle(pa):
    rng = np.random.default_rng(5)
    K = 2000
    g, o = _seed_both(pa, rng, K, log2_slots=13)
    n = 30000
    ids = _gen.zipf_ids(rng, n, K + 400)
    names = _gen.key_names(ids)
    a, t, e = _gen.dirty_states(rng, n)
    now = _gen.T0 + 9 * SEC
    out = g.upsert_soa(names, a, t, e, now)
    merged = o.upsert_soa(names, a, t, e, now)
    assert np.array_equal((out["status"] & 0x7F) == 1, merged.astype(bool))
    assert_same_dump(gpu_dump(g), o.dump())


def _mixed_stream(rng, n, K, hot_frac=0.0):
    ids = _gen.zipf_ids(rng, n, K)
    if hot_frac:
        ids[rng.random(n) < hot_frac] = 7
    names = _gen.key_names(ids)
    kind = (rng.random(n) < 0.5).astype(np.uint8)          # 0 take, 1 receive
    now = _gen.T0 + np.arange(n, dtype=np.int64) * 20
    freq = np.full(n, 100, np.int64)
    per = np.full(n, SEC, np.int64)
    odd = rng.random(n) < 0.05
    freq[odd] = rng.choice([0, 3, 7, -5, 1 << 40], int(odd.sum()))
    per[odd] = rng.choice([SEC, 1, 0, 60 * SEC], int(odd.sum()))
    cnt = np.ones(n, np.uint64)
    cnt[rng.random(n) < 0.05] = 3
    a, t, e = _gen.clean_states(rng, n)
    a = (a.view(np.float64) / 1e4).view(np.uint64).copy()   # keep tokens in play
    t = (t.view(np.float64) / 1e4).view(np.uint64).copy()
    e = e >> 12
    return kind, names, now, freq, per, cnt, a, t, e


@pytest.mark.parametrize("hot", [0.0, 0.3])
def test_mixed_stream_vs_oracle(pa, hot):
    """Take + Merge interleaved, per-bucket order; hot=0.3 puts ~30% of the
    ops on one bucket (long segment -> k_fold_wave)."""
    rng = np.random.default_rng(11 + int(hot * 10))
    n, K = 60000, 5000
    args = _mixed_stream(rng, n, K, hot)
    g = pa.GPURepo(log2_slots=14)
    o = O.Repo()
    out = g.apply_mixed(*args)
    ref = o.apply_mixed(*args)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["remaining"], ref["remaining"])
    take = args[0] == 0
    assert np.array_equal(out["have"][take], ref["have"][take])
    assert assert_replies(out, ref, args[0]) == int(take.sum()) + \
        int((((ref["status"] & 0x7F) == 2) | ((ref["status"] & 0x7F) == 3)).sum())
    assert_same_dump(gpu_dump(g), o.dump())


def test_mixed_stream_hot_buckets_block_fold(pa):
    """Several buckets with 10^4..10^5 ops each (k_fold_block windows), rate
    changes and merges interleaved: exact vs the oracle."""
    rng = np.random.default_rng(77)
    n, K = 300000, 50
    args = list(_mixed_stream(rng, n, K, 0.4))
    g = pa.GPURepo(log2_slots=10)
    o = O.Repo()
    out = g.apply_mixed(*args)
    ref = o.apply_mixed(*args)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["remaining"], ref["remaining"])
    take = args[0] == 0
    assert np.array_equal(out["have"][take], ref["have"][take])
    assert assert_replies(out, ref, args[0]) > 0      # k_huge_outputs writes them too
    assert_same_dump(gpu_dump(g), o.dump())


def reply_mask(kind, status):
    """Ops whose phip_results.reply is written (include/patrolhip.h): Takes
    and Upserts (the state after them, what UpsertBucket broadcasts) and
    incasts (the local state, repo.go:86-90)."""
    st = np.asarray(status) & 0x7F
    kind = np.asarray(kind)
    return (kind == 0) | (kind == 2) | (st == 2) | (st == 3)


def assert_replies(out, ref, kind, tag=None):
    """Every reply state, `created` included, equals the oracle's."""
    rep = reply_mask(kind, ref["status"])
    r = out["reply"][rep]
    for f, k in (("a", "reply_added"), ("t", "reply_taken"), ("e", "reply_elapsed"),
                 ("c", "reply_created")):
        bad = np.nonzero(r[f] != ref[k][rep])[0]
        assert bad.size == 0, (tag, f, int(np.nonzero(rep)[0][bad[0]]))
    return int(rep.sum())


def _check_mixed(pa, args, log2_slots, reply=False):
    g = pa.GPURepo(log2_slots=log2_slots)
    o = O.Repo()
    out = g.apply_mixed(*args)
    ref = o.apply_mixed(*args)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["remaining"], ref["remaining"])
    take = args[0] == 0
    assert np.array_equal(out["have"][take], ref["have"][take])
    if reply:
        assert ((ref["status"] & 0x7F) == 2).any()
        assert assert_replies(out, ref, args[0]) > 0
    assert_same_dump(gpu_dump(g), o.dump())


def test_mixed_hot_adversarial_all_fold_kinds(pa):
    """Thread, wave and workgroup folds on one stream with every op kind:
    Take (odd rates), Receive of dirty states (incast replies, -0.0, NaN,
    negatives) and Upsert, with 3 buckets hot enough for k_fold_block
    (about 75k, 50k and 35k ops: over the 32768-op huge threshold)."""
    rng = np.random.default_rng(5150)
    n, K = 500000, 3000
    args = list(_mixed_stream(rng, n, K))
    ids = _gen.zipf_ids(rng, n, K)
    hot = rng.random(n)
    ids[hot < 0.15] = 11
    ids[(hot >= 0.15) & (hot < 0.25)] = 12
    ids[(hot >= 0.25) & (hot < 0.32)] = 13
    args[1] = _gen.key_names(ids)
    args[0] = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.5, 0.4, 0.1])
    a, t, e = _gen.dirty_states(rng, n, 0.1)
    args[6], args[7], args[8] = a, t, e
    _check_mixed(pa, args, 13, reply=True)


def test_small_batches_one_launch_vs_large_path_and_oracle(pa):
    """Ordered batches of <= 1024 host ops run as one launch (k_small_mixed).
    A stream of small batches exercises every op kind: odd rates, dirty
    states with incast replies, upserts, new short and long names repeated
    inside a batch, and a bucket with more than 32 ops in one batch (the
    wave fold). Each batch must give the same statuses, remaining, have and
    replies, and the same table, on the small path, on the large path
    (PHIP_CFG_NO_SMALL) and in the oracle."""
    rng = np.random.default_rng(9090)
    small = pa.GPURepo(log2_slots=12, arena_bytes=1 << 16)
    large = pa.GPURepo(log2_slots=12, arena_bytes=1 << 16, small=False)
    o = O.Repo()
    longs = [b"a-long-bucket-name-for-the-arena-%03d" % k for k in range(40)]
    t0 = _gen.T0
    for step, n in enumerate([1, 2, 33, 500, 1024, 1025, 700, 64, 1024]):
        args = list(_mixed_stream(rng, n, 300))
        names = list(args[1])
        for k in np.nonzero(rng.random(n) < 0.1)[0]:
            names[k] = longs[int(rng.integers(0, len(longs)))]
        hot = rng.random(n) < 0.2
        for k in np.nonzero(hot)[0]:
            names[k] = b"hot-bucket"
        args[1] = names
        args[0] = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.5, 0.4, 0.1])
        a, t, e = _gen.dirty_states(rng, n, 0.1)
        args[6], args[7], args[8] = a, t, e
        args[2] = t0 + step * SEC + np.arange(n, dtype=np.int64) * 1000
        outs = [r.apply_mixed(*args) for r in (small, large)]
        ref = o.apply_mixed(*args)
        take = args[0] == 0
        for out in outs:
            assert np.array_equal(out["status"], ref["status"]), step
            assert np.array_equal(out["remaining"], ref["remaining"]), step
            assert np.array_equal(out["have"][take], ref["have"][take]), step
            assert_replies(out, ref, args[0], step)
    want = o.dump()
    assert_same_dump(gpu_dump(small), want)
    assert_same_dump(gpu_dump(large), want)
    assert len(small) == len(large) == len(want)


def test_small_receive_upsert_datagrams_one_launch_vs_large_path(pa):
    """Host Receive / Upsert / datagram batches of <= 1024 messages run as one
    launch too (small_uniform, small_datagrams): statuses, incast replies,
    the short-datagram stop and the table equal the large paths' and the
    oracle's."""
    import struct
    rng = np.random.default_rng(4242)
    small = pa.GPURepo(log2_slots=12, arena_bytes=1 << 16)
    large = pa.GPURepo(log2_slots=12, arena_bytes=1 << 16, small=False)
    o = O.Repo()
    longs = [b"receive-path-long-name-for-the-arena-%02d" % k for k in range(20)]
    for step, n in enumerate([1, 40, 777, 1024, 1025, 300]):
        ids = _gen.zipf_ids(rng, n, 500)
        names = [longs[i % 20] if i % 7 == 0 else b"r%d" % i for i in ids]
        a, t, e = _gen.dirty_states(rng, n, 0.15)
        now = _gen.T0 + step * SEC
        mode = step % 3
        if mode == 0:
            outs = [r.receive_soa(names, a, t, e, now) for r in (small, large)]
            st, ra, rt, re_ = o.receive_soa(names, a, t, e, now)
            rep = (st & 0x7F) == 2
            for out in outs:
                assert np.array_equal(out["status"], st), step
                r = out["reply"][rep]
                assert np.array_equal(r["a"], ra[rep]) and np.array_equal(r["t"], rt[rep]), step
                assert np.array_equal(r["e"], re_[rep]), step
        elif mode == 1:
            outs = [r.upsert_soa(names, a, t, e, now) for r in (small, large)]
            merged = o.upsert_soa(names, a, t, e, now)
            assert np.array_equal(outs[0]["status"], outs[1]["status"]), step
            assert np.array_equal((outs[0]["status"] & 0x7F) == 1, merged.astype(bool)), step
        else:
            dgs = [struct.pack(">QQQ", int(a[i]), int(t[i]), int(e[i]) & (2**64 - 1))
                   + bytes([len(names[i])]) + names[i] for i in range(n)]
            cut = n // 2
            dgs[cut] = dgs[cut][:20]                      # io.ErrShortBuffer there
            outs = [r.receive_datagrams(dgs, now) for r in (small, large)]
            st, _, _, _ = o.receive_soa(names[:cut], a[:cut], t[:cut], e[:cut], now)
            for out in outs:
                assert out["stop"] == cut, step
                assert np.array_equal(out["status"][:cut], st), step
                assert out["status"][cut] == 4 and (out["status"][cut + 1:] == 5).all(), step
    want = o.dump()
    assert_same_dump(gpu_dump(small), want)
    assert_same_dump(gpu_dump(large), want)


def test_mixed_c3_shape_clamped_clock(pa):
    """The bench's C3 shape: replica elapsed far ahead of the local clock, so
    Take's `last` is clamped to now (bucket.go:199-201) and tokens come only
    from merged added/taken; one bucket carries ~12% of 250k ops."""
    rng = np.random.default_rng(31337)
    n, K = 250000, 20000
    ids = _gen.zipf_ids(rng, n, K)
    names = _gen.key_names(ids)
    kind = (rng.random(n) < 0.5).astype(np.uint8)
    now = _gen.T0 + np.arange(n, dtype=np.int64) * 20
    freq = np.full(n, 100, np.int64)
    per = np.full(n, SEC, np.int64)
    cnt = np.ones(n, np.uint64)
    a, t, e = _gen.clean_states(rng, n)
    _check_mixed(pa, [kind, names, now, freq, per, cnt, a, t, e], 16)


def test_take_clock_extremes(pa):
    """Take's clock arithmetic at the int64 edges (bucket.go:198-207):
    created + elapsed overflowing either way, now.Sub saturating, negative
    clocks, with every fold kind (1, 40 and 20000 ops per bucket)."""
    rng = np.random.default_rng(2718)
    I64 = np.iinfo(np.int64)
    edge = np.array([I64.min, I64.min + 1, -(1 << 62), -SEC, -1, 0, 1, SEC, 1 << 62,
                     I64.max - 1, I64.max], np.int64)
    K = 60
    names = [b"edge%d" % k for k in range(K)]
    created = edge[rng.integers(0, len(edge), K)]
    elapsed = edge[rng.integers(0, len(edge), K)]
    added = (rng.random(K) * 50).view(np.uint64)
    taken = (rng.random(K) * 10).view(np.uint64)
    reps = np.concatenate([np.full(20, 1), np.full(30, 40), np.full(10, 20000)])
    ids = np.repeat(np.arange(K), reps)
    rng.shuffle(ids)
    n = len(ids)
    nm = [names[i] for i in ids]
    kind = (rng.random(n) < 0.8).astype(np.uint8) ^ 1        # mostly Take
    now = edge[rng.integers(0, len(edge), n)].copy()
    mid = rng.random(n) < 0.5
    now[mid] = rng.integers(-(1 << 62), 1 << 62, int(mid.sum()))
    freq = rng.choice(np.array([1, 3, 100, 1 << 40, -7], np.int64), n)
    per = rng.choice(np.array([SEC, 1, 3 * SEC, I64.max, I64.min], np.int64), n)
    cnt = rng.choice(np.array([0, 1, 2, 5], np.uint64), n)
    a = (rng.random(n) * 60).view(np.uint64)
    t = (rng.random(n) * 20).view(np.uint64)
    e = edge[rng.integers(0, len(edge), n)]
    g = pa.GPURepo(log2_slots=10)
    o = O.Repo()
    g.seed(names, added, taken, elapsed, created)
    o.seed(names, added, taken, elapsed, created)
    out = g.apply_mixed(kind, nm, now, freq, per, cnt, a, t, e)
    ref = o.apply_mixed(kind, nm, now, freq, per, cnt, a, t, e)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["remaining"], ref["remaining"])
    tk = kind == 0
    assert np.array_equal(out["have"][tk], ref["have"][tk])
    assert_same_dump(gpu_dump(g), o.dump())


@pytest.mark.parametrize("freq,per", [(100, SEC), (-5, SEC), (7, 0), (3, -SEC)])
def test_hot_bucket_quiet_window_skips(pa, freq, per):
    """k_fold_block skips windows its summary proves quiet: one uniform rate
    per run (positive, negative and zero intervals), jittered clocks (now not
    monotone), merges carrying -0.0, NaN and negatives, an incast now and
    then; 3 buckets of ~40k ops each (about 20 windows of 2048)."""
    rng = np.random.default_rng(abs(freq) * 7 + 3)
    n = 120000
    ids = rng.integers(0, 3, n)
    names = [b"hot%d" % i for i in ids]
    kind = (rng.random(n) < 0.3).astype(np.uint8)          # 70% Take
    now = _gen.T0 + np.arange(n, dtype=np.int64) * 50_000 + rng.integers(-2 * MS, 2 * MS, n)
    fr = np.full(n, freq, np.int64)
    pe = np.full(n, per, np.int64)
    cnt = np.ones(n, np.uint64)
    a, t, e = _gen.dirty_states(rng, n, 0.02)
    a = (np.abs(a.view(np.float64)) / 1e5).view(np.uint64).copy()
    t = (np.abs(t.view(np.float64)) / 1e5).view(np.uint64).copy()
    e = e >> 20
    _check_mixed(pa, [kind, names, now, fr, pe, cnt, a, t, e], 10, reply=True)


@pytest.mark.parametrize("variant", ["below", "over_capacity", "negzero", "rates", "seeded"])
def test_hot_bucket_absorbing_merges(pa, variant):
    """k_fold_block absorbs merges into the running replica maximum when a
    window's Takes are provably denied (window_absorbable): the C3 shape with
    replica `elapsed` below the local clock, so merges raise the hot buckets
    all the time while Takes refill now and then.  Variants that break the
    max(R, G) identity must switch the segment to exact runs: replicas whose
    tokens exceed capacity (negative refill lowers `added`), -0.0 replica
    fields, and windows of mixed rates; 'seeded' starts from existing
    buckets.  Three buckets of ~45k ops each plus a cold tail."""
    rng = np.random.default_rng({"below": 1, "over_capacity": 2, "negzero": 3, "rates": 4,
                                 "seeded": 5}[variant])
    n = 150000
    ids = np.where(rng.random(n) < 0.9, rng.integers(0, 3, n), rng.integers(3, 3000, n))
    names = [b"hot%d" % i if i < 3 else b"b%d" % i for i in ids]
    kind = (rng.random(n) < 0.5).astype(np.uint8)
    now = _gen.T0 + np.arange(n, dtype=np.int64) * 20_000
    fr = np.full(n, 100, np.int64)
    pe = np.full(n, SEC, np.int64)
    cnt = np.ones(n, np.uint64)
    taken = rng.integers(0, 10**4, n).astype(np.float64)
    added = taken + rng.random(n) * 100
    if variant == "over_capacity":
        sel = rng.random(n) < 0.001
        added[sel] = taken[sel] + 150.0
    a, t = added.view(np.uint64).copy(), taken.view(np.uint64).copy()
    e = (rng.random(n) * (now - _gen.T0)).astype(np.int64)
    if variant == "negzero":
        sel = (rng.random(n) < 0.0005) & (kind == 1)
        t[sel] = np.uint64(0x8000000000000000)
    if variant == "rates":
        sel = rng.random(n) < 0.002
        fr[sel] = 7
        cnt[rng.random(n) < 0.002] = 2
    args = [kind, names, now, fr, pe, cnt, a, t, e]
    if variant != "seeded":
        _check_mixed(pa, args, 12, reply=False)
        return
    g = pa.GPURepo(log2_slots=12)
    o = O.Repo()
    seed = [b"hot0", b"hot1", b"hot2"]
    sa = np.array([50.0, 0.0, 1e4 + 99.5]).view(np.uint64)
    st = np.array([10.0, 0.0, 1e4]).view(np.uint64)
    for r in (g, o):
        r.seed(seed, sa, st, [0, 0, 0], [_gen.T0 - SEC] * 3)
    out = g.apply_mixed(*args)
    ref = o.apply_mixed(*args)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["remaining"], ref["remaining"])
    take = kind == 0
    assert np.array_equal(out["have"][take], ref["have"][take])
    assert_same_dump(gpu_dump(g), o.dump())


def test_tag_collisions_names_always_compared(pa):
    """With the probe tag cut to 3 bits nearly every lookup meets other names
    with an equal tag: results must still be exact."""
    rng = np.random.default_rng(21)
    n, K = 20000, 600
    g = pa.GPURepo(log2_slots=12, debug_tag_bits=3)
    o = O.Repo()
    ids = _gen.zipf_ids(rng, n, K)
    names = _gen.key_names(ids)
    a, t, e = _gen.clean_states(rng, n)
    now = _gen.T0
    out = g.receive_soa(names, a, t, e, now)
    st, _, _, _ = o.receive_soa(names, a, t, e, now)
    assert np.array_equal(out["status"], st)
    args = _mixed_stream(rng, n, K)
    out = g.apply_mixed(*args)
    ref = o.apply_mixed(*args)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["remaining"], ref["remaining"])
    assert_same_dump(gpu_dump(g), o.dump())


def test_long_names_and_edges(pa):
    """Names of 0..231 bytes (arena path above 23), arbitrary bytes."""
    rng = np.random.default_rng(31)
    base = [b"", b"a", b"x" * 23, b"y" * 24, b"z" * 231, bytes(range(1, 40)), b"\x00" * 30,
            b"\x00" * 31, b"same-prefix-16-bytes-AAAAAAAA", b"same-prefix-16-bytes-AAAAAAAB"]
    base += [bytes(rng.integers(0, 256, int(rng.integers(0, 232)), dtype=np.uint8)) for _ in range(300)]
    n = 5000
    names = [base[i] for i in rng.integers(0, len(base), n)]
    a, t, e = _gen.clean_states(rng, n)
    g = pa.GPURepo(log2_slots=12, arena_bytes=1 << 20)
    o = O.Repo()
    out = g.receive_soa(names, a, t, e, _gen.T0)
    st, _, _, _ = o.receive_soa(names, a, t, e, _gen.T0)
    assert np.array_equal(out["status"], st)
    assert_same_dump(gpu_dump(g), o.dump())
    for nm in base[:10]:
        got, want = g.get(nm), o.get(nm)
        assert (got is None) == (want is None)
        if got:
            assert (got.added, got.taken, got.elapsed, got.created) == want


@pytest.mark.parametrize("form", ["soa", "wire"])
def test_hot_long_names(pa, form):
    """Skewed batches (hot directory on) of 15..60-byte names that share their
    first 16 bytes and differ only in the tail: the directory's match of an
    arena name (LDS tail words up to 40 bytes, the arena beyond) is exact."""
    import struct
    rng = np.random.default_rng(43)
    K, n = 3000, 1 << 18
    lens = rng.integers(15, 61, K)
    names_k = [(b"shared-prefix-AB" + (b"%d" % k).rjust(max(int(L) - 16, 0), b"-"))[-int(L):]
               if L < 16 else (b"%d" % k).rjust(int(L), b"~") for k, L in enumerate(lens)]
    assert len(set(names_k)) == K
    g = pa.GPURepo(log2_slots=14, arena_bytes=1 << 20)
    o = O.Repo()
    for step in range(2):
        ids = _gen.zipf_ids(rng, n, K)
        names = [names_k[i] for i in ids]
        a, t, e = _gen.clean_states(rng, n)
        now = _gen.T0 + step
        if form == "soa":
            out = g.receive_soa(names, a, t, e, now)
        else:
            dgs = [struct.pack(">QQQ", int(a[i]), int(t[i]), int(e[i]) & (2**64 - 1))
                   + bytes([len(names[i])]) + names[i] for i in range(n)]
            out = g.receive_datagrams(dgs, now)
        st, _, _, _ = o.receive_soa(names, a, t, e, now)
        assert np.array_equal(out["status"], st)
        if step == 1:
            hot, folded = g.last_stats()[:2]
            assert hot > 0 and folded > n // 4   # the directory carried the hot names
    assert_same_dump(gpu_dump(g), o.dump())


def test_datagram_path_matches_soa_path(pa):
    """Raw wire datagrams (device decode) == pre-decoded states."""
    import struct
    rng = np.random.default_rng(41)
    n, K = 50000, 3000
    ids = _gen.zipf_ids(rng, n, K)
    names = _gen.key_names(ids)
    a, t, e = _gen.dirty_states(rng, n, 0.05)
    dgs = [struct.pack(">QQQ", int(a[i]), int(t[i]), int(e[i]) & (2**64 - 1)) + bytes([len(names[i])]) + names[i]
           for i in range(n)]
    g = pa.GPURepo(log2_slots=13)
    o = O.Repo()
    out = g.receive_datagrams(dgs, _gen.T0)
    st, ra, rt, re, stop = o.receive(dgs, _gen.T0)
    assert out["stop"] == stop == n
    assert np.array_equal(out["status"], st)
    assert_same_dump(gpu_dump(g), o.dump())


@pytest.mark.parametrize("path", ["receive", "mixed", "seed"])
def test_table_full_refused_without_growth(pa, path):
    """PHIP_CFG_NO_GROW: a batch whose new buckets would pass the load limit
    is refused before any of them is claimed (PHIP_ERR_FULL).  The table then
    holds what it held plus the merges into existing buckets (merges commute),
    no slot is left claimed or flagged as new, and later batches that fit
    still work bit-exactly."""
    rng = np.random.default_rng(0)
    g = pa.GPURepo(log2_slots=8, max_load_pct=50, grow=False)     # 128 buckets allowed
    o = O.Repo()
    names1 = _gen.key_names(range(100))
    a, t, e = _gen.clean_states(rng, 100)
    g.receive_soa(names1, a, t, e, _gen.T0)
    o.receive_soa(names1, a, t, e, _gen.T0)
    new = _gen.key_names(range(1000, 1100))
    old = [names1[i] for i in rng.integers(0, 100, 60)]
    names2 = old + new
    rng.shuffle(names2)
    a2, t2, e2 = _gen.clean_states(rng, len(names2))
    with pytest.raises(pa.PatrolHipError) as ei:
        if path == "receive":
            g.receive_soa(names2, a2, t2, e2, _gen.T0 + SEC)
        elif path == "mixed":
            k = np.ones(len(names2), np.uint8)
            z = np.zeros(len(names2), np.int64)
            g.apply_mixed(k, names2, z + _gen.T0 + SEC, z, z, z.astype(np.uint64), a2, t2, e2)
        else:
            g.seed(names2, a2, t2, e2, np.full(len(names2), _gen.T0 + SEC, np.int64))
    assert ei.value.code == -3
    assert len(g) == 100
    if path == "receive":   # the fast path merged the clean prefix's existing buckets
        keep = [i for i, nm in enumerate(names2) if nm in set(names1)]
        o.receive_soa([names2[i] for i in keep], a2[keep], t2[keep], e2[keep], _gen.T0 + SEC)
    assert_same_dump(gpu_dump(g), o.dump())
    # the table still works: a batch that fits creates and merges exactly
    names3 = old[:10] + new[:20]
    a3, t3, e3 = _gen.clean_states(rng, len(names3))
    out = g.receive_soa(names3, a3, t3, e3, _gen.T0 + 2 * SEC)
    st, _, _, _ = o.receive_soa(names3, a3, t3, e3, _gen.T0 + 2 * SEC)
    assert np.array_equal(out["status"], st)
    assert len(g) == 120
    assert_same_dump(gpu_dump(g), o.dump())


@pytest.mark.parametrize("hot_name", [b"one-new-hot-bucket", b"one-new-hot-bucket-" + b"L" * 60])
def test_near_full_table_one_new_hot_name_fits(pa, hot_name):
    """PHIP_CFG_NO_GROW, a table a few buckets below its load limit, and a
    fast batch whose 60000 messages all name one new bucket:
    the insert step bounds its reservation by the batch's distinct missing
    names (one), so the batch is applied instead of refused, exactly.  With
    a long name (arena-held, > 22 bytes) and an arena of 64 KiB, the arena
    bytes are counted once too (60000 x 79 bytes would not fit)."""
    rng = np.random.default_rng(21)
    g = pa.GPURepo(log2_slots=16, max_load_pct=90, grow=False,      # 58982 buckets allowed
                   arena_bytes=1 << 16)
    o = O.Repo()
    K = 58900
    names = _gen.key_names(range(K))
    z = np.zeros(K, np.uint64)
    g.seed(names, z, z, np.zeros(K, np.int64), np.full(K, _gen.T0, np.int64))
    o.seed(names, z, z, np.zeros(K, np.int64), np.full(K, _gen.T0, np.int64))
    n = 60000
    hot = [hot_name] * n
    for i in rng.integers(0, n, 500):
        hot[i] = names[int(i) % K]                 # some existing buckets too
    a, t, e = _gen.clean_states(rng, n)
    out = g.receive_soa(hot, a, t, e, _gen.T0 + SEC)
    st, _, _, _ = o.receive_soa(hot, a, t, e, _gen.T0 + SEC)
    assert np.array_equal(out["status"], st)
    assert len(g) == K + 1
    assert_same_dump(gpu_dump(g), o.dump())


@pytest.mark.parametrize("tag_bits", [0, 12])
def test_table_grows_vs_oracle(pa, tag_bits):
    """Go's map never refuses a bucket (repo.go:204-207): a 2^10-slot table
    takes 60k buckets by rehashing into larger tables (k_rehash) through the
    fast Receive path (small and large miss lists), the ordered path and
    seeding, bit-exact throughout (statuses, `created`, the final table)."""
    rng = np.random.default_rng(303 + tag_bits)
    g = pa.GPURepo(log2_slots=10, debug_tag_bits=tag_bits)
    o = O.Repo()
    # small miss list (k_receive_list) on a table that must grow
    names = _gen.key_names(rng.integers(0, 3000, 9000))
    a, t, e = _gen.clean_states(rng, len(names))
    out = g.receive_soa(names, a, t, e, _gen.T0)
    st, _, _, _ = o.receive_soa(names, a, t, e, _gen.T0)
    assert np.array_equal(out["status"], st)
    # large miss list (k_dedupe + second fast pass)
    ids = _gen.zipf_ids(rng, 200_000, 40_000) + 3000
    names = [(b"a-long-name-that-lives-in-the-arena-%d" % i) if i % 53 == 0 else b"b%d" % i
             for i in ids]
    a, t, e = _fast_dirty_states(rng, len(names))
    out = g.receive_soa(names, a, t, e, _gen.T0 + SEC)
    st, _, _, _ = o.receive_soa(names, a, t, e, _gen.T0 + SEC)
    assert np.array_equal(out["status"], st)
    # ordered path creating buckets (slots resolved again after the rehash)
    args = _mixed_stream(rng, 100_000, 60_000)
    out = g.apply_mixed(*args)
    ref = o.apply_mixed(*args)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["remaining"], ref["remaining"])
    # seeding into a table that must grow
    sn = _gen.key_names(np.arange(500_000, 520_000))
    sa, stt, se = _gen.clean_states(rng, len(sn))
    sc = np.full(len(sn), _gen.T0 + 5 * SEC, np.int64)
    g.seed(sn, sa, stt, se, sc)
    o.seed(sn, sa, stt, se, sc)
    assert len(g) == len(o) > 50_000
    assert g.capacity * 9 // 10 >= len(g) and g.capacity >= 1 << 16 and g.last_stats()[3] >= 2
    assert_same_dump(gpu_dump(g), o.dump())
    g.close()


@pytest.mark.parametrize("grow", [True, False])
def test_long_name_arena_growth(pa, grow):
    """The long-name arena is reserved before any name is claimed: with
    growth a 256-byte arena takes thousands of 23..231-byte names exactly;
    without it the batch is refused (PHIP_ERR_ARENA) with no bucket created
    and no record pointing at another name's bytes."""
    rng = np.random.default_rng(17)
    g = pa.GPURepo(log2_slots=14, arena_bytes=256, grow=grow)
    o = O.Repo()
    short = _gen.key_names(range(50))
    a, t, e = _gen.clean_states(rng, 50)
    g.receive_soa(short, a, t, e, _gen.T0)
    o.receive_soa(short, a, t, e, _gen.T0)
    longs = [bytes(rng.integers(97, 123, int(rng.integers(23, 232)), dtype=np.uint8)) for _ in range(3000)]
    names = [longs[i] for i in rng.integers(0, len(longs), 20000)] + short[:10]
    a, t, e = _gen.clean_states(rng, len(names))
    if grow:
        out = g.receive_soa(names, a, t, e, _gen.T0 + SEC)
        st, _, _, _ = o.receive_soa(names, a, t, e, _gen.T0 + SEC)
        assert np.array_equal(out["status"], st)
        for nm in longs[:20]:
            got, want = g.get(nm), o.get(nm)
            assert (got.added, got.taken, got.elapsed, got.created) == want
    else:
        with pytest.raises(pa.PatrolHipError) as ei:
            g.receive_soa(names, a, t, e, _gen.T0 + SEC)
        assert ei.value.code == -4
        assert len(g) == 50
        o.receive_soa(names[-10:], a[-10:], t[-10:], e[-10:], _gen.T0 + SEC)
    assert_same_dump(gpu_dump(g), o.dump())


def test_merge_laws_at_scale(pa):
    """Size-independent properties at 4M messages: a batch applied twice is
    idempotent, and a shuffled batch gives the same table (clean domain)."""
    rng = np.random.default_rng(51)
    K, n = 200000, 4_000_000
    ids = _gen.zipf_ids(rng, n, K)
    names = _gen.key_names(ids)
    a, t, e = _gen.clean_states(rng, n)
    g1 = pa.GPURepo(log2_slots=19)
    g1.receive_soa(names, a, t, e, _gen.T0)
    d1 = gpu_dump(g1)
    g1.receive_soa(names, a, t, e, _gen.T0 + 1)
    assert gpu_dump(g1) == d1
    perm = rng.permutation(n)
    g2 = pa.GPURepo(log2_slots=19)
    g2.receive_soa([names[i] for i in perm], a[perm], t[perm], e[perm], _gen.T0)
    d2 = gpu_dump(g2)
    # created differs only by the clock each batch saw; compare replicated fields
    assert {k: v[:3] for k, v in d1.items()} == {k: v[:3] for k, v in d2.items()}


@pytest.mark.parametrize("n,short_at", [(60000, None), (60000, 41234), (1 << 21, None),
                                        (1 << 21, 1500000)])
def test_datagram_fast_path_vs_oracle(pa, n, short_at):
    """Wire datagrams on the fast path (k_classify_wire + k_receive_fast
    reading the datagrams in place; the hot directory from 2^16 messages):
    NaN / +-Inf / negatives, new buckets, 15-22 byte and arena names, and a
    malformed datagram that ends the batch (io.ErrShortBuffer)."""
    import struct
    rng = np.random.default_rng(n + (short_at or 0))
    K = 20000
    g, o = _seed_both(pa, rng, K, log2_slots=16)
    ids = _gen.zipf_ids(rng, n, K + 2000)
    names = [(b"a-much-longer-bucket-name-%d" % i) if i % 97 == 0 else
             (b"medium-name-%d" % i) if i % 89 == 0 else (b"b%d" % i) for i in ids]
    a, t, e = _fast_dirty_states(rng, n)
    dgs = [struct.pack(">QQQ", int(a[i]), int(t[i]), int(e[i]) & (2**64 - 1)) +
           bytes([len(names[i])]) + names[i] for i in range(n)]
    if short_at is not None:
        dgs[short_at] = dgs[short_at][:25 + len(names[short_at]) - 1]   # length byte lies
    out = g.receive_datagrams(dgs, _gen.T0 + 3 * SEC)
    st, _, _, _, stop = o.receive(dgs, _gen.T0 + 3 * SEC)
    assert out["stop"] == stop == (n if short_at is None else short_at)
    assert np.array_equal(out["status"], st)
    assert_same_dump(gpu_dump(g), o.dump())


@pytest.mark.parametrize("dirty", [False, True])
def test_mixed_large_batch_vs_oracle(pa, dirty):
    """Ordered batches at 2^21 ops over a Zipf key set, so the hottest
    buckets take the huge-segment path (gathered runs, windowed block folds
    with quiet-window skipping): C3 shape, plus a dirty variant with every op
    kind (Take at several rates, Receive of dirty states with incast replies,
    Upsert) and new buckets."""
    rng = np.random.default_rng(2024 + dirty)
    n, K = 1 << 21, 40000
    ids = _gen.zipf_ids(rng, n, K + 5000)
    names = _gen.key_names(ids)
    now = _gen.T0 + np.arange(n, dtype=np.int64) * 20
    if not dirty:
        kind = (rng.random(n) < 0.5).astype(np.uint8)
        freq = np.full(n, 100, np.int64)
        per = np.full(n, SEC, np.int64)
        cnt = np.ones(n, np.uint64)
        a, t, e = _gen.clean_states(rng, n)
    else:
        kind = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.5, 0.45, 0.05])
        freq = rng.choice(np.array([1, 3, 100, 1000], np.int64), n)
        per = rng.choice(np.array([MS, SEC, 7 * SEC], np.int64), n)
        cnt = rng.integers(1, 4, n).astype(np.uint64)
        a, t, e = _gen.dirty_states(rng, n, 0.02)
    _check_mixed(pa, [kind, names, now, freq, per, cnt, a, t, e], 17, reply=dirty)


@pytest.mark.parametrize("wire", [False, True])
@pytest.mark.parametrize("first", [0, 131000, 131072 + 5, 1500001])
def test_receive_clean_prefix_then_ordered_vs_oracle(pa, wire, first):
    """A 2^21-message batch (hot directory on) whose first incast or -0.0
    sits at `first`: the clean prefix is merged on the fast path, everything
    from `first` on by the ordered path from the state the prefix left,
    replies included.  Wire variant: a malformed datagram after the dirty
    ones ends the batch."""
    import struct
    rng = np.random.default_rng(first + 3 * wire)
    K = 20000
    g, o = _seed_both(pa, rng, K, log2_slots=16)
    n = 1 << 21
    ids = _gen.zipf_ids(rng, n, K + 2000)
    names = _gen.key_names(ids)
    a, t, e = _fast_dirty_states(rng, n)
    later = np.sort(rng.integers(first + 1, n - 100, 40))
    if first % 2:
        a[first] = np.uint64(0x8000000000000000)           # -0.0 first
    else:
        a[first], t[first], e[first] = 0, 0, 0               # incast first
    a[later[:20]], t[later[:20]], e[later[:20]] = 0, 0, 0    # incasts (replies)
    t[later[20:]] = np.uint64(0x8000000000000000)            # -0.0
    now = _gen.T0 + 4 * SEC
    if wire:
        dgs = [struct.pack(">QQQ", int(a[i]), int(t[i]), int(e[i]) & (2**64 - 1)) +
               bytes([len(names[i])]) + names[i] for i in range(n)]
        short = n - 50
        dgs[short] = dgs[short][:20]
        out = g.receive_datagrams(dgs, now)
        st, ra, rt, re, stop = o.receive(dgs, now)
        assert out["stop"] == stop == short
    else:
        out = g.receive_soa(names, a, t, e, now)
        st, ra, rt, re = o.receive_soa(names, a, t, e, now)
    assert np.array_equal(out["status"], st)
    rep = (st & 0x7F) == 2
    assert rep.sum() > 0
    assert np.array_equal(out["reply"]["a"][rep], ra[rep])
    assert np.array_equal(out["reply"]["t"][rep], rt[rep])
    assert np.array_equal(out["reply"]["e"][rep], re[rep])
    assert_same_dump(gpu_dump(g), o.dump())


def test_export_datagrams_are_marshal_binary(pa):
    """Egress batch (phip_export_datagrams): every named bucket's state as the
    byte-identical MarshalBinary datagram (bucket.go:51-68) of the oracle's
    state after the same batches; absent names give found = 0.  Short,
    15-22 byte and arena names, NaN / -0.0 / negative states."""
    import struct
    rng = np.random.default_rng(91)
    K = 5000
    g, o = _seed_both(pa, rng, K, log2_slots=14)
    n = 40000
    ids = _gen.zipf_ids(rng, n, K + 800)
    names = [(b"an-arena-length-bucket-name-%d" % i) if i % 13 == 0 else
             (b"medium-name-%d" % i) if i % 11 == 0 else (b"b%d" % i) for i in ids]
    a, t, e = _gen.dirty_states(rng, n, 0.05)
    g.receive_soa(names, a, t, e, _gen.T0 + SEC)
    o.receive_soa(names, a, t, e, _gen.T0 + SEC)
    ask = sorted(set(names))[:3000] + [b"absent-%d" % i for i in range(50)] + [b"b0", b"b0"]
    rng.shuffle(ask)
    dgs, found = g.export_datagrams(ask)
    for nm, d, f in zip(ask, dgs, found):
        st = o.get(nm)
        assert bool(f) == (st is not None), nm
        if st is None:
            assert d == bytes(25 + len(nm))
            continue
        want = struct.pack(">QQQ", st[0], st[1], st[2] & (2**64 - 1)) + bytes([len(nm)]) + nm
        assert d == want, (nm, d.hex(), want.hex())


def test_snapshot_restore_round_trip(pa, tmp_path):
    """phip_snapshot / phip_restore: a restored handle has the same buckets
    (arena names included) and keeps behaving exactly like the original:
    the same later batch (inserts, incasts, -0.0, Takes) gives the same
    outputs and the same table, which also equals the oracle's.  A handle of
    another table size refuses the image."""
    rng = np.random.default_rng(93)
    K = 4000
    g, o = _seed_both(pa, rng, K, log2_slots=14)
    n = 30000
    ids = _gen.zipf_ids(rng, n, K + 600)
    names = [(b"an-arena-length-bucket-name-%d" % i) if i % 7 == 0 else (b"b%d" % i) for i in ids]
    a, t, e = _gen.dirty_states(rng, n, 0.05)
    g.receive_soa(names, a, t, e, _gen.T0 + SEC)
    o.receive_soa(names, a, t, e, _gen.T0 + SEC)
    path = str(tmp_path / "table.snap")
    g.snapshot(path)
    r = pa.GPURepo(log2_slots=14)
    r.restore(path)
    assert len(r) == len(g)
    d0 = gpu_dump(g)
    assert gpu_dump(r) == d0
    ids2 = _gen.zipf_ids(rng, n, K + 1200)
    names2 = [(b"an-arena-length-bucket-name-%d" % i) if i % 7 == 0 else (b"b%d" % i) for i in ids2]
    kind = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.5, 0.45, 0.05])
    now = _gen.T0 + 2 * SEC + np.arange(n, dtype=np.int64) * 1000
    freq = rng.choice(np.array([1, 100, 1000], np.int64), n)
    per = np.full(n, SEC, np.int64)
    cnt = rng.integers(1, 3, n).astype(np.uint64)
    a2, t2, e2 = _gen.dirty_states(rng, n, 0.02)
    outs = [x.apply_mixed(kind, names2, now, freq, per, cnt, a2, t2, e2) for x in (g, r)]
    for k in ("status", "remaining", "have"):
        assert np.array_equal(outs[0][k], outs[1][k]), k
    o.apply_mixed(kind, names2, now, freq, per, cnt, a2, t2, e2)
    assert gpu_dump(r) == gpu_dump(g)
    assert_same_dump(gpu_dump(r), o.dump())
    # a handle opened at another size takes the image's table size
    other = pa.GPURepo(log2_slots=11)
    other.restore(path)
    assert other.capacity == g.capacity and gpu_dump(other) == d0


# ------------------------------------------------ C1 (BASELINE configs[0]) --
@pytest.mark.parametrize("dist", ["zipf", "uniform"])
def test_c1_receive_vs_oracle(pa, dist):
    """SURVEY C1, the reference's CPU case: 1M replica states merged into a
    pre-populated 100k-bucket repo (Receive path: GetBucket + Merge,
    repo.go:78-79), Zipf(1.1) and uniform, every status and the final state
    of every bucket bit-exact."""
    rng = np.random.default_rng(101 if dist == "zipf" else 102)
    K, n = 100_000, 1_000_000
    g, o = _seed_both(pa, rng, K, log2_slots=18)
    ids = _gen.zipf_ids(rng, n, K) if dist == "zipf" else rng.integers(0, K, n)
    names = _gen.key_names(ids)
    a, t, e = _gen.clean_states(rng, n)
    now = _gen.T0 + 7 * SEC
    out = g.receive_soa(names, a, t, e, now)
    st, _, _, _ = o.receive_soa(names, a, t, e, now)
    assert np.array_equal(out["status"], st)
    assert (st == 1).all()
    assert_same_dump(gpu_dump(g), o.dump())


def test_c1_upsert_vs_oracle(pa):
    """SURVEY C1's Upsert path: 1M distinct states through
    LocalRepo.UpsertBucket (repo.go:215-235: insert as-is on a miss, Merge
    under the write lock on a hit) into the 100k-bucket repo, 5% new names."""
    rng = np.random.default_rng(103)
    K, n = 100_000, 1_000_000
    g, o = _seed_both(pa, rng, K, log2_slots=18)
    ids = _gen.zipf_ids(rng, n, K + 5000)
    names = _gen.key_names(ids)
    a, t, e = _gen.dirty_states(rng, n)
    now = _gen.T0 + 9 * SEC
    st = g.upsert_soa(names, a, t, e, now)["status"]
    merged = o.upsert_soa(names, a, t, e, now).astype(bool)
    assert np.array_equal(st, np.where(merged, 1, 8 | 0x80).astype(np.uint8))
    assert (~merged).sum() > 1000
    assert_same_dump(gpu_dump(g), o.dump())


# ----------------------------------------- insert-heavy (many misses) ----
@pytest.mark.parametrize("wire,tag_bits", [(False, 0), (True, 0), (False, 14)])
def test_insert_heavy_batch_vs_oracle(pa, wire, tag_bits):
    """A batch whose names are mostly new (a node starting nearly empty; the
    C2 insert-on-miss variant): >= 2^16 misses take finish_many_misses
    (one message per distinct name into the insert pipeline, then a second
    fast pass over the prefix).  Statuses (PHIP_ST_CREATED on the lowest-seq
    message of each new bucket), replies and the final table equal the
    oracle's.  tag_bits=14 forces shared tags, so k_dedupe drops names that
    the general insert path must then create."""
    import struct
    rng = np.random.default_rng(77 + tag_bits + wire)
    K = 1000
    names0 = _gen.key_names(np.arange(K))
    a0, t0, e0 = _gen.clean_states(rng, K)
    created = _gen.T0 - rng.integers(0, SEC, K)
    g = pa.GPURepo(log2_slots=18, debug_tag_bits=tag_bits)
    g.seed(names0, a0, t0, e0, created)
    o = O.Repo()
    o.seed(names0, a0, t0, e0, created)
    n = 300_000
    ids = _gen.zipf_ids(rng, n, 60_000)
    names = [(b"a-long-replicated-bucket-name-%d" % i) if i % 71 == 0 else b"b%d" % i
             for i in ids]
    a, t, e = _fast_dirty_states(rng, n)
    now = _gen.T0 + 11 * SEC
    if wire:
        dgs = [struct.pack(">QQQ", int(a[i]), int(t[i]), int(e[i]) & (2**64 - 1)) +
               bytes([len(names[i])]) + names[i] for i in range(n)]
        out = g.receive_datagrams(dgs, now)
        st, _, _, _, stop = o.receive(dgs, now)
        assert out["stop"] == stop == n
    else:
        out = g.receive_soa(names, a, t, e, now)
        st, _, _, _ = o.receive_soa(names, a, t, e, now)
    assert np.array_equal(out["status"], st)
    assert int(((st & 0x80) != 0).sum()) > 10_000
    assert_same_dump(gpu_dump(g), o.dump())
    g.close()


@pytest.mark.parametrize("tag_bits", [0, 14])
def test_mixed_stream_many_new_buckets_vs_oracle(pa, tag_bits):
    """An ordered Take/Merge stream on an empty table with >= 2^16 distinct
    names: resolve_all creates one message per name (k_dedupe) and resolves
    the rest; `created` is still the first op's clock for every bucket and
    shared tags (tag_bits=14) still resolve exactly."""
    rng = np.random.default_rng(91 + tag_bits)
    n, K = 400_000, 150_000
    args = _mixed_stream(rng, n, K)
    g = pa.GPURepo(log2_slots=19, debug_tag_bits=tag_bits)
    o = O.Repo()
    out = g.apply_mixed(*args)
    ref = o.apply_mixed(*args)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["remaining"], ref["remaining"])
    assert int(((ref["status"] & 0x80) != 0).sum()) > 40_000   # all 400k ops miss first
    assert_same_dump(gpu_dump(g), o.dump())
    g.close()


def test_seed_many_names_with_duplicates(pa):
    """phip_seed of >= 2^16 names (the large-miss resolve path), some named
    twice: the last entry of a name wins, as NewLocalRepo's map build does."""
    rng = np.random.default_rng(5)
    K = 120_000
    ids = np.concatenate([np.arange(K), rng.integers(0, K, 5000)])
    names = _gen.key_names(ids)
    a, t, e = _gen.clean_states(rng, len(ids))
    created = _gen.T0 + rng.integers(0, SEC, len(ids))
    g = pa.GPURepo(log2_slots=18)
    g.seed(names, a, t, e, created)
    o = O.Repo()
    o.seed(names, a, t, e, created)
    assert len(g) == K
    assert_same_dump(gpu_dump(g), o.dump())
    g.close()


def test_empty_batches_are_no_ops(pa):
    """n = 0 on every batched entry point: PHIP_OK, nothing created, nothing
    read (the Go loops simply do not iterate)."""
    g = pa.GPURepo(log2_slots=10)
    g.seed([b"b1"], [0x3FF0000000000000], [0], [5], [_gen.T0])
    before = gpu_dump(g)
    out = g.receive_datagrams([], _gen.T0)
    assert out["stop"] == 0 and len(out["status"]) == 0
    assert len(g.receive_soa([], [], [], [], _gen.T0)["status"]) == 0
    assert len(g.upsert_soa([], [], [], [], _gen.T0)["status"]) == 0
    e = np.zeros(0, np.int64)
    res = g.apply_mixed(np.zeros(0, np.uint8), [], e, e, e, np.zeros(0, np.uint64),
                        np.zeros(0, np.uint64), np.zeros(0, np.uint64), e)
    assert len(res["status"]) == 0
    ring = pa.Ring(g, nslots=2, max_msgs=4)
    slot, n = ring.fill([])
    ring.submit(slot, n)
    assert len(ring.receive(slot, n, _gen.T0)["status"]) == 0
    ring.close()
    assert gpu_dump(g) == before
    g.close()
