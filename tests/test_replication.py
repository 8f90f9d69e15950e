"""What the drop-in handlers send to peers, from the same batched launch as
the ops themselves (include/patrolhip.h phip_results.reply, phip_take_reply):

* the Take batcher returns, per request, whether its GetBucket created the
  bucket (ReplicatedRepo.GetBucket then broadcasts a zero-state incast,
  repo.go:96-106) and the MarshalBinary datagram of the state right after
  the Take, which UpsertBucket broadcasts (api.go:67-74, repo.go:123-158);
  checked against the oracle run in arrival order;
* GetBucket as a zero-state Receive (a pure find-or-create, repo.go:189-211):
  existence, state and `created`, and no state change;
* closing a batcher while callers are blocked in it;
* placement: names crafted to share a home slot under one seed pile up on
  one probe chain only under that seed (Go's map seeds its hash per
  process, repo.go:175), and results never depend on the seed.
"""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import go_semantics as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests import _gen  # noqa: E402

SEC = 10**9


@pytest.fixture(scope="module")
def pa():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import patrol_amd
    return patrol_amd


def marshal(name: bytes, a_bits: int, t_bits: int, e: int) -> bytes:
    """Bucket.MarshalBinary (bucket.go:51-68), the Python restatement."""
    b = G.Bucket(name=name.decode("latin-1"), added=G.b2f(a_bits), taken=G.b2f(t_bits), elapsed=e)
    return b.marshal()


@pytest.mark.parametrize("window_us", [0, 40])
def test_batcher_take_reply_vs_oracle(pa, window_us):
    """Threads issue Takes through phip_batcher_take_reply; every request's
    remaining/ok, created flag, post-Take state and datagram equal the
    oracle running the requests one by one in arrival order."""
    threads, per_thread, K = 32, 120, 90
    repo = pa.GPURepo(log2_slots=12)
    # a third of the buckets exist before (some with state), the rest are new
    pre = [b"b%d" % k for k in range(0, K, 3)]
    rng = np.random.default_rng(100 + window_us)
    st = [int(x) for x in rng.integers(0, 4, len(pre))]
    added = [G.f2b(float(x)) for x in st]
    repo.seed(pre, added, [0] * len(pre), [0] * len(pre), [_gen.T0] * len(pre))
    o = O.Repo()
    o.seed(pre, added, [0] * len(pre), [0] * len(pre), [_gen.T0] * len(pre))
    b = pa.TakeBatcher(repo, window_us=window_us)
    plan = []
    for tid in range(threads):
        ids = _gen.zipf_ids(rng, per_thread, K)
        now = _gen.T0 + np.sort(rng.integers(0, 3 * SEC, per_thread))
        freq = rng.choice(np.array([100, 5, 3, 0], np.int64), per_thread)
        plan.append([(b"b%d" % ids[k], int(now[k]), int(freq[k]), SEC, int(rng.integers(1, 3)))
                     for k in range(per_thread)])
    results = [[] for _ in range(threads)]
    start = threading.Barrier(threads)

    def worker(tid):
        start.wait()
        for req in plan[tid]:
            results[tid].append((req, b.take_reply(*req)))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    b.close()
    allr = sorted((r["seq"], req, r) for rs in results for req, r in rs)
    n = len(allr)
    assert [x[0] for x in allr] == list(range(n))
    names = [x[1][0] for x in allr]
    ref = o.apply_mixed(np.zeros(n, np.uint8), names, [x[1][1] for x in allr],
                        [x[1][2] for x in allr], [x[1][3] for x in allr], [x[1][4] for x in allr],
                        np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(n, np.int64))
    created = 0
    for i, (_, req, r) in enumerate(allr):
        s = int(ref["status"][i])
        assert r["remaining"] == int(ref["remaining"][i]), i
        assert r["ok"] == ((s & 0x7F) == G.TAKE_OK), i
        assert r["created"] == bool(s & G.CREATED), i
        created += r["created"]
        want = (int(ref["reply_added"][i]), int(ref["reply_taken"][i]), int(ref["reply_elapsed"][i]),
                int(ref["reply_created"][i]))
        got = r["state"]
        assert (got.added, got.taken, got.elapsed, got.created) == want, i
        assert r["datagram"] == marshal(req[0], *want[:3]), i
    # each new bucket is created by exactly one request, the earliest of its name
    assert created == K - len(pre)
    assert {k: (v.added, v.taken, v.elapsed, v.created) for k, v in repo.dump().items()} == o.dump()
    repo.close()


def test_batcher_api_take_reply_table(pa):
    """api_test.go:34-73 through phip_batcher_api_take_reply: codes and bodies
    as the reference, a 400 sends nothing, every other request carries its
    post-Take datagram, and only a bucket's first request is its creator."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "api_table.json")) as f:
        g = json.load(f)
    repo = pa.GPURepo(log2_slots=10)
    sb = g["seed_bucket"]
    repo.seed([sb["name"].encode()], [0], [0], [0], [sb["created"]])
    b = pa.TakeBatcher(repo, window_us=10)
    seen = {sb["name"].encode()}
    for r in g["requests"]:
        name = r["name"].encode()
        code, body, rep = b.api_take_reply(name, r["rate"].encode(), r["count"].encode(), r["now"])
        assert (code, body) == (r["code"], r["body"]), r
        if code == 400:
            assert rep["datagram"] == b"" and not rep["created"]
            continue
        assert rep["created"] == (name not in seen)
        seen.add(name)
        st = rep["state"]
        assert rep["datagram"] == marshal(name, st.added, st.taken, st.elapsed)
        cur = repo.get(name)
        assert (cur.added, cur.taken, cur.elapsed, cur.created) == \
            (st.added, st.taken, st.elapsed, st.created)
    b.close()
    repo.close()


@pytest.mark.parametrize("small", [True, False])
def test_getbucket_is_zero_state_receive(pa, small):
    """LocalRepo.GetBucket (repo.go:189-211) as a zero-state Receive: found
    buckets report their state (INCAST_REPLY when non-zero, NOREPLY when
    zero) and are not changed; a missing one is created with created = now
    (NOREPLY | CREATED); the table equals the oracle's after the same calls."""
    repo = pa.GPURepo(log2_slots=10, small=small)
    o = O.Repo()
    names = [b"live", b"zero", b"neg"]
    a = [G.f2b(5.0), 0, G.f2b(-1.0)]
    t = [G.f2b(2.0), 0, G.f2b(-3.0)]
    e = [77, 0, -5]
    c = [_gen.T0 - 5, _gen.T0 - 6, _gen.T0 - 7]
    repo.seed(names, a, t, e, c)
    o.seed(names, a, t, e, c)
    now = _gen.T0 + 123
    ask = [b"live", b"zero", b"neg", b"new-one", b"new-one", b"live"]
    z = np.zeros(len(ask), np.uint64)
    out = repo.receive_soa(ask, z, z, np.zeros(len(ask), np.int64), now)
    kind = np.ones(len(ask), np.uint8)
    ref = o.apply_mixed(kind, ask, np.full(len(ask), now, np.int64), z.view(np.int64),
                        z.view(np.int64), z, z, z, np.zeros(len(ask), np.int64))
    assert np.array_equal(out["status"], ref["status"])
    assert list(out["status"] & 0x7F) == [2, 3, 2, 3, 3, 2]
    assert list(out["status"] & 0x80) == [0, 0, 0, 0x80, 0, 0]
    r = out["reply"]
    for i in range(len(ask)):
        assert (int(r["a"][i]), int(r["t"][i]), int(r["e"][i]), int(r["c"][i])) == \
            (int(ref["reply_added"][i]), int(ref["reply_taken"][i]),
             int(ref["reply_elapsed"][i]), int(ref["reply_created"][i])), i
    assert int(r["c"][3]) == now
    assert {k: (v.added, v.taken, v.elapsed, v.created) for k, v in repo.dump().items()} == o.dump()
    repo.close()


def test_batcher_close_while_callers_blocked(pa):
    """phip_batcher_close with many callers blocked in take(): it runs the
    queued requests, every caller returns its result, and the batcher is
    freed only after the last of them left."""
    for rep in range(5):
        repo = pa.GPURepo(log2_slots=10)
        b = pa.TakeBatcher(repo, window_us=100000)   # a batch closes 0.1 s after its first take
        out = []
        lock = threading.Lock()

        def worker(k):
            r = b.take(b"c%d" % (k % 7), _gen.T0 + k, 100, SEC, 1)
            with lock:
                out.append(r)

        ts = [threading.Thread(target=worker, args=(k,)) for k in range(48)]
        for t in ts:
            t.start()
        time.sleep(0.02)
        b.close()              # stops the window early, runs the queue
        for t in ts:
            t.join(timeout=30)
        assert not any(t.is_alive() for t in ts)
        assert len(out) == 48 and sorted(r[2] for r in out) == list(range(48))
        repo.close()


def _fnv_matrix(names):
    """FNV-1a 64 of equal-length names (uint8 matrix [n, L]) with numpy."""
    h = np.full(names.shape[0], 0xcbf29ce484222325, np.uint64)
    p = np.uint64(0x100000001b3)
    for j in range(names.shape[1]):
        h = (h ^ names[:, j].astype(np.uint64)) * p
    return h


def _home(tags, seed, L):
    x = tags ^ np.uint64(seed)
    x ^= x >> np.uint64(33)
    x *= np.uint64(0xff51afd7ed558ccd)
    x ^= x >> np.uint64(33)
    x *= np.uint64(0xc4ceb9fe1a85ec53)
    x ^= x >> np.uint64(33)
    return x >> np.uint64(64 - L)


def test_crafted_home_collisions_only_under_their_seed(pa):
    """300 names chosen to share one home slot of a 2^10-slot table under
    the unseeded placement (seed 0) form one 300-long probe chain there; in
    a handle with its own random seed they scatter (short chains).  Both
    tables hold the same buckets with the same states."""
    L, m = 10, 300
    ids = np.arange(600_000, dtype=np.int64)
    cand = np.empty((ids.size, 10), np.uint8)
    cand[:, 0] = ord("x")
    for k in range(9):                       # names x000000000 .. x000599999
        cand[:, 9 - k] = 48 + (ids // 10**k) % 10
    with np.errstate(over="ignore"):
        homes = _home(_fnv_matrix(cand), 0, L)
    target = np.bincount(homes.astype(np.int64)).argmax()
    pick = np.nonzero(homes == target)[0][:m]
    assert pick.size == m
    names = [bytes(cand[i]) for i in pick]
    rng = np.random.default_rng(8)
    a, t, e = _gen.clean_states(rng, len(names))
    stats, dumps = {}, {}
    for label, seed in (("fixed0", 0), ("random", None)):
        repo = pa.GPURepo(log2_slots=L, hash_seed=seed, grow=False)
        repo.receive_soa(names, a, t, e, _gen.T0)
        stats[label] = repo.table_stats()
        dumps[label] = {k: (v.added, v.taken, v.elapsed, v.created) for k, v in repo.dump().items()}
        repo.close()
    assert stats["fixed0"]["buckets"] == stats["random"]["buckets"] == m
    assert stats["fixed0"]["max_probe"] >= m - 1          # the crafted chain
    assert stats["random"]["max_probe"] < 32              # 300 of 1024 slots, scattered
    assert dumps["fixed0"] == dumps["random"]


@pytest.mark.parametrize("tag_bits", [3, 0])
def test_seeded_placement_vs_oracle(pa, tag_bits):
    """Random seeds (and 3-bit tags, forcing tag collisions everywhere):
    receive, mixed and growth give the oracle's results under any seed."""
    rng = np.random.default_rng(31 + tag_bits)
    o = O.Repo()
    repos = [pa.GPURepo(log2_slots=8, debug_tag_bits=tag_bits, hash_seed=s)
             for s in (None, 0x9E3779B97F4A7C15, 1)]
    for step in range(3):
        n = 3000
        ids = _gen.zipf_ids(rng, n, 600)
        names = _gen.key_names(ids + 600 * step)
        kind = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.5, 0.4, 0.1])
        now = _gen.T0 + step * SEC + np.arange(n, dtype=np.int64) * 1000
        freq = np.full(n, 100, np.int64)
        per = np.full(n, SEC, np.int64)
        cnt = np.ones(n, np.uint64)
        a, t, e = _gen.dirty_states(rng, n, 0.1)
        args = (kind, names, now, freq, per, cnt, a, t, e)
        ref = o.apply_mixed(*args)
        for r in repos:
            out = r.apply_mixed(*args)
            assert np.array_equal(out["status"], ref["status"]), step
            assert np.array_equal(out["remaining"], ref["remaining"]), step
    want = o.dump()
    for r in repos:
        assert {k: (v.added, v.taken, v.elapsed, v.created) for k, v in r.dump().items()} == want
        assert r.last_stats()[3] > 0     # the 2^8-slot tables grew (rehash under the seed)
        r.close()
