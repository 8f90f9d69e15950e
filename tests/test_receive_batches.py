"""Large Receive batches (>= 2^16 messages: the hot directory, the clean
prefix through the fast path, the dirty suffix through the ordered path)
against the oracle, called synchronously and queued (PHIP_RECV_ASYNC: each
batch finished by the handle's next call or flush).

Bar: bit-exact statuses, incast replies and tables (repo.go:54-92,
bucket.go:240-263).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import _gen  # noqa: E402

SEC = 10**9
NEG0 = np.uint64(0x8000000000000000)


@pytest.fixture(scope="module")
def pa():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import patrol_amd
    return patrol_amd


def dump(repo):
    d = {k: (v.added, v.taken, v.elapsed, v.created) for k, v in repo.dump().items()}
    assert len(repo) == len(d)
    return d


def same(g, o):
    assert len(g) == len(o)
    bad = [k for k in o if g.get(k) != o[k]]
    assert not bad, [(k, g.get(k), o[k]) for k in bad[:5]]


def f64(x):
    return np.float64(x).view(np.uint64)


def seeded(pa, rng, K, log2_slots=17, negative=0.0, **kw):
    """K buckets b0..b{K-1} on the GPU (two handles: host batches, and device
    batches queued) and in the oracle; a fraction `negative` of them holds
    negative added/taken (where a -0.0 replica's place in the batch decides
    the sign of zero)."""
    kw.setdefault("isolate", True)   # (every batch's dirty buckets apart: test_dirty_isolation_policy
    #                                    covers the default, adaptive policy)
    names = _gen.key_names(np.arange(K))
    a, t, e = _gen.clean_states(rng, K)
    neg = rng.random(K) < negative
    a[neg] = (-np.abs(a[neg].view(np.float64)) - 1.0).view(np.uint64)
    t[neg] = (-np.abs(t[neg].view(np.float64)) - 2.0).view(np.uint64)
    created = _gen.T0 - rng.integers(0, SEC, K)
    gs = pa.GPURepo(log2_slots=log2_slots, **kw)
    gc = pa.GPURepo(log2_slots=log2_slots, **kw)
    for g in (gs, gc):
        g.seed(names, a, t, e, created)
    o = O.Repo()
    o.seed(names, a, t, e, created)
    return gs, gc, o


def device_batch(names, a, t, e):
    import torch
    dev = torch.device("cuda", 0)
    n = len(names)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in names])
    tb = torch.from_numpy(np.frombuffer(b"".join(names) + b"\0" * 8, np.uint8).copy()).to(dev)
    to = torch.from_numpy(offs.astype(np.int32)).to(dev)
    ta, tt, te = (torch.from_numpy(x.view(np.int64).copy()).to(dev) for x in (a, t, e))
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    reply = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    return dict(n=n, tb=tb, to=to, ta=ta, tt=tt, te=te, status=status, reply=reply)


def queue_batch(g, b, now):
    g.receive_soa(b["tb"], b["ta"], b["tt"], b["te"], now, name_offs=b["to"], n=b["n"],
                  status=b["status"], device=True, reply=b["reply"], queue=True)


def check(res_status, res_reply, st, ra, rt, re):
    assert np.array_equal(res_status, st), np.nonzero(res_status != st)[0][:8]
    rep = (st & 0x7F) == 2
    assert np.array_equal(res_reply[0][rep], ra[rep])
    assert np.array_equal(res_reply[1][rep], rt[rep])
    assert np.array_equal(res_reply[2][rep], re[rep])


def run_all(gs, gc, o, names, a, t, e, now):
    """gs: the host-pointer call; gc: the device batch queued, then flushed."""
    out = gs.receive_soa(names, a, t, e, now)
    b = device_batch(names, a, t, e)
    queue_batch(gc, b, now)
    gc.flush()
    st, ra, rt, re = o.receive_soa(names, a, t, e, now)
    check(out["status"], (out["reply"]["a"], out["reply"]["t"], out["reply"]["e"]), st, ra, rt, re)
    r = b["reply"].cpu().numpy()
    check(b["status"].cpu().numpy(), (r[:, 0].view(np.uint64), r[:, 1].view(np.uint64), r[:, 2]),
          st, ra, rt, re)
    return st


def sprinkle(rng, ids, a, t, e, K, *, incast_hot=0, incast_cold=0, incast_new=0, negzero=0):
    """Dirty messages at random positions: incasts (all-zero states) naming
    the hottest ids, random existing ids and absent ids; -0.0 fields."""
    n = ids.size
    hot = np.bincount(ids, minlength=1).argsort()[::-1][:4]
    for cnt, pool in ((incast_hot, hot), (incast_cold, None), (incast_new, "new")):
        pos = rng.choice(n, cnt, replace=False) if cnt else []
        for p in pos:
            if pool is None:
                ids[p] = rng.integers(0, K)
            elif isinstance(pool, str):
                ids[p] = K + 10**6 + rng.integers(0, 50)
            else:
                ids[p] = pool[rng.integers(0, len(pool))]
            a[p], t[p], e[p] = 0, 0, 0
    if negzero:
        pos = rng.choice(n, negzero, replace=False)
        for p in pos:
            (a if rng.random() < 0.5 else t)[p] = NEG0


@pytest.mark.parametrize("kind", ["incast_hot", "incast_cold_new", "negzero", "dirty_mix"])
def test_large_dirty_batches_vs_oracle(pa, kind):
    rng = np.random.default_rng({"incast_hot": 21, "incast_cold_new": 22, "negzero": 23,
                                 "dirty_mix": 24}[kind])
    K = 20000
    gs, gc, o = seeded(pa, rng, K, negative=0.3 if kind == "negzero" else 0.0)
    n = 1 << 18
    ids = _gen.zipf_ids(rng, n, K + 2000)   # ~some new keys: the miss path too
    a, t, e = _gen.clean_states(rng, n)
    if kind == "incast_hot":
        sprinkle(rng, ids, a, t, e, K, incast_hot=5)
    elif kind == "incast_cold_new":
        sprinkle(rng, ids, a, t, e, K, incast_cold=40, incast_new=20)
    elif kind == "negzero":
        # replicas +0 / -0 / small negatives racing on buckets whose local
        # state is negative: Go keeps the first zero it sees
        z = rng.random(n) < 0.02
        a[z] = np.where(rng.random(int(z.sum())) < 0.5, np.uint64(0), NEG0)
        z = rng.random(n) < 0.02
        t[z] = np.where(rng.random(int(z.sum())) < 0.5, np.uint64(0), NEG0)
        sprinkle(rng, ids, a, t, e, K, incast_hot=2, incast_cold=5)
    else:
        a, t, e = _gen.dirty_states(rng, n)
    names = _gen.key_names(ids)
    now = _gen.T0 + 5 * SEC
    run_all(gs, gc, o, names, a, t, e, now)
    same(dump(gs), o.dump())
    same(dump(gc), o.dump())
    # a clean batch after it (the next epoch) over the same keys
    a2, t2, e2 = _gen.clean_states(rng, n)
    run_all(gs, gc, o, names, a2, t2, e2, now + SEC)
    same(dump(gs), o.dump())


def test_large_dirty_batch_with_many_new_buckets(pa):
    """Over 2^16 new names (the dedupe and a second fast pass) with incasts
    and -0.0 fields on new and existing buckets."""
    rng = np.random.default_rng(31)
    K = 5000
    gs, gc, o = seeded(pa, rng, K, log2_slots=16)
    n = 1 << 19
    ids = np.concatenate([_gen.zipf_ids(rng, n // 2, K),
                          K + rng.permutation(n // 2)[: n // 2] % (3 * n // 8)])
    ids = ids[rng.permutation(n)]
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_hot=3, incast_cold=30, negzero=40)
    # incasts naming new buckets (created by an earlier message or by them)
    pos = rng.choice(n, 40, replace=False)
    a[pos], t[pos], e[pos] = 0, 0, 0
    names = _gen.key_names(ids)
    run_all(gs, gc, o, names, a, t, e, _gen.T0 + 3 * SEC)
    same(dump(gs), o.dump())
    same(dump(gc), o.dump())


@pytest.mark.parametrize("tag_bits", [9, 14])
def test_large_dirty_batch_narrow_tags(pa, tag_bits):
    """Tags truncated so that names share them (names are always compared)."""
    rng = np.random.default_rng(40 + tag_bits)
    K = 20000
    gs, gc, o = seeded(pa, rng, K, debug_tag_bits=tag_bits)
    n = 1 << 17
    ids = _gen.zipf_ids(rng, n, K + 1000)
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_hot=2, incast_cold=20, incast_new=5, negzero=10)
    names = _gen.key_names(ids)
    run_all(gs, gc, o, names, a, t, e, _gen.T0 + SEC)
    same(dump(gs), o.dump())


def test_large_dirty_batch_table_grows(pa):
    """The batch's new buckets rehash the table in the middle of the batch."""
    rng = np.random.default_rng(51)
    K = 3000
    gs, gc, o = seeded(pa, rng, K, log2_slots=12)
    n = 1 << 17
    ids = np.where(rng.random(n) < 0.5, _gen.zipf_ids(rng, n, K), K + rng.integers(0, 20000, n))
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_hot=3, incast_cold=30, negzero=20)
    names = _gen.key_names(ids)
    cap0 = gs.capacity
    run_all(gs, gc, o, names, a, t, e, _gen.T0 + SEC)
    assert gs.capacity > cap0
    same(dump(gs), o.dump())


def test_queued_batches_back_to_back_many(pa):
    """Twelve queued device batches in a row, each finished by the next call:
    clean ones, ones with new buckets, ones with incasts and -0.0 fields
    (the queued front of the next batch is queued again after such a
    batch's work); every batch's outputs checked after the flush."""
    rng = np.random.default_rng(61)
    K = 4000
    gs, gc, o = seeded(pa, rng, K, log2_slots=14)
    n = 1 << 16
    bs, refs = [], []
    for j in range(12):
        ids = _gen.zipf_ids(rng, n, K + (300 if j % 3 == 1 else 0))
        a, t, e = _gen.clean_states(rng, n)
        if j % 4 == 2:
            sprinkle(rng, ids, a, t, e, K, incast_hot=1, incast_cold=5, negzero=5)
        names = _gen.key_names(ids)
        b = device_batch(names, a, t, e)
        queue_batch(gc, b, _gen.T0 + j * SEC)
        bs.append(b)
        refs.append(o.receive_soa(names, a, t, e, _gen.T0 + j * SEC))
    gc.flush()
    for b, (st, ra, rt, re) in zip(bs, refs):
        r = b["reply"].cpu().numpy()
        check(b["status"].cpu().numpy(), (r[:, 0].view(np.uint64), r[:, 1].view(np.uint64), r[:, 2]),
              st, ra, rt, re)
    same(dump(gc), o.dump())


@pytest.mark.parametrize("queue", [False, True])
def test_back_to_back_device_batches(pa, queue):
    """Three device-resident batches back to back through phip_receive_soa
    (no host copy): one with new buckets, one with incasts and -0.0 fields
    late in the batch, one clean; statuses and replies checked per batch.
    queue: PHIP_RECV_ASYNC, each batch finished by the next call, the last
    by flush()."""
    import torch
    rng = np.random.default_rng(71)
    K = 30000
    gs, gc, o = seeded(pa, rng, K, log2_slots=17)
    n = 1 << 18
    dev = torch.device("cuda", 0)
    batches = []
    for j in range(3):
        ids = _gen.zipf_ids(rng, n, K + (3000 if j == 0 else 0))
        a, t, e = _gen.clean_states(rng, n)
        if j == 1:
            late = np.arange(n - 5000, n)
            pos = rng.choice(late, 30, replace=False)
            a[pos], t[pos], e[pos] = 0, 0, 0
            pos = rng.choice(late, 30, replace=False)
            t[pos] = NEG0
        batches.append((ids, a, t, e))
    outs = []
    for j, (ids, a, t, e) in enumerate(batches):
        names = _gen.key_names(ids)
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum([len(s) for s in names])
        blob = np.frombuffer(b"".join(names) + b"\0" * 8, np.uint8)
        tb = torch.from_numpy(blob.copy()).to(dev)
        to = torch.from_numpy(offs.astype(np.int32)).to(dev)
        ta, tt, te = (torch.from_numpy(x.view(np.int64).copy()).to(dev) for x in (a, t, e))
        status = torch.zeros(n, dtype=torch.uint8, device=dev)
        reply = torch.zeros((n, 4), dtype=torch.int64, device=dev)
        gs.receive_soa(tb, ta, tt, te, _gen.T0 + j * SEC, name_offs=to, n=n, status=status,
                       device=True, reply=reply, queue=queue)
        outs.append((status, reply, tb, to, ta, tt, te))
    gs.flush()
    torch.cuda.synchronize()
    for j, (ids, a, t, e) in enumerate(batches):
        names = _gen.key_names(ids)
        st, ra, rt, re = o.receive_soa(names, a, t, e, _gen.T0 + j * SEC)
        status, reply = outs[j][0].cpu().numpy(), outs[j][1].cpu().numpy()
        assert np.array_equal(status, st), (j, np.nonzero(status != st)[0][:8])
        rep = (st & 0x7F) == 2
        assert np.array_equal(reply[rep, 0].view(np.uint64), ra[rep])
        assert np.array_equal(reply[rep, 1].view(np.uint64), rt[rep])
        assert np.array_equal(reply[rep, 2], re[rep])
    same(dump(gs), o.dump())


def test_queued_batch_finished_by_other_calls(pa):
    """A queued batch (PHIP_RECV_ASYNC) with incasts is finished by whatever
    call comes next on the handle: a lookup sees its merges and replays."""
    import torch
    rng = np.random.default_rng(81)
    K = 10000
    gs, gc, o = seeded(pa, rng, K, log2_slots=16)
    n = 1 << 17
    ids = _gen.zipf_ids(rng, n, K + 500)
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_hot=2, incast_cold=10, negzero=10)
    names = _gen.key_names(ids)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum([len(s) for s in names])
    dev = torch.device("cuda", 0)
    tb = torch.from_numpy(np.frombuffer(b"".join(names) + b"\0" * 8, np.uint8).copy()).to(dev)
    to = torch.from_numpy(offs.astype(np.int32)).to(dev)
    ta, tt, te = (torch.from_numpy(x.view(np.int64).copy()).to(dev) for x in (a, t, e))
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    gs.receive_soa(tb, ta, tt, te, _gen.T0, name_offs=to, n=n, status=status, device=True,
                   queue=True)
    st, _, _, _ = o.receive_soa(names, a, t, e, _gen.T0)
    hot = names[int(np.bincount(ids).argmax())]
    got = gs.get(hot)   # finishes the queued batch first
    want = o.dump()[hot]
    assert (got.added, got.taken, got.elapsed) == want[:3]
    assert np.array_equal(status.cpu().numpy(), st)
    same(dump(gs), o.dump())


@pytest.mark.parametrize("first_call", ["flush", "len", "receive"])
def test_queued_batch_error_reported_by_next_call(pa, first_call):
    """A queued batch that cannot be finished (PHIP_CFG_NO_GROW: its new
    buckets would pass the load limit) returns its error from the handle's
    next call, or, when that call is phip_len (which has no status), from
    the call after it; a queued receive that meets it returns it and queues
    nothing.  As for a synchronous batch, the fast path has merged the
    messages naming existing buckets and no new bucket is created; the
    handle keeps working."""
    rng = np.random.default_rng(91)
    K = 300
    names0 = _gen.key_names(np.arange(K))
    a0, t0, e0 = _gen.clean_states(rng, K)
    created = _gen.T0 - rng.integers(0, SEC, K)
    g = pa.GPURepo(log2_slots=10, max_load_pct=50, grow=False)   # 512 buckets allowed
    g.seed(names0, a0, t0, e0, created)
    o = O.Repo()
    o.seed(names0, a0, t0, e0, created)
    n = 1 << 16
    ids = rng.integers(0, K, n)
    ids[rng.choice(n, 400, replace=False)] = K + np.arange(400)   # 400 new names: over the limit
    names = _gen.key_names(ids)
    a, t, e = _gen.clean_states(rng, n)
    b1 = device_batch(names, a, t, e)   # held: a queued batch's inputs stay put until it is finished
    queue_batch(g, b1, _gen.T0)
    ids2 = rng.integers(0, K + 100, n)
    names2 = _gen.key_names(ids2)
    a2, t2, e2 = _gen.clean_states(rng, n)
    b = device_batch(names2, a2, t2, e2)
    if first_call == "len":
        assert len(g) == K   # finishes the batch; its error waits for the next call
    with pytest.raises(pa.PatrolHipError) as ei:
        if first_call == "receive":
            queue_batch(g, b, _gen.T0 + SEC)   # not queued: the error is the batch before's
        else:
            g.flush()
    assert ei.value.code == -3
    g.flush()   # reported once
    del b1
    keep = np.nonzero(ids < K)[0]
    o.receive_soa([names[i] for i in keep], a[keep], t[keep], e[keep], _gen.T0)
    same(dump(g), o.dump())
    # the handle still works: a queued batch that fits, then its flush
    b["status"].zero_()
    queue_batch(g, b, _gen.T0 + SEC)
    g.flush()
    st, ra, rt, re = o.receive_soa(names2, a2, t2, e2, _gen.T0 + SEC)
    r = b["reply"].cpu().numpy()
    check(b["status"].cpu().numpy(), (r[:, 0].view(np.uint64), r[:, 1].view(np.uint64), r[:, 2]),
          st, ra, rt, re)
    assert len(g) == K + 100
    same(dump(g), o.dump())


def test_queued_batch_outputs_final_when_next_call_returns(pa):
    """A queued batch with a late dirty suffix (incasts, -0.0 in its last
    messages: the ordered path's folds write those statuses and replies) is
    finished by the next queued receive; its outputs are read right after
    that call returns, on another stream, with no flush in between
    (phip_engine.hip finish_pending: the leftover work is waited for)."""
    import torch
    rng = np.random.default_rng(95)
    K = 20000
    gs, gc, o = seeded(pa, rng, K, log2_slots=16)
    n = 1 << 17
    ids = _gen.zipf_ids(rng, n, K + 200)
    a, t, e = _gen.clean_states(rng, n)
    late = np.arange(n - 3000, n)
    pos = rng.choice(late, 40, replace=False)
    a[pos], t[pos], e[pos] = 0, 0, 0
    pos = rng.choice(late, 40, replace=False)
    t[pos] = NEG0
    names = _gen.key_names(ids)
    b1 = device_batch(names, a, t, e)
    queue_batch(gc, b1, _gen.T0)
    ids2 = _gen.zipf_ids(rng, n, K)
    a2, t2, e2 = _gen.clean_states(rng, n)
    names2 = _gen.key_names(ids2)
    b2 = device_batch(names2, a2, t2, e2)
    queue_batch(gc, b2, _gen.T0 + SEC)   # finishes b1 before it returns
    with torch.cuda.stream(torch.cuda.Stream()):
        s1 = b1["status"].cpu().numpy()
        r1 = b1["reply"].cpu().numpy()
    st, ra, rt, re = o.receive_soa(names, a, t, e, _gen.T0)
    check(s1, (r1[:, 0].view(np.uint64), r1[:, 1].view(np.uint64), r1[:, 2]), st, ra, rt, re)
    gc.flush()
    st2, ra2, rt2, re2 = o.receive_soa(names2, a2, t2, e2, _gen.T0 + SEC)
    r2 = b2["reply"].cpu().numpy()
    check(b2["status"].cpu().numpy(), (r2[:, 0].view(np.uint64), r2[:, 1].view(np.uint64), r2[:, 2]),
          st2, ra2, rt2, re2)
    same(dump(gc), o.dump())


@pytest.mark.parametrize("queue", [True, False])
def test_corrupted_offset_column_is_an_error_not_a_fault(pa, queue):
    """A device batch whose name offset column is corrupted (one entry far
    past the blob: what a queued batch's freed and reused column reads as)
    with names_len given (the binding's default: the blob's size): the
    classification finds the first malformed entry, no kernel reads the blob
    there, and the call (queued: the call that finishes it) returns
    PHIP_ERR_INVALID.  The batch stops at that message as Go's loop stops at
    a short datagram: the messages before it are received, it reads
    PHIP_ST_SHORT and the rest PHIP_ST_NOT_PROCESSED; the handle keeps
    working (bucket.go:71-91, repo.go:70-74)."""
    rng = np.random.default_rng(97)
    K = 8000
    gs, gc, o = seeded(pa, rng, K, log2_slots=15)
    g = gc if queue else gs
    n = 1 << 17
    ids = _gen.zipf_ids(rng, n, K + 100)
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_cold=5)
    names = _gen.key_names(ids)
    b = device_batch(names, a, t, e)
    k = 70001
    b["to"][k] = 0x7FFF0000   # message k-1 ends past the blob, message k starts there
    stop = k - 1
    with pytest.raises(pa.PatrolHipError) as ei:
        if queue:
            queue_batch(g, b, _gen.T0)
            g.flush()
        else:
            g.receive_soa(b["tb"], b["ta"], b["tt"], b["te"], _gen.T0, name_offs=b["to"],
                          n=n, status=b["status"], device=True, reply=b["reply"])
    assert ei.value.code == -1
    st, ra, rt, re = o.receive_soa(names[:stop], a[:stop], t[:stop], e[:stop], _gen.T0)
    got = b["status"].cpu().numpy()
    assert np.array_equal(got[:stop], st), np.nonzero(got[:stop] != st)[0][:8]
    assert got[stop] == 4 and (got[stop + 1:] == 5).all()
    same(dump(g), o.dump())
    # the handle keeps working: the same batch with the column repaired
    b2 = device_batch(names, a, t, e)
    if queue:
        queue_batch(g, b2, _gen.T0 + SEC)
        g.flush()
    else:
        g.receive_soa(b2["tb"], b2["ta"], b2["tt"], b2["te"], _gen.T0 + SEC, name_offs=b2["to"],
                      n=n, status=b2["status"], device=True, reply=b2["reply"])
    o.receive_soa(names, a, t, e, _gen.T0 + SEC)
    same(dump(g), o.dump())


def test_corrupted_offsets_ordered_batch_refused_whole(pa):
    """phip_apply_mixed with device pointers and names_len: a corrupted
    offset column refuses the whole batch (PHIP_ERR_INVALID) before anything
    is applied or created; the handle keeps working."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(99)
    K = 5000
    gs, gc, o = seeded(pa, rng, K, log2_slots=15)
    before = dump(gs)
    n = 1 << 16
    ids = _gen.zipf_ids(rng, n, K + 50)
    names = _gen.key_names(ids)
    b = device_batch(names, *_gen.clean_states(rng, n))
    kind = torch.ones(n, dtype=torch.uint8, device=dev)
    kind[::2] = 0
    now = torch.full((n,), _gen.T0, dtype=torch.int64, device=dev)
    freq = torch.full((n,), 100, dtype=torch.int64, device=dev)
    per = torch.full((n,), SEC, dtype=torch.int64, device=dev)
    cnt = torch.ones(n, dtype=torch.int64, device=dev)
    b["to"][n // 2] = 0x40000000
    with pytest.raises(pa.PatrolHipError) as ei:
        gs.apply_mixed_device(n, kind, b["tb"], b["to"], now, freq, per, cnt, b["ta"], b["tt"],
                              b["te"], status=b["status"])
    assert ei.value.code == -1
    same(dump(gs), before)
    g2 = gs.get(names[0])
    assert g2 is not None


def dirty_mask(a, t, e):
    """The messages whose place in the batch matters (k_classify): incasts
    (both floats zero, elapsed 0) and -0.0 fields."""
    return ((a == 0) & (t == 0) & (e == 0)) | (a == NEG0) | (t == NEG0)


def deferred_count(names, dirty):
    """Entries of the ordered sub-batch (dirty_finish): per dirty bucket,
    one merge of its clean messages before its first dirty message (if any),
    then every dirty message, each followed by one merge of the clean
    messages after it and before the bucket's next dirty message (if any)."""
    pos = {}
    for i, x in enumerate(names):
        pos.setdefault(x, []).append(i)
    total = 0
    for x, ps in pos.items():
        d = dirty[ps]
        if not d.any():
            continue
        total += int(d.sum())
        run = False
        for k in range(len(ps)):
            if d[k]:
                run = False
            elif not run:
                run = True
                total += 1
    return total


@pytest.mark.parametrize("seed", [61, 62])
def test_dirty_buckets_deferred_alone(pa, seed):
    """Dirty-bucket isolation: a batch with a few incasts (hot, cold and new
    buckets) and -0.0 fields, the first of them near its start, sends only
    the messages of the buckets those name through the ordered path (in
    their order); every other message is merged by the fast path.  Called
    synchronously and queued; bit-exact against the oracle, and the ordered
    path's share is exactly the dirty messages plus one merge per run of
    clean messages between them (last_stats()[4])."""
    rng = np.random.default_rng(seed)
    K = 20000
    gs, gc, o = seeded(pa, rng, K, negative=0.3)
    n = 1 << 18
    ids = _gen.zipf_ids(rng, n, K + 2000)
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_hot=1 if seed == 61 else 0, incast_cold=30,
             incast_new=10, negzero=20)
    ids[7] = 12345
    a[7], t[7], e[7] = 0, 0, 0                     # an incast at message 7
    names = _gen.key_names(ids)
    dirty = dirty_mask(a, t, e)
    assert 0 < dirty.sum() <= 4096 and np.argmax(dirty) <= 7
    want = deferred_count(names, dirty)
    assert want <= 3 * int(dirty.sum())
    run_all(gs, gc, o, names, a, t, e, _gen.T0 + 2 * SEC)
    assert gs.last_stats()[4] == want
    assert gc.last_stats()[4] == want
    same(dump(gs), o.dump())
    same(dump(gc), o.dump())


def test_dirty_buckets_over_cap_keep_prefix_rule(pa):
    """More than 4096 dirty messages: the batch keeps the prefix rule (the
    ordered path from the first dirty message on)."""
    rng = np.random.default_rng(63)
    K = 20000
    gs, gc, o = seeded(pa, rng, K)
    n = 1 << 17
    ids = _gen.zipf_ids(rng, n, K + 500)
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_cold=4500, negzero=200)
    names = _gen.key_names(ids)
    dirty = dirty_mask(a, t, e)
    assert dirty.sum() > 4096
    run_all(gs, gc, o, names, a, t, e, _gen.T0 + SEC)
    assert gs.last_stats()[4] == n - int(np.argmax(dirty))
    same(dump(gs), o.dump())
    same(dump(gc), o.dump())


def test_dirty_long_name_keeps_prefix_rule(pa):
    """A dirty message whose name is longer than 14 bytes (the dirty set
    compares short names only): the batch keeps the prefix rule."""
    rng = np.random.default_rng(64)
    K = 20000
    gs, gc, o = seeded(pa, rng, K)
    n = 1 << 17
    ids = _gen.zipf_ids(rng, n, K + 500)
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_cold=20)
    names = _gen.key_names(ids)
    for p in rng.choice(n, 50, replace=False):
        names[p] = b"a-much-longer-bucket-name-%d" % (p % 7)   # (some of them dirty)
    p = int(rng.integers(n // 4, n // 2))
    names[p] = b"a-much-longer-bucket-name-3"
    a[p], t[p], e[p] = 0, 0, 0
    dirty = dirty_mask(a, t, e)
    run_all(gs, gc, o, names, a, t, e, _gen.T0 + SEC)
    assert gs.last_stats()[4] == n - int(np.argmax(dirty))
    same(dump(gs), o.dump())
    same(dump(gc), o.dump())


def test_dirty_bucket_isolation_over_a_clean_batch_and_repeat(pa):
    """A clean batch after a deferred one (the deferred list's counters start
    again from zero), then the dirty batch again on the queued handle twice
    in a row (parity counter sets)."""
    import torch
    rng = np.random.default_rng(65)
    K = 10000
    gs, gc, o = seeded(pa, rng, K)
    n = 1 << 17
    now = _gen.T0
    for r in range(4):
        ids = _gen.zipf_ids(rng, n, K + 300)
        a, t, e = _gen.clean_states(rng, n)
        if r != 1:
            sprinkle(rng, ids, a, t, e, K, incast_cold=15, incast_new=5, negzero=5)
        names = _gen.key_names(ids)
        want = deferred_count(names, dirty_mask(a, t, e))
        now += SEC
        bs = []
        for _ in range(2):   # two queued copies back to back (the second sees the first's state)
            b = device_batch(names, a, t, e)
            queue_batch(gc, b, now)
            bs.append(b)
        gc.flush()
        gs.receive_soa(names, a, t, e, now)
        gs.receive_soa(names, a, t, e, now)
        assert gs.last_stats()[4] == want
        o.receive_soa(names, a, t, e, now)
        st, ra, rt, re = o.receive_soa(names, a, t, e, now)
        r_ = bs[1]["reply"].cpu().numpy()
        check(bs[1]["status"].cpu().numpy(),
              (r_[:, 0].view(np.uint64), r_[:, 1].view(np.uint64), r_[:, 2]), st, ra, rt, re)
        torch.cuda.synchronize()
        same(dump(gs), o.dump())
        same(dump(gc), o.dump())


@pytest.mark.parametrize("short_at", [None, 150000])
def test_dirty_buckets_datagrams(pa, short_at):
    """The same isolation for raw datagrams (phip_receive_datagrams, the
    sub-batch read from the wire): a few incasts and -0.0 fields on hot,
    cold and new buckets, bit-exact statuses, incast replies and tables
    against the oracle's datagram loop; with a short datagram the batch
    stops there (dirty messages past it are never applied)."""
    import struct
    rng = np.random.default_rng(71 if short_at is None else 72)
    K = 20000
    gs, gc, o = seeded(pa, rng, K, negative=0.3)
    n = 1 << 18
    ids = _gen.zipf_ids(rng, n, K + 2000)
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_hot=1, incast_cold=30, incast_new=10, negzero=20)
    names = _gen.key_names(ids)
    dgs = [struct.pack(">QQQ", int(a[i]), int(t[i]), int(e[i]) & (2**64 - 1)) +
           bytes([len(names[i])]) + names[i] for i in range(n)]
    if short_at is not None:
        dgs[short_at] = dgs[short_at][:20]
    now = _gen.T0 + SEC
    out = gs.receive_datagrams(dgs, now)
    st, ra, rt, re, stop = o.receive(dgs, now)
    assert out["stop"] == stop == (n if short_at is None else short_at)
    check(out["status"], (out["reply"]["a"], out["reply"]["t"], out["reply"]["e"]), st, ra, rt, re)
    if short_at is None:
        assert gs.last_stats()[4] == deferred_count(names, dirty_mask(a, t, e))
    same(dump(gs), o.dump())


@pytest.mark.parametrize("queue", [False, True])
def test_dirty_bucket_cells_that_read_as_incasts(pa, queue):
    """A cell's merge whose maxima read (+0, +0, 0) -- clean messages
    (-5, +0, 0) and (+0, -3, 0) of a bucket whose state is negative -- would
    read as an incast if it went through the ordered path as one message; it
    is split into two merges of the same effect (dirty_finish).  Bucket b0:
    incast, the two clean messages, incast (their cell after the first
    incast); bucket b1: the two clean messages before its first incast (its
    pre cell).  The final incasts see a zero state: PHIP_ST_INCAST_NOREPLY,
    as the Go loop gives; the oracle agrees on every status and reply."""
    rng = np.random.default_rng(81)
    K = 5000
    names0 = _gen.key_names(np.arange(K))
    a0, t0, e0 = _gen.clean_states(rng, K)
    neg = np.float64(-10.0).view(np.uint64)
    a0[:2], t0[:2], e0[:2] = neg, neg, -5
    created = np.full(K, _gen.T0 - SEC, np.int64)
    g = pa.GPURepo(log2_slots=15, isolate=True)
    g.seed(names0, a0, t0, e0, created)
    o = O.Repo()
    o.seed(names0, a0, t0, e0, created)
    n = 1 << 16
    ids = 2 + rng.integers(0, K - 2, n)
    a, t, e = _gen.clean_states(rng, n)
    m5, m3 = np.float64(-5.0).view(np.uint64), np.float64(-3.0).view(np.uint64)
    seq = {  # position: (bucket, a, t, e)
        1000: (0, 0, 0, 0), 1010: (0, m5, 0, 0), 1020: (0, 0, m3, 0), 1030: (0, 0, 0, 0),
        2000: (1, m5, 0, 0), 2005: (1, 0, m3, 0), 2010: (1, 0, 0, 0),
    }
    for p, (b, x, y, z) in seq.items():
        ids[p], a[p], t[p], e[p] = b, x, y, z
    names = _gen.key_names(ids)
    now = _gen.T0
    if queue:
        bt = device_batch(names, a, t, e)
        queue_batch(g, bt, now)
        g.flush()
        r = bt["reply"].cpu().numpy()
        got = (bt["status"].cpu().numpy(), (r[:, 0].view(np.uint64), r[:, 1].view(np.uint64), r[:, 2]))
    else:
        out = g.receive_soa(names, a, t, e, now)
        got = (out["status"], (out["reply"]["a"], out["reply"]["t"], out["reply"]["e"]))
    st, ra, rt, re = o.receive_soa(names, a, t, e, now)
    check(got[0], got[1], st, ra, rt, re)
    assert st[1030] == 3 and st[2010] == 3   # PHIP_ST_INCAST_NOREPLY: the state is zero
    assert g.last_stats()[4] >= 6            # the split merges went through the sub-batch
    same(dump(g), o.dump())


def test_dirty_isolation_policy(pa):
    """The default policy: a handle sets a batch's dirty buckets apart only
    after a batch that held a dirty message (a clean batch would pay the
    isolation kernels for nothing), until 256 clean batches in a row.  The
    first dirty batch of a fresh handle takes the prefix rule, the next one
    is isolated, and a handle that only ever saw clean batches never
    launches the isolation kernels; bit-exact against the oracle throughout."""
    rng = np.random.default_rng(91)
    K = 20000
    gs, _, o = seeded(pa, rng, K, isolate=False)
    n = 1 << 17
    now = _gen.T0
    for r, want_iso in ((0, False), (1, True)):
        ids = _gen.zipf_ids(rng, n, K + 500)
        a, t, e = _gen.clean_states(rng, n)
        sprinkle(rng, ids, a, t, e, K, incast_cold=20, negzero=10)
        names = _gen.key_names(ids)
        dirty = dirty_mask(a, t, e)
        now += SEC
        out = gs.receive_soa(names, a, t, e, now)
        st, ra, rt, re = o.receive_soa(names, a, t, e, now)
        check(out["status"], (out["reply"]["a"], out["reply"]["t"], out["reply"]["e"]), st, ra, rt, re)
        want = deferred_count(names, dirty) if want_iso else n - int(np.argmax(dirty))
        assert gs.last_stats()[4] == want, (r, gs.last_stats())
        same(dump(gs), o.dump())
    # clean batches on a fresh handle: no isolation kernel runs
    g2 = pa.GPURepo(log2_slots=17)
    g2.set_timing(True)
    ids = _gen.zipf_ids(rng, n, K)
    a, t, e = _gen.clean_states(rng, n)
    g2.receive_soa(_gen.key_names(ids), a, t, e, now)
    names_run = [nm for nm, _ in g2.timings()]
    assert "k_receive_fast" in names_run and "k_dirty_build" not in names_run, names_run
