"""Large ordered batches against the oracle: C3's shape
with refilling Takes on a seeded table, every op kind with dirty states and
long names beside hot buckets, a Receive batch whose dirty suffix is most of
it, and a 2^22-op device batch through phip_apply_mixed.  Bit for bit:
statuses, remaining, have, reply states and the whole table
(bucket.go:186-263, repo.go:54-92, repo.go:189-235).  (Written for round 6's
hot split of the ordered path, which was measured slower and reverted; the
batches stay as ordered-path parity cases.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import _gen  # noqa: E402
from tests.test_gpu_parity import (_mixed_stream, assert_replies, assert_same_dump,  # noqa: E402
                                   gpu_dump)

SEC = 10**9


@pytest.fixture(scope="module")
def pa():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import patrol_amd
    return patrol_amd


def run_both(pa, args, log2_slots, reply=True, seed=None, **kw):
    """The batch through the GPU (large path and, where it applies, the
    one-launch small path is bypassed by size) and through the oracle, from
    the same seeded buckets."""
    o = O.Repo()
    gs = [pa.GPURepo(log2_slots=log2_slots, **kw)]
    if seed is not None:
        for r in gs + [o]:
            r.seed(*seed)
    ref = o.apply_mixed(*args)
    take = np.asarray(args[0]) == 0
    for g, sp in zip(gs, ("default",)):
        out = g.apply_mixed(*args)
        assert np.array_equal(out["status"], ref["status"]), (sp, np.nonzero(out["status"] != ref["status"])[0][:8])
        assert np.array_equal(out["remaining"], ref["remaining"]), sp
        assert np.array_equal(out["have"][take], ref["have"][take]), sp
        if reply:
            assert_replies(out, ref, args[0], sp)
    want = o.dump()
    for g in gs:
        assert_same_dump(gpu_dump(g), want)
    return ref


@pytest.mark.parametrize("seed", [1, 2])
def test_ordered_zipf_mixed_stream(pa, seed):
    """C3's shape at 2^18 ops: Take(100:1s) + clean merges, Zipf over 20k
    buckets, replica clocks below the local clock (Takes refill, succeed and
    deny), some buckets created by the batch."""
    rng = np.random.default_rng(100 + seed)
    n, K = 1 << 18, 20000
    ids = _gen.zipf_ids(rng, n, K + 500)
    names = _gen.key_names(ids)
    kind = (rng.random(n) < 0.5).astype(np.uint8)
    now = _gen.T0 + np.arange(n, dtype=np.int64) * 20_000
    freq = np.full(n, 100, np.int64)
    per = np.full(n, SEC, np.int64)
    cnt = np.ones(n, np.uint64)
    taken = rng.integers(0, 10**4, n).astype(np.float64)
    a = (taken + rng.random(n) * 100).view(np.uint64)
    t = taken.view(np.uint64)
    e = (rng.random(n) * (now - _gen.T0)).astype(np.int64)
    names0 = _gen.key_names(np.arange(K))
    z = np.zeros(K, np.uint64)
    run_both(pa, [kind, names, now, freq, per, cnt, a, t, e], 16,
             seed=(names0, z, z, np.zeros(K, np.int64), np.full(K, _gen.T0 - SEC, np.int64)))


def test_ordered_adversarial_all_kinds(pa):
    """Every op kind (Take with odd rates, Receive of dirty states: incasts,
    -0.0, NaN, negatives; Upsert), three buckets hot enough for the block
    folds, long (arena) names that are never hot, and many new buckets."""
    rng = np.random.default_rng(7)
    n, K = 300000, 3000
    args = list(_mixed_stream(rng, n, K))
    ids = _gen.zipf_ids(rng, n, K)
    r = rng.random(n)
    ids[r < 0.12] = 11
    ids[(r >= 0.12) & (r < 0.2)] = 12
    ids[(r >= 0.2) & (r < 0.26)] = 13
    names = _gen.key_names(ids)
    longs = [b"a-long-bucket-name-never-hot-%04d" % k for k in range(30)]
    for k in np.nonzero(rng.random(n) < 0.05)[0]:
        names[k] = longs[k % 30]
    names[-1] = b"x" * 14   # a 14-byte name (the longest short one)
    args[1] = names
    args[0] = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.5, 0.4, 0.1])
    a, t, e = _gen.dirty_states(rng, n, 0.1)
    args[6], args[7], args[8] = a, t, e
    run_both(pa, args, 13)


def test_ordered_receive_suffix(pa):
    """A large Receive batch whose first dirty message is early: its suffix
    (most of the batch) takes the ordered path (incast replies on hot and
    cold buckets, -0.0 fields)."""
    from tests.test_receive_batches import sprinkle
    rng = np.random.default_rng(33)
    K = 20000
    names0 = _gen.key_names(np.arange(K))
    a0, t0, e0 = _gen.clean_states(rng, K)
    created = _gen.T0 - rng.integers(0, SEC, K)
    n = 1 << 18
    ids = _gen.zipf_ids(rng, n, K + 300)
    a, t, e = _gen.clean_states(rng, n)
    sprinkle(rng, ids, a, t, e, K, incast_hot=3, incast_cold=20, negzero=20)
    a[5], t[5], e[5] = 0, 0, 0   # first dirty message: the rest is ordered
    names = _gen.key_names(ids)
    o = O.Repo()
    o.seed(names0, a0, t0, e0, created)
    st, ra, rt, re = o.receive_soa(names, a, t, e, _gen.T0 + SEC)
    want = o.dump()
    for sp in ("default",):
        g = pa.GPURepo(log2_slots=16)
        g.seed(names0, a0, t0, e0, created)
        out = g.receive_soa(names, a, t, e, _gen.T0 + SEC)
        assert np.array_equal(out["status"], st), sp
        rep = (st & 0x7F) == 2
        assert np.array_equal(out["reply"]["a"][rep], ra[rep]), sp
        assert np.array_equal(out["reply"]["e"][rep], re[rep]), sp
        assert_same_dump(gpu_dump(g), want)


def test_ordered_device_batch_4m(pa):
    """A 2^22-op device batch through
    phip_apply_mixed with device pointers, against the oracle."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(4)
    n, K = 1 << 22, 100000
    ids = _gen.zipf_ids(rng, n, K)
    names = _gen.key_names(ids)
    kind = (rng.random(n) < 0.5).astype(np.uint8)
    now = _gen.T0 + np.arange(n, dtype=np.int64) * 20
    a, t, e = _gen.clean_states(rng, n)
    e = (rng.random(n) * (now - _gen.T0)).astype(np.int64)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in names])
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    tb = T(np.frombuffer(b"".join(names) + b"\0" * 8, np.uint8).copy())
    to = T(offs.astype(np.int32))
    cols = dict(kind=T(kind), now=T(now), freq=T(np.full(n, 100, np.int64)),
                per=T(np.full(n, SEC, np.int64)), cnt=T(np.ones(n, np.int64)),
                a=T(a.view(np.int64)), t=T(t.view(np.int64)), e=T(e))
    o = O.Repo()
    ref = o.apply_mixed(kind, names, now, np.full(n, 100, np.int64), np.full(n, SEC, np.int64),
                        np.ones(n, np.uint64), a, t, e)
    want = o.dump()
    for sp in (None,):
        g = pa.GPURepo(log2_slots=18)
        st = torch.zeros(n, dtype=torch.uint8, device=dev)
        rm = torch.zeros(n, dtype=torch.int64, device=dev)
        hv = torch.zeros(n, dtype=torch.int64, device=dev)
        g.apply_mixed_device(n, cols["kind"], tb, to, cols["now"], cols["freq"], cols["per"],
                             cols["cnt"], cols["a"], cols["t"], cols["e"], status=st, remaining=rm,
                             have=hv)
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), ref["status"]), sp
        assert np.array_equal(rm.cpu().numpy().view(np.uint64), ref["remaining"]), sp
        take = kind == 0
        assert np.array_equal(hv.cpu().numpy().view(np.uint64)[take], ref["have"][take]), sp
        assert_same_dump(gpu_dump(g), want)
        g.close()
