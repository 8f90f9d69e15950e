"""Pin the oracle before trusting it (CPU only).

1. The pure-Python restatement (oracle/go_semantics.py) reproduces the
   reference's own tests: bucket_test.go:35-66 (Take known answers),
   bucket_test.go:68-114 (Merge CRDT laws, here with fixed seeds),
   bucket_test.go:10-34 (codec round trip), api_test.go:34-73 (HTTP table).
2. The C++ restatement (oracle/liboracle.so) reproduces every golden fixture
   in tests/golden/ bit-for-bit, and agrees with the Python restatement on
   fresh random cases.
"""
import json
import math
import os
import random
import struct

import numpy as np
import pytest

from oracle import go_semantics as G
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SEC, MS = 10**9, 10**6


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def hb(s):
    return int(s, 16)


# ---------------------------------------------------------------- (1) ----
def test_take_known_answer_reference_table():
    """bucket_test.go:35-66 verbatim: Rate{5, 1s}, 8 sequential steps."""
    rate = G.Rate(5, SEC)
    interval = rate.interval()
    assert interval == 200 * MS
    b = G.Bucket(created=1_600_000_000 * SEC)
    now = b.created
    table = [(MS, 1, True, 4), (MS, 1, True, 3), (MS, 3, True, 0), (interval, 1, True, 0),
             (interval, 2, False, 1), (MS, 1, True, 0), (MS, 1, False, 0), (SEC, 0, True, 5)]
    for dt, n, ok, rem in table:
        now += dt
        r, o, _ = b.take(now, rate, n)
        assert (o, r) == (ok, rem)
    # final state added=12.0 taken=7.0 elapsed=1.405e9
    assert (b.added, b.taken, b.elapsed) == (12.0, 7.0, 1_405_000_000)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_merge_crdt_laws_reference_shape(seed):
    """bucket_test.go:68-114 with a fixed seed (the reference seeds from time)."""
    rng = random.Random(seed)
    buckets = [G.Bucket(added=rng.random(), taken=rng.random(), elapsed=rng.getrandbits(63))
               for _ in range(100)]
    seq = G.Bucket()
    for b in buckets:
        seq.merge(seq, b)
    for _ in range(300):
        rng.shuffle(buckets)
        r = G.Bucket()
        for b in buckets:
            r.merge(b, b)
        assert (r.added, r.taken, r.elapsed) == (seq.added, seq.taken, seq.elapsed)


def test_codec_round_trip_quickcheck():
    """bucket_test.go:10-34: Marshal→Unmarshal is lossless (bitwise for floats)."""
    rng = random.Random(7)
    for _ in range(5000):
        name = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 232))).decode("latin-1")
        b = G.Bucket(name=name, added=G.b2f(rng.getrandbits(64)), taken=G.b2f(rng.getrandbits(64)),
                     elapsed=rng.randrange(-(1 << 63), 1 << 63))
        d = G.Bucket()
        assert d.unmarshal(b.marshal())
        assert (d.name, G.f2b(d.added), G.f2b(d.taken), d.elapsed) == \
               (b.name, G.f2b(b.added), G.f2b(b.taken), b.elapsed)
    with pytest.raises(ValueError):
        G.Bucket(name="x" * 232).marshal()


def test_api_reference_table():
    """api_test.go:34-73 (the HTTP layer is out of scope; the handler logic is not)."""
    repo = G.LocalRepo(G.Bucket(name="foo", created=1))
    assert G.api_take(repo, "A" * 232, "", "", 10) == (400, "bucket name larger than 231")
    assert G.api_take(repo, "default-rate", "", "", 10) == (429, "0")
    assert G.api_take(repo, "default-count", "2:s", "", 10) == (200, "1")
    assert G.api_take(repo, "pass", "2:s", "1", 10) == (200, "1")
    assert G.api_take(repo, "fail", "0:s", "1", 10) == (429, "0")


# ---------------------------------------------------------------- (2) ----
def test_c_oracle_take_known_answer_fixture():
    g = load("take_known_answer.json")
    st = [0.0, 0.0, 0]
    for s in g["steps"]:
        rem, ok, have = O.take_fields(st, g["created"], s["now"], g["freq"], g["per"], s["take"])
        assert (ok, rem) == (s["ok"], s["rem"])
        assert G.f2b(have) == hb(s["have"])
        assert (G.f2b(st[0]), G.f2b(st[1]), st[2]) == (hb(s["added"]), hb(s["taken"]), s["b_elapsed"])


def test_c_oracle_codec_fixture():
    import ctypes as C
    L = O.lib()
    g = load("codec.json")
    for c in g["round_trip"]:
        name = bytes.fromhex(c["name"])
        out = C.create_string_buffer(256)
        n = L.orc_marshal(name, len(name), G.b2f(hb(c["added"])), G.b2f(hb(c["taken"])),
                          c["elapsed"], out)
        assert out.raw[:n].hex() == c["datagram"]
        a, t, e, nl = C.c_double(), C.c_double(), C.c_int64(), C.c_uint32()
        nm = C.create_string_buffer(256)
        d = bytes.fromhex(c["datagram"])
        assert L.orc_unmarshal(d, len(d), C.byref(a), C.byref(t), C.byref(e), nm, C.byref(nl)) == 0
        assert (G.f2b(a.value), G.f2b(t.value), e.value, nm.raw[:nl.value]) == \
               (hb(c["added"]), hb(c["taken"]), c["elapsed"], name)
    for c in g["malformed"]:
        d = bytes.fromhex(c["datagram"])
        a, t, e, nl = C.c_double(), C.c_double(), C.c_int64(), C.c_uint32()
        nm = C.create_string_buffer(256)
        rc = L.orc_unmarshal(d, len(d), C.byref(a), C.byref(t), C.byref(e), nm, C.byref(nl))
        assert (rc == 0) == c["ok"]
        if c.get("name"):
            assert nm.raw[:nl.value].hex() == c["name"]


def test_c_oracle_merge_fixture():
    import ctypes as C
    L = O.lib()
    for s in load("merge_sequences.json")["sequences"]:
        a = C.c_double(G.b2f(hb(s["init"][0])))
        t = C.c_double(G.b2f(hb(s["init"][1])))
        e = C.c_int64(s["init"][2])
        for m in s["msgs"]:
            L.orc_merge_fields(C.byref(a), C.byref(t), C.byref(e), G.b2f(hb(m[0])), G.b2f(hb(m[1])), m[2])
        assert (G.f2b(a.value), G.f2b(t.value), e.value) == \
               (hb(s["final"][0]), hb(s["final"][1]), s["final"][2])


def test_c_oracle_parse_rate_fixture():
    for c in load("parse_rate.json")["cases"]:
        f, p, rc = O.parse_rate(c["rate"].encode("utf-8"))
        assert (f, p, rc == 0) == (c["freq"], c["per"], c["ok"]), c


def test_c_oracle_api_fixture():
    g = load("api_table.json")
    repo = O.Repo()
    sb = g["seed_bucket"]
    repo.seed([sb["name"].encode()], [0], [0], [0], [sb["created"]])
    for r in g["requests"]:
        code, body = repo.api_take(r["name"].encode(), r["rate"].encode(), r["count"].encode(), r["now"])
        assert (code, body) == (r["code"], r["body"]), r


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


def test_c_oracle_mixed_fixture():
    for tr in load("mixed_traces.json")["traces"]:
        repo = O.Repo()
        out = repo.apply_mixed(*_mixed_arrays(tr["ops"]))
        for i, r in enumerate(tr["results"]):
            assert out["status"][i] == r["status"], (i, tr["ops"][i])
            if "remaining" in r:
                assert int(out["remaining"][i]) == r["remaining"]
                assert int(out["have"][i]) == hb(r["have"])
            if "reply" in r:
                assert [int(out["reply_added"][i]), int(out["reply_taken"][i]),
                        int(out["reply_elapsed"][i])] == [hb(r["reply"][0]), hb(r["reply"][1]), r["reply"][2]]
        dump = repo.dump()
        want = {k.encode(): (hb(v[0]), hb(v[1]), v[2], v[3]) for k, v in tr["final"].items()}
        assert dump == want


def test_c_oracle_receive_fixture():
    for b in load("receive_batches.json")["batches"]:
        repo = O.Repo()
        if b["seed"]:
            repo.seed([s["name"].encode() for s in b["seed"]], [hb(s["added"]) for s in b["seed"]],
                      [hb(s["taken"]) for s in b["seed"]], [s["elapsed"] for s in b["seed"]],
                      [s["created"] for s in b["seed"]])
        dgs = [bytes.fromhex(d) for d in b["datagrams"]]
        st, ra, rt, re, stop = repo.receive(dgs, b["now"])
        assert list(st) == b["status"]
        for i, r in enumerate(b["replies"]):
            if r:
                assert [int(ra[i]), int(rt[i]), int(re[i])] == [hb(r[0]), hb(r[1]), r[2]]
        want = {k.encode(): (hb(v[0]), hb(v[1]), v[2], v[3]) for k, v in b["final"].items()}
        assert repo.dump() == want


def test_c_vs_python_take_random():
    """Fresh random Take/merge chains: the two restatements agree bitwise."""
    rng = random.Random(11)
    sp = [0.0, -0.0, 1.0, -1.0, math.inf, -math.inf, math.nan, 1e300, -1e-300, 100.0]
    for _ in range(2000):
        created = rng.randrange(-(1 << 62), 1 << 62)
        pb = G.Bucket(created=created, added=rng.choice(sp + [rng.random() * 200]),
                      taken=rng.choice(sp + [rng.random() * 200]),
                      elapsed=rng.choice([0, rng.randrange(0, 1 << 62), (1 << 63) - 1]))
        st = [pb.added, pb.taken, pb.elapsed]
        for _ in range(10):
            now = created + rng.randrange(-(1 << 40), 1 << 63 if rng.random() < 0.1 else 1 << 40)
            now = max(-(1 << 63), min((1 << 63) - 1, now))
            freq = rng.choice([0, 1, 3, 5, 100, -7, 1 << 62, -(1 << 63)])
            per = rng.choice([0, SEC, 3, -SEC, 1 << 62, -(1 << 63)])
            n = rng.choice([0, 1, 2, 100, 1 << 63, (1 << 64) - 1])
            r1, o1, h1 = pb.take(now, G.Rate(freq, per), n)
            r2, o2, h2 = O.take_fields(st, created, now, freq, per, n)
            assert (r1, o1, G.f2b(h1)) == (r2, o2, G.f2b(h2))
            assert (G.f2b(pb.added), G.f2b(pb.taken), pb.elapsed) == (G.f2b(st[0]), G.f2b(st[1]), st[2])


def test_go_u64_conversion_edges():
    for x in [0.0, -0.0, -0.5, -1.0, -1.7, 0.9, 2.0**63, 2.0**63 + 2048, 2.0**64, 1e300, -1e300,
              math.nan, math.inf, -math.inf, 18446744073709549568.0, -9223372036854775808.0]:
        assert O.go_f64_to_u64(x) == G.go_f64_to_u64(x), x
    assert G.go_f64_to_u64(-1.7) == (1 << 64) - 1
    assert G.go_f64_to_u64(math.nan) == 1 << 63
    assert G.go_f64_to_u64(2.0**64) == 1 << 63


def test_fnv1a():
    assert O.fnv1a64(b"") == 0xCBF29CE484222325
    assert O.fnv1a64(b"a") == 0xAF63DC4C8601EC8C
    for s in [b"foo", b"b123", b"x" * 231]:
        assert O.fnv1a64(s) == G.fnv1a64(s)


def test_bench_mixed_mt_matches_serial_stream_order():
    """The CPU baseline's multi-threaded mixed stream (orc_bench_mixed_mt:
    each bucket's ops on one worker in stream order) gives exactly the
    single-threaded stream's statuses, remaining and table."""
    import numpy as np
    from oracle import oracle as O
    from tests import _gen
    rng = np.random.default_rng(12)
    n, K = 20000, 500
    ids = _gen.zipf_ids(rng, n, K)
    names = _gen.key_names(ids)
    blob, offs = O._names_blob(names)
    kind = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.5, 0.4, 0.1])
    now = _gen.T0 + np.arange(n, dtype=np.int64) * 1000
    freq = np.full(n, 100, np.int64)
    per = np.full(n, 10**9, np.int64)
    cnt = np.ones(n, np.uint64)
    a, t, e = _gen.dirty_states(rng, n, 0.1)
    outs = []
    for th in (1, 7):
        r = O.Repo()
        st = np.zeros(n, np.uint8)
        rm = np.zeros(n, np.uint64)
        f = r.L.orc_bench_mixed if th == 1 else r.L.orc_bench_mixed_mt
        extra = () if th == 1 else (th,)
        f(r.h, kind, blob, offs, n, now, freq, per, cnt, a, t, e, st, rm, *extra)
        outs.append((st, np.where(kind == 0, rm, 0), r.dump()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]
