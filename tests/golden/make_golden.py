"""Generate the golden fixtures under tests/golden/ from the pure-Python
restatement of the Go reference (oracle/go_semantics.py).

The Go reference itself cannot run in this container (no Go toolchain: see
DESIGN.md §2).  These vectors are therefore produced by the Python
restatement, which tests/test_oracle.py first pins against the reference's
own known-answer tests (bucket_test.go, api_test.go), and they are then used
to check the C++ oracle and the HIP engine bit-for-bit.

Run:  python tests/golden/make_golden.py   (deterministic; fixed seeds)
"""
from __future__ import annotations

import json
import math
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import go_semantics as G  # noqa: E402

SEC = 10**9
MS = 10**6
T0 = 1_700_000_000_000_000_000   # synthetic clock origin (ns), as SURVEY §8d


def bits(x: float) -> str:
    return "%016x" % G.f2b(x)


def special_floats():
    return [0.0, -0.0, 1.0, -1.0, 0.5, 1e-310, -1e-310, 5e-324, 1.7976931348623157e308,
            math.inf, -math.inf, math.nan, G.b2f(0xFFF8000000000000), G.b2f(0x7FF0000000000001),
            G.b2f(0xFFF0000000000001), 100.0, 99.99999999999999, 1e6, 2.0**63, 2.0**64,
            -2.0**63, -0.3, -1.7, 3.0]


def take_known_answer():
    """bucket_test.go:35-66, replayed with intermediate states."""
    rate = G.Rate(5, SEC)
    interval = rate.interval()
    rows = [(MS, 1, True, 4), (MS, 1, True, 3), (MS, 3, True, 0), (interval, 1, True, 0),
            (interval, 2, False, 1), (MS, 1, True, 0), (MS, 1, False, 0), (SEC, 0, True, 5)]
    b = G.Bucket(created=T0)
    now = T0
    out = []
    for dt, n, ok, rem in rows:
        now += dt
        r, o, have = b.take(now, rate, n)
        assert (o, r) == (ok, rem), (dt, n, o, r)
        out.append(dict(elapsed_ns=dt, take=n, ok=ok, rem=rem, now=now, have=bits(have),
                        added=bits(b.added), taken=bits(b.taken), b_elapsed=b.elapsed))
    return dict(source="bucket_test.go:35-66", freq=5, per=SEC, created=T0, steps=out)


def codec_vectors(rng):
    cases = []
    names = [b"", b"a", b"foo", b"b1234567", bytes(range(32, 64)), b"x" * 231, b"\x00\xff\x80"]
    for nm in names:
        for a in special_floats()[:8]:
            e = rng.randrange(-(1 << 63), 1 << 63)
            t = rng.choice(special_floats())
            b = G.Bucket(name=nm.decode("latin-1"), added=a, taken=t, elapsed=e)
            cases.append(dict(name=nm.hex(), added=bits(a), taken=bits(t), elapsed=e,
                              datagram=b.marshal().hex()))
    for _ in range(200):
        nm = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40)))
        a = G.b2f(rng.getrandbits(64))
        t = G.b2f(rng.getrandbits(64))
        e = rng.randrange(-(1 << 63), 1 << 63)
        b = G.Bucket(name=nm.decode("latin-1"), added=a, taken=t, elapsed=e)
        cases.append(dict(name=nm.hex(), added=bits(a), taken=bits(t), elapsed=e,
                          datagram=b.marshal().hex()))
    # malformed inputs for UnmarshalBinary (bucket.go:72-87)
    bad = []
    full = G.Bucket(name="hello", added=1.0, taken=2.0, elapsed=3).marshal()
    for cut in [0, 1, 24, 25, 26, 29]:
        d = full[:cut]
        ok = G.Bucket().unmarshal(d)
        bad.append(dict(datagram=d.hex(), ok=ok))
    trailing = full + b"trailing-bytes"
    bb = G.Bucket()
    ok = bb.unmarshal(trailing)
    bad.append(dict(datagram=trailing.hex(), ok=ok, name=bb.name.encode("latin-1").hex()))
    return dict(source="bucket.go:51-91", round_trip=cases, malformed=bad)


def merge_sequences(rng):
    """Sequential Merge folds (bucket.go:240-263) incl. ±0/NaN/negatives."""
    sp = special_floats()
    seqs = []
    for k in range(300):
        init = G.Bucket(added=rng.choice(sp), taken=rng.choice(sp),
                        elapsed=rng.choice([0, -5, 7, -(1 << 63), (1 << 63) - 1]))
        if k % 3 == 0:
            init = G.Bucket()
        msgs = []
        for _ in range(rng.randrange(1, 12)):
            if rng.random() < 0.6:
                a, t = rng.choice(sp), rng.choice(sp)
            else:
                a, t = rng.random() * 10 - 2, rng.random() * 10 - 2
            e = rng.choice([0, 3, -3, rng.randrange(-(1 << 63), 1 << 63)])
            msgs.append((a, t, e))
        b = G.Bucket(added=init.added, taken=init.taken, elapsed=init.elapsed)
        for a, t, e in msgs:
            b.merge(G.Bucket(added=a, taken=t, elapsed=e))
        seqs.append(dict(init=[bits(init.added), bits(init.taken), init.elapsed],
                         msgs=[[bits(a), bits(t), e] for a, t, e in msgs],
                         final=[bits(b.added), bits(b.taken), b.elapsed]))
    return dict(source="bucket.go:240-263", sequences=seqs)


def parse_rate_table():
    cases = ["", "5", "5:s", "5:1s", "2:s", "0:s", "100:1s", "3:1s", "10:m", "1:h", "7:ms",
             "7:µs", "7:μs", "7:us", "7:ns", "1:1.5h", "4:2h45m", "-5:s", "+5:s", "5:-1s",
             "abc:s", "5:abc", "5:", ":s", "99999999999999999999:s", "-99999999999999999999:s",
             "9223372036854775807:s", "5:1.0000000001s", "5:.5s", "5:5.s", "5:.s", "5:1",
             "5:0", "5:-0", "5:1e3s", "1:2562047h47m16.854775807s", "1:2562047h47m16.854775808s",
             "1:9223372036854775807ns", "1:9223372036854775808ns", "1:-9223372036854775808ns",
             "50:1s", "1_000:s", " 5:s", "5: s", "5:s:extra", "12345678901234567890:s",
             "123456789012345678:s", "5:3m20.5s", "5:0.000000001s", "5:1.23456789012ms"]
    out = []
    for c in cases:
        r, ok = G.parse_rate(c)
        out.append(dict(rate=c, freq=r.freq, per=r.per, ok=ok))
    return dict(source="bucket.go:102-123", cases=out)


def api_table():
    """api_test.go:34-73 plus handler edge cases (api.go:51-86)."""
    now = T0
    repo = G.LocalRepo(G.Bucket(name="foo", created=now))
    reqs = [("A" * 232, "", ""), ("default-rate", "", ""), ("default-count", "2:s", ""),
            ("pass", "2:s", "1"), ("fail", "0:s", "1"), ("A" * 231, "1:s", ""),
            ("big", "10:s", "99999999999999999999"), ("zero", "10:s", "0"),
            ("neg", "-3:s", "1"), ("bad", "x:s", "1"), ("huge", "99999999999999999999:s", "5"),
            ("foo", "5:s", "2"), ("foo", "5:s", "2"), ("foo", "5:s", "2")]
    out = []
    for i, (name, rate, count) in enumerate(reqs):
        code, body = G.api_take(repo, name, rate, count, now + i * MS)
        out.append(dict(name=name, rate=rate, count=count, now=now + i * MS, code=code, body=body))
    expect = {0: (400, G.ERR_NAME_TOO_LARGE), 1: (429, "0"), 2: (200, "1"), 3: (200, "1"),
              4: (429, "0")}
    for i, (c, b) in expect.items():     # the reference's own assertions
        assert (out[i]["code"], out[i]["body"]) == (c, b), (i, out[i])
    return dict(source="api_test.go:34-73", seed_bucket=dict(name="foo", created=now), requests=out)


def mixed_traces(rng):
    """Ordered Take/Merge streams over a few buckets (api.go:67-74, repo.go:78-90);
    traces 40.. also carry UpsertBucket ops (kind 2, repo.go:215-235)."""
    traces = []
    rates = [(100, SEC), (5, SEC), (3, SEC), (0, SEC), (7, 0), (2, 3), (1, MS), (-5, SEC),
             (10, -SEC), (-1, -(1 << 63)), (1 << 62, SEC), (9, 60 * SEC)]
    sp = special_floats()
    for k in range(52):
        names = ["k%d" % j for j in range(rng.randrange(1, 5))]
        now = T0 + rng.randrange(0, 10**12)
        ops = []
        for _ in range(rng.randrange(5, 60)):
            name = rng.choice(names)
            now += rng.choice([0, 1, 7, MS, 10 * MS, 200 * MS, SEC, -5 * MS])
            if rng.random() < 0.6:
                f, p = rng.choice(rates) if rng.random() < 0.5 else rates[k % len(rates)]
                n = rng.choice([0, 1, 1, 1, 2, 3, 10, 1 << 63, (1 << 64) - 1])
                ops.append(dict(kind=0, name=name, now=now, freq=f, per=p, count=n))
            else:
                if rng.random() < 0.3:
                    a, t, e = rng.choice(sp), rng.choice(sp), rng.choice([0, 5, -5, SEC])
                elif rng.random() < 0.2:
                    a, t, e = 0.0, rng.choice([0.0, -0.0]), 0
                else:
                    t = float(rng.randrange(0, 50))
                    a = t + rng.random() * 10
                    e = rng.randrange(0, 10 * SEC)
                kind = 2 if k >= 40 and rng.random() < 0.35 else 1
                ops.append(dict(kind=kind, name=name, now=now, added=bits(a), taken=bits(t),
                                elapsed=e))
        repo = G.LocalRepo()
        res = []
        for op in ops:
            if op["kind"] == 0:
                st, rem, have = repo.take(op["name"], op["now"], G.Rate(op["freq"], op["per"]),
                                          op["count"])
                res.append(dict(status=st, remaining=rem, have=bits(have)))
            elif op["kind"] == 2:
                remote = G.Bucket(name=op["name"], added=G.b2f(int(op["added"], 16)),
                                  taken=G.b2f(int(op["taken"], 16)), elapsed=op["elapsed"])
                res.append(dict(status=repo.upsert(remote, op["now"])))
            else:
                remote = G.Bucket(name=op["name"], added=G.b2f(int(op["added"], 16)),
                                  taken=G.b2f(int(op["taken"], 16)), elapsed=op["elapsed"])
                st, reply = repo.receive_one(remote, op["now"])
                r = dict(status=st)
                if reply:
                    r["reply"] = ["%016x" % reply[0], "%016x" % reply[1], reply[2]]
                res.append(r)
        final = {nm: [bits(b.added), bits(b.taken), b.elapsed, b.created]
                 for nm, b in sorted(repo.buckets.items())}
        traces.append(dict(ops=ops, results=res, final=final))
    return dict(source="bucket.go:186-263, repo.go:54-92,179-235, api.go:67-74", traces=traces)


def receive_batches(rng):
    """Receive loop over datagram batches (repo.go:54-92) incl. incast and short."""
    batches = []
    for k in range(20):
        seed = []
        for j in range(rng.randrange(0, 4)):
            seed.append(dict(name="s%d" % j, added=bits(float(j)), taken=bits(0.0),
                             elapsed=j, created=T0 - SEC))
        repo = G.LocalRepo(*[G.Bucket(name=s["name"], added=G.b2f(int(s["added"], 16)),
                                      taken=0.0, elapsed=s["elapsed"], created=s["created"])
                             for s in seed])
        dgs = []
        pool = ["s0", "s1", "s2", "n0", "n1", "n2", "n3"]
        for _ in range(rng.randrange(1, 40)):
            nm = rng.choice(pool)
            r = rng.random()
            if r < 0.25:
                b = G.Bucket(name=nm)                          # incast request
            elif r < 0.3:
                b = G.Bucket(name=nm, added=-0.0)              # IsZero with -0
            else:
                b = G.Bucket(name=nm, added=rng.random() * 100, taken=rng.random() * 50,
                             elapsed=rng.randrange(0, 10**9))
            dgs.append(b.marshal())
        if k % 5 == 4:
            pos = rng.randrange(0, len(dgs))
            dgs.insert(pos, dgs[pos][:rng.randrange(0, 25)])   # short datagram
        if k % 7 == 3:
            dgs.append(dgs[0] + b"junk")                       # trailing bytes ignored
        now = T0 + k * SEC
        res = repo.receive(dgs, now)
        final = {nm: [bits(b.added), bits(b.taken), b.elapsed, b.created]
                 for nm, b in sorted(repo.buckets.items())}
        batches.append(dict(seed=seed, now=now, datagrams=[d.hex() for d in dgs],
                            status=[s for s, _ in res],
                            replies=[["%016x" % r[0], "%016x" % r[1], r[2]] if r else None
                                     for _, r in res],
                            final=final))
    return dict(source="repo.go:54-92,108-120,160-169", batches=batches)


def write(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=None, separators=(",", ":"), ensure_ascii=True)
        f.write("\n")


def main():
    write("take_known_answer.json", take_known_answer())
    write("codec.json", codec_vectors(random.Random(1)))
    write("merge_sequences.json", merge_sequences(random.Random(2)))
    write("parse_rate.json", parse_rate_table())
    write("api_table.json", api_table())
    write("mixed_traces.json", mixed_traces(random.Random(3)))
    write("receive_batches.json", receive_batches(random.Random(4)))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
