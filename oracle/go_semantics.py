"""ORACLE — test infrastructure only.

An independent pure-Python restatement of calavera/patrol's bucket-state hot
path, written separately from oracle/patrol_oracle.cc so the two can
cross-check each other.  It generates the golden vectors under tests/golden/
(see tests/golden/make_golden.py).  Python floats are IEEE-754 binary64 with
correctly rounded + - / and ordered comparisons, i.e. the same arithmetic Go
uses on amd64 for bucket.go; Go's int64 wrap-around and conversion rules are
emulated explicitly.

Parity pinning: checked against the reference's own tests
(bucket_test.go:35-66, :68-114, :10-34; api_test.go:34-73) in
tests/test_oracle.py.  Never imported by the product path.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

MASK64 = (1 << 64) - 1
INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1

BUCKET_FIXED_SIZE = 8 + 8 + 8 + 1          # bucket.go:36
BUCKET_PACKET_SIZE = 256                   # bucket.go:41
MAX_BUCKET_NAME_LENGTH = BUCKET_PACKET_SIZE - BUCKET_FIXED_SIZE   # bucket.go:44
ERR_NAME_TOO_LARGE = "bucket name larger than %d" % MAX_BUCKET_NAME_LENGTH  # bucket.go:48


def f2b(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def b2f(b: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", b & MASK64))[0]


def wrap64(v: int) -> int:
    v &= MASK64
    return v - (1 << 64) if v >> 63 else v


def _cvttsd2sq(x: float) -> int:
    """x86-64 CVTTSD2SQ: trunc toward zero, NaN/out-of-range -> 0x8000..."""
    if not (-9223372036854775808.0 <= x < 9223372036854775808.0):
        return INT64_MIN
    return int(x)


def go_f64_to_u64(x: float) -> int:
    """Go uint64(float64) as compiled for amd64 (ssagen floatToUint)."""
    if x < 9223372036854775808.0:
        return _cvttsd2sq(x) & MASK64
    return (_cvttsd2sq(x - 9223372036854775808.0) & MASK64) | (1 << 63)


# --------------------------------------------------------------- Rate ----
@dataclass
class Rate:                       # bucket.go:96-99
    freq: int = 0
    per: int = 0

    def is_zero(self) -> bool:    # bucket.go:126-128
        return self.freq == 0 or self.per == 0

    def interval(self) -> int:    # bucket.go:146-148, Go truncating int64 division
        q = abs(self.per) // abs(self.freq)
        if (self.per < 0) != (self.freq < 0):
            q = -q
        return wrap64(q)

    def tokens(self, d: int) -> float:   # bucket.go:132-143
        if self.is_zero():
            return 0.0
        iv = self.interval()
        if iv == 0:
            return 0.0
        return float(d) / float(iv)


def go_parse_uint10(s: str):
    """strconv.ParseUint(s, 10, 64) -> (value, ok): syntax 0, range MaxUint64."""
    if s == "":
        return 0, False
    n = 0
    for c in s:
        if not ("0" <= c <= "9"):
            return 0, False
        n = n * 10 + (ord(c) - 48)
        if n > MASK64:
            return MASK64, False
    return n, True


def go_atoi(s: str):
    """strconv.Atoi on 64-bit -> (value, ok)."""
    if 0 < len(s) < 19:
        t = s
        if t[0] in "+-":
            t = t[1:]
            if not t:
                return 0, False
        v = 0
        for c in t:
            if not ("0" <= c <= "9"):
                return 0, False
            v = v * 10 + ord(c) - 48
        return (-v if s[0] == "-" else v), True
    if s == "":
        return 0, False
    neg = s[0] == "-"
    t = s[1:] if s[0] in "+-" else s
    # ParseUint scans left to right: syntax and range errors in the order met.
    n = 0
    rng = False
    if t == "":
        return 0, False
    for c in t:
        if not ("0" <= c <= "9"):
            return 0, False
        n = n * 10 + ord(c) - 48
        if n > MASK64:
            rng = True
            n = MASK64
            break
    if not neg and n >= (1 << 63):
        return INT64_MAX, False
    if neg and n > (1 << 63):
        return INT64_MIN, False
    if rng:
        return (INT64_MIN if neg else INT64_MAX), False
    return (-n if neg else n), True


_UNITS = {"ns": 1, "us": 1000, "µs": 1000, "μs": 1000, "ms": 10**6,
          "s": 10**9, "m": 60 * 10**9, "h": 3600 * 10**9}


def go_parse_duration(s: str):
    """time.ParseDuration -> (ns, ok); any error gives 0 like Go."""
    b = s.encode("utf-8")
    neg = False
    if b[:1] in (b"-", b"+"):
        neg = b[:1] == b"-"
        b = b[1:]
    if b == b"0":
        return 0, True
    if b == b"":
        return 0, False
    d = 0
    while b:
        if not (b[:1] == b"." or b"0" <= b[:1] <= b"9"):
            return 0, False
        i, v = 0, 0
        while i < len(b) and 48 <= b[i] <= 57:
            if v > (1 << 63) // 10:
                return 0, False
            v = v * 10 + b[i] - 48
            if v > (1 << 63):
                return 0, False
            i += 1
        pre = i > 0
        b = b[i:]
        post = False
        f, scale = 0, 1.0
        if b[:1] == b".":
            b = b[1:]
            j, over = 0, False
            while j < len(b) and 48 <= b[j] <= 57:
                if not over:
                    if f > ((1 << 63) - 1) // 10:
                        over = True
                    else:
                        y = f * 10 + b[j] - 48
                        if y > (1 << 63):
                            over = True
                        else:
                            f = y
                            scale *= 10
                j += 1
            post = j > 0
            b = b[j:]
        if not pre and not post:
            return 0, False
        k = 0
        while k < len(b) and not (b[k] == 46 or 48 <= b[k] <= 57):
            k += 1
        if k == 0:
            return 0, False
        unit = _UNITS.get(b[:k].decode("utf-8", "replace"))
        b = b[k:]
        if unit is None:
            return 0, False
        if v > (1 << 63) // unit:
            return 0, False
        v *= unit
        if f > 0:
            v += int(float(f) * (float(unit) / scale))
            if v > (1 << 63):
                return 0, False
        d += v
        if d > (1 << 63):
            return 0, False
    if neg:
        return wrap64(-d), True
    if d > (1 << 63) - 1:
        return 0, False
    return d, True


def parse_rate(v: str):
    """bucket.go:102-123 -> (Rate, ok) with the value Go returns beside err."""
    ps = v.split(":", 1)
    if len(ps) == 1:
        ps.append("1s")
    freq, ok = go_atoi(ps[0])
    if not ok:
        return Rate(freq, 0), False
    unit = ps[1]
    if unit in ("ns", "us", "µs", "ms", "s", "m", "h"):   # bucket.go:117
        unit = "1" + unit
    per, ok = go_parse_duration(unit)
    return Rate(freq, per), ok


# ------------------------------------------------------------- Bucket ----
@dataclass
class Bucket:                     # bucket.go:20-32 (created: int64 ns)
    name: str = ""
    added: float = 0.0
    taken: float = 0.0
    elapsed: int = 0
    created: int = 0

    def is_zero(self) -> bool:    # bucket.go:165-170
        return self.added == 0 and self.taken == 0 and self.elapsed == 0

    def merge(self, *others: "Bucket") -> None:   # bucket.go:240-263
        for o in others:
            if o is self:
                continue
            if self.added < o.added:
                self.added = o.added
            if self.taken < o.taken:
                self.taken = o.taken
            if self.elapsed < o.elapsed:
                self.elapsed = o.elapsed

    def take(self, now: int, r: Rate, n: int):     # bucket.go:186-225
        capacity = float(r.freq)
        if self.added == 0:
            self.added = capacity
        last = self.created + self.elapsed          # exact (time.Time range)
        if now < last:
            last = now
        tokens = self.added - self.taken
        dt = now - last
        dt = max(INT64_MIN, min(INT64_MAX, dt))     # time.Time.Sub saturates
        added = r.tokens(dt)
        missing = capacity - tokens
        if added > missing:
            added = missing
        taken = float(n)
        have = tokens + added
        if taken > have:
            return go_f64_to_u64(have), False, have
        self.elapsed = wrap64(self.elapsed + dt)
        self.added += added
        self.taken += taken
        rem = self.added - self.taken
        return go_f64_to_u64(rem), True, rem

    def marshal(self) -> bytes:    # bucket.go:51-68
        nb = self.name.encode("latin-1") if isinstance(self.name, str) else self.name
        if len(nb) > MAX_BUCKET_NAME_LENGTH:
            raise ValueError(ERR_NAME_TOO_LARGE)
        return (struct.pack(">QQQ", f2b(self.added), f2b(self.taken), self.elapsed & MASK64)
                + bytes([len(nb)]) + nb)

    def unmarshal(self, data: bytes) -> bool:      # bucket.go:71-91
        if len(data) < BUCKET_FIXED_SIZE:
            return False
        a, t, e = struct.unpack(">QQQ", data[:24])
        self.added, self.taken, self.elapsed = b2f(a), b2f(t), wrap64(e)
        nl = data[24]
        if len(data) - 25 < nl:
            return False
        self.name = data[25:25 + nl].decode("latin-1")
        return True


# Status codes (mirror include/patrolhip.h).
MERGED, INCAST_REPLY, INCAST_NOREPLY, SHORT, NOT_PROCESSED, TAKE_OK, TAKE_DENIED = 1, 2, 3, 4, 5, 6, 7
UPSERT_INSERTED = 8
CREATED = 0x80


class LocalRepo:                  # repo.go:171-235
    def __init__(self, *bs: Bucket):
        self.buckets = {b.name: b for b in bs}

    def get_bucket(self, name: str, clock: int):    # repo.go:189-211
        b = self.buckets.get(name)
        if b is not None:
            return b, True
        b = Bucket(name=name, created=clock)
        self.buckets[name] = b
        return b, False

    def upsert_bucket(self, b: Bucket, clock: int):  # repo.go:215-235
        prev = self.buckets.get(b.name)
        if prev is b:
            return prev, True
        if prev is None:
            b.created = clock
            self.buckets[b.name] = b
            return b, False
        prev.merge(b)
        return prev, True

    def receive_one(self, remote: Bucket, now: int):  # repo.go:78-90
        local, existed = self.get_bucket(remote.name, now)
        reply = None
        if not remote.is_zero():
            local.merge(remote)
            st = MERGED
        elif existed and not local.is_zero():
            st = INCAST_REPLY
            reply = (f2b(local.added), f2b(local.taken), local.elapsed)
        else:
            st = INCAST_NOREPLY
        return st | (0 if existed else CREATED), reply

    def receive(self, datagrams, now: int):          # repo.go:54-92
        out, remote, stopped = [], Bucket(), False
        for d in datagrams:
            if stopped:
                out.append((NOT_PROCESSED, None))
                continue
            if not remote.unmarshal(d):
                out.append((SHORT, None))
                stopped = True
                continue
            out.append(self.receive_one(remote, now))
        return out

    def take(self, name: str, now: int, r: Rate, n: int):   # api.go:67-74
        b, existed = self.get_bucket(name, now)
        rem, ok, have = b.take(now, r, n)
        return (TAKE_OK if ok else TAKE_DENIED) | (0 if existed else CREATED), rem, have

    def upsert(self, remote: Bucket, now: int):      # repo.go:215-235, a distinct state
        _, merged = self.upsert_bucket(remote, now)
        return MERGED if merged else (UPSERT_INSERTED | CREATED)

    def apply_mixed(self, ops):
        """ops: (kind, name, now, freq, per, count, added_bits, taken_bits, elapsed)
        in index order; kind 0 Take, 1 Receive, 2 Upsert.  Returns per op
        (status, remaining, have_bits, reply)."""
        out = []
        for kind, name, now, freq, per, count, ab, tb, e in ops:
            if kind == 0:
                st, rem, have = self.take(name, now, Rate(freq, per), count)
                out.append((st, rem, f2b(have), None))
                continue
            remote = Bucket(name=name, added=b2f(ab), taken=b2f(tb), elapsed=e)
            if kind == 2:
                out.append((self.upsert(remote, now), 0, 0, None))
            else:
                st, reply = self.receive_one(remote, now)
                out.append((st, 0, 0, reply))
        return out


def api_take(repo: LocalRepo, name: str, rate: str, count: str, now: int):
    """api.go:51-86 -> (status code, body)."""
    if len(name.encode("utf-8")) > MAX_BUCKET_NAME_LENGTH:
        return 400, ERR_NAME_TOO_LARGE
    r, _ = parse_rate(rate)
    n, _ = go_parse_uint10(count)
    if n == 0:
        n = 1
    b, _ = repo.get_bucket(name, now)
    rem, ok, _ = b.take(now, r, n)
    return (200 if ok else 429), str(rem)


def fnv1a64(data: bytes) -> int:
    h = 0xCBF29CE484222325
    for c in data:
        h ^= c
        h = (h * 0x100000001B3) & MASK64
    return h
