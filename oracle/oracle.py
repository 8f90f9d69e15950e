"""ORACLE — test infrastructure only.

ctypes/numpy wrapper over oracle/liboracle.so (the C++ restatement of the Go
reference, oracle/patrol_oracle.cc).  Loaded by tests/, by
__graft_entry__.smoke() as the checker and by bench.py's cpu_baseline leg;
never by the product path (patrol_amd/).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile liboracle.so from oracle/patrol_oracle.cc (make)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = C.CDLL(_LIB_PATH)
    vp = C.c_void_p
    L.orc_repo_new.restype = vp
    L.orc_repo_free.argtypes = [vp]
    L.orc_repo_len.argtypes = [vp]
    L.orc_repo_len.restype = C.c_size_t
    L.orc_repo_seed.argtypes = [vp, u8p, u32p, C.c_uint32, u64p, u64p, i64p, i64p]
    L.orc_receive.argtypes = [vp, u8p, u64p, C.c_uint32, C.c_int64, u8p, u64p, u64p, i64p]
    L.orc_receive.restype = C.c_uint32
    L.orc_receive_soa.argtypes = [vp, u8p, u32p, C.c_uint32, u64p, u64p, i64p, C.c_int64,
                                  u8p, u64p, u64p, i64p]
    L.orc_upsert_soa.argtypes = [vp, u8p, u32p, C.c_uint32, u64p, u64p, i64p, C.c_int64, u8p]
    L.orc_apply_mixed.argtypes = [vp, u8p, u8p, u32p, C.c_uint32, i64p, i64p, i64p, u64p,
                                  u64p, u64p, i64p, u8p, u64p, u64p, u64p, u64p, i64p, i64p]
    L.orc_get.argtypes = [vp, C.c_char_p, C.c_uint32, C.POINTER(C.c_uint64),
                          C.POINTER(C.c_uint64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.orc_get.restype = C.c_int
    L.orc_dump.argtypes = [vp, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                           C.c_void_p, C.c_void_p, C.c_uint64]
    L.orc_dump.restype = C.c_int64
    L.orc_parse_rate.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.orc_parse_rate.restype = C.c_int
    L.orc_parse_uint10.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_uint64)]
    L.orc_go_f64_to_u64.argtypes = [C.c_double]
    L.orc_go_f64_to_u64.restype = C.c_uint64
    L.orc_rate_interval.argtypes = [C.c_int64, C.c_int64]
    L.orc_rate_interval.restype = C.c_int64
    L.orc_rate_tokens.argtypes = [C.c_int64, C.c_int64, C.c_int64]
    L.orc_rate_tokens.restype = C.c_double
    L.orc_take_fields.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double),
                                  C.POINTER(C.c_int64), C.c_int64, C.c_int64, C.c_int64,
                                  C.c_int64, C.c_uint64, C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_double)]
    L.orc_take_fields.restype = C.c_int
    L.orc_merge_fields.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double),
                                   C.POINTER(C.c_int64), C.c_double, C.c_double, C.c_int64]
    L.orc_marshal.argtypes = [C.c_char_p, C.c_uint32, C.c_double, C.c_double, C.c_int64,
                              C.c_char_p]
    L.orc_marshal.restype = C.c_int
    L.orc_unmarshal.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_double),
                                C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_char_p,
                                C.POINTER(C.c_uint32)]
    L.orc_unmarshal.restype = C.c_int
    L.orc_api_take.argtypes = [vp, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_char_p,
                               C.c_uint32, C.c_int64, C.c_char_p, C.POINTER(C.c_uint32)]
    L.orc_api_take.restype = C.c_int
    L.orc_bench_receive.argtypes = [vp, u8p, u32p, C.c_uint64, u64p, u64p, i64p, C.c_int64,
                                    C.c_int]
    L.orc_bench_receive.restype = C.c_double
    L.orc_bench_mixed.argtypes = [vp, u8p, u8p, u32p, C.c_uint32, i64p, i64p, i64p, u64p, u64p,
                                  u64p, i64p, u8p, u64p]
    L.orc_bench_mixed.restype = C.c_double
    L.orc_bench_mixed_mt.argtypes = [vp, u8p, u8p, u32p, C.c_uint32, i64p, i64p, i64p, u64p,
                                     u64p, u64p, i64p, u8p, u64p, C.c_int]
    L.orc_bench_mixed_mt.restype = C.c_double
    L.orc_check_dump.argtypes = [vp, u8p, u64p, C.c_uint64, u64p, u64p, i64p, i64p,
                                 C.POINTER(C.c_uint64)]
    L.orc_check_dump.restype = C.c_uint64
    L.orc_fnv1a64.argtypes = [C.c_char_p, C.c_uint32]
    L.orc_fnv1a64.restype = C.c_uint64
    _lib = L
    return L


def _names_blob(names):
    """list[bytes] -> (blob uint8, offsets uint32[n+1])."""
    offs = np.zeros(len(names) + 1, dtype=np.uint32)
    if names:
        offs[1:] = np.cumsum([len(x) for x in names], dtype=np.uint64).astype(np.uint32)
    blob = np.frombuffer(b"".join(names), dtype=np.uint8).copy() if names else np.zeros(1, np.uint8)
    if blob.size == 0:
        blob = np.zeros(1, np.uint8)
    return blob, offs


class Repo:
    """The Go LocalRepo (repo.go:171-235) restated in C++."""

    def __init__(self):
        self.L = lib()
        self.h = self.L.orc_repo_new()

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_repo_free(self.h)
            self.h = None

    def __len__(self):
        return int(self.L.orc_repo_len(self.h))

    def seed(self, names, added_bits, taken_bits, elapsed, created):
        blob, offs = _names_blob(names)
        self.L.orc_repo_seed(self.h, blob, offs, len(names),
                             np.ascontiguousarray(added_bits, np.uint64),
                             np.ascontiguousarray(taken_bits, np.uint64),
                             np.ascontiguousarray(elapsed, np.int64),
                             np.ascontiguousarray(created, np.int64))

    def receive(self, datagrams, now):
        """datagrams: list[bytes] -> (status u8[n], reply a/t/e arrays, stop index)."""
        n = len(datagrams)
        offs = np.zeros(n + 1, np.uint64)
        if n:
            offs[1:] = np.cumsum([len(d) for d in datagrams])
        blob = np.frombuffer(b"".join(datagrams) or b"\0", np.uint8).copy()
        st = np.zeros(max(n, 1), np.uint8)
        ra = np.zeros(max(n, 1), np.uint64)
        rt = np.zeros(max(n, 1), np.uint64)
        re = np.zeros(max(n, 1), np.int64)
        stop = self.L.orc_receive(self.h, blob, offs, n, int(now), st, ra, rt, re)
        return st[:n], ra[:n], rt[:n], re[:n], int(stop)

    def receive_soa(self, names, added_bits, taken_bits, elapsed, now):
        n = len(names)
        blob, offs = _names_blob(names)
        st = np.zeros(max(n, 1), np.uint8)
        ra = np.zeros(max(n, 1), np.uint64)
        rt = np.zeros(max(n, 1), np.uint64)
        re = np.zeros(max(n, 1), np.int64)
        self.L.orc_receive_soa(self.h, blob, offs, n, np.ascontiguousarray(added_bits, np.uint64),
                               np.ascontiguousarray(taken_bits, np.uint64),
                               np.ascontiguousarray(elapsed, np.int64), int(now), st, ra, rt, re)
        return st[:n], ra[:n], rt[:n], re[:n]

    def upsert_soa(self, names, added_bits, taken_bits, elapsed, now):
        n = len(names)
        blob, offs = _names_blob(names)
        m = np.zeros(max(n, 1), np.uint8)
        self.L.orc_upsert_soa(self.h, blob, offs, n, np.ascontiguousarray(added_bits, np.uint64),
                              np.ascontiguousarray(taken_bits, np.uint64),
                              np.ascontiguousarray(elapsed, np.int64), int(now), m)
        return m[:n]

    def apply_mixed(self, kind, names, now, freq, per, count, added_bits, taken_bits, elapsed):
        n = len(names)
        blob, offs = _names_blob(names)
        z = max(n, 1)
        st = np.zeros(z, np.uint8)
        rem = np.zeros(z, np.uint64)
        have = np.zeros(z, np.uint64)
        ra = np.zeros(z, np.uint64)
        rt = np.zeros(z, np.uint64)
        re = np.zeros(z, np.int64)
        rc = np.zeros(z, np.int64)

        def a(x, t):
            x = np.ascontiguousarray(x, t)
            return x if x.size else np.zeros(1, t)
        self.L.orc_apply_mixed(self.h, a(kind, np.uint8), blob, offs, n, a(now, np.int64),
                               a(freq, np.int64), a(per, np.int64), a(count, np.uint64),
                               a(added_bits, np.uint64), a(taken_bits, np.uint64),
                               a(elapsed, np.int64), st, rem, have, ra, rt, re, rc)
        return dict(status=st[:n], remaining=rem[:n], have=have[:n], reply_added=ra[:n],
                    reply_taken=rt[:n], reply_elapsed=re[:n], reply_created=rc[:n])

    def get(self, name: bytes):
        a, t, e, c = C.c_uint64(), C.c_uint64(), C.c_int64(), C.c_int64()
        ok = self.L.orc_get(self.h, name, len(name), C.byref(a), C.byref(t), C.byref(e), C.byref(c))
        if not ok:
            return None
        return a.value, t.value, e.value, c.value

    def dump(self):
        """-> dict(name bytes -> (added bits, taken bits, elapsed, created))."""
        need = self.L.orc_dump(self.h, None, 0, None, None, None, None, None, 0)
        total = -need - 1
        n = len(self)
        names = np.zeros(max(total, 1), np.uint8)
        offs = np.zeros(n + 1, np.uint64)
        a = np.zeros(max(n, 1), np.uint64)
        t = np.zeros(max(n, 1), np.uint64)
        e = np.zeros(max(n, 1), np.int64)
        c = np.zeros(max(n, 1), np.int64)
        got = self.L.orc_dump(self.h, names.ctypes.data, names.size, offs.ctypes.data,
                              a.ctypes.data, t.ctypes.data, e.ctypes.data, c.ctypes.data, n)
        assert got == n, (got, n)
        nb = names.tobytes()
        return {nb[int(offs[i]):int(offs[i + 1])]: (int(a[i]), int(t[i]), int(e[i]), int(c[i]))
                for i in range(n)}

    def check_dump(self, names, offs, added, taken, elapsed, created):
        """Differences between a table dump given as arrays (GPURepo.dump_arrays)
        and this repo -> (count, index of the first differing entry)."""
        fb = C.c_uint64()
        bad = self.L.orc_check_dump(self.h, np.ascontiguousarray(names, np.uint8),
                                    np.ascontiguousarray(offs, np.uint64), len(offs) - 1,
                                    np.ascontiguousarray(added, np.uint64),
                                    np.ascontiguousarray(taken, np.uint64),
                                    np.ascontiguousarray(elapsed, np.int64),
                                    np.ascontiguousarray(created, np.int64), C.byref(fb))
        return int(bad), int(fb.value)

    def api_take(self, name: bytes, rate: bytes, count: bytes, now: int):
        body = C.create_string_buffer(64)
        bl = C.c_uint32()
        code = self.L.orc_api_take(self.h, name, len(name), rate, len(rate), count, len(count),
                                   int(now), body, C.byref(bl))
        return code, body.raw[:bl.value].decode()


def parse_rate(s: bytes):
    f, p = C.c_int64(), C.c_int64()
    rc = lib().orc_parse_rate(s, len(s), C.byref(f), C.byref(p))
    return f.value, p.value, rc


def take_fields(state, created, now, freq, per, n):
    """state: [added f64, taken f64, elapsed i64] mutated; -> (remaining, ok, have)."""
    a, t, e = C.c_double(state[0]), C.c_double(state[1]), C.c_int64(state[2])
    rem, have = C.c_uint64(), C.c_double()
    ok = lib().orc_take_fields(C.byref(a), C.byref(t), C.byref(e), int(created), int(now),
                               int(freq), int(per), int(n), C.byref(rem), C.byref(have))
    state[0], state[1], state[2] = a.value, t.value, e.value
    return rem.value, bool(ok), have.value


def go_f64_to_u64(x: float) -> int:
    return int(lib().orc_go_f64_to_u64(float(x)))


def fnv1a64(b: bytes) -> int:
    return int(lib().orc_fnv1a64(b, len(b)))
