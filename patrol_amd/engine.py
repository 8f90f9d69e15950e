"""Python mirror of Patrol's Repo seam over libpatrolhip.

Patrol (Go) exposes its bucket map through the `Repo` interface
(repo.go:15-18) and drives it from two loops: the UDP `Receive` loop
(repo.go:54-92) and the HTTP `takeBucket` handler (api.go:51-86).  A
device-resident table cannot hand out mutable `*Bucket` pointers, so the
unit of work here is a batch of ops, each with the exact Go semantics in
batch order (include/patrolhip.h).  This module is a thin ctypes layer used by
the tests and bench.py; a Go deployment binds the same C ABI with cgo
(INTEGRATION.md).

Arrays may be numpy (host) or torch CUDA tensors (device, zero-copy: the
call then passes PHIP_DEVICE_PTRS).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import (DEVICE_PTRS, phip_config, phip_msgs, phip_ops, phip_results, phip_state,
                   phip_take_reply)


class PatrolHipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libpatrolhip error {code} ({_lib.PHIP_ERR.get(code, '?')}): {msg}")
        self.code = code


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _ptr(x):
    if x is None:
        return None
    if _is_torch(x):
        return x.data_ptr()
    return x.ctypes.data


def _names_len(names, names_len=None):
    """phip_msgs / phip_ops names_len of a device names blob: the length the
    device checks every name offset against (patrolhip.h), by default the
    blob's own size; 0 (or a blob past 4 GiB) leaves the offsets unchecked."""
    if names_len is not None:
        return int(names_len)
    nb = int(names.numel() * names.element_size()) if _is_torch(names) else int(names.nbytes)
    return nb if 0 < nb < (1 << 32) else 0


def _np(x, dtype):
    if x is None:
        return None
    a = np.ascontiguousarray(x, dtype=dtype)
    return a if a.size else np.zeros(1, dtype)


def names_blob(names: Sequence[bytes]):
    """list[bytes] -> (blob uint8 (8 bytes of read slack), offsets uint32[n+1])."""
    offs = np.zeros(len(names) + 1, dtype=np.uint32)
    if len(names):
        offs[1:] = np.cumsum(np.fromiter((len(x) for x in names), np.int64, len(names)))
    blob = np.zeros(int(offs[-1]) + 8, dtype=np.uint8)
    if offs[-1]:
        blob[:offs[-1]] = np.frombuffer(b"".join(names), dtype=np.uint8)
    return blob, offs


@dataclass
class BucketState:
    """A Bucket's replicated fields plus its local `created` (bucket.go:20-32)."""
    added: int      # float64 bits
    taken: int      # float64 bits
    elapsed: int    # ns
    created: int    # ns since the Unix epoch

    @property
    def added_f(self) -> float:
        return float(np.array([self.added], np.uint64).view(np.float64)[0])

    @property
    def taken_f(self) -> float:
        return float(np.array([self.taken], np.uint64).view(np.float64)[0])


class GPURepo:
    """A device-resident bucket map (the LocalRepo of repo.go:171-235)."""

    def __init__(self, device: int = 0, log2_slots: int = 20, arena_bytes: int = 1 << 24,
                 max_load_pct: int = 90, debug_tag_bits: int = 0, grow: bool = True,
                 small: bool = True, hash_seed: int | None = None, isolate: bool = False):
        """hash_seed: None = a random placement seed per handle (the default,
        as Go's map seeds its hash per process); an int pins it
        (PHIP_CFG_FIXED_SEED; 0 = the unseeded placement).  isolate: set every
        Receive batch's dirty buckets apart (PHIP_CFG_ISOLATE; by default only
        after a dirty batch)."""
        self.L = _lib.load()
        flags = (0 if grow else _lib.CFG_NO_GROW) | (0 if small else _lib.CFG_NO_SMALL)
        if isolate:
            flags |= _lib.CFG_ISOLATE
        if hash_seed is not None:
            flags |= _lib.CFG_FIXED_SEED
        cfg = phip_config(device, log2_slots, arena_bytes, max_load_pct, debug_tag_bits, flags, 0,
                          (hash_seed or 0) & (2**64 - 1))
        h = C.c_void_p()
        rc = self.L.phip_open(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise PatrolHipError(rc, "phip_open failed")
        self.h = h
        self.device = device
        self.owned = True

    @classmethod
    def wrap(cls, handle, device: int):
        """A GPURepo over a handle someone else owns (a GPUGroup member)."""
        r = cls.__new__(cls)
        r.L, r.h, r.device, r.owned = _lib.load(), C.c_void_p(handle), device, False
        return r

    # ------------------------------------------------------------ basics --
    def close(self):
        if getattr(self, "h", None) and getattr(self, "owned", True):
            self.L.phip_close(self.h)
        self.h = None
        self._queued = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self.L.phip_len(self.h))

    @property
    def capacity(self) -> int:
        return int(self.L.phip_capacity(self.h))

    def _check(self, rc: int, allow=()):
        if rc < 0 and rc not in allow:
            raise PatrolHipError(rc, self.L.phip_last_error(self.h).decode(errors="replace"))
        return rc

    def flush(self):
        rc = self.L.phip_flush(self.h)
        self._queued = None   # the queued batch is finished (or failed)
        self._check(rc)

    def set_stream(self, stream=None):
        """Run the handle's work on `stream` (a torch.cuda.Stream, a raw
        hipStream_t int, or None for the handle's own stream).  Device-pointer
        calls whose inputs torch produces on that stream then need no
        synchronisation between the two."""
        raw = getattr(stream, "cuda_stream", stream)
        self._check(self.L.phip_set_stream(self.h, C.c_void_p(raw) if raw else None))

    def use_torch_stream(self):
        """set_stream(torch's current stream on this device).  torch's default
        stream has the handle 0, which means "the handle's own stream" here:
        make a dedicated torch stream current first (torch.cuda.set_stream)."""
        import torch
        s = torch.cuda.current_stream(self.device)
        if not s.cuda_stream:
            raise ValueError("torch's current stream is the default stream; set a torch.cuda.Stream first")
        self.set_stream(s)

    def set_timing(self, on, accumulate: bool = False):
        """Event timing per kernel; accumulate=True keeps every call's
        timings until timings() is read (for a timed loop)."""
        self.L.phip_set_timing(self.h, (2 if accumulate else 1) if on else 0)

    def last_stats(self):
        """(hot-directory entries, messages folded through it, misses) of the
        last fast-path Receive batch, the table's growths since open, and the
        batch's messages that went through the ordered path."""
        out = (C.c_uint64 * 5)()
        k = self.L.phip_last_stats(self.h, out, 5)
        return tuple(int(out[i]) for i in range(k))

    def table_stats(self):
        """dict(buckets, slots, max_probe, sum_probe): probe distances of the
        buckets from their home slots (phip_table_stats)."""
        out = (C.c_uint64 * 4)()
        k = self._check(self.L.phip_table_stats(self.h, out, 4))
        keys = ("buckets", "slots", "max_probe", "sum_probe")
        return {keys[i]: int(out[i]) for i in range(k)}

    def timings(self, max_entries: int = 1 << 14):
        names = (C.c_char_p * max_entries)()
        ms = (C.c_float * max_entries)()
        k = self.L.phip_last_timings(self.h, names, ms, max_entries)
        return [(names[i].decode(), float(ms[i])) for i in range(k)]

    # -------------------------------------------------------------- repo --
    def seed(self, names: Sequence[bytes], added, taken, elapsed, created):
        """NewLocalRepo(clock, bs...) (repo.go:179-185): buckets as given."""
        blob, offs = names_blob(names)
        n = len(names)
        st = np.zeros(max(n, 1), dtype=[("a", "<u8"), ("t", "<u8"), ("e", "<i8"), ("c", "<i8")])
        st["a"][:n], st["t"][:n] = np.asarray(added, np.uint64), np.asarray(taken, np.uint64)
        st["e"][:n], st["c"][:n] = np.asarray(elapsed, np.int64), np.asarray(created, np.int64)
        self._check(self.L.phip_seed(self.h, blob.ctypes.data, offs.ctypes.data, n,
                                     st.ctypes.data, 0))

    def seed_device(self, names, name_offs, states, n: int):
        """phip_seed with device pointers: names (uint8 CUDA tensor), name_offs
        (n+1 int32/uint32), states (n x 4 int64: added bits, taken bits,
        elapsed, created)."""
        self._check(self.L.phip_seed(self.h, _ptr(names), _ptr(name_offs), n, _ptr(states),
                                     DEVICE_PTRS))

    def get(self, name: bytes):
        """Lookup without creating (None when absent)."""
        s = phip_state()
        rc = self._check(self.L.phip_get(self.h, name, len(name), C.byref(s)))
        if rc == 0:
            return None
        return BucketState(s.added, s.taken, s.elapsed, s.created)

    def export_datagrams(self, names: Sequence[bytes]):
        """Egress batch: each named bucket's current state as its MarshalBinary
        datagram (bucket.go:51-68).  -> (list of datagrams, found uint8[n]);
        an absent bucket's datagram is zero bytes."""
        n = len(names)
        blob, offs = names_blob(names)
        out = np.zeros(25 * n + int(offs[-1]) + 1, np.uint8)
        found = np.zeros(max(n, 1), np.uint8)
        self._check(self.L.phip_export_datagrams(self.h, blob.ctypes.data, offs.ctypes.data, n,
                                                 out.ctypes.data, found.ctypes.data, 0))
        raw = out.tobytes()
        dgs = [raw[25 * i + int(offs[i]):25 * (i + 1) + int(offs[i + 1])] for i in range(n)]
        return dgs, found[:n]

    def export_states_device(self, names, name_offs, n: int):
        """phip_export_datagrams with device pointers (names uint8 CUDA tensor,
        name_offs int32[n+1]): each named bucket's MarshalBinary datagram
        (bucket.go:51-68) written on the device, then its three big-endian
        words read back as (added bits, taken bits, elapsed) int64 tensors and
        found (bool), all on the device.  An absent bucket reads as zeros."""
        import torch
        dev = names.device
        offs64 = name_offs.to(torch.int64)
        total = int(offs64[-1] - offs64[0])
        out = torch.zeros(_lib.BUCKET_FIXED_SIZE * max(n, 1) + total + 8, dtype=torch.uint8,
                          device=dev)
        found = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        self._check(self.L.phip_export_datagrams(self.h, _ptr(names), _ptr(name_offs), n,
                                                 _ptr(out), _ptr(found), DEVICE_PTRS))
        base = _lib.BUCKET_FIXED_SIZE * torch.arange(n, dtype=torch.int64, device=dev) + \
            (offs64[:-1] - offs64[0])
        words = out[base.unsqueeze(1) + torch.arange(24, device=dev).unsqueeze(0)]   # [n, 24]
        w = words.view(n, 3, 8).flip(2).contiguous().view(torch.int64).view(n, 3)   # big-endian
        return w[:, 0], w[:, 1], w[:, 2], found[:n].bool()

    def snapshot(self, path=None):
        """The table as a raw image (phip_snapshot); written to `path` if given,
        else returned as a uint8 array."""
        nb = int(self.L.phip_snapshot_bytes(self.h))
        if nb == 0:
            raise PatrolHipError(-1, "phip_snapshot_bytes failed")
        buf = np.empty(nb, np.uint8)
        self._check(self.L.phip_snapshot(self.h, buf.ctypes.data, nb))
        if path is None:
            return buf
        buf.tofile(path)
        return None

    def restore(self, src):
        """Load a snapshot (a path or a uint8 array) into this handle, which must
        have the snapshot's log2_slots (phip_restore)."""
        buf = np.fromfile(src, np.uint8) if isinstance(src, (str, bytes, os.PathLike)) else \
            np.ascontiguousarray(src, np.uint8)
        self._check(self.L.phip_restore(self.h, buf.ctypes.data, buf.size))

    def dump_arrays(self):
        """Every bucket as arrays (unordered): (names uint8, offs uint64[n+1],
        added bits, taken bits, elapsed, created) -- for tables too large for
        a dict."""
        n, nb = C.c_uint64(), C.c_uint64()
        self._check(self.L.phip_dump(self.h, None, 0, None, None, 0, C.byref(n), C.byref(nb)))
        cnt = n.value
        names = np.zeros(max(nb.value, 1), np.uint8)
        offs = np.zeros(cnt + 1, np.uint64)
        st = np.zeros(max(cnt, 1), dtype=[("a", "<u8"), ("t", "<u8"), ("e", "<i8"), ("c", "<i8")])
        self._check(self.L.phip_dump(self.h, names.ctypes.data, names.size, offs.ctypes.data,
                                     st.ctypes.data, cnt, C.byref(n), C.byref(nb)))
        st = st[:n.value]
        return (names, offs[:n.value + 1], np.ascontiguousarray(st["a"]),
                np.ascontiguousarray(st["t"]), np.ascontiguousarray(st["e"]),
                np.ascontiguousarray(st["c"]))

    def dump(self):
        """{name: BucketState} of every bucket."""
        n, nb = C.c_uint64(), C.c_uint64()
        self._check(self.L.phip_dump(self.h, None, 0, None, None, 0, C.byref(n), C.byref(nb)))
        cnt = n.value
        names = np.zeros(max(nb.value, 1), np.uint8)
        offs = np.zeros(cnt + 1, np.uint64)
        st = np.zeros(max(cnt, 1), dtype=[("a", "<u8"), ("t", "<u8"), ("e", "<i8"), ("c", "<i8")])
        self._check(self.L.phip_dump(self.h, names.ctypes.data, names.size, offs.ctypes.data,
                                     st.ctypes.data, cnt, C.byref(n), C.byref(nb)))
        raw = names.tobytes()
        return {raw[int(offs[i]):int(offs[i + 1])]:
                BucketState(int(st["a"][i]), int(st["t"][i]), int(st["e"][i]), int(st["c"][i]))
                for i in range(n.value)}

    # ---------------------------------------------------------- hot path --
    @staticmethod
    def _results(n, want_remaining=False, want_reply=False):
        status = np.zeros(max(n, 1), np.uint8)
        rem = np.zeros(max(n, 1), np.uint64) if want_remaining else None
        have = np.zeros(max(n, 1), np.uint64) if want_remaining else None
        reply = (np.zeros(max(n, 1), dtype=[("a", "<u8"), ("t", "<u8"), ("e", "<i8"), ("c", "<i8")])
                 if want_reply else None)
        res = phip_results(status.ctypes.data, _ptr(rem), _ptr(have), _ptr(reply))
        return res, status, rem, have, reply

    def receive_datagrams(self, datagrams: Sequence[bytes], now: int):
        """ReplicatedRepo.Receive over raw datagrams (repo.go:54-92).

        Returns dict(status, reply, stop) — `stop` is the index of the first
        malformed datagram (the Go loop returns io.ErrShortBuffer there) or n.
        """
        n = len(datagrams)
        offs = np.zeros(n + 1, np.uint64)
        if n:
            offs[1:] = np.cumsum([len(d) for d in datagrams])
        blob = np.zeros(int(offs[-1]) + 8, np.uint8)
        if offs[-1]:
            blob[:offs[-1]] = np.frombuffer(b"".join(datagrams), np.uint8)
        res, status, _, _, reply = self._results(n, want_reply=True)
        stop = C.c_uint32()
        self._check(self.L.phip_receive_datagrams(self.h, blob.ctypes.data, offs.ctypes.data, n,
                                                  int(now), C.byref(res), C.byref(stop), 0),
                    allow=(-5,))
        return dict(status=status[:n], reply=reply[:n], stop=stop.value)

    def receive_datagrams_device(self, data, offs, n: int, now: int, status=None):
        """phip_receive_datagrams with device pointers: data (uint8 CUDA tensor
        of back-to-back datagrams, 8 bytes of slack), offs (int64[n+1]).
        Returns the index of the first malformed datagram (n if none)."""
        res = phip_results(_ptr(status), None, None, None)
        stop = C.c_uint32(0)
        rc = self.L.phip_receive_datagrams(self.h, _ptr(data), _ptr(offs), n, int(now),
                                           C.byref(res), C.byref(stop), DEVICE_PTRS)
        if rc not in (0, -5):
            self._check(rc)
        return stop.value

    def receive_soa(self, names, added, taken, elapsed, now: int, name_offs=None, n=None,
                    status=None, device=False, reply=None, queue=False, names_len=None):
        """Receive over decoded states.  With device=True every array is a torch
        CUDA tensor (names = uint8 blob, name_offs = int32/uint32 offsets;
        reply: an int64 [n, 4] tensor for the phip_state replies).
        queue=True (device only): PHIP_RECV_ASYNC, the batch is finished by
        the handle's next call or flush(); the binding holds the batch's
        tensors until the next receive or flush(), so that the caching
        allocator cannot hand their memory to another tensor meanwhile.
        names_len (device only): the blob length the device checks the name
        offsets against (phip_msgs.names_len); default the blob's size, 0 =
        unchecked."""
        fl = _lib.RECV_ASYNC if queue else 0
        if device:
            m = phip_msgs(n, _names_len(names, names_len), _ptr(names), _ptr(name_offs),
                          _ptr(added), _ptr(taken), _ptr(elapsed))
            res = phip_results(_ptr(status), None, None, _ptr(reply))
            rc = self.L.phip_receive_soa(self.h, C.byref(m), int(now), C.byref(res),
                                         DEVICE_PTRS | fl)
            self._queued = ((names, name_offs, added, taken, elapsed, status, reply)
                            if queue and rc == 0 else None)
            self._check(rc)
            return None
        n = len(names)
        blob, offs = names_blob(names)
        a, t, e = _np(added, np.uint64), _np(taken, np.uint64), _np(elapsed, np.int64)
        m = phip_msgs(n, 0, blob.ctypes.data, offs.ctypes.data, a.ctypes.data, t.ctypes.data,
                      e.ctypes.data)
        res, st, _, _, reply = self._results(n, want_reply=True)
        self._check(self.L.phip_receive_soa(self.h, C.byref(m), int(now), C.byref(res), fl))
        return dict(status=st[:n], reply=reply[:n])

    def upsert_soa(self, names, added, taken, elapsed, now: int):
        """LocalRepo.UpsertBucket for each state (repo.go:215-235)."""
        n = len(names)
        blob, offs = names_blob(names)
        a, t, e = _np(added, np.uint64), _np(taken, np.uint64), _np(elapsed, np.int64)
        m = phip_msgs(n, 0, blob.ctypes.data, offs.ctypes.data, a.ctypes.data, t.ctypes.data,
                      e.ctypes.data)
        res, st, _, _, _ = self._results(n)
        self._check(self.L.phip_upsert_soa(self.h, C.byref(m), int(now), C.byref(res), 0))
        return dict(status=st[:n])

    def apply_mixed(self, kind, names, now, freq=None, per=None, count=None, added=None,
                    taken=None, elapsed=None):
        """Ordered TAKE/RECEIVE/UPSERT stream (api.go:67-74, repo.go:78-90, :215-235)."""
        n = len(names)
        blob, offs = names_blob(names)
        arrs = dict(kind=_np(kind, np.uint8), now=_np(now, np.int64), freq=_np(freq, np.int64),
                    per=_np(per, np.int64), count=_np(count, np.uint64),
                    added=_np(added, np.uint64), taken=_np(taken, np.uint64),
                    elapsed=_np(elapsed, np.int64))
        ops = phip_ops(n, 0, _ptr(arrs["kind"]), blob.ctypes.data, offs.ctypes.data,
                       _ptr(arrs["now"]), _ptr(arrs["freq"]), _ptr(arrs["per"]), _ptr(arrs["count"]),
                       _ptr(arrs["added"]), _ptr(arrs["taken"]), _ptr(arrs["elapsed"]))
        res, st, rem, have, reply = self._results(n, want_remaining=True, want_reply=True)
        self._check(self.L.phip_apply_mixed(self.h, C.byref(ops), C.byref(res), 0))
        return dict(status=st[:n], remaining=rem[:n], have=have[:n], reply=reply[:n])

    def apply_mixed_device(self, n, kind, names, name_offs, now, freq=None, per=None, count=None,
                           added=None, taken=None, elapsed=None, status=None, remaining=None,
                           have=None, names_len=None):
        """apply_mixed with every array a torch CUDA tensor (PHIP_DEVICE_PTRS);
        names_len as receive_soa's."""
        ops = phip_ops(n, _names_len(names, names_len), _ptr(kind), _ptr(names), _ptr(name_offs),
                       _ptr(now), _ptr(freq),
                       _ptr(per), _ptr(count), _ptr(added), _ptr(taken), _ptr(elapsed))
        res = phip_results(_ptr(status), _ptr(remaining), _ptr(have), None)
        self._check(self.L.phip_apply_mixed(self.h, C.byref(ops), C.byref(res), DEVICE_PTRS))

    def take(self, names, now, freq, per, count):
        """Batched Bucket.Take via GetBucket (create) then Take: (remaining, ok)."""
        n = len(names)
        blob, offs = names_blob(names)
        now, freq, per = _np(now, np.int64), _np(freq, np.int64), _np(per, np.int64)
        count = _np(count, np.uint64)
        rem = np.zeros(max(n, 1), np.uint64)
        ok = np.zeros(max(n, 1), np.uint8)
        self._check(self.L.phip_take(self.h, blob.ctypes.data, offs.ctypes.data, n, now.ctypes.data,
                                     freq.ctypes.data, per.ctypes.data, count.ctypes.data,
                                     rem.ctypes.data, ok.ctypes.data, 0))
        return rem[:n], ok[:n].astype(bool)

    def api_take(self, name: bytes, rate: bytes, count: bytes, now: int):
        """API.takeBucket (api.go:51-86): (HTTP status, body)."""
        body = C.create_string_buffer(64)
        bl = C.c_uint32()
        code = self._check(self.L.phip_api_take(self.h, name, len(name), rate, len(rate), count,
                                                len(count), int(now), body, C.byref(bl)))
        return code, body.raw[:bl.value].decode()


class GPUGroup:
    """A shard group over RCCL (phip_group_*, include/patrolhip.h): the
    buckets hash-sharded by name over several GPUs, owner-routed Receive and
    anti-entropy in the C library (no torch on the data path).

    open_all(devices): one process, every listed GPU (ncclCommInitAll);
    open_rank(repo, uid, nranks, rank): one process per GPU around `repo`
    (ncclCommInitRank), `uid` from unique_id() on rank 0."""

    def __init__(self, g, L, repos):
        self.g, self.L, self.repos = g, L, repos

    @staticmethod
    def unique_id() -> bytes:
        L = _lib.load()
        buf = C.create_string_buffer(_lib.GROUP_ID_BYTES)
        rc = L.phip_group_unique_id(buf)
        if rc != 0:
            raise PatrolHipError(rc, "phip_group_unique_id failed")
        return buf.raw

    @classmethod
    def open_all(cls, devices, log2_slots: int = 20, arena_bytes: int = 1 << 24,
                 max_load_pct: int = 90):
        L = _lib.load()
        cfg = phip_config(0, log2_slots, arena_bytes, max_load_pct, 0, 0, 0, 0)
        devs = (C.c_int32 * len(devices))(*devices)
        g = C.c_void_p()
        rc = L.phip_group_open_all(C.byref(cfg), devs, len(devices), C.byref(g))
        if rc != 0:
            raise PatrolHipError(rc, "phip_group_open_all failed")
        repos = [GPURepo.wrap(L.phip_group_handle(g, i), devices[i]) for i in range(len(devices))]
        return cls(g, L, repos)

    @classmethod
    def open_rank(cls, repo: "GPURepo", uid: bytes, nranks: int, rank: int):
        L = repo.L
        g = C.c_void_p()
        rc = L.phip_group_open_rank(repo.h, uid, nranks, rank, C.byref(g))
        if rc != 0:
            raise PatrolHipError(rc, "phip_group_open_rank failed")
        return cls(g, L, [repo])

    @property
    def world(self) -> int:
        return int(self.L.phip_group_world(self.g))

    def _check(self, rc):
        if rc != 0:
            raise PatrolHipError(rc, self.L.phip_group_last_error(self.g).decode(errors="replace"))

    def receive(self, batches, now: int, combine: bool = True, rccl_self: bool = False,
                small_chunks: bool = False):
        """batches: one (names uint8, name_offs int32[n+1], added, taken, elapsed)
        tuple of CUDA tensors per local member -> (sent, merged) lists.
        rccl_self (PHIP_GROUP_RCCL_SELF, testing): every segment, the
        member's own included, travels through ncclSend/ncclRecv.
        small_chunks (PHIP_GROUP_SMALL_CHUNKS, testing): the pipelined
        exchange runs in chunks of 4096 messages."""
        k = len(batches)
        msgs = (phip_msgs * k)()
        for i, (names, offs, a, t, e) in enumerate(batches):
            msgs[i] = phip_msgs(offs.numel() - 1, _names_len(names), _ptr(names), _ptr(offs), _ptr(a), _ptr(t),
                                _ptr(e))
        sent, merged = (C.c_uint64 * k)(), (C.c_uint64 * k)()
        flags = DEVICE_PTRS | (_lib.ROUTE_COMBINE if combine else 0) | \
            (_lib.GROUP_RCCL_SELF if rccl_self else 0) | \
            (_lib.GROUP_SMALL_CHUNKS if small_chunks else 0)
        self._check(self.L.phip_group_receive(self.g, msgs, int(now), sent, merged, flags))
        return [int(x) for x in sent], [int(x) for x in merged]

    def set_timing(self, on: bool = True):
        """phip_group_set_timing: per-stage event timing of later calls."""
        self._check(self.L.phip_group_set_timing(self.g, 1 if on else 0))

    def stage_ms(self, i: int = 0):
        """phip_group_stage_ms: member i's busy ms of the last call per stage
        -> dict(pack, exchange, merge) (anti-entropy: local join, all-reduce,
        apply)."""
        ms = (C.c_float * 3)()
        self._check(self.L.phip_group_stage_ms(self.g, i, ms))
        return dict(pack=float(ms[0]), exchange=float(ms[1]), merge=float(ms[2]))

    def rccl_info(self, i: int = 0):
        """phip_group_rccl_info: the RCCL member i runs on -> dict(version,
        comm_count, lib_path, mapped): `mapped` lists every librccl this
        process has mapped (/proc/self/maps), to show one copy is shared."""
        v, c = C.c_int32(), C.c_int32()
        buf = C.create_string_buffer(4096)
        self._check(self.L.phip_group_rccl_info(self.g, i, C.byref(v), C.byref(c), buf, 4096))
        mapped = set()
        try:
            with open("/proc/self/maps") as f:
                for line in f:
                    p = line.split()[-1] if len(line.split()) >= 6 else ""
                    if "librccl" in p:
                        mapped.add(os.path.realpath(p))
        except OSError:
            pass
        return dict(version=int(v.value), comm_count=int(c.value),
                    lib_path=os.path.realpath(buf.value.decode()) if buf.value else None,
                    mapped=sorted(mapped))

    def anti_entropy(self, replicas):
        """replicas: one contiguous int64 CUDA tensor [R, 3, B] per local member."""
        R, three, B = replicas[0].shape
        ptrs = (C.c_void_p * len(replicas))(*[x.data_ptr() for x in replicas])
        self._check(self.L.phip_group_anti_entropy(self.g, ptrs, R, B, DEVICE_PTRS))

    def close(self):
        if getattr(self, "g", None):
            for r in self.repos:
                if not r.owned:
                    r.h = None
            self.L.phip_group_close(self.g)
            self.g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TakeBatcher:
    """Request-coalescing Take batcher over a GPURepo (phip_batcher_*,
    include/patrolhip.h): the drop-in form of the POST /take handler
    (api.go:51-86) for one-request-per-thread callers.  take()/api_take()
    block until the request's batch ran; they release the GIL (ctypes), so
    many Python threads can wait at once."""

    def __init__(self, repo: "GPURepo", window_us: int = 20, max_batch: int = 0):
        self.repo, self.L = repo, repo.L
        b = C.c_void_p()
        cfg = _lib.phip_batcher_config(window_us, max_batch)
        repo._check(self.L.phip_batcher_open(repo.h, C.byref(cfg), C.byref(b)))
        self.b = b

    def close(self):
        if getattr(self, "b", None):
            self.L.phip_batcher_close(self.b)
            self.b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def take(self, name: bytes, now: int, freq: int, per: int, count: int):
        """-> (remaining, ok, arrival seq)."""
        rem, ok, seq = C.c_uint64(), C.c_uint8(), C.c_uint64()
        rc = self.L.phip_batcher_take(self.b, name, len(name), int(now), int(freq), int(per),
                                      int(count), C.byref(rem), C.byref(ok), C.byref(seq))
        if rc != 0:
            raise PatrolHipError(rc, "phip_batcher_take failed")
        return rem.value, bool(ok.value), seq.value

    def api_take(self, name: bytes, rate: bytes, count: bytes, now: int):
        """API.takeBucket through the batcher: (HTTP status, body)."""
        body = C.create_string_buffer(64)
        bl = C.c_uint32()
        code = self.L.phip_batcher_api_take(self.b, name, len(name), rate, len(rate), count,
                                            len(count), int(now), body, C.byref(bl))
        if code < 0:
            raise PatrolHipError(code, "phip_batcher_api_take failed")
        return code, body.raw[:bl.value].decode()

    @staticmethod
    def _reply(r):
        st = r.state
        return dict(remaining=int(r.remaining), ok=bool(r.ok), created=bool(r.created),
                    seq=int(r.seq), state=BucketState(st.added, st.taken, st.elapsed, st.created),
                    datagram=bytes(r.datagram[:r.datagram_len]))

    def take_reply(self, name: bytes, now: int, freq: int, per: int, count: int):
        """A Take with everything the handler replicates (phip_batcher_take_reply):
        dict(remaining, ok, created, seq, state, datagram)."""
        r = phip_take_reply()
        rc = self.L.phip_batcher_take_reply(self.b, name, len(name), int(now), int(freq), int(per),
                                            int(count), C.byref(r))
        if rc != 0:
            raise PatrolHipError(rc, "phip_batcher_take_reply failed")
        return self._reply(r)

    def api_take_reply(self, name: bytes, rate: bytes, count: bytes, now: int):
        """API.takeBucket plus its replication (phip_batcher_api_take_reply):
        (HTTP status, body, reply dict)."""
        body = C.create_string_buffer(64)
        bl = C.c_uint32()
        r = phip_take_reply()
        code = self.L.phip_batcher_api_take_reply(self.b, name, len(name), rate, len(rate), count,
                                                  len(count), int(now), body, C.byref(bl),
                                                  C.byref(r))
        if code < 0:
            raise PatrolHipError(code, "phip_batcher_api_take_reply failed")
        return code, body.raw[:bl.value].decode(), self._reply(r)

    def stats(self):
        """dict(batches, requests, max_batch, gpu_ns, errors)."""
        out = (C.c_uint64 * 5)()
        k = self.L.phip_batcher_stats(self.b, out, 5)
        keys = ("batches", "requests", "max_batch", "gpu_ns", "errors")
        return {keys[i]: int(out[i]) for i in range(k)}


class Ring:
    """Pinned ingest ring over a GPURepo (phip_ring_*, include/patrolhip.h):
    the batched form of the Receive goroutine (repo.go:54-92).  Slots are
    filled in host memory (fill(), or recv() from a UDP socket), submitted
    (an async host->device copy on the ring's own stream) and received in
    order; submitting slot k+1 before receiving slot k overlaps its copy with
    slot k's merge."""

    def __init__(self, repo: "GPURepo", nslots: int = 3, max_msgs: int = 1 << 16,
                 max_bytes: int | None = None):
        self.repo, self.L = repo, repo.L
        self.max_msgs = max_msgs
        self.max_bytes = max_bytes if max_bytes is not None else 256 * max_msgs
        r = C.c_void_p()
        repo._check(self.L.phip_ring_open(repo.h, nslots, max_msgs, self.max_bytes, C.byref(r)))
        self.r = r
        self._views = {}

    def close(self):
        if getattr(self, "r", None):
            self.L.phip_ring_close(self.r)
            self.r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def acquire(self):
        """-> (slot, bytes view uint8[max_bytes], offs view uint64[max_msgs+1])."""
        slot, b, o = C.c_uint32(), C.c_void_p(), C.c_void_p()
        self.repo._check(self.L.phip_ring_acquire(self.r, C.byref(slot), C.byref(b), C.byref(o)))
        bv = np.ctypeslib.as_array(C.cast(b, C.POINTER(C.c_uint8)), (self.max_bytes,))
        ov = np.ctypeslib.as_array(C.cast(o, C.POINTER(C.c_uint64)), (self.max_msgs + 1,))
        return slot.value, bv, ov

    def fill(self, datagrams: Sequence[bytes]):
        """Acquire a slot and pack `datagrams` into it -> (slot, n)."""
        slot, bv, ov = self.acquire()
        n = len(datagrams)
        if n > self.max_msgs:
            raise ValueError("batch larger than the ring's slots")
        ov[0] = 0
        if n:
            ov[1:n + 1] = np.cumsum([len(d) for d in datagrams])
            bv[:int(ov[n])] = np.frombuffer(b"".join(datagrams), np.uint8)
        return slot, n

    def recv(self, sock, timeout_ms: int = 3000, peers: bool = True):
        """Acquire a slot and fill it from a UDP socket (phip_udp_recv_batch)
        -> (slot, n, peers uint8[n, PEER_BYTES] or None)."""
        slot, bv, ov = self.acquire()
        pbuf = np.zeros((self.max_msgs, _lib.PEER_BYTES), np.uint8) if peers else None
        n = C.c_uint32()
        self.repo._check(self.L.phip_udp_recv_batch(sock.fileno(), bv.ctypes.data, self.max_bytes,
                                                    ov.ctypes.data, self.max_msgs, _ptr(pbuf),
                                                    int(timeout_ms), C.byref(n)))
        return slot, n.value, (pbuf[:n.value] if peers else None)

    def submit(self, slot: int, n: int):
        self.repo._check(self.L.phip_ring_submit(self.r, slot, n))

    def receive(self, slot: int, n: int, now: int, want_reply: bool = True,
                want_status: bool = True, status=None):
        """-> dict(status, reply, stop) as GPURepo.receive_datagrams.
        `status`: a caller uint8[>= n] array to fill instead of a new one."""
        if status is not None:
            res, reply = phip_results(status.ctypes.data, None, None, None), None
        elif want_status or want_reply:
            res, status, _, _, reply = GPURepo._results(n, want_reply=want_reply)
        else:
            res, reply = None, None
        stop = C.c_uint32()
        self.repo._check(self.L.phip_ring_receive(self.r, slot, int(now),
                                                  C.byref(res) if res is not None else None,
                                                  C.byref(stop)), allow=(-5,))
        return dict(status=status[:n] if status is not None else None,
                    reply=reply[:n] if reply is not None else None, stop=stop.value)


def udp_send_batch(sock, data: bytes | np.ndarray, offs: np.ndarray, peers=None,
                   peer_stride: int = 0) -> int:
    """sendmmsg of datagrams data[offs[i]:offs[i+1]] (phip_udp_send_batch)."""
    L = _lib.load()
    buf = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else data
    offs = np.ascontiguousarray(offs, np.uint64)
    sent = C.c_uint32()
    rc = L.phip_udp_send_batch(sock.fileno(), buf.ctypes.data if buf.size else None,
                               offs.ctypes.data, len(offs) - 1, _ptr(peers), peer_stride,
                               C.byref(sent))
    if rc != 0:
        raise PatrolHipError(rc, "sendmmsg failed")
    return sent.value


def udp_recv_batch(sock, max_msgs: int, timeout_ms: int = 3000, cap: int | None = None):
    """recvmmsg into plain host arrays (phip_udp_recv_batch) ->
    (list of datagrams, peers uint8[n, PEER_BYTES])."""
    L = _lib.load()
    cap = cap if cap is not None else 256 * max_msgs
    buf = np.zeros(cap + 8, np.uint8)
    offs = np.zeros(max_msgs + 1, np.uint64)
    peers = np.zeros((max(max_msgs, 1), _lib.PEER_BYTES), np.uint8)
    n = C.c_uint32()
    rc = L.phip_udp_recv_batch(sock.fileno(), buf.ctypes.data, cap, offs.ctypes.data, max_msgs,
                               peers.ctypes.data, int(timeout_ms), C.byref(n))
    if rc != 0:
        raise PatrolHipError(rc, "recvmmsg failed")
    k = n.value
    return [bytes(buf[int(offs[i]):int(offs[i + 1])]) for i in range(k)], peers[:k]


def incast_replies(data: np.ndarray, offs: np.ndarray, status, reply, peers=None):
    """phip_incast_replies -> (packed replies uint8, offs uint64[m+1], peers or None)."""
    L = _lib.load()
    n = len(offs) - 1
    status = np.ascontiguousarray(status, np.uint8)
    cap = 256 * max(n, 1)
    out = np.zeros(cap, np.uint8)
    oo = np.zeros(n + 1, np.uint64)
    op = np.zeros((max(n, 1), _lib.PEER_BYTES), np.uint8) if peers is not None else None
    m = C.c_uint32()
    rc = L.phip_incast_replies(data.ctypes.data, offs.ctypes.data, n, status.ctypes.data,
                               reply.ctypes.data, _ptr(peers), out.ctypes.data, cap,
                               oo.ctypes.data, _ptr(op), C.byref(m))
    if rc != 0:
        raise PatrolHipError(rc, "incast replies")
    k = m.value
    return out[:int(oo[k])], oo[:k + 1], (op[:k] if op is not None else None)


def parse_rate(s: bytes):
    """ParseRate (bucket.go:102-123): (freq, per_ns, ok) with Go's error values."""
    L = _lib.load()
    f, p = C.c_int64(), C.c_int64()
    rc = L.phip_parse_rate(s, len(s), C.byref(f), C.byref(p))
    return f.value, p.value, rc == 0


def marshal(name: bytes, state: BucketState) -> bytes:
    """Bucket.MarshalBinary (bucket.go:51-68)."""
    L = _lib.load()
    out = C.create_string_buffer(256)
    st = phip_state(state.added, state.taken, state.elapsed, state.created)
    n = L.phip_marshal(name, len(name), C.byref(st), out)
    if n < 0:
        raise PatrolHipError(n, "bucket name larger than 231")
    return out.raw[:n]
