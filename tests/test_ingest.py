"""Batched UDP ingest: the socket edge (recvmmsg /
sendmmsg / incast reply marshalling, host only) and the pinned ingest ring
(phip_ring_*, GPU).

The reference reads one datagram per iteration into a 256-byte buffer
(repo.go:54-73,108-120) and unicasts each incast reply (repo.go:86-90,
160-169).  The batched pipeline must hand the engine the same bytes the Go
loop would see, in arrival order, and send back the same reply datagrams.
Bar: bit-exact (bytes, statuses, replies, final table).
"""
import socket
import struct

import numpy as np
import pytest

from oracle import go_semantics as G
from oracle import oracle as O
from tests import _gen

SEC = 10**9


@pytest.fixture(scope="module")
def lib():
    import patrol_amd
    patrol_amd.load()
    return patrol_amd


def _pair():
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.bind(("127.0.0.1", 0))
    return rx, tx


def _peer_addr(rec):
    """sockaddr_in inside a PHIP_PEER_BYTES record -> (host, port)."""
    fam = struct.unpack_from("=H", rec, 0)[0]
    assert fam == socket.AF_INET
    port = struct.unpack_from(">H", rec, 2)[0]
    return socket.inet_ntoa(bytes(rec[4:8])), port


def _datagram(name: bytes, a: int, t: int, e: int) -> bytes:
    return struct.pack(">QQQ", a, t, e & (2**64 - 1)) + bytes([len(name)]) + name


# ------------------------------------------------------------ host only ---
def test_recv_batch_packs_datagrams_in_arrival_order(lib):
    rx, tx = _pair()
    try:
        rng = np.random.default_rng(3)
        sent = []
        for i in range(700):
            name = b"b%d" % rng.integers(0, 10**6)
            d = _datagram(name, int(rng.integers(0, 2**63)), int(rng.integers(0, 2**63)),
                          int(rng.integers(-2**62, 2**62)))
            if i % 50 == 7:
                d = d[:20]                              # malformed: shorter than the header
            if i % 61 == 3:
                d = d + bytes(300)                      # longer than Go's 256-byte buffer
            sent.append(d)
            tx.sendto(d, rx.getsockname())
        got, peers = [], []
        while len(got) < len(sent):
            dg, pr = lib.udp_recv_batch(rx, 256, timeout_ms=2000)
            assert dg, "datagrams lost on loopback"
            got += dg
            peers += [_peer_addr(p) for p in pr]
        # ReadFrom into a 256-byte buffer: a longer datagram arrives cut to 256
        assert got == [d[:256] for d in sent]
        assert set(peers) == {tx.getsockname()}
    finally:
        rx.close()
        tx.close()


def test_recv_batch_timeout_is_not_an_error(lib):
    rx, tx = _pair()
    try:
        dg, pr = lib.udp_recv_batch(rx, 64, timeout_ms=50)
        assert dg == [] and len(pr) == 0
    finally:
        rx.close()
        tx.close()


def test_recv_batch_respects_caps(lib):
    rx, tx = _pair()
    try:
        for i in range(40):
            tx.sendto(_datagram(b"b%d" % i, i, i, i), rx.getsockname())
        import time
        time.sleep(0.05)
        dg, _ = lib.udp_recv_batch(rx, 16, timeout_ms=1000)      # message cap
        assert [d[25:] for d in dg] == [b"b%d" % i for i in range(16)]
        # byte cap: a datagram is only read while a whole 256-byte window is free
        dg, _ = lib.udp_recv_batch(rx, 64, timeout_ms=1000, cap=512)
        assert 1 <= len(dg) < 24
        assert [d[25:] for d in dg] == [b"b%d" % i for i in range(16, 16 + len(dg))]
        used = sum(len(d) for d in dg)
        assert used <= 512 and used + 256 > 512
        dg, _ = lib.udp_recv_batch(rx, 64, timeout_ms=1000)
        assert [d[25:] for d in dg][-1] == b"b39"
    finally:
        rx.close()
        tx.close()


def test_incast_replies_marshal_like_go(lib):
    """phip_incast_replies = Bucket.MarshalBinary (bucket.go:51-68) of the
    reply state under each INCAST_REPLY datagram's name, in batch order."""
    rng = np.random.default_rng(5)
    n = 300
    names = [b"b%d" % i if i % 7 else b"long-bucket-name-%d" % i for i in range(n)]
    dgs = [_datagram(nm, 0, 0, 0) for nm in names]
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(d) for d in dgs])
    data = np.frombuffer(b"".join(dgs), np.uint8).copy()
    status = rng.choice([1, 2, 3, 2 | 0x80], n).astype(np.uint8)
    reply = np.zeros(n, dtype=[("a", "<u8"), ("t", "<u8"), ("e", "<i8"), ("c", "<i8")])
    reply["a"] = rng.integers(0, 2**63, n, dtype=np.uint64)
    reply["t"] = rng.integers(0, 2**63, n, dtype=np.uint64)
    reply["e"] = rng.integers(-2**62, 2**62, n)
    peers = rng.integers(0, 256, (n, 128)).astype(np.uint8)
    out, oo, op = lib.incast_replies(data, offs, status, reply, peers)
    want = [i for i in range(n) if (status[i] & 0x7F) == 2]
    exp = []
    for i in want:
        b = G.Bucket(names[i].decode("latin-1"))
        b.added, b.taken = G.b2f(int(reply["a"][i])), G.b2f(int(reply["t"][i]))
        b.elapsed = int(reply["e"][i])
        exp.append(b.marshal())
    assert len(oo) == len(want) + 1
    assert [bytes(out[int(oo[k]):int(oo[k + 1])]) for k in range(len(want))] == exp
    assert np.array_equal(op, peers[want])


def test_send_batch_to_one_peer_and_to_each_peer(lib):
    rx1, tx = _pair()
    rx2 = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx2.bind(("127.0.0.1", 0))
    try:
        dgs = [_datagram(b"b%d" % i, i, 2 * i, 3 * i) for i in range(500)]
        offs = np.zeros(len(dgs) + 1, np.uint64)
        offs[1:] = np.cumsum([len(d) for d in dgs])
        data = np.frombuffer(b"".join(dgs), np.uint8).copy()
        # stride 0: the whole egress batch to one peer (one sendmmsg run)
        _, pr = _recv_some(lib, rx1, tx, [b"x"])
        peer1 = pr[0].copy()   # tx's address as recvmmsg reports it
        # address records for rx1 and rx2, alternating
        p1 = _sockaddr(rx1.getsockname())
        p2 = _sockaddr(rx2.getsockname())
        assert lib.udp_send_batch(tx, data, offs, p1[None, :], 0) == len(dgs)
        got = _drain(lib, rx1, len(dgs))
        assert got == dgs
        peers = np.stack([p1 if i % 2 == 0 else p2 for i in range(len(dgs))])
        assert lib.udp_send_batch(tx, data, offs, peers, 128) == len(dgs)
        assert _drain(lib, rx1, 250) == dgs[0::2]
        assert _drain(lib, rx2, 250) == dgs[1::2]
        assert _peer_addr(peer1) == tx.getsockname()
    finally:
        rx1.close()
        rx2.close()
        tx.close()


def _sockaddr(addr):
    rec = np.zeros(128, np.uint8)
    struct.pack_into("=H", rec, 0, socket.AF_INET)
    struct.pack_into(">H", rec, 2, addr[1])
    rec[4:8] = np.frombuffer(socket.inet_aton(addr[0]), np.uint8)
    return rec


def _recv_some(lib, rx, tx, payloads):
    for p in payloads:
        tx.sendto(p, rx.getsockname())
    return lib.udp_recv_batch(rx, len(payloads), timeout_ms=2000)


def _drain(lib, rx, n):
    got = []
    while len(got) < n:
        dg, _ = lib.udp_recv_batch(rx, n - len(got), timeout_ms=2000)
        assert dg, "datagrams lost on loopback"
        got += dg
    return got


# ----------------------------------------------------------------- GPU ---
def _batches(rng, K, nb, n):
    """nb batches of wire datagrams: clean merges, new buckets, incasts,
    -0.0 / NaN fields, long names, and one malformed datagram in batch 2."""
    out = []
    for b in range(nb):
        ids = _gen.zipf_ids(rng, n, K + 500)
        names = [(b"a-long-replicated-bucket-name-%d" % i) if i % 53 == 0 else b"b%d" % i
                 for i in ids]
        a, t, e = _gen.dirty_states(rng, n) if b % 2 else _gen.clean_states(rng, n)
        dgs = [_datagram(names[i], int(a[i]), int(t[i]), int(e[i])) for i in range(n)]
        if b % 3 == 1:     # incast requests: all-zero states
            for i in range(0, n, 37):
                dgs[i] = _datagram(names[i], 0, 0, 0)
        if b == 2:
            dgs[n // 2] = dgs[n // 2][:24]
        out.append(dgs)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("n", [40000, 700])
def test_ring_pipeline_vs_oracle(lib, n):
    """Slots submitted one ahead of the receive (copy k+1 overlaps merge k):
    statuses, replies, stop index and the final table equal the oracle's
    Receive loop over the same datagrams (700: small slots, merged from the
    pinned host bytes in one launch)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(21)
    K = 5000
    names = _gen.key_names(np.arange(K))
    a, t, e = _gen.clean_states(rng, K)
    created = _gen.T0 - rng.integers(0, SEC, K)
    g = lib.GPURepo(log2_slots=15)
    g.seed(names, a, t, e, created)
    o = O.Repo()
    o.seed(names, a, t, e, created)
    batches = _batches(rng, K, 6, n)
    ring = lib.Ring(g, nslots=3, max_msgs=n)
    pending = []
    for k, dgs in enumerate(batches):
        slot, n = ring.fill(dgs)
        ring.submit(slot, n)
        pending.append((slot, n, k))
        if len(pending) == 2:
            slot0, n0, k0 = pending.pop(0)
            _check_batch(ring.receive(slot0, n0, _gen.T0 + k0 * SEC), o, batches[k0], k0)
    for slot0, n0, k0 in pending:
        _check_batch(ring.receive(slot0, n0, _gen.T0 + k0 * SEC), o, batches[k0], k0)
    gd = {k: (v.added, v.taken, v.elapsed, v.created) for k, v in g.dump().items()}
    assert gd == o.dump()
    ring.close()
    g.close()


def _check_batch(out, o, dgs, k):
    st, ra, rt, re, stop = o.receive(dgs, _gen.T0 + k * SEC)
    assert out["stop"] == stop
    assert np.array_equal(out["status"], st), k
    rep = (st & 0x7F) == 2
    assert rep.any() or k % 3 != 1
    assert np.array_equal(out["reply"]["a"][rep], ra[rep])
    assert np.array_equal(out["reply"]["t"][rep], rt[rep])
    assert np.array_equal(out["reply"]["e"][rep], re[rep])


@pytest.mark.gpu
def test_ring_slot_states(lib):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = lib.GPURepo(log2_slots=10)
    ring = lib.Ring(g, nslots=2, max_msgs=8)
    s0, n0 = ring.fill([_datagram(b"b1", 1, 0, 0)])
    s1, n1 = ring.fill([_datagram(b"b2", 2, 0, 0)])
    with pytest.raises(lib.PatrolHipError):      # both slots held
        ring.acquire()
    ring.submit(s0, n0)
    ring.submit(s1, n1)
    with pytest.raises(lib.PatrolHipError):      # out of submission order
        ring.receive(s1, n1, _gen.T0)
    assert list(ring.receive(s0, n0, _gen.T0)["status"]) == [1 | 0x80]
    assert list(ring.receive(s1, n1, _gen.T0)["status"]) == [1 | 0x80]
    assert len(g) == 2
    ring.close()
    g.close()


@pytest.mark.gpu
def test_udp_round_trip_through_ring(lib):
    """Peer -> recvmmsg into a ring slot -> GPU Receive -> incast replies
    marshalled and sent back with sendmmsg: the peer gets exactly the
    datagrams the Go loop's unicast would send (repo.go:86-90)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(8)
    K = 300
    names = _gen.key_names(np.arange(K))
    a, t, e = _gen.clean_states(rng, K)
    created = np.full(K, _gen.T0)
    g = lib.GPURepo(log2_slots=12)
    g.seed(names, a, t, e, created)
    o = O.Repo()
    o.seed(names, a, t, e, created)
    rx, tx = _pair()
    try:
        ids = rng.integers(0, K + 50, 600)
        ma, mt, me = _gen.clean_states(rng, 600)
        dgs = [_datagram(b"b%d" % i, 0, 0, 0) if j % 3 == 0 else
               _datagram(b"b%d" % i, int(ma[j]), int(mt[j]), int(me[j])) for j, i in enumerate(ids)]
        for d in dgs:
            tx.sendto(d, rx.getsockname())
        ring = lib.Ring(g, nslots=2, max_msgs=1024)
        got = []
        now = _gen.T0 + SEC
        all_replies = []
        while len(got) < len(dgs):
            slot, n, peers = ring.recv(rx, timeout_ms=2000)
            assert n, "datagrams lost on loopback"
            ring.submit(slot, n)
            out = ring.receive(slot, n, now)
            batch = dgs[len(got):len(got) + n]
            st, ra, rt, re, stop = o.receive(batch, now)
            assert np.array_equal(out["status"], st)
            data = np.frombuffer(b"".join(batch), np.uint8).copy()
            offs = np.zeros(n + 1, np.uint64)
            offs[1:] = np.cumsum([len(d) for d in batch])
            rep, roffs, rpeers = lib.incast_replies(data, offs, out["status"], out["reply"], peers)
            m = len(roffs) - 1
            if m:
                assert lib.udp_send_batch(rx, rep, roffs, rpeers, 128) == m
            for i in np.nonzero((st & 0x7F) == 2)[0]:
                b = G.Bucket(batch[i][25:].decode("latin-1"))
                b.added, b.taken, b.elapsed = G.b2f(int(ra[i])), G.b2f(int(rt[i])), int(re[i])
                all_replies.append(b.marshal())
            got += batch
        ring.close()
        back = _drain(lib, tx, len(all_replies)) if all_replies else []
        assert back == all_replies
        assert len(all_replies) > 50
    finally:
        rx.close()
        tx.close()
        g.close()


@pytest.mark.gpu
def test_bad_offsets_are_refused_before_any_device_read(lib):
    """Decreasing datagram offsets from the host would send the kernels
    outside the copied bytes: phip_ring_submit and phip_receive_datagrams
    refuse them (PHIP_ERR_INVALID), and the slot stays usable."""
    import ctypes as C
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = lib.GPURepo(log2_slots=10)
    ring = lib.Ring(g, nslots=2, max_msgs=8)
    slot, bv, ov = ring.acquire()
    d = [_datagram(b"b%d" % i, i + 1, 0, 0) for i in range(3)]
    blob = b"".join(d)
    bv[:len(blob)] = np.frombuffer(blob, np.uint8)
    ov[:4] = [0, len(d[0]), 5, len(blob)]                 # offs[2] < offs[1]
    with pytest.raises(lib.PatrolHipError) as ex:
        ring.submit(slot, 3)
    assert ex.value.code == -1
    ov[:4] = np.cumsum([0] + [len(x) for x in d])
    ring.submit(slot, 3)
    assert list(ring.receive(slot, 3, _gen.T0)["status"]) == [1 | 0x80] * 3
    offs = np.array([0, 40, 20, 60], np.uint64)
    data = np.zeros(72, np.uint8)
    rc = g.L.phip_receive_datagrams(g.h, data.ctypes.data, offs.ctypes.data, 3, _gen.T0, None,
                                    None, 0)
    assert rc == -1
    ring.close()
    g.close()
