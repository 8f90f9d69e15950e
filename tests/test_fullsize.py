"""Parity at the BASELINE configurations' full sizes, generated exactly as
bench.py generates them (same functions, seeds and shapes), checked against
the oracle (oracle/liboracle.so) on the same inputs:

* C2 (BASELINE configs[1]): 10M seeded buckets in 2^25 slots, one 100M-message
  Zipf(1.1) batch through phip_receive_soa (the timed step of bench.py):
  every status and the whole 10M-bucket table bit-exact;
* C3 (configs[2]): 50M mixed Take(100:1s)/Merge ops through phip_apply_mixed,
  with the replica clock below the local one (Takes refill, succeed, deny)
  and ahead of it: every status, `remaining`, `have` and the table.

The oracle runs the Go loop one message at a time (about 5M ops/s), so each
test takes tens of seconds on the host.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402

T0 = 1_700_000_000_000_000_000


@pytest.fixture(scope="module")
def env():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    import patrol_amd
    return torch, bench, patrol_amd


def _seeded(torch, bench, pa, dev, K, L, stream):
    """bench.py's table: K buckets b0..b{K-1}, zero state, created T0."""
    repo = pa.GPURepo(device=0, log2_slots=L, arena_bytes=1 << 20)
    repo.set_stream(stream)
    keys = torch.arange(K, dtype=torch.int64, device=dev)
    kb, ko = bench.names_for_ids(torch, keys)
    st = torch.zeros((K, 4), dtype=torch.int64, device=dev)
    st[:, 3] = T0
    torch.cuda.synchronize()
    repo.seed_device(kb, ko, st, K)
    assert len(repo) == K
    o = O.Repo()
    z = np.zeros(K, np.uint64)
    o.L.orc_repo_seed(o.h, kb.cpu().numpy(), ko.cpu().numpy().view(np.uint32), K, z, z,
                      np.zeros(K, np.int64), np.full(K, T0, np.int64))
    return repo, o


def _check_table(repo, o):
    names, offs, a, t, e, c = repo.dump_arrays()
    assert len(offs) - 1 == len(repo) == len(o)
    bad, first = o.check_dump(names, offs, a, t, e, c)
    assert bad == 0, (bad, first, bytes(names[offs[first]:offs[first + 1]]) if first < len(offs) - 1
                      else None)


@pytest.mark.timeout(900)
def test_c2_full_size_vs_oracle(env):
    torch, bench, pa = env
    dev = torch.device("cuda", 0)
    K, n, L = 10_000_000, 100_000_000, 25
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        gen = torch.Generator(device=dev).manual_seed(1234)     # bench.py, rank 0
        repo, o = _seeded(torch, bench, pa, dev, K, L, s)
        ids = bench.zipf_ids(torch, gen, n, K, 1.1, dev)
        blob, offs = bench.names_for_ids(torch, ids)
        del ids
        a, t, e = bench.replica_states(torch, gen, n, 0, dev)
        status = torch.empty(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        repo.receive_soa(blob, a, t, e, T0, name_offs=offs, n=n, status=status, device=True)
        torch.cuda.synchronize()
        hot, hits, misses = repo.last_stats()[:3]
        assert hot > 300 and hits > n // 2 and misses == 0     # the timed path ran
        g_st = status.cpu().numpy()
        blob_h, offs_h = blob.cpu().numpy(), offs.cpu().numpy().view(np.uint32)
        a_h, t_h, e_h = (x.cpu().numpy() for x in (a, t, e))
    del blob, offs, a, t, e, status
    torch.cuda.empty_cache()
    print("[c2] GPU batch done; oracle running", flush=True)
    o_st = np.zeros(n, np.uint8)
    o.L.orc_receive_soa(o.h, blob_h, offs_h, n, a_h.view(np.uint64), t_h.view(np.uint64), e_h, T0,
                        o_st, np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.int64))
    assert np.array_equal(g_st, o_st)
    assert (o_st == 1).all()
    del blob_h, offs_h, a_h, t_h, e_h, g_st, o_st
    print("[c2] statuses equal; comparing the table", flush=True)
    _check_table(repo, o)
    repo.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("clock", ["below", "ahead"])
def test_c3_full_size_vs_oracle(env, clock):
    """bench.py --workload c3 (--c3-clock below|ahead): the warmup batch, then
    the first timed batch, each through phip_apply_mixed and the oracle."""
    torch, bench, pa = env
    import argparse
    dev = torch.device("cuda", 0)
    K, n, L = 10_000_000, 50_000_000, 25
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        gen = torch.Generator(device=dev).manual_seed(1234)
        repo, o = _seeded(torch, bench, pa, dev, K, L, s)
        args = argparse.Namespace(ops=n, zipf=1.1, warmup=1, steps=1, c3_clock=clock)
        c = bench.c3_inputs(args, torch, dev, K, 0, gen)
        host = {k: c[k].cpu().numpy() for k in ("blob", "kind", "freq", "per", "cnt")}
        offs_h = c["offs"].cpu().numpy().view(np.uint32)
        status = torch.empty(n, dtype=torch.uint8, device=dev)
        rem = torch.empty(n, dtype=torch.int64, device=dev)
        have = torch.empty(n, dtype=torch.int64, device=dev)
        stats = []
        for j, (now, a, t, e) in enumerate(c["steps"]):
            torch.cuda.synchronize()
            repo.apply_mixed_device(n, c["kind"], c["blob"], c["offs"], now, c["freq"], c["per"],
                                    c["cnt"], a, t, e, status=status, remaining=rem, have=have)
            torch.cuda.synchronize()
            g = [x.cpu().numpy() for x in (status, rem, have)]
            now_h, a_h, t_h, e_h = (x.cpu().numpy() for x in (now, a, t, e))
            st = np.zeros(n, np.uint8)
            orem = np.zeros(n, np.uint64)
            ohave = np.zeros(n, np.uint64)
            r = [np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.int64)]
            o.L.orc_apply_mixed(o.h, host["kind"], host["blob"], offs_h, n, now_h, host["freq"],
                                host["per"], host["cnt"].view(np.uint64), a_h.view(np.uint64),
                                t_h.view(np.uint64), e_h, st, orem, ohave, *r)
            assert np.array_equal(g[0], st), j
            take = host["kind"] == 0
            assert np.array_equal(g[1].view(np.uint64)[take], orem[take]), j
            assert np.array_equal(g[2].view(np.uint64)[take], ohave[take]), j
            stats.append((int((st == 6).sum()), int((st == 7).sum())))
            print(f"[c3 {clock}] batch {j} equal: {stats[-1][0]} Takes ok, {stats[-1][1]} denied",
                  flush=True)
            del g, now_h, a_h, t_h, e_h, st, orem, ohave, r
    # the input the step was meant to exercise: both outcomes of Take occur
    ok, denied = stats[-1]
    assert ok > 0 and denied > 0, stats
    if clock == "below":
        assert ok > n // 20, stats       # Takes refill and succeed
    _check_table(repo, o)
    repo.close()
