"""The shard group through the C ABI (phip_group_*): owner-routed
Receive and anti-entropy over RCCL with no torch.distributed on the data
path, against the oracle.  The box has one GPU, so the group is world 1 in
both forms (ncclCommInitAll over [0]; ncclCommInitRank with 1 rank); the
multi-rank exchange glue is covered on CPU (test_shard.py, gloo world 2)
and the N-GPU runs are the driver's.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import _gen  # noqa: E402


@pytest.fixture(scope="module")
def pa():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import patrol_amd
    return patrol_amd


def _batch(rng, n, K, dev, dirty=0.0):
    from patrol_amd.engine import names_blob
    ids = _gen.zipf_ids(rng, n, K)
    names = [(b"an-arena-length-bucket-name-%d" % i) if i % 97 == 0 else b"b%d" % i for i in ids]
    a, t, e = _gen.dirty_states(rng, n, dirty) if dirty else _gen.clean_states(rng, n)
    blob, offs = names_blob(names)
    dv = [torch.from_numpy(blob).to(dev), torch.from_numpy(offs.view(np.int32)).to(dev)]
    dv += [torch.from_numpy(x.view(np.int64)).to(dev) for x in (a, t, e)]
    return names, a, t, e, dv


def _dump(repo):
    return {k: (v.added, v.taken, v.elapsed, v.created) for k, v in repo.dump().items()}


@pytest.mark.parametrize("mode,rccl_self,small", [("all", False, False), ("rank", False, False),
                                                   ("all", True, False), ("rank", True, False),
                                                   ("rank", True, True)])
def test_group_receive_vs_oracle(pa, mode, rccl_self, small):
    """Two owner-routed batches (the second large enough for the sender-side
    combine) merged through phip_group_receive equal the oracle's Receive of
    the same messages.  rccl_self (PHIP_GROUP_RCCL_SELF): the member's own
    segment travels through grouped ncclSend/ncclRecv to itself, so the
    per-peer exchange of the multi-GPU group (segment plan, counts, dtypes,
    offsets) runs on this one GPU.  small (PHIP_GROUP_SMALL_CHUNKS): the
    exchange is pipelined in chunks of 4096 messages, so the 2^21 batch runs
    512 pack / exchange rounds over the two send sets."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(61)
    if mode == "all":
        g = pa.GPUGroup.open_all([0], log2_slots=14)
        repo = g.repos[0]
    else:
        repo = pa.GPURepo(log2_slots=14)
        g = pa.GPUGroup.open_rank(repo, pa.GPUGroup.unique_id(), 1, 0)
    assert g.world == 1
    o = O.Repo()
    for k, n in enumerate((5000, 1 << 21)):
        names, a, t, e, dv = _batch(rng, n, 20000, dev)
        torch.cuda.synchronize()
        sent, merged = g.receive([dv], _gen.T0 + k, combine=True, rccl_self=rccl_self,
                                 small_chunks=small)
        assert sent == merged and 0 < merged[0] <= n
        if not rccl_self:
            assert merged[0] == n         # one owner: merged as it came, no pack
        elif n >= 1 << 20:
            assert merged[0] < n          # hot names were combined at the sender
        o.receive_soa(names, a, t, e, _gen.T0 + k)
    got = _dump(repo)
    want = o.dump()
    assert len(got) == len(want)
    assert all(got.get(k) == v for k, v in want.items())
    g.close()
    if mode == "rank":
        repo.close()


def test_group_anti_entropy_equals_torch_restatement(pa):
    from patrol_amd import shard
    R, B = 5, 4000
    rng = np.random.default_rng(3)
    x = torch.zeros((R, 3, B), dtype=torch.int64)
    for k in range(R):
        taken = rng.integers(0, 10**6, B).astype(np.float64)
        x[k, 0] = shard.e_encode(torch.from_numpy((taken + rng.random(B) * 100).view(np.int64)))
        x[k, 1] = shard.e_encode(torch.from_numpy(taken.view(np.int64)))
        x[k, 2] = torch.from_numpy(rng.integers(0, 1 << 40, B))
    want = shard.anti_entropy(x.clone())
    g = pa.GPUGroup.open_all([0], log2_slots=10)
    xd = x.cuda()
    torch.cuda.synchronize()
    g.anti_entropy([xd])
    torch.cuda.synchronize()
    assert torch.equal(xd.cpu(), want)
    g.close()


@pytest.mark.parametrize("world,dirty", [(2, 0.0), (2, 0.05), (3, 0.0), (3, 0.05)])
def test_shared_device_group_receive_vs_oracle(pa, world, dirty):
    """A group of `world` shards on one GPU (phip_group_open_all with the
    device listed `world` times): the multi-member exchange (split sizes,
    each source's segment, sources merged in rank order) without RCCL, which
    takes one rank per device.  Member i sends batch i; every bucket lands
    on its owner, the members' tables together equal the oracle's Receive of
    batch 0, then 1, ... (per-bucket order), and a batch with incasts and
    -0.0 fields is packed without the sender-side combine."""
    from patrol_amd import shard
    from oracle import go_semantics as G
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(700 + world)
    g = pa.GPUGroup.open_all([0] * world, log2_slots=14)
    assert g.world == world
    o = O.Repo()
    for k, n in enumerate((3000, 1 << 20)):
        per = [_batch(rng, n, 30000, dev, dirty) for _ in range(world)]
        torch.cuda.synchronize()
        sent, merged = g.receive([b[4] for b in per], _gen.T0 + k, combine=True)
        assert sum(sent) == sum(merged) and sum(merged) <= world * n
        for names, a, t, e, _ in per:
            o.receive_soa(names, a, t, e, _gen.T0 + k)
    want = o.dump()
    got = {}
    for r, repo in enumerate(g.repos):
        d = _dump(repo)
        for name in d:
            h = torch.tensor([int(np.array([G.fnv1a64(name)], np.uint64).view(np.int64)[0])])
            assert int(shard.owner_of(h, world)) == r
        got.update(d)
    assert len(got) == len(want)
    assert all(got.get(k) == v for k, v in want.items())
    g.close()


@pytest.mark.parametrize("dirty", [0.0, 0.02])
def test_shared_device_group_receive_pipelined_vs_oracle(pa, dirty):
    """The pipelined exchange over many rounds (PHIP_GROUP_SMALL_CHUNKS:
    chunks of 4096 messages) in a group of three shards on one GPU whose
    members hold batches of different lengths, one of them empty: every
    member runs the longest batch's number of rounds (the chunk counts ride
    on the split-size exchange), sends empty chunks past its own batch, and
    the owners' tables together equal the oracle's Receive of batch 0, 1, 2
    in order.  With incasts and -0.0 fields the chunks holding them are
    packed without the combine."""
    from patrol_amd import shard
    from oracle import go_semantics as G
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(900 + int(dirty * 100))
    world = 3
    g = pa.GPUGroup.open_all([0] * world, log2_slots=14)
    o = O.Repo()
    for k, sizes in enumerate(((30000, 5000, 0), (1 << 20, 70000, 4097))):
        per = [_batch(rng, n, 30000, dev, dirty) if n else None for n in sizes]
        empty = [torch.zeros(8, dtype=torch.uint8, device=dev), torch.zeros(1, dtype=torch.int32, device=dev)]
        empty += [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(3)]
        torch.cuda.synchronize()
        sent, merged = g.receive([b[4] if b else empty for b in per], _gen.T0 + k, combine=True,
                                 small_chunks=True)
        assert sum(sent) == sum(merged) and sum(merged) <= sum(sizes)
        # an owner receives chunk by chunk, sources in rank order within a
        # chunk: the oracle applies the same interleaving (each source's
        # order is kept, as Patrol's peers' datagrams interleave)
        C = 4096
        for c in range(max((n + C - 1) // C for n in sizes)):
            for b, n in zip(per, sizes):
                if b and c * C < n:
                    sl = slice(c * C, min(n, (c + 1) * C))
                    o.receive_soa(b[0][sl], b[1][sl], b[2][sl], b[3][sl], _gen.T0 + k)
    want = o.dump()
    got = {}
    for r, repo in enumerate(g.repos):
        d = _dump(repo)
        for name in d:
            h = torch.tensor([int(np.array([G.fnv1a64(name)], np.uint64).view(np.int64)[0])])
            assert int(shard.owner_of(h, world)) == r
        got.update(d)
    assert len(got) == len(want)
    assert all(got.get(k) == v for k, v in want.items())
    g.close()


def test_shared_device_group_anti_entropy(pa):
    from patrol_amd import shard
    R, B, world = 3, 5000, 3
    rng = np.random.default_rng(17)
    xs = []
    for _ in range(world):
        x = torch.zeros((R, 3, B), dtype=torch.int64)
        for k in range(R):
            taken = rng.integers(0, 10**6, B).astype(np.float64)
            x[k, 0] = shard.e_encode(torch.from_numpy((taken + rng.random(B) * 100).view(np.int64)))
            x[k, 1] = shard.e_encode(torch.from_numpy(taken.view(np.int64)))
            x[k, 2] = torch.from_numpy(rng.integers(0, 1 << 40, B))
        xs.append(x)
    want = shard.anti_entropy(torch.cat(xs).clone())[:R]
    g = pa.GPUGroup.open_all([0] * world, log2_slots=10)
    xd = [x.cuda() for x in xs]
    torch.cuda.synchronize()
    g.anti_entropy(xd)
    torch.cuda.synchronize()
    for x in xd:
        assert torch.equal(x.cpu(), want)
    g.close()
