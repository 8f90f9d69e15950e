"""Multi-GPU shard layer: owner routing and anti-entropy.

One process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm,
xGMI between the GPUs of a node); the same code runs on "gloo" with CPU
tensors for the CPU tests.

* Buckets are sharded by name: owner(name) = ((fnv1a64(name) >> 32) * world)
  >> 32, independent of the slot hash inside a shard (phip_device.hpp), so a
  shard's table stays uniformly loaded.
* route_messages(): the one exchange step of the merge path.  Each rank
  stable-partitions its decoded replica messages by owner and one
  all_to_all_single per column moves them to their owners (per-source order
  kept, sources concatenated by rank: the merges are order-free in the clean
  domain, and per-bucket Take order is preserved because a bucket's ops all
  come from one source queue).
* anti_entropy(): the simulated cluster replicas of BASELINE configs[4].
  Replica states are E-encoded (the order-preserving key of
  phip_device.hpp, mirrored in torch by e_encode), so the CvRDT join of any
  number of replicas is an elementwise max: a local max over the replicas
  resident on this GPU, then one all_reduce(MAX) on int64 bit patterns
  (E XOR 2^63 turns the unsigned order into the signed one RCCL reduces).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from . import _lib

SIGN = -(1 << 63)                       # 0x8000000000000000 as int64
INF_BITS = 0x7FF0000000000000
NAN_BASE = 0xFFE0000000000002 - (1 << 64)
NAN_PER_SIGN = (1 << 52) - 1


def hash_names(blob: torch.Tensor, offs: torch.Tensor, repo=None) -> torch.Tensor:
    """FNV-1a 64 per name (phip_hash_names) as an int64 tensor on blob's device."""
    n = offs.numel() - 1
    L = _lib.load()
    out = torch.empty(max(n, 1), dtype=torch.int64, device=blob.device)
    if blob.is_cuda:
        if repo is None:
            raise ValueError("device hashing needs a GPURepo handle")
        offs32 = offs.to(torch.int32)
        rc = L.phip_hash_names(repo.h, blob.data_ptr(), offs32.data_ptr(), n, out.data_ptr(),
                               _lib.DEVICE_PTRS)
    else:
        b = blob.contiguous().numpy()
        o = offs.to(torch.int64).numpy().astype(np.uint32)
        rc = L.phip_hash_names(None, b.ctypes.data, o.ctypes.data, n, out.data_ptr(), 0)
    if rc != 0:
        raise RuntimeError(f"phip_hash_names failed: {rc}")
    return out[:n]


def owner_of(h: torch.Tensor, world: int) -> torch.Tensor:
    """Shard map: ((h >> 32) * world) >> 32 on the unsigned hash."""
    hi = (h >> 32) & 0xFFFFFFFF
    return ((hi * world) >> 32).to(torch.int64)


def _gather_names(blob, offs, order):
    starts = offs[:-1][order].to(torch.int64)
    lens = (offs[1:] - offs[:-1])[order].to(torch.int64)
    total = int(lens.sum())
    new_offs = torch.zeros(order.numel() + 1, dtype=torch.int64, device=blob.device)
    new_offs[1:] = torch.cumsum(lens, 0)
    seg = torch.repeat_interleave(torch.arange(order.numel(), device=blob.device), lens)
    idx = starts[seg] + (torch.arange(total, device=blob.device) - new_offs[:-1][seg])
    return blob[idx], lens, new_offs


def route_messages(blob, offs, added, taken, elapsed, group=None, repo=None, h=None):
    """All-to-all the decoded messages to their owner ranks.

    blob uint8 / offs int64[n+1] / added, taken, elapsed int64 (float64 bit
    patterns for added/taken).  Returns the same five arrays for the messages
    this rank owns.
    """
    world = dist.get_world_size(group)
    packed = pack_by_owner(blob, offs, added, taken, elapsed, world, h=h, repo=repo)
    return exchange_packed(*packed, group=group)


def _a2a(out, inp, r_splits=None, s_splits=None, group=None):
    """all_to_all_single; gloo (the CPU rehearsal backend) takes CPU tensors
    only, so CUDA tensors are staged through host memory there."""
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), r_splits, s_splits, group=group)
        out.copy_(o)
        return
    dist.all_to_all_single(out, inp, r_splits, s_splits, group=group)


def pack_by_owner(blob, offs, added, taken, elapsed, world, h=None, repo=None):
    """The pack step of owner routing restated with torch ops: the
    owner-major, per-owner stable layout phip_route_pack writes (without its
    sender-side combine).  Returns (names, lens int32, added, taken, elapsed,
    counts int64[world], name_bytes int64[world])."""
    if h is None:
        h = hash_names(blob, offs, repo)
    own = owner_of(h, world)
    order = torch.sort(own, stable=True).indices
    nb, lens, _ = _gather_names(blob, offs, order)
    cnt = torch.bincount(own, minlength=world).to(torch.int64)
    nbytes = torch.zeros(world, dtype=torch.int64, device=blob.device)
    nbytes.index_add_(0, own, (offs[1:] - offs[:-1]).to(torch.int64))
    return nb, lens.to(torch.int32), added[order], taken[order], elapsed[order], cnt, nbytes


def exchange_packed(s_names, s_lens, s_a, s_t, s_e, cnt, nbytes, group=None):
    """The exchange step of owner routing: one all-to-all of the (messages,
    name bytes) split sizes, then one all-to-all per column of the
    owner-major send buffers (phip_route_pack's or pack_by_owner's layout).
    Returns (names with 8 bytes of read slack, int32 offsets[m+1], added,
    taken, elapsed) of the m messages this rank owns, sources concatenated
    by rank, each source's in its order."""
    world = dist.get_world_size(group)
    dev = s_names.device
    sizes = torch.stack([cnt, nbytes], 1)                  # [world, 2]
    recv_sizes = torch.empty_like(sizes)
    _a2a(recv_sizes, sizes, group=group)
    (sc, sb), (rc_, rb) = torch.cat([sizes, recv_sizes], 1).t().reshape(2, 2, world).tolist()

    def a2a(x, s_splits, r_splits, slack=0):
        total = sum(r_splits)
        out = torch.zeros(total + slack, dtype=x.dtype, device=dev)
        _a2a(out[:total], x[:sum(s_splits)], r_splits, s_splits, group=group)
        return out if slack else out[:total]

    r_lens = a2a(s_lens, sc, rc_)
    # 8 bytes of read slack past the last name (the ABI's blob rule)
    r_blob = a2a(s_names, sb, rb, slack=8)
    r_a, r_t, r_e = a2a(s_a, sc, rc_), a2a(s_t, sc, rc_), a2a(s_e, sc, rc_)
    # name offsets in the received blob: one int32 scan of the lengths
    r_offs = torch.zeros(r_lens.numel() + 1, dtype=torch.int32, device=dev)
    torch.cumsum(r_lens, 0, dtype=torch.int32, out=r_offs[1:])
    return r_blob, r_offs, r_a, r_t, r_e


def route_pack_native(blob, offs, added, taken, elapsed, repo, world, combine=False):
    """phip_route_pack on the GPU (owner hash, stable owner-major pack of
    names, lengths and states in two passes; with combine=True a clean
    batch's hot names are max-combined at the sender, PHIP_ROUTE_COMBINE).
    Returns the send buffers and split sizes exchange_packed() takes."""
    from .engine import phip_msgs
    dev = blob.device
    n = offs.numel() - 1
    L = _lib.load()
    offs32 = offs if offs.dtype == torch.int32 else offs.to(torch.int32)
    s_names = torch.empty(max(blob.numel(), 1), dtype=torch.uint8, device=dev)
    s_lens = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    s_a = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    s_t = torch.empty_like(s_a)
    s_e = torch.empty_like(s_a)
    cnt = torch.zeros(world, dtype=torch.int64, device=dev)
    nbytes = torch.zeros(world, dtype=torch.int64, device=dev)
    m = phip_msgs(n, 0, blob.data_ptr(), offs32.data_ptr(), added.data_ptr(), taken.data_ptr(),
                  elapsed.data_ptr())
    rc = L.phip_route_pack(repo.h, C.byref(m), world, s_names.data_ptr(), s_lens.data_ptr(),
                           s_a.data_ptr(), s_t.data_ptr(), s_e.data_ptr(), cnt.data_ptr(),
                           nbytes.data_ptr(),
                           _lib.DEVICE_PTRS | (_lib.ROUTE_COMBINE if combine else 0))
    if rc != 0:
        raise RuntimeError(f"phip_route_pack failed: {rc}")
    return s_names, s_lens, s_a, s_t, s_e, cnt, nbytes


def route_messages_native(blob, offs, added, taken, elapsed, repo, group=None, combine=False):
    """route_messages with the partition on the GPU (route_pack_native), then
    the all-to-all of each column over RCCL (exchange_packed).  Same result
    as route_messages(); with combine=True every owner's merged state is the
    same with fewer messages moved.  repo's stream must be torch's current
    stream (GPURepo.use_torch_stream) or the inputs complete."""
    world = dist.get_world_size(group)
    packed = route_pack_native(blob, offs, added, taken, elapsed, repo, world, combine)
    return exchange_packed(*packed, group=group)


# ---------------------------------------------------------- E-encoding ----
def e_encode(bits: torch.Tensor) -> torch.Tensor:
    """float64 bit patterns (int64) -> E codes (int64 holding the u64 code).

    Mirrors phip_device.hpp enc_f64: unsigned order negatives < +0 < -0 <
    positives < NaNs, a bijection on all 2^64 patterns."""
    b = bits.to(torch.int64)
    mag = b & 0x7FFFFFFFFFFFFFFF
    neg = b < 0
    is_nan = mag > INF_BITS
    nan_idx = mag - INF_BITS - 1 + torch.where(neg, NAN_PER_SIGN, 0)
    out = torch.where(neg, torch.where(mag == 0, INF_BITS + 1, INF_BITS - mag),
                      torch.where(mag == 0, INF_BITS, INF_BITS + 1 + mag))
    out = torch.where(is_nan, NAN_BASE + nan_idx, out)
    return out


def e_decode(code: torch.Tensor) -> torch.Tensor:
    """Inverse of e_encode."""
    e = code.to(torch.int64)
    u_lt = lambda a, c: (a ^ SIGN) < (c ^ SIGN)   # unsigned a < c on int64 storage
    inf = torch.full_like(e, INF_BITS)
    out = torch.where(u_lt(e, inf), SIGN | (INF_BITS - e), torch.zeros_like(e))
    out = torch.where(e == INF_BITS, torch.zeros_like(e), out)
    out = torch.where(e == INF_BITS + 1, torch.full_like(e, SIGN), out)
    pos = (~u_lt(e, torch.full_like(e, INF_BITS + 2))) & u_lt(e, torch.full_like(e, NAN_BASE))
    out = torch.where(pos, e - INF_BITS - 1, out)
    idx = e - NAN_BASE
    isn = ~u_lt(e, torch.full_like(e, NAN_BASE))
    nanv = torch.where(idx < NAN_PER_SIGN, INF_BITS + 1 + idx, SIGN | (INF_BITS + 1 + idx - NAN_PER_SIGN))
    return torch.where(isn, nanv, out)


def to_signed_order(code: torch.Tensor) -> torch.Tensor:
    return code ^ SIGN


def is_nan_code(code: torch.Tensor) -> torch.Tensor:
    """E codes of NaNs are the top of the unsigned order (>= NAN_BASE)."""
    return (code ^ SIGN) >= (NAN_BASE ^ SIGN)


def anti_entropy_native(replicas: torch.Tensor, repo, group=None, timings=None) -> torch.Tensor:
    """anti_entropy on the GPU through libpatrolhip, in place: one pass over
    the local replicas (k_ae_local_max), one RCCL all-reduce(MAX) of the
    [3, B] join, one pass writing every replica (k_ae_apply).  Same result
    as anti_entropy().  With a list `timings` (and repo.set_timing(True)) the
    two kernels' (name, ms) are appended to it."""
    if not replicas.is_cuda or replicas.dtype != torch.int64 or not replicas.is_contiguous():
        raise ValueError("anti_entropy_native needs a contiguous int64 CUDA tensor [R, 3, B]")
    R, three, B = replicas.shape
    assert three == 3
    L = _lib.load()
    m = torch.empty((3, B), dtype=torch.int64, device=replicas.device)
    rc = L.phip_ae_local_max(repo.h, replicas.data_ptr(), R, B, m.data_ptr(), _lib.DEVICE_PTRS)
    if rc != 0:
        raise RuntimeError(f"phip_ae_local_max failed: {rc}")
    if timings is not None:
        timings += repo.timings()
    if dist.is_initialized():
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    rc = L.phip_ae_apply(repo.h, replicas.data_ptr(), R, B, m.data_ptr(), _lib.DEVICE_PTRS)
    if rc != 0:
        raise RuntimeError(f"phip_ae_apply failed: {rc}")
    if timings is not None:
        timings += repo.timings()
    return replicas


def anti_entropy(replicas: torch.Tensor, group=None) -> torch.Tensor:
    """One anti-entropy round over every replica of the job.

    replicas: [R_local, 3, B] int64 -- E codes of added and taken, and plain
    int64 elapsed, for B buckets aligned by index across replicas.  Each
    replica ends as if it had Bucket.Merge'd (bucket.go:240-263) every other
    replica's state into its own, in any order: a NaN replica value is never
    adopted (Go's `<` is false) but a replica's own NaN sticks, so
        result_i = max(E(own_i), max_j E'(r_j)),   E'(NaN) = 0 = E(-Inf).
    That is exact for replicas without -0.0 fields (a -0.0 vs +0.0 tie is
    first-seen in Go, hence order dependent; Patrol's own Take/Merge never
    produce -0.0).  Returns [R_local, 3, B]; one round converges.
    """
    s = replicas.clone()
    ep = s[:, 0:2]
    ep = torch.where(is_nan_code(ep), torch.zeros_like(ep), ep)
    m = torch.cat([to_signed_order(ep), s[:, 2:3]], dim=1).max(dim=0).values   # [3, B]
    if dist.is_initialized():
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    own = torch.cat([to_signed_order(s[:, 0:2]), s[:, 2:3]], dim=1)
    out = torch.maximum(own, m.unsqueeze(0))
    out[:, 0:2] = to_signed_order(out[:, 0:2])
    return out
