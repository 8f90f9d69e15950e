"""ctypes binding of libpatrolhip (include/patrolhip.h).

The library is built in-tree (patrol_amd/libpatrolhip.so, see Makefile /
__graft_entry__.build()).  There is no fallback: if the shared object is
missing or fails to load, importing the engine raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# PATROLHIP_LIB: a tuning build of the same sources (tools/build_variants.sh).
LIB_PATH = os.environ.get("PATROLHIP_LIB") or os.path.join(HERE, "libpatrolhip.so")

# Every symbol include/patrolhip.h declares (tests/test_abi.py checks both ways).
EXPORTS = [
    "phip_abi_version", "phip_build_id", "phip_open", "phip_close", "phip_last_error", "phip_flush", "phip_len",
    "phip_capacity", "phip_seed", "phip_get", "phip_dump", "phip_receive_datagrams",
    "phip_receive_soa", "phip_upsert_soa", "phip_apply_mixed", "phip_take", "phip_parse_rate",
    "phip_marshal", "phip_api_take", "phip_last_timings", "phip_set_timing", "phip_last_stats", "phip_hash_names",
    "phip_ae_local_max", "phip_ae_apply", "phip_ae_join", "phip_set_stream", "phip_route_pack",
    "phip_export_datagrams", "phip_snapshot_bytes", "phip_snapshot", "phip_restore",
    "phip_ring_open", "phip_ring_close", "phip_ring_acquire", "phip_ring_submit",
    "phip_ring_receive", "phip_udp_recv_batch", "phip_incast_replies", "phip_udp_send_batch",
    "phip_batcher_open", "phip_batcher_close", "phip_batcher_take", "phip_batcher_api_take",
    "phip_batcher_stats", "phip_batcher_take_reply", "phip_batcher_api_take_reply",
    "phip_table_stats", "phip_group_unique_id", "phip_group_open_all", "phip_group_open_rank",
    "phip_group_close", "phip_group_last_error", "phip_group_world", "phip_group_local",
    "phip_group_handle", "phip_group_receive", "phip_group_anti_entropy",
    "phip_group_set_timing", "phip_group_stage_ms", "phip_group_rccl_info",
]

PHIP_OK = 0
PHIP_ERR = {-1: "INVALID", -2: "HIP", -3: "FULL", -4: "ARENA", -5: "SHORT_BUFFER",
            -6: "NAME_TOO_LARGE", -7: "NO_DEVICE", -8: "IO", -9: "BUSY", -10: "RCCL"}
GROUP_ID_BYTES = 128
PEER_BYTES = 128   # PHIP_PEER_BYTES = sizeof(struct sockaddr_storage)
ST_MERGED, ST_INCAST_REPLY, ST_INCAST_NOREPLY, ST_SHORT, ST_NOT_PROCESSED = 1, 2, 3, 4, 5
ST_TAKE_OK, ST_TAKE_DENIED, ST_UPSERT_INSERTED, ST_CREATED = 6, 7, 8, 0x80
OP_TAKE, OP_RECEIVE, OP_UPSERT = 0, 1, 2
DEVICE_PTRS = 0x1
CFG_NO_GROW = 0x1
CFG_NO_SMALL = 0x2
CFG_FIXED_SEED = 0x4
CFG_ISOLATE = 0x8
ROUTE_COMBINE = 0x2
GROUP_RCCL_SELF = 0x4
GROUP_SMALL_CHUNKS = 0x8
RECV_ASYNC = 0x20
PACKET_SIZE = 256
BUCKET_FIXED_SIZE = 25   # PHIP_BUCKET_FIXED_SIZE: added, taken, elapsed, name length


class phip_config(C.Structure):
    _fields_ = [("device", C.c_int32), ("log2_slots", C.c_uint32), ("arena_bytes", C.c_uint64),
                ("max_load_pct", C.c_uint32), ("debug_tag_bits", C.c_uint32),
                ("flags", C.c_uint32), ("reserved", C.c_uint32), ("hash_seed", C.c_uint64)]


class phip_state(C.Structure):
    _fields_ = [("added", C.c_uint64), ("taken", C.c_uint64), ("elapsed", C.c_int64),
                ("created", C.c_int64)]


class phip_msgs(C.Structure):
    # names_len: the names blob's byte length, 0 = unchecked (patrolhip.h)
    _fields_ = [("n", C.c_uint32), ("names_len", C.c_uint32), ("names", C.c_void_p),
                ("name_offs", C.c_void_p), ("added", C.c_void_p), ("taken", C.c_void_p),
                ("elapsed", C.c_void_p)]


class phip_ops(C.Structure):
    _fields_ = [("n", C.c_uint32), ("names_len", C.c_uint32), ("kind", C.c_void_p),
                ("names", C.c_void_p), ("name_offs", C.c_void_p), ("now", C.c_void_p),
                ("freq", C.c_void_p), ("per", C.c_void_p), ("count", C.c_void_p),
                ("added", C.c_void_p), ("taken", C.c_void_p), ("elapsed", C.c_void_p)]


class phip_batcher_config(C.Structure):
    _fields_ = [("window_us", C.c_uint32), ("max_batch", C.c_uint32)]


class phip_take_reply(C.Structure):
    _fields_ = [("remaining", C.c_uint64), ("ok", C.c_uint8), ("created", C.c_uint8),
                ("datagram_len", C.c_uint16), ("reserved", C.c_uint32), ("seq", C.c_uint64),
                ("state", phip_state), ("datagram", C.c_uint8 * 256)]


class phip_results(C.Structure):
    _fields_ = [("status", C.c_void_p), ("remaining", C.c_void_p), ("have", C.c_void_p),
                ("reply", C.c_void_p)]


_lib = None


def build_id() -> str:
    """phip_build_id() of the loaded library (a hash of its sources)."""
    return load().phip_build_id().decode()


def load(path: str = LIB_PATH):
    """Load libpatrolhip.so (raises OSError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"libpatrolhip.so not built at {path}: run `make -C patrol_amd` "
                      "or __graft_entry__.build()")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same
    # soname as /opt/rocm's), and whichever is loaded first serves both.  The
    # engine shares streams and device memory with torch, so torch's runtime
    # must be the one: load it before this library when torch is present.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    vp, u32, u64, i64 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int64
    L.phip_abi_version.restype = C.c_int
    L.phip_build_id.restype = C.c_char_p
    L.phip_open.argtypes = [C.POINTER(phip_config), C.POINTER(vp)]
    L.phip_close.argtypes = [vp]
    L.phip_close.restype = None
    L.phip_last_error.argtypes = [vp]
    L.phip_last_error.restype = C.c_char_p
    L.phip_flush.argtypes = [vp]
    L.phip_len.argtypes = [vp]
    L.phip_len.restype = u64
    L.phip_capacity.argtypes = [vp]
    L.phip_capacity.restype = u64
    L.phip_seed.argtypes = [vp, vp, vp, u32, vp, u32]
    L.phip_get.argtypes = [vp, C.c_char_p, u32, C.POINTER(phip_state)]
    L.phip_dump.argtypes = [vp, vp, u64, vp, vp, u64, C.POINTER(u64), C.POINTER(u64)]
    L.phip_export_datagrams.argtypes = [vp, vp, vp, u32, vp, vp, u32]
    L.phip_snapshot_bytes.argtypes = [vp]
    L.phip_snapshot_bytes.restype = u64
    L.phip_snapshot.argtypes = [vp, vp, u64]
    L.phip_restore.argtypes = [vp, vp, u64]
    L.phip_receive_datagrams.argtypes = [vp, vp, vp, u32, i64, C.POINTER(phip_results),
                                         C.POINTER(u32), u32]
    L.phip_receive_soa.argtypes = [vp, C.POINTER(phip_msgs), i64, C.POINTER(phip_results), u32]
    L.phip_upsert_soa.argtypes = [vp, C.POINTER(phip_msgs), i64, C.POINTER(phip_results), u32]
    L.phip_apply_mixed.argtypes = [vp, C.POINTER(phip_ops), C.POINTER(phip_results), u32]
    L.phip_take.argtypes = [vp, vp, vp, u32, vp, vp, vp, vp, vp, vp, u32]
    L.phip_parse_rate.argtypes = [C.c_char_p, u32, C.POINTER(i64), C.POINTER(i64)]
    L.phip_marshal.argtypes = [C.c_char_p, u32, C.POINTER(phip_state), C.c_char_p]
    L.phip_api_take.argtypes = [vp, C.c_char_p, u32, C.c_char_p, u32, C.c_char_p, u32, i64,
                                C.c_char_p, C.POINTER(u32)]
    L.phip_last_timings.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.c_int]
    L.phip_hash_names.argtypes = [vp, vp, vp, u32, vp, u32]
    L.phip_set_timing.argtypes = [vp, C.c_int]
    L.phip_set_timing.restype = None
    L.phip_last_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.c_int]
    L.phip_last_stats.restype = C.c_int
    L.phip_ae_local_max.argtypes = [vp, vp, u32, u64, vp, u32]
    L.phip_ae_apply.argtypes = [vp, vp, u32, u64, vp, u32]
    L.phip_ae_join.argtypes = [vp, vp, u32, u64, u32]
    L.phip_set_stream.argtypes = [vp, vp]
    L.phip_route_pack.argtypes = [vp, C.POINTER(phip_msgs), u32, vp, vp, vp, vp, vp, vp, vp, u32]
    L.phip_ring_open.argtypes = [vp, u32, u32, u64, C.POINTER(vp)]
    L.phip_ring_close.argtypes = [vp]
    L.phip_ring_close.restype = None
    L.phip_ring_acquire.argtypes = [vp, C.POINTER(u32), C.POINTER(vp), C.POINTER(vp)]
    L.phip_ring_submit.argtypes = [vp, u32, u32]
    L.phip_ring_receive.argtypes = [vp, u32, i64, C.POINTER(phip_results), C.POINTER(u32)]
    L.phip_udp_recv_batch.argtypes = [C.c_int, vp, u64, vp, u32, vp, C.c_int, C.POINTER(u32)]
    L.phip_incast_replies.argtypes = [vp, vp, u32, vp, vp, vp, vp, u64, vp, vp, C.POINTER(u32)]
    L.phip_udp_send_batch.argtypes = [C.c_int, vp, vp, u32, vp, u32, C.POINTER(u32)]
    L.phip_batcher_open.argtypes = [vp, C.POINTER(phip_batcher_config), C.POINTER(vp)]
    L.phip_batcher_close.argtypes = [vp]
    L.phip_batcher_close.restype = None
    L.phip_batcher_take.argtypes = [vp, C.c_char_p, u32, i64, i64, i64, u64, C.POINTER(u64),
                                    C.POINTER(C.c_uint8), C.POINTER(u64)]
    L.phip_batcher_api_take.argtypes = [vp, C.c_char_p, u32, C.c_char_p, u32, C.c_char_p, u32,
                                        i64, C.c_char_p, C.POINTER(u32)]
    L.phip_batcher_stats.argtypes = [vp, C.POINTER(u64), C.c_int]
    L.phip_batcher_take_reply.argtypes = [vp, C.c_char_p, u32, i64, i64, i64, u64,
                                          C.POINTER(phip_take_reply)]
    L.phip_batcher_api_take_reply.argtypes = [vp, C.c_char_p, u32, C.c_char_p, u32, C.c_char_p,
                                              u32, i64, C.c_char_p, C.POINTER(u32),
                                              C.POINTER(phip_take_reply)]
    L.phip_table_stats.argtypes = [vp, C.POINTER(u64), C.c_int]
    L.phip_group_unique_id.argtypes = [C.c_char_p]
    L.phip_group_open_all.argtypes = [C.POINTER(phip_config), C.POINTER(C.c_int32), u32,
                                      C.POINTER(vp)]
    L.phip_group_open_rank.argtypes = [vp, C.c_char_p, u32, u32, C.POINTER(vp)]
    L.phip_group_close.argtypes = [vp]
    L.phip_group_close.restype = None
    L.phip_group_last_error.argtypes = [vp]
    L.phip_group_last_error.restype = C.c_char_p
    L.phip_group_world.argtypes = [vp]
    L.phip_group_world.restype = u32
    L.phip_group_local.argtypes = [vp]
    L.phip_group_local.restype = u32
    L.phip_group_handle.argtypes = [vp, u32]
    L.phip_group_handle.restype = vp
    L.phip_group_receive.argtypes = [vp, C.POINTER(phip_msgs), i64, C.POINTER(u64),
                                     C.POINTER(u64), u32]
    L.phip_group_anti_entropy.argtypes = [vp, C.POINTER(vp), u32, u64, u32]
    # (round 5's entry points: a variant library built from older sources for
    # an A/B run, PATROLHIP_LIB, lacks them)
    if hasattr(L, "phip_group_set_timing"):
        L.phip_group_set_timing.argtypes = [vp, C.c_int]
        L.phip_group_stage_ms.argtypes = [vp, u32, C.POINTER(C.c_float)]
        L.phip_group_rccl_info.argtypes = [vp, u32, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                           C.c_char_p, u32]
    _lib = L
    return L
