"""patrol_amd — MI355X-native bucket-state engine for Patrol (calavera/patrol).

The product is libpatrolhip (HIP kernels for gfx950 behind the C ABI in
include/patrolhip.h).  This package holds its sources (csrc/), the in-tree
build (Makefile -> libpatrolhip.so) and a thin Python binding used by tests
and bench.py.
"""
from ._lib import EXPORTS, LIB_PATH, build_id, load  # noqa: F401
from .engine import (BucketState, GPUGroup, GPURepo, PatrolHipError, Ring, TakeBatcher,  # noqa: F401
                     incast_replies, marshal, names_blob, parse_rate, udp_recv_batch,
                     udp_send_batch)

__all__ = ["GPURepo", "GPUGroup", "BucketState", "PatrolHipError", "Ring", "TakeBatcher", "parse_rate", "marshal",
           "names_blob", "udp_recv_batch", "udp_send_batch", "incast_replies", "load", "LIB_PATH",
           "EXPORTS"]
