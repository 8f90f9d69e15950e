"""The drop-in boundary without a GPU: libpatrolhip loads, exports exactly the
C ABI that include/patrolhip.h declares, and its host-only entry points
(ParseRate, MarshalBinary) match the golden fixtures.  No device calls."""
import json
import os
import re
import subprocess

import pytest

import patrol_amd
from patrol_amd import _lib
from oracle import go_semantics as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def header_functions():
    src = open(os.path.join(ROOT, "include", "patrolhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(phip_[a-z_0-9]+)\s*\(", src)))


def test_library_built_in_tree():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build()"


def test_exports_match_header():
    declared = header_functions()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = sorted(set(m for m in re.findall(r"\bT (phip_[a-z_0-9]+)", out)))
    assert declared == exported
    assert sorted(_lib.EXPORTS) == declared
    L = _lib.load()
    for name in declared:
        assert hasattr(L, name)
    assert L.phip_abi_version() == 3


def test_config_struct_layout():
    """phip_config as the header lays it out (a cgo binding mirrors it)."""
    import ctypes as C
    assert C.sizeof(_lib.phip_config) == 40
    assert _lib.phip_config.flags.offset == 24
    assert _lib.phip_config.hash_seed.offset == 32
    # phip_take_reply: remaining, ok, created, datagram_len, reserved, seq, state, datagram
    assert C.sizeof(_lib.phip_take_reply) == 8 + 8 + 8 + 32 + 256
    assert _lib.phip_take_reply.state.offset == 24
    assert _lib.phip_take_reply.datagram.offset == 56


def test_seeded_mix_host_copy():
    """The placement mix (phip_kernels.hpp seeded_mix: murmur3 fmix64 of
    tag ^ seed) is a bijection that spreads tags differing in one bit."""
    M = (1 << 64) - 1

    def mix(t, s):
        x = t ^ s
        x ^= x >> 33
        x = (x * 0xff51afd7ed558ccd) & M
        x ^= x >> 33
        x = (x * 0xc4ceb9fe1a85ec53) & M
        x ^= x >> 33
        return x
    import random
    rng = random.Random(3)
    tags = [rng.getrandbits(64) for _ in range(2000)]
    seed = rng.getrandbits(64)
    assert len({mix(t, seed) for t in tags}) == len(tags)
    # one flipped input bit flips about half of the output bits
    flips = [bin(mix(t, seed) ^ mix(t ^ (1 << (k % 64)), seed)).count("1") for k, t in enumerate(tags)]
    assert 28 < sum(flips) / len(flips) < 36


def test_library_is_gfx950_code_object():
    """The kernels embedded in the .so are compiled for gfx950 (MI355X)."""
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_parse_rate_matches_golden():
    with open(os.path.join(GOLD, "parse_rate.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        assert patrol_amd.parse_rate(c["rate"].encode("utf-8")) == (c["freq"], c["per"], c["ok"]), c


def test_marshal_matches_golden():
    with open(os.path.join(GOLD, "codec.json")) as f:
        cases = json.load(f)["round_trip"]
    for c in cases:
        st = patrol_amd.BucketState(int(c["added"], 16), int(c["taken"], 16), c["elapsed"], 0)
        assert patrol_amd.marshal(bytes.fromhex(c["name"]), st).hex() == c["datagram"]
    with pytest.raises(patrol_amd.PatrolHipError):
        patrol_amd.marshal(b"x" * 232, patrol_amd.BucketState(0, 0, 0, 0))


def test_open_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(patrol_amd.PatrolHipError) as e:
        patrol_amd.GPURepo(log2_slots=10)
    assert e.value.code == -7


def test_e_encoding_is_order_preserving_bijection():
    """Host copy of the device key encoding (phip_device.hpp enc_f64/dec_f64):
    bijective, and max() of codes equals Go's merge for every non -0 replica."""
    import random
    S = 1 << 63
    INF = 0x7FF0000000000000

    def enc(b):
        mag = b & ~S
        if mag > INF:
            idx = mag - INF - 1 + ((1 << 52) - 1 if b & S else 0)
            return 0xFFE0000000000002 + idx
        if b & S:
            return INF + 1 if mag == 0 else INF - mag
        return INF if mag == 0 else INF + 1 + mag

    rng = random.Random(5)
    specials = [0, S, 1, S | 1, INF, S | INF, INF + 1, S | (INF + 1), 0x7FFFFFFFFFFFFFFF,
                0xFFFFFFFFFFFFFFFF, G.f2b(1.0), G.f2b(-1.0), G.f2b(2.5)]
    vals = specials + [rng.getrandbits(64) for _ in range(3000)]
    codes = [enc(v) for v in vals]
    assert len(set(codes)) == len(set(vals))
    for _ in range(20000):
        b, o = rng.choice(vals), rng.choice(vals)
        if o == S:      # -0.0 replicas take the ordered path
            continue
        bb, ob = G.b2f(b), G.b2f(o)
        want = G.f2b(ob) if bb < ob else b        # bucket.go:250-252
        oc = 0 if (o & ~S) > INF else enc(o)      # NaN replica: never adopted
        assert max(enc(b), oc) == enc(want), (hex(b), hex(o))


def test_flag_constants_match_header():
    """Every PHIP_* flag the Python binding passes has the header's value
    (a cgo binding reads them from the header itself)."""
    src = open(os.path.join(ROOT, "include", "patrolhip.h")).read()
    defs = {m.group(1): int(m.group(2), 16)
            for m in re.finditer(r"#define PHIP_([A-Z_0-9]+)\s+(0x[0-9a-fA-F]+)u", src)}
    for name, want in (("DEVICE_PTRS", "DEVICE_PTRS"), ("RECV_ASYNC", "RECV_ASYNC"),
                       ("CFG_NO_GROW", "CFG_NO_GROW"), ("CFG_NO_SMALL", "CFG_NO_SMALL"),
                       ("CFG_FIXED_SEED", "CFG_FIXED_SEED"), ("CFG_ISOLATE", "CFG_ISOLATE")):
        assert name in defs, name
        assert getattr(_lib, want) == defs[name], (name, getattr(_lib, want), defs[name])
