"""odp_packet_parse / odp_packet_parse_multi (packet.h; odp_packet.c:1986-2075)
on the GPU parser, against the oracle's restatement of the same function.

CPU: the oracle's packet_parse is pinned on its receive parse (which the
reference's own fixtures pin, tests/test_oracle_golden.py): from offset 0
with ODP_PROTO_ETH it must give the receive path's parse result; from an
offset k behind k junk bytes the same result shifted by k; from the L3
header with ODP_PROTO_IPV4 / IPV6 the same L3/L4 result without the L2 part.

GPU: packets of the runtime (odp/rt.h) parsed by odp_packet_parse_multi with
every start protocol, parse layer and checksum option mix; the parse result
each packet then carries (odpg_packet_view) must equal the oracle's bit for
bit, and the call must stop at the same packet (the first that fails)."""
import ctypes as C

import numpy as np
import pytest

import oracle
import rulesets
from helpers import ALL_CHKSUM, IFL, golden_frames, pack
from odp_amd import _lib as L

PROTO_ETH, PROTO_IPV4, PROTO_IPV6 = 1, 2, 3
L2_BITS = sum(1 << IFL[n] for n in ("l2", "eth", "jumbo", "eth_bcast", "eth_mcast"))


def _corpus(n=3000, seed=5):
    _, g = golden_frames()
    return list(g) + rulesets.mutate_corpus(n, seed=seed)


def _meta0(n):
    m = np.zeros(n, oracle.META_DT)
    m["l2_offset"] = m["l3_offset"] = m["l4_offset"] = 0xFFFF
    return m


def _parse_all(frames, offsets, proto, layer, chk):
    """oracle packet_parse on every packet (restarting after each failure)"""
    buf, desc = pack(frames)
    meta = _meta0(len(frames))
    ret = np.zeros(len(frames), np.int32)
    i = 0
    while i < len(frames):
        sub = meta[i:].copy()
        n, r = oracle.packet_parse_multi(buf, desc[i:], offsets[i:], proto, layer, chk, sub)
        meta[i:] = sub
        ret[i:i + min(n + 1, len(frames) - i)] = r[:min(n + 1, len(frames) - i)]
        i += n + 1
    return meta, ret


def test_oracle_parse_from_l2_equals_receive_parse():
    # empty frames excluded: odp_packet_parse refuses an offset at or past
    # the end (packet_map fails), the receive path parses them
    frames = [f for f in _corpus() if f]
    buf, desc = pack(frames)
    rx = oracle.classify(L.odpg_rules_t(default_cos=-1, error_cos=-1), buf, len(frames),
                         desc=desc, opt=ALL_CHKSUM, classify=False)
    meta, ret = _parse_all(frames, np.zeros(len(frames), np.uint32), PROTO_ETH, L.LAYER_ALL, 15)
    assert np.array_equal(meta.view(np.uint8), rx["meta"].view(np.uint8))
    # -1 exactly where the receive parse returned non-zero
    assert np.array_equal(ret != 0, (rx["out"] & L.ODPG_OUT_PARSE_ERR) != 0)
    assert 0 < (ret != 0).sum() < len(frames)


def test_oracle_parse_at_offset_is_shifted():
    frames = _corpus(1500, seed=9)
    rng = np.random.default_rng(3)
    k = rng.integers(0, 48, len(frames)).astype(np.uint32)
    shifted = [bytes(rng.integers(0, 256, int(x), dtype=np.uint8)) + f for x, f in zip(k, frames)]
    m0, r0 = _parse_all(frames, np.zeros(len(frames), np.uint32), PROTO_ETH, L.LAYER_ALL, 15)
    m1, r1 = _parse_all(shifted, k, PROTO_ETH, L.LAYER_ALL, 15)
    assert np.array_equal(r0, r1)
    for f in ("input_flags", "flags"):
        assert np.array_equal(m0[f], m1[f])
    for f in ("l2_offset", "l3_offset", "l4_offset"):
        v = m0[f].astype(np.int64)
        assert np.array_equal(np.where(v == 0xFFFF, 0xFFFF, v + k), m1[f])


@pytest.mark.parametrize("proto,etype", [(PROTO_IPV4, 0x0800), (PROTO_IPV6, 0x86DD)])
def test_oracle_parse_from_l3(proto, etype):
    frames = [f for f in _corpus(4000, seed=13) if len(f) > 14 and f[12:14] ==
              etype.to_bytes(2, "big")]
    assert len(frames) > 100
    m0, r0 = _parse_all(frames, np.zeros(len(frames), np.uint32), PROTO_ETH, L.LAYER_ALL, 15)
    m1, r1 = _parse_all(frames, np.full(len(frames), 14, np.uint32), proto, L.LAYER_ALL, 15)
    assert np.array_equal(r0, r1)
    assert np.array_equal(m0["input_flags"] & ~np.uint64(L2_BITS), m1["input_flags"])
    assert np.array_equal(m0["flags"], m1["flags"])
    assert np.all(m1["l2_offset"] == 0xFFFF)
    assert np.array_equal(m0["l3_offset"], m1["l3_offset"])
    assert np.array_equal(m0["l4_offset"], m1["l4_offset"])


def test_oracle_parse_refusals():
    buf, desc = pack([bytes(64)])
    for proto, layer, off in ((0, 4, 0), (1, 0, 0), (1, 4, 64), (1, 4, 100)):
        meta = _meta0(1)
        n, r = oracle.packet_parse_multi(buf, desc, np.array([off], np.uint32), proto, layer,
                                         0, meta)
        assert n == 0 and r[0] == -1
        assert meta["l3_offset"][0] == 0xFFFF            # untouched


# ---- GPU: the runtime's odp_packet_parse_multi ----------------------------
class PoolParam(C.Structure):
    _fields_ = [("type", C.c_int), ("buf", C.c_uint32 * 3), ("pkt", C.c_uint32 * 7),
                ("reserved", C.c_uint64 * 8)]


class ParseParam(C.Structure):
    """odp_packet_parse_param_t"""
    _fields_ = [("proto", C.c_int), ("last_layer", C.c_int), ("chksums", C.c_uint32)]


@pytest.fixture(scope="module")
def rt():
    lib = C.CDLL(L.LIB_PATH)
    lib.odp_pool_create.restype = C.c_void_p
    lib.odp_packet_alloc.restype = C.c_void_p
    lib.odp_packet_data.restype = C.c_void_p
    inst = C.c_uint64()
    assert lib.odp_init_global(C.byref(inst), None, None) == 0
    pp = PoolParam()
    lib.odp_pool_param_init(C.byref(pp))
    pp.pkt[0] = 1 << 16
    pool = lib.odp_pool_create(b"parse", C.byref(pp))
    assert pool
    yield lib, pool
    lib.odp_pool_destroy(C.c_void_p(pool))


def _gpu_parse(lib, pool, frames, offsets, proto, layer, chk):
    pk = (C.c_void_p * len(frames))()
    for i, f in enumerate(frames):
        pk[i] = lib.odp_packet_alloc(C.c_void_p(pool), len(f))
        assert pk[i]
        C.memmove(lib.odp_packet_data(C.c_void_p(pk[i])), f, len(f))
    offs = (C.c_uint32 * len(frames))(*[int(x) for x in offsets])
    prm = ParseParam(proto, layer, chk)
    meta = _meta0(len(frames))
    ret = np.zeros(len(frames), np.int32)
    i = 0
    while i < len(frames):           # restart after each failing packet
        n = lib.odp_packet_parse_multi(C.byref(pk, i * 8), C.byref(offs, i * 4),
                                       len(frames) - i, C.byref(prm))
        assert n >= 0
        if i + n < len(frames):
            ret[i + n] = -1
        i += n + 1
    view = L.odpg_packet_t()
    for i in range(len(frames)):
        assert lib.odpg_packet_view(C.c_void_p(pk[i]), C.byref(view)) == 0
        C.memmove(meta[i:i + 1].ctypes.data, C.byref(view.meta), C.sizeof(L.odpg_meta_t))
        lib.odp_packet_free(C.c_void_p(pk[i]))
    return meta, ret


@pytest.mark.gpu
@pytest.mark.parametrize("proto,layer,chk", [
    (PROTO_ETH, L.LAYER_ALL, 15), (PROTO_ETH, L.LAYER_L4, 2 | 4), (PROTO_ETH, L.LAYER_L3, 1),
    (PROTO_ETH, L.LAYER_L2, 15), (PROTO_IPV4, L.LAYER_ALL, 15), (PROTO_IPV6, L.LAYER_ALL, 15),
    (PROTO_IPV4, L.LAYER_L3, 0)])
def test_gpu_packet_parse_matches_oracle(rt, proto, layer, chk):
    lib, pool = rt
    frames = _corpus(2500, seed=17 + proto * 8 + layer)
    rng = np.random.default_rng(proto * 100 + layer)
    if proto == PROTO_ETH:
        k = rng.integers(0, 40, len(frames)).astype(np.uint32)
        frames = [bytes(rng.integers(0, 256, int(x), dtype=np.uint8)) + f
                  for x, f in zip(k, frames)]
    else:
        k = np.full(len(frames), 14, np.uint32)         # the L3 header (or junk there)
        k[::7] = 0                                       # and at the frame start
        frames = [f if len(f) > 20 else f + bytes(24) for f in frames]
    want_m, want_r = _parse_all(frames, k, proto, layer, chk)
    got_m, got_r = _gpu_parse(lib, pool, frames, k, proto, layer, chk)
    assert np.array_equal(got_r, want_r), np.nonzero(got_r != want_r)[0][:8]
    bad = np.nonzero(np.any(got_m.view(np.uint8).reshape(len(frames), -1) !=
                            want_m.view(np.uint8).reshape(len(frames), -1), axis=1))[0]
    assert not len(bad), (bad[:4], got_m[bad[:2]], want_m[bad[:2]])
    assert 0 < (want_r != 0).sum() < len(frames)
