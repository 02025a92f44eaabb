"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU restatement
(``oracle/build/libodp_oracle.so``, built from ``oracle/odp_oracle.c``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module; the product (``odp_amd``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libodp_oracle.so")


def build():
    subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)


def _load():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    lib.oracle_classify.restype = i32
    lib.oracle_classify.argtypes = [vp, vp, vp, u32, u32, u64, i32, i32, vp, vp, vp, vp]
    lib.oracle_classify_mt.restype = i32
    lib.oracle_classify_mt.argtypes = [vp, vp, vp, u32, u32, u64, i32, i32, vp, i32, u32, vp]
    lib.oracle_chksum_ones_comp16.restype = C.c_uint16
    lib.oracle_chksum_ones_comp16.argtypes = [vp, u32]
    lib.oracle_crc32c.restype = u32
    lib.oracle_crc32c.argtypes = [vp, u32, u32]
    lib.oracle_thash.restype = u32
    lib.oracle_thash.argtypes = [vp, u32]
    lib.oracle_helper_udp_tcp_chksum.restype = i32
    lib.oracle_helper_udp_tcp_chksum.argtypes = [vp, u32, u32, u32, i32, i32, i32, vp]
    lib.oracle_l3fwd.restype = i32
    lib.oracle_l3fwd.argtypes = [vp, u32, vp, vp, u32, u32, i32, i32, vp]
    lib.oracle_l3fwd_reps.restype = i32
    lib.oracle_l3fwd_reps.argtypes = [vp, u32, vp, vp, u32, u32, i32, i32, vp, u32, vp]
    lib.oracle_tx_prepare.restype = i32
    lib.oracle_tx_prepare.argtypes = [vp, vp, u32, u32, vp, vp, vp]
    lib.oracle_packet_parse_multi.restype = i32
    lib.oracle_packet_parse_multi.argtypes = [vp, vp, u32, vp, i32, i32, u32, vp, vp]
    lib.oracle_fib_lookup.restype = i32
    lib.oracle_fib_lookup.argtypes = [vp, u32, vp, u32, vp, vp]
    return lib


lib = _load()

META_DT = np.dtype([("input_flags", "<u8"), ("flags", "<u4"), ("l2_offset", "<u2"),
                    ("l3_offset", "<u2"), ("l4_offset", "<u2"), ("cls_mark", "<u2"),
                    ("reserved", "<u4")])
DESC_DT = np.dtype([("offset", "<u4"), ("len", "<u4")])


def classify(rules, frames, num, stride=0, desc=None, opt=0, layer=4, classify=True,
             num_cos=None):
    """Run the CPU restatement. `rules` is an odpg_rules_t (ctypes struct)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    dptr = None
    if desc is not None:
        desc = np.ascontiguousarray(desc, dtype=DESC_DT)
        dptr = desc.ctypes.data
    out = np.zeros(num, np.uint32)
    mark = np.zeros(num, np.uint16)
    meta = np.zeros(num, META_DT)
    ncos = rules.num_cos if num_cos is None else num_cos
    stats = np.zeros(4 + ncos, np.uint64)
    lib.oracle_classify(C.byref(rules), frames.ctypes.data, dptr, stride, num, opt, layer,
                        int(bool(classify)), out.ctypes.data, mark.ctypes.data,
                        meta.ctypes.data, stats.ctypes.data)
    return {"out": out, "mark": mark, "meta": meta, "stats": stats}


def classify_mt(rules, frames, num, stride=0, desc=None, opt=0, layer=4, classify=True,
                nthreads=1, reps=1, cpus=None):
    """Threads on contiguous slices, `reps` passes; thread t pinned to cpus[t]."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    dptr = None
    if desc is not None:
        desc = np.ascontiguousarray(desc, dtype=DESC_DT)
        dptr = desc.ctypes.data
    out = np.zeros(num, np.uint32)
    cp = None
    if cpus is not None:
        cp = np.ascontiguousarray(cpus[:nthreads], dtype=np.int32)
        assert len(cp) == nthreads
    n = lib.oracle_classify_mt(C.byref(rules), frames.ctypes.data, dptr, stride, num, opt,
                               layer, int(bool(classify)), out.ctypes.data, nthreads, reps,
                               cp.ctypes.data if cp is not None else None)
    return out, n


def packet_parse_multi(frames, desc, offsets, proto, layer, chksums, meta):
    """odp_packet_parse_multi restated (odp_packet.c:1986-2075): parses from
    offsets[i] with odp_proto_t `proto` up to `layer`, checksum bits
    (ipv4 1, udp 2, tcp 4, sctp 8). `meta` (META_DT, updated in place) holds
    each packet's metadata before the call. Returns (first failing index or
    num, per-packet return values)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=DESC_DT)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32)
    ret = np.zeros(len(desc), np.int32)
    n = lib.oracle_packet_parse_multi(frames.ctypes.data, desc.ctypes.data, len(desc),
                                      offs.ctypes.data, proto, layer, chksums,
                                      meta.ctypes.data, ret.ctypes.data)
    return n, ret


def ones_comp16(data: bytes) -> int:
    b = np.frombuffer(bytes(data), np.uint8)
    return lib.oracle_chksum_ones_comp16(b.ctypes.data if len(b) else None, len(b))


def crc32c(data: bytes, init=0xFFFFFFFF) -> int:
    b = np.frombuffer(bytes(data), np.uint8)
    return lib.oracle_crc32c(b.ctypes.data if len(b) else None, len(b), init)


HELPER_GENERATE, HELPER_VERIFY, HELPER_RETURN = 0, 1, 2


def helper_udp_tcp_chksum(frame, l3, l4, ipv6, tcp, op=HELPER_VERIFY):
    """odph_udp_tcp_chksum() restated (helper/chksum.c:265-353). Returns
    (rc, checksum, frame bytes after the op)."""
    b = np.frombuffer(bytes(frame), np.uint8).copy()
    ck = np.zeros(1, np.uint16)
    rc = lib.oracle_helper_udp_tcp_chksum(b.ctypes.data, len(b), l3, l4, int(bool(ipv6)),
                                          int(bool(tcp)), op,
                                          None if op == HELPER_VERIFY else ck.ctypes.data)
    return rc, int(ck[0]), bytes(b)


def thash(words) -> int:
    a = np.ascontiguousarray(words, dtype=np.uint32)
    return lib.oracle_thash(a.ctypes.data, len(a))


def l3fwd(routes, param, frames, stride, num, src_port=0, error_check=False):
    """example/l3fwd restatement. `routes` is a ctypes array of odpg_route_t
    (add order), `param` an odpg_fwd_param_t. Returns (out_port, rewritten
    frames); the input array is not modified. rc -1 = unsupported route set."""
    fr = np.array(frames, dtype=np.uint8, copy=True)
    out = np.zeros(num, np.int32)
    rc = lib.oracle_l3fwd(C.cast(routes, C.c_void_p) if len(routes) else None, len(routes),
                          C.byref(param), fr.ctypes.data, stride, num, src_port,
                          int(bool(error_check)), out.ctypes.data)
    if rc:
        raise ValueError("route set outside the restated domain")
    return out, fr


def l3fwd_passes(routes, param, frames, stride, num, reps):
    """`reps` passes of the l3fwd restatement over a private copy of
    `frames`, the trie / warmed flow cache built once before them (as
    l3fwd's init does): returns the seconds the passes took (CPU baseline)."""
    fr = np.array(frames, dtype=np.uint8, copy=True)
    out = np.zeros(num, np.int32)
    ns = C.c_uint64(0)
    rc = lib.oracle_l3fwd_reps(C.cast(routes, C.c_void_p) if len(routes) else None, len(routes),
                               C.byref(param), fr.ctypes.data, stride, num, 0, 0,
                               out.ctypes.data, reps, C.byref(ns))
    if rc:
        raise ValueError("route set outside the restated domain")
    return ns.value * 1e-9


def fib_lookup(routes, ips):
    """Build the l3fwd LPM trie from `routes` (add order) and look up `ips`:
    returns (port, valid) arrays, exactly as fib_tbl_lookup reports them."""
    ips = np.ascontiguousarray(ips, dtype=np.uint32)
    port = np.zeros(len(ips), np.int32)
    valid = np.zeros(len(ips), np.int32)
    rc = lib.oracle_fib_lookup(C.cast(routes, C.c_void_p) if len(routes) else None, len(routes),
                               ips.ctypes.data, len(ips), port.ctypes.data, valid.ctypes.data)
    if rc:
        raise ValueError("trie pool overflow")
    return port, valid.astype(bool)


class TxCfg(C.Structure):
    """odpg_tx_cfg_t (include/odpg_tx.h)"""
    _fields_ = [("pktout_cfg", C.c_uint64), ("pktout_capa", C.c_uint64),
                ("hash_proto", C.c_uint32), ("num_qs", C.c_uint32), ("index", C.c_uint32),
                ("reserved", C.c_uint32)]


TX_META_DT = np.dtype([("l3_offset", "<u2"), ("l4_offset", "<u2"), ("flags", "<u4")])
PKTOUT_LOOP_CAPA = (1 << 5) | (1 << 6) | (1 << 7) | (1 << 8)


def tx_prepare(frames, num, stride=0, desc=None, meta=None, pktout_cfg=0,
               pktout_capa=PKTOUT_LOOP_CAPA, hash_proto=0, num_qs=1, index=0):
    """loopback_send()'s checksum insertion + queue pick restated
    (pktio/loop.c:415-523). Returns (out words, rewritten copy of frames)."""
    fr = np.array(frames, dtype=np.uint8, copy=True)
    dptr = mptr = None
    if desc is not None:
        desc = np.ascontiguousarray(desc, dtype=DESC_DT)
        dptr = desc.ctypes.data
    if meta is not None:
        meta = np.ascontiguousarray(meta, dtype=TX_META_DT)
        mptr = meta.ctypes.data
    out = np.zeros(num, np.uint32)
    cfg = TxCfg(pktout_cfg, pktout_capa, hash_proto, num_qs, index, 0)
    if lib.oracle_tx_prepare(fr.ctypes.data, dptr, stride, num, mptr, C.byref(cfg),
                             out.ctypes.data):
        raise ValueError("num_qs must be >= 1")
    return out, fr
