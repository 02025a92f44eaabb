"""Shared test helpers: frame packing, flag names, oracle-vs-GPU comparison."""
import json
import os

import numpy as np

from odp_amd import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "reference_fixtures.json")))

DESC_DT = np.dtype([("offset", "<u4"), ("len", "<u4")])

# _odp_packet_input_flags_t bit positions (packet_inline_types.h:60-113)
IFL = dict(dst_queue=0, cls_mark=1, flow_hash=2, timestamp=3, l2=4, l3=5, l4=6, eth=7,
           eth_bcast=8, eth_mcast=9, jumbo=10, vlan=11, vlan_qinq=12, snap=13, arp=14,
           ipv4=15, ipv6=16, ip_bcast=17, ip_mcast=18, ipfrag=19, ipopt=20, ipsec=21,
           ipsec_ah=22, ipsec_esp=23, udp=24, tcp=25, sctp=26, icmp=27, no_next_hdr=28,
           l3_chksum_done=32, l4_chksum_done=33, ipsec_udp=34, udp_chksum_zero=35)

ALL_CHKSUM = L.PKTIN_IPV4_CHKSUM | L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM | L.PKTIN_SCTP_CHKSUM


def has(meta_row, name):
    return bool((int(meta_row["input_flags"]) >> IFL[name]) & 1)


def pack(frames, align=64, tail=128):
    """Variable-length frames -> (flat uint8 buffer, desc array); 64-B aligned
    offsets like pool segments; trailing slack so 16-B chunk reads stay inside."""
    offs, lens, parts, pos = [], [], [], 0
    for f in frames:
        f = bytes(f)
        offs.append(pos)
        lens.append(len(f))
        pad = (-len(f)) % align
        parts.append(f + bytes(pad))
        pos += len(f) + pad
    buf = np.frombuffer(b"".join(parts) + bytes(tail), np.uint8).copy()
    desc = np.zeros(len(frames), DESC_DT)
    desc["offset"] = offs
    desc["len"] = lens
    return buf, desc


def golden_frames(names=None):
    names = sorted(GOLDEN["frames"]) if names is None else names
    return names, [bytes.fromhex(GOLDEN["frames"][n]) for n in names]


def assert_same(a, b, what=""):
    """Bit-exact comparison of two result dicts (out/mark/meta/stats)."""
    for k in ("out", "mark", "meta", "stats"):
        if k in a and k in b:
            x, y = a[k], b[k]
            if k == "stats" and len(x) != len(y):
                # the compiled table drops never-referenced trailing CoS slots
                m = min(len(x), len(y))
                tail = x[m:] if len(x) > m else y[m:]
                assert not np.any(tail), f"{what}: non-zero counters past CoS {m - 4}"
                x, y = x[:m], y[:m]
            if k == "meta":
                x = x.view(np.uint8).reshape(len(x), -1)
                y = y.view(np.uint8).reshape(len(y), -1)
            if not np.array_equal(x, y):
                bad = np.nonzero(np.any((x != y).reshape(len(x), -1), axis=1))[0] \
                    if x.ndim else []
                raise AssertionError(f"{what}: '{k}' differs at {len(bad)} entries, "
                                     f"first {bad[:8]}: {x[bad[:4]]} vs {y[bad[:4]]}")


def expected_counters(o, num_cos):
    """The sharded-counter fold (odpg.h) an oracle run implies: its pktio and
    CoS counters, and per (CoS, hash queue) the packets the classifier handed
    to a queue (ret 0: a CoS, no drop action; _odp_cls_enq ->
    _odp_cos_queue_stats_add, odp_classification_internal.h:64-78)."""
    out = np.asarray(o["out"], np.uint32)
    cos = out & 0xFFFF
    ok = (cos < num_cos) & ((out & L.ODPG_OUT_CLS_DROP) == 0)
    q = np.zeros((num_cos, L.COS_QUEUE_MAX), np.uint64)
    np.add.at(q, (cos[ok], (out[ok] >> 24) & 31), 1)
    st = np.asarray(o["stats"], np.uint64)
    cs = np.zeros(num_cos, np.uint64)
    m = min(num_cos, len(st) - 4)
    cs[:m] = st[4:4 + m]
    assert not np.any(st[4 + m:]), "oracle counts a CoS past the table"
    return {"pktio": st[:4].copy(), "cos": cs, "queue": q}


def assert_counters(f, e, what=""):
    for k in ("pktio", "cos", "queue"):
        if not np.array_equal(f[k], e[k]):
            bad = np.argwhere(f[k] != e[k])[:6]
            raise AssertionError(f"{what}: counters '{k}' differ at {bad.tolist()}: "
                                 f"{[int(f[k][tuple(b)]) for b in bad]} vs "
                                 f"{[int(e[k][tuple(b)]) for b in bad]}")


TBL_XWALK, TBL_XGF, TBL_XMASK = 0x200, 0x800, 0x1000    # odpg_internal.h table forms


def table_flags(rules):
    """dtable_hdr_t.flags of the compiled image (odpg_rules_compile: a
    16-byte image header, then the table header, flags at +12)"""
    from odp_amd import gpu
    img = gpu.compile_rules(rules)
    return int.from_bytes(img[28:32], "little")


def make_c_tests():
    """make -C tests/c under a file lock: xdist workers running two tests that
    build it must not relink a test program the other is executing"""
    import fcntl
    import subprocess
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c")
    with open(os.path.join(d, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", d], check=True, capture_output=True)
