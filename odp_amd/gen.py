"""Synthetic traffic and rule sets for the BASELINE.json configurations.

Frames are built vectorised in numpy with valid IPv4 header and UDP/TCP
checksums (RFC 1071), laid out either at a fixed 64-byte stride (C1/C2/C4)
or in a 64-byte-aligned buffer with (offset, len) descriptors (IMIX, C3).
The shapes follow SURVEY.md §8(d).
"""
from __future__ import annotations

import numpy as np

ETH_IPV4 = 0x0800
ETH_IPV6 = 0x86DD
PROTO_TCP = 6
PROTO_UDP = 17

DESC_DT = np.dtype([("offset", "<u4"), ("len", "<u4")])


def xorshift64(seed, n):
    """Deterministic u64 stream (xorshift64), vectorised over blocks."""
    out = np.empty(n, np.uint64)
    x = np.uint64(seed) if seed else np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        # generate a short serial seed table, then use a counter-based mix for the rest
        for i in range(min(n, 64)):
            x ^= (x << np.uint64(13)) & np.uint64(0xFFFFFFFFFFFFFFFF)
            x ^= x >> np.uint64(7)
            x ^= (x << np.uint64(17)) & np.uint64(0xFFFFFFFFFFFFFFFF)
            out[i] = x
        if n > 64:
            idx = np.arange(64, n, dtype=np.uint64)
            z = idx * np.uint64(0x9E3779B97F4A7C15) + out[idx % np.uint64(64)]
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out[64:] = z ^ (z >> np.uint64(31))
    return out


def _be16(a, off, v):
    v = np.asarray(v, dtype=np.uint32)
    a[:, off] = (v >> 8) & 0xFF
    a[:, off + 1] = v & 0xFF


def _be32(a, off, v):
    v = np.asarray(v, dtype=np.uint64)
    for k in range(4):
        a[:, off + k] = (v >> np.uint64(24 - 8 * k)) & np.uint64(0xFF)


def ones_sum(a, lo, hi, extra=None):
    """One's-complement 16-bit sum (unfolded, int64) of bytes [lo, hi) per row."""
    seg = a[:, lo:hi].astype(np.int64)
    if seg.shape[1] % 2:
        seg = np.concatenate([seg, np.zeros((seg.shape[0], 1), np.int64)], axis=1)
    s = (seg[:, 0::2] << 8).sum(axis=1) + seg[:, 1::2].sum(axis=1)
    if extra is not None:
        s = s + extra
    return s


def fold(s):
    s = np.asarray(s, dtype=np.int64)
    while np.any(s >> 16):
        s = (s & 0xFFFF) + (s >> 16)
    return s


def csum(s):
    return (~fold(s)) & 0xFFFF


def ipv4_frames(n, length, src, dst, proto, sport, dport, *, smac=None, dmac=None, ttl=64,
                tos=0, ident=None, payload_seed=1, vlan=None, l4_csum=True, ip_csum=True):
    """Eth/[VLAN]/IPv4/UDP|TCP frames of `length` bytes each, shape (n, length)."""
    length = int(length)
    l2 = 14 + (4 if vlan is not None else 0)
    l4h = 8 if proto == PROTO_UDP else 20
    assert length >= l2 + 20 + l4h
    a = np.zeros((n, length), np.uint8)
    dm = np.array(dmac if dmac is not None else [0x02, 0x00, 0x00, 0x00, 0x00, 0x01], np.uint8)
    sm = np.array(smac if smac is not None else [0x02, 0x00, 0x00, 0x00, 0x00, 0x02], np.uint8)
    a[:, 0:6] = dm
    a[:, 6:12] = sm
    if vlan is not None:
        _be16(a, 12, 0x8100)
        _be16(a, 14, vlan)
        _be16(a, 16, ETH_IPV4)
    else:
        _be16(a, 12, ETH_IPV4)
    o = l2
    tot_len = length - l2
    a[:, o] = 0x45
    a[:, o + 1] = tos
    _be16(a, o + 2, tot_len)
    _be16(a, o + 4, np.arange(n) & 0xFFFF if ident is None else ident)
    a[:, o + 8] = ttl
    a[:, o + 9] = proto
    _be32(a, o + 12, src)
    _be32(a, o + 16, dst)
    l4 = o + 20
    _be16(a, l4, sport)
    _be16(a, l4 + 2, dport)
    # deterministic payload
    pl = length - (l4 + l4h)
    if pl > 0:
        r = xorshift64(payload_seed, n * ((pl + 7) // 8)).view(np.uint8)
        a[:, l4 + l4h:] = r[: n * pl].reshape(n, pl)
    if proto == PROTO_UDP:
        _be16(a, l4 + 4, length - l4)
    else:
        _be32(a, l4 + 4, np.arange(n, dtype=np.uint64) * np.uint64(7919))
        a[:, l4 + 12] = 0x50
        a[:, l4 + 13] = 0x18
        _be16(a, l4 + 14, 8192)
    if ip_csum:
        _be16(a, o + 10, csum(ones_sum(a, o, o + 20)))
    if l4_csum:
        pseudo = ones_sum(a, o + 12, o + 20) + proto + (length - l4)
        c = csum(ones_sum(a, l4, length, pseudo))
        if proto == PROTO_UDP:
            c = np.where(c == 0, 0xFFFF, c)
            _be16(a, l4 + 6, c)
        else:
            _be16(a, l4 + 16, c)
    return a


def ipv6_frames(n, length, src_lo, dst_lo, proto, sport, dport, *, payload_seed=2, l4_csum=True):
    """Eth/IPv6/UDP|TCP frames; addresses 2001:db8::<src_lo> / 2001:db8:1::<dst_lo>."""
    length = int(length)
    l4h = 8 if proto == PROTO_UDP else 20
    assert length >= 14 + 40 + l4h
    a = np.zeros((n, length), np.uint8)
    a[:, 0:6] = [0x02, 0, 0, 0, 0, 1]
    a[:, 6:12] = [0x02, 0, 0, 0, 0, 2]
    _be16(a, 12, ETH_IPV6)
    o = 14
    a[:, o] = 0x60
    _be16(a, o + 4, length - o - 40)
    a[:, o + 6] = proto
    a[:, o + 7] = 64
    a[:, o + 8:o + 12] = [0x20, 0x01, 0x0d, 0xb8]
    _be32(a, o + 20, src_lo)
    a[:, o + 24:o + 28] = [0x20, 0x01, 0x0d, 0xb8]
    a[:, o + 28] = 0
    a[:, o + 29] = 1
    _be32(a, o + 36, dst_lo)
    l4 = o + 40
    _be16(a, l4, sport)
    _be16(a, l4 + 2, dport)
    pl = length - (l4 + l4h)
    if pl > 0:
        r = xorshift64(payload_seed, n * ((pl + 7) // 8)).view(np.uint8)
        a[:, l4 + l4h:] = r[: n * pl].reshape(n, pl)
    if proto == PROTO_UDP:
        _be16(a, l4 + 4, length - l4)
    else:
        a[:, l4 + 12] = 0x50
        a[:, l4 + 13] = 0x10
    if l4_csum:
        pseudo = ones_sum(a, o + 8, o + 40) + proto + (length - l4)
        c = csum(ones_sum(a, l4, length, pseudo))
        if proto == PROTO_UDP:
            c = np.where(c == 0, 0xFFFF, c)
            _be16(a, l4 + 6, c)
        else:
            _be16(a, l4 + 16, c)
    return a


def ip4(s):
    p = [int(x) for x in s.split(".")]
    return (p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3]


def be_bytes(v, n):
    return int(v).to_bytes(n, "big")


# ---- BASELINE.json configurations -----------------------------------------
C_SEED = 0x0DDC0FFEE


def c1_frames(n, seed=C_SEED):
    """C1: 64 B IPv4/UDP, 50 % src 10.10.10.x (matches the one PMR), 50 % 10.1.x.x."""
    r = xorshift64(seed, n)
    half = (r & np.uint64(1)).astype(bool)
    lo = ((r >> np.uint64(8)) & np.uint64(0xFFFF)).astype(np.uint64)
    src = np.where(half, np.uint64(ip4("10.10.10.0")) + (lo & np.uint64(0xFF)),
                   np.uint64(ip4("10.1.0.0")) + lo)
    dst = np.full(n, ip4("10.0.0.100"), np.uint64)
    return ipv4_frames(n, 64, src, dst, PROTO_UDP, 1024, 2048).reshape(-1)


def c2_frames(n, seed=C_SEED):
    """C2: 64 B IPv4/UDP, src 10.0.R16, dst 10.1.R16, sport R16, dport R & 63."""
    r = xorshift64(seed, n)
    m16 = np.uint64(0xFFFF)
    src = np.uint64(ip4("10.0.0.0")) + (r & m16)
    dst = np.uint64(ip4("10.1.0.0")) + ((r >> np.uint64(16)) & m16)
    sport = (r >> np.uint64(32)) & m16
    dport = (r >> np.uint64(48)) & np.uint64(63)
    return ipv4_frames(n, 64, src, dst, PROTO_UDP, sport, dport).reshape(-1)


def c2_dport(a, j):
    return (a + 8 * j) & 63


def build_c1_rules(cls, pktio):
    """example/classifier run script rule: ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1
    (example/classifier/odp_classifier_run.sh:17-19)."""
    default = cls.cos_create("DefaultCos", queue=cls.queue(0))
    q1 = cls.cos_create("CoSqueue1", queue=cls.queue(1))
    assert default and q1
    assert cls.default_cos_set(pktio, default) == 0
    pmr = cls.pmr_create([cls.Term(cls.PMR_SIP_ADDR, be_bytes(ip4("10.10.10.0"), 4),
                                   be_bytes(0xFFFFFF00, 4))], default, q1)
    assert pmr
    return {"default": default, "queue1": q1, "pmr": pmr}


def build_c2_rules(cls, pktio, stats=False):
    """C2: 64 PMRs in the reference limits (64 CoS, <= 8 PMR per CoS):
    default -> 8 x SIP_ADDR 10.0.(a<<5).0/19 -> L1[a] -> 7 x UDP_DPORT -> 55 leaves."""
    default = cls.cos_create("c2_default", queue=cls.queue(0), stats_enable=stats)
    l1 = [cls.cos_create(f"c2_l1_{a}", queue=cls.queue(1 + a), stats_enable=stats)
          for a in range(8)]
    leaves = [cls.cos_create(f"c2_leaf_{k}", queue=cls.queue(9 + k), stats_enable=stats)
              for k in range(55)]
    assert default and all(l1) and all(leaves)
    assert cls.default_cos_set(pktio, default) == 0
    pmrs = []
    for a in range(8):
        pmrs.append(cls.pmr_create([cls.Term(cls.PMR_SIP_ADDR,
                                             be_bytes(ip4("10.0.0.0") | (a << 13), 4),
                                             be_bytes(0xFFFFE000, 4))], default, l1[a]))
    for a in range(8):
        for j in range(7):
            leaf = leaves[(a * 7 + j) % 55]
            pmrs.append(cls.pmr_create([cls.Term(cls.PMR_UDP_DPORT, be_bytes(c2_dport(a, j), 2),
                                                 b"\xff\xff")], l1[a], leaf))
    assert all(pmrs) and len(pmrs) == 64
    return {"default": default, "l1": l1, "leaves": leaves, "pmrs": pmrs}


def build_c4_rules(cls, pktio, n_l1=32, per_l1=31):
    """C4 (raised limits, cls.set_limits before any create): default ->
    32 x SIP_ADDR /21 -> L1[a] -> 31 x UDP_DPORT -> 992 leaves = 1024 PMRs."""
    default = cls.cos_create("c4_default", queue=cls.queue(0))
    l1 = [cls.cos_create(f"c4_l1_{a}", queue=cls.queue(1 + a)) for a in range(n_l1)]
    pmrs = []
    for a in range(n_l1):
        pmrs.append(cls.pmr_create([cls.Term(cls.PMR_SIP_ADDR,
                                             be_bytes(ip4("10.0.0.0") | (a << 11), 4),
                                             be_bytes(0xFFFFF800, 4))], default, l1[a]))
    k = 0
    for a in range(n_l1):
        for j in range(per_l1):
            leaf = cls.cos_create(f"c4_leaf_{k}", queue=cls.queue(100 + k))
            k += 1
            pmrs.append(cls.pmr_create([cls.Term(cls.PMR_UDP_DPORT,
                                                 be_bytes((a + 2 * j) & 63, 2), b"\xff\xff")],
                                       l1[a], leaf))
    assert default and all(l1) and all(pmrs)
    assert cls.default_cos_set(pktio, default) == 0
    return {"default": default, "l1": l1, "pmrs": pmrs}


# ---- C2x: C2's shape over the other term kinds --------------------------------
# "a second rule-mix variant should cover the other
# terms (DMAC, ETHTYPE_0/X, VLAN_ID/PCP, IPPROTO, IP_DSCP, SIP6/DIP6,
# CUSTOM_FRAME/L3) with VLAN/QinQ/IPv6 frames". 64-byte frames (68
# algorithmic bytes per packet, as C2); QinQ + IPv6 does not fit 64 bytes, so
# the QinQ frames carry IPv4.
C2X_VIDS = (10, 20, 30, 40, 50, 60, 70, 80)


def c2x_frames(n, seed=C_SEED):
    """C2x traffic, 64 B frames with valid checksums: 35 % Eth/IPv4/UDP,
    15 % Eth/IPv4/TCP, 15 % VLAN/IPv4/UDP (VID from 16 values, half of them
    ruled), 5 % QinQ/IPv4/UDP, 20 % Eth/IPv6/UDP, 5 % IPv4 multicast, 5 %
    IPv4/UDP with DSCP 10. Ports and addresses as C2."""
    r = xorshift64(seed ^ 0xC2C2, n)
    m16 = np.uint64(0xFFFF)
    kind = (r % np.uint64(20)).astype(np.int64)
    src = np.uint64(ip4("10.0.0.0")) + ((r >> np.uint64(8)) & m16)
    dst = np.uint64(ip4("10.1.0.0")) + ((r >> np.uint64(24)) & m16)
    sport = ((r >> np.uint64(40)) & m16).astype(np.int64)
    dport = ((r >> np.uint64(56)) & np.uint64(63)).astype(np.int64)
    vid = np.array(C2X_VIDS + tuple(v + 1 for v in C2X_VIDS))[(r >> np.uint64(20)) & np.uint64(15)]
    a = np.empty((n, 64), np.uint8)

    def put(sel, f):
        idx = np.nonzero(sel)[0]
        if len(idx):
            a[idx] = f(idx)
    put(kind < 7, lambda i: ipv4_frames(len(i), 64, src[i], dst[i], PROTO_UDP, sport[i], dport[i]))
    put((kind >= 7) & (kind < 10),
        lambda i: ipv4_frames(len(i), 64, src[i], dst[i], PROTO_TCP, sport[i], dport[i]))
    put((kind >= 10) & (kind < 13),
        lambda i: ipv4_frames(len(i), 64, src[i], dst[i], PROTO_UDP, sport[i], dport[i],
                              vlan=vid[i] | (3 << 13)))

    def qinq(i):
        f = ipv4_frames(len(i), 64, src[i], dst[i], PROTO_UDP, sport[i], dport[i], vlan=vid[i])
        # outer 0x88A8 tag in front of the 0x8100 one: the IPv4 header moves
        # 4 bytes down and the frame loses 4 payload bytes (checksums redone)
        g = np.zeros_like(f)
        g[:, :12] = f[:, :12]
        _be16(g, 12, 0x88A8)
        _be16(g, 14, 100)
        g[:, 16:] = f[:, 12:60]
        o, l4 = 22, 42
        _be16(g, o + 2, 64 - o)
        g[:, o + 10:o + 12] = 0
        _be16(g, o + 10, csum(ones_sum(g, o, o + 20)))
        _be16(g, l4 + 4, 64 - l4)
        g[:, l4 + 6:l4 + 8] = 0
        c = csum(ones_sum(g, l4, 64, ones_sum(g, o + 12, o + 20) + PROTO_UDP + (64 - l4)))
        _be16(g, l4 + 6, np.where(c == 0, 0xFFFF, c))
        return g
    put(kind == 13, qinq)
    put((kind >= 14) & (kind < 18),
        lambda i: ipv6_frames(len(i), 64, (r[i] >> np.uint64(8)) & m16, (r[i] >> np.uint64(24)) & m16,
                              PROTO_UDP, sport[i], dport[i]))
    put(kind == 18, lambda i: ipv4_frames(len(i), 64, src[i], np.uint64(ip4("239.1.0.0")) + (dst[i] & m16),
                                          PROTO_UDP, sport[i], dport[i],
                                          dmac=[0x01, 0x00, 0x5E, 0x01, 0x00, 0x01]))
    put(kind == 19, lambda i: ipv4_frames(len(i), 64, src[i], dst[i], PROTO_UDP, sport[i], dport[i],
                                          tos=10 << 2))
    return a.reshape(-1)


def build_c2x_rules(cls, pktio, stats=False):
    """C2x: 62 PMRs over 63 CoS in the reference limits, every level-1 and
    level-2 rule a different term kind than C2's (SIP_ADDR / UDP_DPORT):
    default -> {ETHTYPE_0 VLAN, ETHTYPE_0 QinQ, ETHTYPE_0 IPv6 + IPPROTO,
    DMAC multicast, IP_DSCP + IPPROTO, IPPROTO TCP, IPPROTO UDP} -> VLAN_ID_0,
    VLAN_ID_X + PCP, DIP6 /120 prefixes, CUSTOM_L3, TCP_DPORT, UDP_SPORT +
    CUSTOM_FRAME, ... -> leaves."""
    T = cls.Term
    q = cls.queue
    n = [0]

    def cos(name):
        c = cls.cos_create(name, queue=q(n[0]), stats_enable=stats)
        n[0] += 1
        assert c, name
        return c
    default = cos("c2x_default")
    assert cls.default_cos_set(pktio, default) == 0
    l1 = {k: cos("c2x_" + k) for k in ("vlan", "qinq", "v6", "mcast", "dscp", "tcp", "udp")}
    leaves = [cos(f"c2x_leaf_{k}") for k in range(55)]
    pmrs = []

    def pmr(terms, src, dst):
        h = cls.pmr_create(terms, src, dst)
        assert h, (terms, src, dst)
        pmrs.append(h)
    pmr([T(cls.PMR_ETHTYPE_0, b"\x81\x00", b"\xff\xff")], default, l1["vlan"])
    pmr([T(cls.PMR_ETHTYPE_0, b"\x88\xa8", b"\xff\xff")], default, l1["qinq"])
    pmr([T(cls.PMR_ETHTYPE_0, b"\x86\xdd", b"\xff\xff"), T(cls.PMR_IPPROTO, b"\x11", b"\xff")],
        default, l1["v6"])
    pmr([T(cls.PMR_DMAC, b"\x01\x00\x5e\x00\x00\x00", b"\xff\xff\xff\x80\x00\x00")],
        default, l1["mcast"])
    pmr([T(cls.PMR_IP_DSCP, b"\x0a", b"\x3f"), T(cls.PMR_IPPROTO, b"\x11", b"\xff")],
        default, l1["dscp"])
    pmr([T(cls.PMR_IPPROTO, b"\x06", b"\xff")], default, l1["tcp"])
    pmr([T(cls.PMR_IPPROTO, b"\x11", b"\xff")], default, l1["udp"])
    k = 0

    def leaf():
        nonlocal k
        c = leaves[k % len(leaves)]
        k += 1
        return c
    for v in C2X_VIDS:
        pmr([T(cls.PMR_VLAN_ID_0, be_bytes(v, 2), b"\x0f\xff")], l1["vlan"], leaf())
    for j in range(4):
        pmr([T(cls.PMR_VLAN_ID_X, be_bytes(C2X_VIDS[j], 2), b"\x0f\xff")], l1["qinq"], leaf())
    pmr([T(cls.PMR_VLAN_PCP_0, b"\x00", b"\x07")], l1["qinq"], leaf())
    for j in range(8):
        # 2001:db8:1::/120 + j << 13 .. the generator's dst low 16 bits
        pmr([T(cls.PMR_DIP6_ADDR,
               bytes.fromhex("20010db8000100000000000000000000")[:14] + be_bytes(j << 13, 2),
               b"\xff" * 14 + b"\xe0\x00")], l1["v6"], leaf())
    for j in range(8):
        pmr([T(cls.PMR_UDP_DPORT, be_bytes(8 * j, 2), b"\xff\xf8")], l1["mcast"], leaf())
    for j in range(8):
        pmr([T(cls.PMR_CUSTOM_L3, be_bytes(j << 5, 1), b"\xe0", offset=13)], l1["dscp"], leaf())
    for j in range(8):
        pmr([T(cls.PMR_TCP_DPORT, be_bytes(c2_dport(j, 0) + 8 * j % 64, 2), b"\xff\xff")],
            l1["tcp"], leaf())
    for j in range(8):
        pmr([T(cls.PMR_UDP_SPORT, be_bytes(j << 13, 2), b"\xe0\x00"),
             T(cls.PMR_CUSTOM_FRAME, b"\x08\x00", b"\xff\xff", offset=12)], l1["udp"], leaf())
    return {"default": default, "l1": l1, "leaves": leaves, "pmrs": pmrs}


# ---- C3: IMIX + 256 PMR DAG + RX checksum verify ----------------------------
IMIX_SIZES = (64, 570, 1518)       # 7:4:1, mean 353.83 B


def c3_frames(n, seed=C_SEED, align=64):
    """C3 traffic: IMIX 7:4:1 of 64/570/1518 B, 80 % IPv4 /
    20 % IPv6, 50/50 UDP/TCP (64 B IPv6 frames are UDP: a TCP header does not
    fit), valid checksums except: 0.5 % bad IPv4 header checksum, 0.5 % bad
    L4 checksum, 0.5 % IPv4/UDP checksum 0, 0.5 % IPv4 fragments (MF set).
    Returns (buf u8, desc DESC_DT[n]); frames start `align`-aligned."""
    r = xorshift64(seed ^ 0xC3C3, n)
    r2 = xorshift64(seed ^ 0x5A5A3C3, n)
    sz_i = (r % np.uint64(12)).astype(np.int64)
    size = np.where(sz_i < 7, 64, np.where(sz_i < 11, 570, 1518))
    v6 = ((r >> np.uint64(8)) % np.uint64(5)) == 0
    tcp = (((r >> np.uint64(12)) & np.uint64(1)) == 1) & ~(v6 & (size == 64))
    m16 = np.uint64(0xFFFF)
    src = np.uint64(ip4("10.0.0.0")) + ((r >> np.uint64(16)) & m16)
    dst = np.uint64(ip4("10.1.0.0")) + ((r >> np.uint64(32)) & m16)
    sport = (r2 & m16).astype(np.int64)
    dport = ((r2 >> np.uint64(16)) & np.uint64(63)).astype(np.int64)
    special = ((r2 >> np.uint64(24)) % np.uint64(1000)).astype(np.int64)

    alen = (size + align - 1) // align * align
    offs = np.zeros(n, np.int64)
    if n:
        offs[1:] = np.cumsum(alen)[:-1]
    total = int(alen.sum()) if n else 0
    buf = np.zeros(total + 64, np.uint8)
    desc = np.zeros(n, DESC_DT)
    desc["offset"] = offs
    desc["len"] = size
    for length in IMIX_SIZES:
        for is6 in (False, True):
            for is_tcp in (False, True):
                idx = np.nonzero((size == length) & (v6 == is6) & (tcp == is_tcp))[0]
                if len(idx) == 0:
                    continue
                proto = PROTO_TCP if is_tcp else PROTO_UDP
                if is6:
                    a = ipv6_frames(len(idx), length, src[idx], dst[idx], proto, sport[idx],
                                    dport[idx], payload_seed=int(idx[0]) + 11)
                else:
                    a = ipv4_frames(len(idx), length, src[idx], dst[idx], proto, sport[idx],
                                    dport[idx], payload_seed=int(idx[0]) + 7)
                    sp = special[idx]
                    l4 = 34
                    # fragments (MF), header checksum recomputed
                    fr = np.nonzero((sp >= 15) & (sp < 20))[0]
                    if len(fr):
                        a[fr, 14 + 6] |= 0x20
                        a[fr, 24:26] = 0
                        c = csum(ones_sum(a[fr], 14, 34))
                        a[fr, 24] = (c >> 8) & 0xFF
                        a[fr, 25] = c & 0xFF
                    if not is_tcp:
                        z = np.nonzero((sp >= 10) & (sp < 15))[0]
                        a[z, l4 + 6:l4 + 8] = 0
                    bad3 = np.nonzero(sp < 5)[0]
                    a[bad3, 25] ^= 0x01
                bad4 = np.nonzero((special[idx] >= 5) & (special[idx] < 10))[0]
                a[bad4, length - 1] ^= 0x5A
                rows = offs[idx][:, None] + np.arange(length)[None, :]
                buf[rows] = a
    return buf, desc


def c3_term_menu(cls, k, h):
    """The k-th PMR's terms for the C3 DAG (h: a per-PMR hash). Values are
    drawn from the C3 traffic distributions so every kind both hits and
    misses; the mix covers the slotted, exact-match and generic compare
    paths."""
    T = cls.Term
    x = h & 15
    kind = k % 11
    if kind == 0:
        return [T(cls.PMR_SIP_ADDR, be_bytes(ip4("10.0.0.0") | (x << 12), 4),
                  be_bytes(0xFFFFF000, 4))]
    if kind == 1:
        return [T(cls.PMR_DIP_ADDR, be_bytes(ip4("10.1.0.0") | (x << 12), 4),
                  be_bytes(0xFFFFF000, 4))]
    if kind == 2:
        return [T(cls.PMR_UDP_DPORT, be_bytes(h & 63, 2), b"\xff\xff")]
    if kind == 3:
        return [T(cls.PMR_TCP_DPORT, be_bytes(h & 63, 2), b"\xff\xff")]
    if kind == 4:
        return [T(cls.PMR_IPPROTO, bytes([PROTO_TCP if h & 1 else PROTO_UDP]), b"\xff")]
    if kind == 5:
        return [T(cls.PMR_SIP6_ADDR, bytes(12) + be_bytes(x, 4),
                  bytes(12) + be_bytes(0xF, 4))]
    if kind == 6:
        return [T(cls.PMR_ETHTYPE_0, be_bytes(ETH_IPV6 if h & 1 else ETH_IPV4, 2), b"\xff\xff")]
    if kind == 7:
        return [T(cls.PMR_LEN, int(IMIX_SIZES[h % 3]).to_bytes(4, "little"), b"\xff\xff\xff\xff")]
    if kind == 8:
        return [T(cls.PMR_IP_DSCP, bytes([0]), bytes([0x3F]))]
    if kind == 9:
        return [T(cls.PMR_SIP_ADDR, be_bytes(ip4("10.0.0.0") | (x << 8), 4),
                  be_bytes(0xFFFF0F00, 4)),
                T(cls.PMR_UDP_DPORT, be_bytes(h & 7, 2), be_bytes(7, 2))]
    return [T(cls.PMR_CUSTOM_L3, bytes([PROTO_UDP]), b"\xff", offset=9, val_sz=1)]


def build_c3_rules(cls, pktio, stats=False, seed=0xC3):
    """C3: 256 PMRs as a DAG over 63 CoS (8 PMRs on each
    of CoS 0..31, destination index > source index), CoS 0 the default, CoS
    63 the error CoS (checksum / header errors). Mixed term kinds."""
    coses = [cls.cos_create(f"c3_{i}", queue=cls.queue(i), stats_enable=stats)
             for i in range(63)]
    err = cls.cos_create("c3_error", queue=cls.queue(63), stats_enable=stats)
    assert all(coses) and err
    assert cls.default_cos_set(pktio, coses[0]) == 0
    assert cls.error_cos_set(pktio, err) == 0
    hs = xorshift64(seed, 256)
    pmrs = []
    for c in range(32):
        for j in range(8):
            k = c * 8 + j
            h = int(hs[k] >> np.uint64(8))
            d = c + 1 + (h >> 12) % (62 - c)
            p = cls.pmr_create(c3_term_menu(cls, k, h), coses[c], coses[d], mark=(k + 1) & 0xFFFF)
            assert p, ("pmr", k)
            pmrs.append(p)
    return {"coses": coses, "error": err, "pmrs": pmrs}


# ---- C5: example/l3fwd, 10 M flows over <= 32 routes ------------------------
C5_FLOWS = 10_000_000


def c5_routes(seed=0xC5, n=32):
    """`n` canonical IPv4 routes (host bits zero, depth 8..28) over 10.0.0.0/8,
    nested and overlapping so the newest-first scan order and the LPM trie's
    quirks both matter; output ports 0..3. Returns a list of
    (addr, depth, oif_id, src_mac, dst_mac) in add order."""
    r = xorshift64(seed, n)
    depths = (8, 12, 16, 18, 20, 22, 24, 26, 28)
    out = []
    for k in range(n):
        h = int(r[k])
        d = depths[h % len(depths)]
        addr = (ip4("10.0.0.0") | ((h >> 8) & 0x00FFFFFF)) & ((0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF)
        if k % 4 == 0:      # pin a quarter of them inside 10.1/16 so prefixes nest
            addr = (ip4("10.1.0.0") | ((h >> 8) & 0xFFFF)) & ((0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF)
            d = max(d, 16)
            addr &= (0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF
        port = (h >> 40) & 3
        src = [0x02, 0x00, 0x00, 0x00, 0x10, port]
        dst = [0x02, 0x00, 0x00, 0x01, k, port]
        out.append((addr, d, port, src, dst))
    return out


def c5_frames(n, routes, seed=C_SEED, flows=C5_FLOWS):
    """C5 traffic: 64 B IPv4/UDP|TCP frames, packet i carries flow i % flows
    (distinct 5-tuples: src 172.16.0.0 + flow, sport / dport from the flow
    index); dst inside a random route's subnet for ~97 % of packets, an
    unrouted 192.0.2.x address otherwise. Returns the flat frame buffer."""
    idx = np.arange(n, dtype=np.uint64) % np.uint64(flows)
    r = xorshift64(seed ^ 0xC5C5, n)
    nr = len(routes)
    pick = (r % np.uint64(max(nr, 1))).astype(np.int64)
    addr = np.array([rt[0] for rt in routes] or [0], np.uint64)
    depth = np.array([rt[1] for rt in routes] or [32], np.uint64)
    host = (r >> np.uint64(16)) & ((np.uint64(1) << (np.uint64(32) - depth[pick])) - np.uint64(1))
    dst = addr[pick] | host
    miss = ((r >> np.uint64(56)) % np.uint64(32)) == 0
    dst = np.where(miss, np.uint64(ip4("192.0.2.0")) + (r & np.uint64(0xFF)), dst)
    src = np.uint64(ip4("172.16.0.0")) + idx
    sport = (idx & np.uint64(0xFFFF)).astype(np.int64)
    dport = ((idx >> np.uint64(16)) + np.uint64(1024)).astype(np.int64) & 0xFFFF
    tcp = ((r >> np.uint64(8)) & np.uint64(1)) == 1
    a = np.empty((n, 64), np.uint8)
    for is_tcp in (False, True):
        sel = np.nonzero(tcp == is_tcp)[0]
        if len(sel):
            a[sel] = ipv4_frames(len(sel), 64, src[sel], dst[sel],
                                 PROTO_TCP if is_tcp else PROTO_UDP, sport[sel], dport[sel])
    return a.reshape(-1)
