"""Rule sets and frame corpora shared by the parity tests.

`all_terms_rules` builds a CoS graph that exercises every PMR term the
reference can create (odp_classification.c:661-720), multi-term PMRs, marks,
a DROP CoS, an error CoS and a second rule level, with values taken from the
golden frames so that rules do match part of the corpus.
"""
import numpy as np

from helpers import GOLDEN, golden_frames
from odp_amd import gen


def _b(h):
    return bytes.fromhex(h)


def all_terms_rules(cls, pktio, stats=True):
    T = cls.Term
    q = cls.queue
    default = cls.cos_create("default", queue=q(0), stats_enable=stats)
    error = cls.cos_create("error", queue=q(1), stats_enable=stats)
    drop = cls.cos_create("drop", action=cls.COS_ACTION_DROP, stats_enable=stats)
    mk = lambda name, n: cls.cos_create(name, queue=q(n), stats_enable=stats)  # noqa: E731
    c = {name: mk(name, 10 + i) for i, name in enumerate([
        "vlan", "ipv6", "tcp", "udp", "ipsec", "custom", "l2", "len", "dscp", "mcast",
        "sctp_l3", "vlan_leaf", "udp_leaf", "tcp_leaf", "v6_leaf"])}
    assert cls.default_cos_set(pktio, default) == 0
    assert cls.error_cos_set(pktio, error) == 0
    P = []

    def pmr(terms, src, dst, mark=None):
        h = cls.pmr_create(terms, src, dst, mark=mark)
        assert h, (terms, src, dst)
        P.append(h)
        return h

    # level 1 (default CoS): <= 8 rules, first match wins
    pmr([T(cls.PMR_ETHTYPE_0, b"\x81\x00", b"\xff\xff")], default, c["vlan"], mark=11)
    pmr([T(cls.PMR_ETHTYPE_0, b"\x86\xdd", b"\xff\xff"),
         T(cls.PMR_IPPROTO, b"\x11", b"\xff")], default, c["ipv6"], mark=12)
    pmr([T(cls.PMR_IPPROTO, b"\x06", b"\xff")], default, c["tcp"])
    pmr([T(cls.PMR_IPSEC_SPI, b"\x00\x00\x00\x7b", b"\xff\xff\xff\xff")], default, c["ipsec"], mark=14)
    pmr([T(cls.PMR_DMAC, b"\x01\x00\x5e\x00\x00\x00", b"\xff\xff\xff\x00\x00\x00")],
        default, c["mcast"], mark=15)
    pmr([T(cls.PMR_CUSTOM_FRAME, b"\x88\xb5", b"\xff\xff", offset=12)], default, c["custom"])
    pmr([T(cls.PMR_IP_DSCP, b"\x00", b"\x3f"), T(cls.PMR_IPPROTO, b"\x11", b"\xff"),
         T(cls.PMR_LEN, (1500).to_bytes(4, "little"), b"\xff\xff\xff\xff")], default, c["len"])
    pmr([T(cls.PMR_IPPROTO, b"\x11", b"\xff")], default, c["udp"], mark=0)

    # level 2
    pmr([T(cls.PMR_VLAN_ID_0, b"\x00\x0a", b"\x0f\xff")], c["vlan"], c["vlan_leaf"], mark=21)
    pmr([T(cls.PMR_VLAN_ID_X, b"\x00\x14", b"\xff\xff")], c["vlan"], c["vlan_leaf"], mark=22)
    pmr([T(cls.PMR_ETHTYPE_X, b"\x08\x00", b"\xff\xff"),
         T(cls.PMR_VLAN_PCP_0, b"\x00", b"\x07")], c["vlan"], drop)
    pmr([T(cls.PMR_UDP_DPORT, b"\x00\x3f", b"\xff\xff")], c["udp"], c["udp_leaf"], mark=31)
    pmr([T(cls.PMR_UDP_SPORT, b"\x00\x00", b"\xff\x00")], c["udp"], c["udp_leaf"], mark=32)
    pmr([T(cls.PMR_SIP_ADDR, b"\xc0\xa8\x00\x00", b"\xff\xff\x00\x00"),
         T(cls.PMR_DIP_ADDR, b"\xc0\xa8\x00\x00", b"\xff\xff\x00\x00")], c["udp"], c["l2"])
    pmr([T(cls.PMR_CUSTOM_L3, b"\x40", b"\xff", offset=8)], c["udp"], c["dscp"], mark=33)
    pmr([T(cls.PMR_TCP_DPORT, b"\x00\x00", b"\x00\x00"),
         T(cls.PMR_TCP_SPORT, b"\x04\x00", b"\xff\x00")], c["tcp"], c["tcp_leaf"], mark=41)
    pmr([T(cls.PMR_LD_VNI, b"\x00\x00\x00\x01", b"\xff\xff\xff\xff")], c["tcp"], drop)
    pmr([T(cls.PMR_SIP6_ADDR, bytes(16), bytes(16))], c["ipv6"], c["v6_leaf"], mark=51)
    pmr([T(cls.PMR_DIP6_ADDR, b"\xff" + bytes(15), b"\xff" + bytes(15))], c["ipv6"], c["v6_leaf"])
    pmr([T(cls.PMR_IP_DSCP, b"\x2e", b"\x3f")], c["ipv6"], c["dscp"])
    pmr([T(cls.PMR_IPPROTO, b"\x84", b"\xff")], c["mcast"], c["sctp_l3"], mark=61)
    return {"default": default, "error": error, "drop": drop, "cos": c, "pmrs": P}


def wide_slots_rules(cls, pktio, stats=False):
    """Rules whose terms read more than 16 of the 19 key slots (DMAC, SMAC,
    ETHTYPE_X, VLAN_ID_X, DSCP, every word of SIP6 and DIP6, the L4 ports,
    the IPsec SPI and the frame length): the hit-map table then keeps slots
    16..18 out of its 16-word key vector (xm_kx, classify_gf.hip KX)."""
    T = cls.Term
    q = cls.queue
    default = cls.cos_create("ws_default", queue=q(0), stats_enable=stats)
    leaves = [cls.cos_create(f"ws_{k}", queue=q(1 + k), stats_enable=stats) for k in range(12)]
    assert default and all(leaves)
    assert cls.default_cos_set(pktio, default) == 0
    rules = [
        [T(cls.PMR_DMAC, b"\x02\x00\x00\x00\x00\x01", b"\xff" * 6)],
        [T(cls.PMR_CUSTOM_FRAME, b"\x00\x00\x00\x02", b"\xff\xff\xff\xff", offset=8)],
        [T(cls.PMR_ETHTYPE_X, b"\x08\x00", b"\xff\xff")],
        [T(cls.PMR_VLAN_ID_X, b"\x00\x14", b"\x0f\xff")],
        [T(cls.PMR_IP_DSCP, b"\x0a", b"\x3f"), T(cls.PMR_IPPROTO, b"\x11", b"\xff")],
        [T(cls.PMR_SIP6_ADDR, bytes.fromhex("20010db8000000000000000000000001"), b"\xff" * 16)],
        [T(cls.PMR_DIP6_ADDR, bytes.fromhex("20010db8000100000000000000000002"), b"\xff" * 16)],
        [T(cls.PMR_UDP_DPORT, b"\x00\x35", b"\xff\xff")],
        [T(cls.PMR_IPSEC_SPI, b"\x00\x00\x00\x7b", b"\xff\xff\xff\xff")],
        [T(cls.PMR_LEN, (64).to_bytes(4, "little"), b"\xff\xff\xff\xff"),
         T(cls.PMR_IPPROTO, b"\x06", b"\xff")],
        [T(cls.PMR_UDP_SPORT, b"\x00\x00", b"\xff\x00")],
        [T(cls.PMR_IPPROTO, b"\x11", b"\xff")],
    ]
    # at most 8 PMRs per CoS (the reference's limits): rules 7.. hang below
    # the default CoS's eighth rule (IPPROTO UDP)
    mid = cls.cos_create("ws_mid", queue=q(13), stats_enable=stats)
    assert mid
    P = []
    for k, terms in enumerate(rules[:7]):
        h = cls.pmr_create(terms, default, leaves[k], mark=k + 1)
        assert h, terms
        P.append(h)
    P.append(cls.pmr_create([T(cls.PMR_IPPROTO, b"\x11", b"\xff")], default, mid, mark=40))
    for k, terms in enumerate(rules[7:], 7):
        h = cls.pmr_create(terms, mid, leaves[k], mark=k + 1)
        assert h, terms
        P.append(h)
    assert all(P)
    return {"default": default, "leaves": leaves, "pmrs": P}


def wide_slots_corpus(n, seed=3):
    """Frames for wide_slots_rules: IPv4 UDP / TCP (half of them with the
    ruled DMAC, some VLAN-tagged, DSCP 10 on some), IPv6 UDP with the ruled
    source / destination addresses on some, then the mutation and IMIX edge
    corpora. Returns a list of bytes."""
    rng = np.random.default_rng(seed)
    out = []
    m = n // 3
    for k in range(m):
        kind = int(rng.integers(0, 6))
        sport, dport = int(rng.integers(0, 1 << 16)), int(rng.choice([53, 80, 4000]))
        dm = [0x02, 0, 0, 0, 0, 1 if rng.integers(0, 2) else 9]
        if kind < 4:
            proto = gen.PROTO_TCP if kind == 3 else gen.PROTO_UDP
            length = int(rng.choice([64, 64, 128]))
            f = gen.ipv4_frames(1, length, np.array([gen.ip4("10.0.0.1")], np.uint64),
                                np.array([gen.ip4("10.1.0.1")], np.uint64), proto,
                                np.array([sport]), np.array([dport]), dmac=dm,
                                tos=(10 << 2) if kind == 2 else 0,
                                vlan=int(rng.choice([20, 21])) if kind == 1 else None)
        else:
            f = gen.ipv6_frames(1, 80, np.array([int(rng.choice([1, 5]))], np.uint64),
                                np.array([int(rng.choice([2, 7]))], np.uint64), gen.PROTO_UDP,
                                np.array([sport]), np.array([dport]))
        out.append(bytes(f.reshape(-1)))
    return out + mutate_corpus(m, seed=seed + 1) + imix_edge_corpus(n - 2 * m, seed=seed + 2)


def mutate_corpus(n, seed=7, max_len=220):
    """Golden frames + generated VLAN / QinQ / SNAP / IPv6-ext / fragment frames,
    then random byte flips and truncations (edge cases the reference tests:
    short, ragged, malformed)."""
    rng = np.random.default_rng(seed)
    _, base = golden_frames()
    extra = []
    v4 = gen.ipv4_frames(4, 80, np.array([gen.ip4("192.168.1.1")] * 4, np.uint64),
                         np.array([gen.ip4("192.168.2.2")] * 4, np.uint64), gen.PROTO_UDP,
                         [0x3f, 1024, 63, 7], [63, 2048, 9, 0x3f], vlan=None)
    extra += [bytes(r) for r in v4]
    vl = gen.ipv4_frames(4, 96, np.arange(4, dtype=np.uint64), np.arange(4, dtype=np.uint64),
                         gen.PROTO_TCP, 1024, 80, vlan=0x00a)
    extra += [bytes(r) for r in vl]
    v6 = gen.ipv6_frames(4, 120, np.arange(4, dtype=np.uint64), np.arange(4, dtype=np.uint64),
                         gen.PROTO_UDP, 0x3f, 63)
    extra += [bytes(r) for r in v6]
    # QinQ around an IPv4/UDP frame
    f = bytearray(bytes(v4[0]))
    extra.append(bytes(f[:12]) + b"\x88\xa8\x00\x14\x81\x00\x00\x0a" + bytes(f[12:]))
    # IPv6 with hop-by-hop + routing ext headers then UDP
    f6 = bytearray(bytes(v6[1]))
    ext = bytes([0x2B, 0]) + bytes(6) + bytes([0x11, 0]) + bytes(6)
    f6[20] = 0x00
    f6 = f6[:54] + ext + f6[54:]
    pl = int.from_bytes(f6[18:20], "big") + len(ext)
    f6[18:20] = pl.to_bytes(2, "big")
    extra.append(bytes(f6))
    corpus = base + extra
    out = []
    for i in range(n):
        f = bytearray(corpus[rng.integers(len(corpus))])
        k = rng.integers(10)
        if k < 3:                                  # keep intact
            pass
        elif k < 6:                                # flip 1..3 bytes in the headers
            for _ in range(rng.integers(1, 4)):
                if len(f):
                    j = int(rng.integers(min(len(f), 64)))
                    f[j] = int(rng.integers(256))
        elif k < 8:                                # truncate
            f = f[: int(rng.integers(0, len(f) + 1))]
        elif k < 9:                                # random bytes
            f = bytearray(rng.integers(0, 256, int(rng.integers(0, max_len)), dtype=np.uint8))
        else:                                      # extend with junk
            f = f + bytearray(rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8))
        out.append(bytes(f))
    return out


def plain64_corpus(n, seed=5):
    """64-byte Eth/IPv4/UDP|TCP frames with the edge properties the register
    fast path must reproduce: fragments, broadcast / multicast MAC and IP,
    UDP port 4500 (IPsec NAT-T marker), zero UDP checksum, corrupted IPv4 /
    L4 checksums, plus a share of frames that must leave the fast path
    (short UDP length, oversize tot_len, IHL > 5, VLAN, IPv6)."""
    rng = np.random.default_rng(seed)
    r = rng.integers(0, 1 << 62, size=(n, 4), dtype=np.int64).astype(np.uint64)
    src = np.uint64(gen.ip4("192.168.0.0")) + (r[:, 0] & np.uint64(0xFFFF))
    dst = np.uint64(gen.ip4("192.168.0.0")) + (r[:, 1] & np.uint64(0xFFFF))
    kind = rng.integers(0, 16, n)
    dst = np.where(kind == 1, np.uint64(0xFFFFFFFF), dst)
    dst = np.where(kind == 2, np.uint64(gen.ip4("224.0.0.5")), dst)
    sport = (r[:, 2] & np.uint64(0xFFFF))
    dport = (r[:, 3] & np.uint64(63))
    dport = np.where(kind == 3, np.uint64(4500), dport)
    udp = gen.ipv4_frames(n, 64, src, dst, gen.PROTO_UDP, sport, dport)
    tcp = gen.ipv4_frames(n, 64, src, dst, gen.PROTO_TCP, sport, dport)
    fr = np.where((rng.integers(0, 2, n) == 1)[:, None], tcp, udp)
    fr[kind == 4, 20] |= 0x20                        # more-fragments bit
    f4 = fr[kind == 4]                               # ... with a valid header checksum
    f4[:, 24:26] = 0
    c = gen.csum(gen.ones_sum(f4, 14, 34))
    f4[:, 24] = (c >> 8) & 0xFF
    f4[:, 25] = c & 0xFF
    fr[kind == 4] = f4
    fr[kind == 5, 0:6] = 0xFF                        # broadcast MAC
    fr[kind == 6, 0] |= 0x01                         # multicast MAC
    sel = (kind == 7) & (fr[:, 23] == 17)
    fr[sel, 40:42] = 0                               # UDP checksum 0
    fr[kind == 8, 24] ^= 0x5A                        # bad IPv4 header checksum
    fr[kind == 9, 60] ^= 0x33                        # bad L4 checksum
    sel = (kind == 10) & (fr[:, 23] == 17)
    fr[sel, 38:40] = [0, 4]                          # UDP length < 8 (udp_err)
    fr[kind == 11, 16:18] = [0, 60]                  # tot_len > frame -> ip_err
    fr[kind == 12, 14] = 0x46                        # IHL 6 (options)
    sel = kind == 13                                 # VLAN tag
    fr[sel, 12:14] = [0x81, 0x00]
    sel = kind == 14                                 # IPv6 ethertype
    fr[sel, 12:14] = [0x86, 0xDD]
    # keep whole waves plain too: first half of every 128 frames untouched
    plain_wave = (np.arange(n) % 128) < 64
    base = np.where((rng.integers(0, 2, n) == 1)[:, None], tcp, udp)
    keep = plain_wave & (kind >= 10)
    fr[keep] = base[keep]
    return fr.reshape(-1)


def simple_mixed_rules(cls, pktio, stats=True):
    """Single-compare rules only (TBL_SIMPLE): exact-match groups large enough
    for hash tables, with duplicate values whose first-match order matters,
    small groups that stay linear, ODP_PMR_LEN, a never-matching LD_VNI rule
    and a rule with no terms (matches everything)."""
    T = cls.Term
    q = cls.queue
    mk = lambda name, n: cls.cos_create(name, queue=q(n), stats_enable=stats)  # noqa: E731
    default = mk("default", 0)
    l1 = [mk(f"l1_{i}", 1 + i) for i in range(8)]
    leaves = [mk(f"leaf_{i}", 20 + i) for i in range(40)]
    assert cls.default_cos_set(pktio, default) == 0
    # default: 8 UDP_DPORT rules (hash group), two share the value 7
    dports = [7, 3, 7, 9, 11, 13, 0x3f, 1]
    for i, d in enumerate(dports):
        assert cls.pmr_create([T(cls.PMR_UDP_DPORT, gen.be_bytes(d, 2), b"\xff\xff")],
                              default, l1[i], mark=100 + i)
    # l1[0]: SIP /24 hash group (7 rules) + LEN + never + match-all, order matters
    for i in range(5):
        assert cls.pmr_create([T(cls.PMR_SIP_ADDR, gen.be_bytes(gen.ip4(f"192.168.{i}.0"), 4),
                                 gen.be_bytes(0xFFFFFF00, 4))], l1[0], leaves[i])
    assert cls.pmr_create([T(cls.PMR_LD_VNI, b"\0\0\0\1", b"\xff\xff\xff\xff")], l1[0], leaves[5])
    assert cls.pmr_create([T(cls.PMR_LEN, (64).to_bytes(4, "little"), b"\xff\xff\xff\xff")],
                          l1[0], leaves[6], mark=7)
    assert cls.pmr_create([], l1[0], leaves[7], mark=8)
    # l1[1..7]: TCP/UDP sport groups of 7 (hash) and 2 (linear)
    for a in range(1, 8):
        for j in range(7 if a % 2 else 2):
            assert cls.pmr_create([T(cls.PMR_UDP_SPORT, gen.be_bytes((a * 7 + j) & 0xff, 2),
                                     b"\x00\xff")], l1[a], leaves[(8 + a * 4 + j) % 40])
    return {"default": default}


def random_mixed_rules(cls, pktio, seed, n_cos=24, complex_share=0.3, stats=True):
    """Random CoS DAG (destination index > source index, <= 8 rules per CoS)
    over single-word terms, IPv4 / IPv6 alternative terms and complex PMRs
    (multi-term, CUSTOM_L3 with its length guard, CUSTOM_FRAME), with values
    drawn from mutate_corpus's frames so rules both hit and miss. Exercises
    the hybrid hash walk (TBL_XWALK) against the walk and the oracle."""
    rng = np.random.default_rng(seed)
    T = cls.Term
    ports = [0x3f, 63, 1024, 2048, 80, 9, 7, 0]

    def one():
        k = int(rng.integers(12))
        if k == 0:
            d = int(rng.choice([8, 16, 24, 32]))
            return T(cls.PMR_SIP_ADDR, b"\xc0\xa8\x01\x01", (0xFFFFFFFF << (32 - d) & 0xFFFFFFFF).to_bytes(4, "big"))
        if k == 1:
            return T(cls.PMR_DIP_ADDR, b"\xc0\xa8\x02\x02", b"\xff\xff\xff\x00")
        if k in (2, 3, 4, 5):
            term = [cls.PMR_UDP_DPORT, cls.PMR_UDP_SPORT, cls.PMR_TCP_DPORT, cls.PMR_TCP_SPORT][k - 2]
            m = b"\xff\xff" if rng.integers(2) else b"\x00\xff"
            return T(term, int(rng.choice(ports)).to_bytes(2, "big"), m)
        if k == 6:
            return T(cls.PMR_IPPROTO, bytes([int(rng.choice([6, 17, 0x84]))]), b"\xff")
        if k == 7:
            return T(cls.PMR_IP_DSCP, bytes([int(rng.choice([0, 0x2e]))]), b"\x3f")
        if k == 8:
            et = int(rng.choice([0x0800, 0x86dd, 0x8100, 0x88a8]))
            return T(cls.PMR_ETHTYPE_0, et.to_bytes(2, "big"), b"\xff\xff")
        if k == 9:
            return T(cls.PMR_SIP6_ADDR, bytes(15) + bytes([int(rng.integers(4))]),
                     bytes(15) + b"\x03")
        if k == 10:
            return T(cls.PMR_LEN, int(rng.choice([60, 64, 80, 96, 120])).to_bytes(4, "little"),
                     b"\xff\xff\xff\xff")
        return T(cls.PMR_IPSEC_SPI, b"\x00\x00\x00\x7b", b"\xff\xff\xff\xff")

    def complex_terms():
        k = int(rng.integers(3))
        if k == 0:
            off = int(rng.integers(0, 24))
            sz = int(rng.integers(1, 3))
            return [T(cls.PMR_CUSTOM_L3, bytes(int(v) for v in rng.integers(0, 256, sz)) if rng.integers(3) == 0
                      else bytes([0x40, 0x11][:sz]) if off == 8 else bytes(sz),
                      b"\xff" * sz if rng.integers(2) else b"\x0f" * sz, offset=off, val_sz=sz)]
        if k == 1:
            return [T(cls.PMR_CUSTOM_FRAME, b"\x08\x00", b"\xff\xff", offset=12)]
        return [one(), one()]

    coses = [cls.cos_create(f"r{seed}_{i}", queue=cls.queue(i), stats_enable=stats)
             for i in range(n_cos)]
    err = cls.cos_create(f"r{seed}_err", queue=cls.queue(n_cos), stats_enable=stats)
    assert all(coses) and err
    assert cls.default_cos_set(pktio, coses[0]) == 0
    assert cls.error_cos_set(pktio, err) == 0
    pmrs = []
    for c in range(n_cos // 2):
        for _ in range(int(rng.integers(1, 9))):
            d = int(rng.integers(c + 1, n_cos))
            terms = complex_terms() if rng.random() < complex_share else [one()]
            p = cls.pmr_create(terms, coses[c], coses[d], mark=int(rng.integers(0, 5)))
            if p:
                pmrs.append(p)
    return {"coses": coses, "error": err, "pmrs": pmrs}


def _ip_csum_fix(a):
    """recompute the IPv4 header checksum of a (1, len) Eth/IPv4 frame array"""
    ihl = int(a[0, 14] & 0x0F) * 4
    a[0, 24:26] = 0
    c = int(gen.csum(gen.ones_sum(a, 14, 14 + ihl))[0])
    a[0, 24], a[0, 25] = c >> 8, c & 0xFF


def _edge_frame(rng, clean):
    lens = (64, 65, 66, 67, 70, 73, 74, 75, 80, 127, 128, 129, 191, 570, 1514, 1515, 1518, 2000)
    v6 = rng.integers(3) == 0
    tcp = rng.integers(2) == 0
    proto = gen.PROTO_TCP if tcp else gen.PROTO_UDP
    n = int(lens[rng.integers(len(lens))])
    kind = int(rng.integers(6 if clean else 16))
    if v6 and kind == 5 and clean:
        kind = 0
    dport = 4500 if kind in (5, 14) else int(rng.integers(64))
    sport = int(rng.integers(1 << 16))
    src, dst = (np.array([rng.integers(1 << 32)], np.uint64) for _ in range(2))
    if v6:
        a = gen.ipv6_frames(1, max(n, 74 if tcp else 62), src, dst, proto, sport, dport)
    else:
        a = gen.ipv4_frames(1, n, src, dst, proto, sport, dport)
    l4 = 54 if v6 else 34
    L = a.shape[1]
    if kind == 1:                                    # bad L4 checksum
        j = int(rng.integers(l4, L))
        a[0, j] ^= int(rng.integers(1, 256))
    elif kind == 2:
        if not tcp:
            a[0, l4 + 6:l4 + 8] = 0                  # UDP checksum 0
        elif L > 64:
            a[0, int(rng.integers(64, L))] ^= 0x41   # bad sum in the tail only
    elif kind == 3:
        if v6:
            a[0, 38] = 0xFF                          # multicast destination
        else:
            a[0, 20] |= 0x20                         # more fragments
            _ip_csum_fix(a)
    elif kind == 4:
        a[0, 0:6] = 0xFF if rng.integers(2) else a[0, 0:6] | 1
        if not v6:
            a[0, 30:34] = [0xFF] * 4 if rng.integers(2) else [224, 0, 0, 9]
            _ip_csum_fix(a)
    elif kind == 5:                                  # NAT-T marker present / absent
        if rng.integers(2) and L >= 46:
            a[0, 42:46] = 0
    elif kind == 6:
        if v6:
            a[0, 18:20] = [0xFF, 0x00]               # payload past the frame
        else:
            a[0, 24] ^= 0x5A                         # bad IPv4 header checksum
    elif kind == 7:
        if v6:
            a[0, 20] = 0                             # hop-by-hop next header
        else:
            a[0, 16:18] = [(L - 13) >> 8, (L - 13) & 0xFF]   # tot_len past the frame
            _ip_csum_fix(a)
    elif kind == 8 and not v6:                       # short tot_len, valid header
        t = int(rng.integers(20, L - 13))
        a[0, 16:18] = [t >> 8, t & 0xFF]
        _ip_csum_fix(a)
    elif kind == 9 and not v6:
        a[0, 14] = 0x46                              # IHL 6
        _ip_csum_fix(a)
    elif kind == 10:
        if tcp:
            a[0, l4 + 12] = int(rng.integers(0, 5)) << 4   # data offset < 5
        else:
            a[0, l4 + 4:l4 + 6] = [0, int(rng.integers(0, 8))]   # UDP length < 8
    elif kind == 11:
        a = a[:, :int(rng.integers(14, L))]
    elif kind == 12:
        a = np.concatenate([a[:, :12], np.array([[0x81, 0, 0, 7]], np.uint8), a[:, 12:]], 1)
    elif kind == 13:
        for _ in range(int(rng.integers(1, 4))):
            a[0, int(rng.integers(14, min(L, 80)))] = int(rng.integers(256))
    elif kind == 14 and v6 and tcp:
        a = a[:, :int(rng.integers(64, 74))]         # TCP header past the frame
    elif kind == 15:
        a[0, 20 if v6 else 23] = 1                   # ICMP
        if not v6:
            _ip_csum_fix(a)
    return bytes(a[0])


def imix_edge_corpus(n, seed=3):
    """IMIX-length Eth/IPv4|IPv6/UDP|TCP frames at the edges of the lean
    descriptor kernel's register parse (classify_gf.hip): lengths around the
    64-byte window and 1514 (jumbo), IPv6 TCP data offset in the byte past
    the window, bad / zero / tail-only-bad checksums, fragments, broadcast /
    multicast, NAT-T port 4500, tot_len / payload_len edges, IHL 6, short UDP
    length / TCP data offset, truncations, VLAN, ICMP. Half of the 64-frame
    blocks hold register-parse frames only (whole fast waves), the others
    every kind (generic waves)."""
    rng = np.random.default_rng(seed)
    out = []
    for b0 in range(0, n, 64):
        clean = rng.integers(2) == 0
        out += [_edge_frame(rng, clean) for _ in range(min(64, n - b0))]
    return out
