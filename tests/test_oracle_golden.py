"""Pin the CPU restatement (oracle) against the reference's own fixtures.

Sources (all extracted by tests/golden/make_golden.py as data):
  * parser flag assertions, test/validation/api/pktio/parser.c:225-500
  * one's-complement KATs, test/validation/api/chksum/chksum.c:244-312
  * helper IPv4 checksum KAT, helper/test/chksum.c:118 (0x3965)
  * example/classifier run (udp64.pcap, SIP 10.10.10.0/24 -> queue1):
    odp_classifier_run.sh:17-19, test/example/classifier/pktio_env:21-22
  * valid L3/L4 checksums (incl. SCTP CRC32C) of the golden frames
"""
import numpy as np
import pytest

import oracle
from helpers import ALL_CHKSUM, GOLDEN, golden_frames, has, pack
from odp_amd import _lib as L
from odp_amd import gen


def _default_only(cls, pktin=0):
    p = cls.loop_pktio(pktin=pktin)
    d = cls.cos_create("DefaultCos", queue=cls.queue(0))
    assert cls.default_cos_set(p, d) == 0
    assert cls.pktio_start(p) == 0
    return p, d


def test_chksum_kat_ip_headers():
    for h in GOLDEN["chksum_kat"]["ip_hdr"]:
        assert (~oracle.ones_comp16(bytes.fromhex(h))) & 0xFFFF == 0


def test_chksum_kat_udp():
    for u in GOLDEN["chksum_kat"]["udp"]:
        assert (~oracle.ones_comp16(bytes.fromhex(u))) & 0xFFFF == 0


def test_chksum_kat_udp_long():
    data = bytes.fromhex(GOLDEN["chksum_kat"]["udp_long"])
    assert (~oracle.ones_comp16(data)) & 0xFFFF == GOLDEN["chksum_kat"]["udp_long_res_cpu"]
    # fragmented sum (chksum.c:288-311)
    n = 7
    flen = len(data) // n
    s, off = 0, 0
    for i in range(n):
        ln = len(data) - off if i == n - 1 else flen
        s += oracle.ones_comp16(data[off:off + ln])
        off += ln
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    assert (~s) & 0xFFFF == GOLDEN["chksum_kat"]["udp_long_res_cpu"]


def test_helper_ipv4_csum_kat():
    hdr = bytearray(bytes.fromhex(GOLDEN["helper_ipv4"]["header"]))
    s = (~oracle.ones_comp16(bytes(hdr))) & 0xFFFF          # LE-space
    assert ((s >> 8) | ((s & 0xFF) << 8)) == GOLDEN["helper_ipv4"]["csum"]


def test_parser_flags(fresh_cls):
    p, _ = _default_only(fresh_cls)
    names = sorted(GOLDEN["parser_expect"])
    _, frames = golden_frames(names)
    buf, desc = pack(frames)
    r = oracle.classify(fresh_cls.pktio_rules(p), buf, len(frames), desc=desc)
    for name, m, w in zip(names, r["meta"], r["out"]):
        exp = GOLDEN["parser_expect"][name]
        for f in exp["has"]:
            assert has(m, f), (name, f)
        for f in exp["not"]:
            assert not has(m, f), (name, f)
        assert not (w & L.ODPG_OUT_ERROR), name          # parser.c:217


def test_golden_frames_valid_checksums(fresh_cls):
    """Every golden frame without an Ethernet FCS carries valid checksums."""
    p, _ = _default_only(fresh_cls, pktin=ALL_CHKSUM)
    names, frames = golden_frames()
    buf, desc = pack(frames)
    r = oracle.classify(fresh_cls.pktio_rules(p), buf, len(frames), desc=desc, opt=ALL_CHKSUM)
    for name, w, m in zip(names, r["out"], r["meta"]):
        l3, l4 = L.out_l3(w), L.out_l4(w)
        if name.endswith("_crc"):
            # the 4-byte FCS is inside frame_len, and the platform sums
            # frame_len - l4_offset bytes (odp_packet.c:1914-1919)
            assert l4 == L.ODPG_CHKSUM_BAD and (w & L.ODPG_OUT_ERROR), name
            continue
        assert l3 != L.ODPG_CHKSUM_BAD and l4 != L.ODPG_CHKSUM_BAD, name
        if has(m, "ipv4"):
            assert l3 == L.ODPG_CHKSUM_OK, name
        if (has(m, "udp") or has(m, "tcp") or has(m, "sctp")) and not has(m, "ipfrag"):
            assert l4 == L.ODPG_CHKSUM_OK, name


@pytest.mark.parametrize("pcap", ["classifier_udp64"])
def test_example_classifier_pcap(fresh_cls, pcap):
    """example/classifier with ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1 sends
    >= 100 packets to queue1 and >= 100 to DefaultCos (pktio_env:21-22)."""
    p = fresh_cls.loop_pktio()
    r = gen.build_c1_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    frames = [bytes.fromhex(h) for h in GOLDEN["pcap"][pcap]]
    buf, desc = pack(frames)
    res = oracle.classify(fresh_cls.pktio_rules(p), buf, len(frames), desc=desc)
    cos = res["out"] & 0xFFFF
    q1 = fresh_cls.to_index(r["queue1"])
    dflt = fresh_cls.to_index(r["default"])
    assert (cos == q1).sum() == 100
    assert (cos == dflt).sum() == 100
    assert res["stats"][0] == 200                      # in_packets


def test_perf_pcap_l3fwd_flow(fresh_cls):
    """test/performance/udp64.pcap: 100 x 60 B 10.0.0.1 -> 10.0.0.2 UDP."""
    p, _ = _default_only(fresh_cls, pktin=ALL_CHKSUM)
    frames = [bytes.fromhex(h) for h in GOLDEN["pcap"]["perf_udp64"]]
    assert len(frames) == 100 and all(len(f) == 60 for f in frames)
    buf, desc = pack(frames)
    res = oracle.classify(fresh_cls.pktio_rules(p), buf, len(frames), desc=desc, opt=ALL_CHKSUM)
    assert all(has(m, "ipv4") and has(m, "udp") for m in res["meta"])


def test_crc32c_known_answer():
    # RFC 3720 B.4: CRC32C of 32 zero bytes = 0x8A9136AA (with ~init/~final)
    assert (~oracle.crc32c(bytes(32), 0xFFFFFFFF)) & 0xFFFFFFFF == 0x8A9136AA
    assert (~oracle.crc32c(bytes([0xFF] * 32), 0xFFFFFFFF)) & 0xFFFFFFFF == 0x62A8AB43


def test_c3_traffic_shape(fresh_cls):
    """The C3 generator's mix as the oracle sees it: IMIX mean near 353.8 B,
    ~20 % IPv6 (L3 checksum UNKNOWN), ~0.5 % bad L3 / ~0.5 % bad L4
    checksums (all routed to the error CoS), several CoS of the DAG hit."""
    from odp_amd import _lib as L
    from odp_amd import gen
    opt = L.PKTIN_IPV4_CHKSUM | L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM
    p = fresh_cls.loop_pktio(pktin=opt)
    r = gen.build_c3_rules(fresh_cls, p, stats=True)
    assert len(r["pmrs"]) == 256
    assert fresh_cls.pktio_start(p) == 0
    n = 40000
    buf, desc = gen.c3_frames(n)
    assert abs(desc["len"].mean() - 353.83) < 8
    assert (desc["offset"] % 16 == 0).all()
    o = oracle.classify(fresh_cls.pktio_rules(p), buf, n, desc=desc, opt=opt)
    out = o["out"]
    l3 = (out >> 16) & 3
    l4 = (out >> 18) & 3
    assert 0.15 < (l3 == 0).mean() < 0.25
    assert 0.002 < (l3 == 2).mean() < 0.01 and 0.002 < (l4 == 2).mean() < 0.01
    err = (out >> 20) & 1
    assert ((out & 0xFFFF)[err == 1] == 63).all()       # error CoS
    assert len(np.unique(out & 0xFFFF)) > 8
