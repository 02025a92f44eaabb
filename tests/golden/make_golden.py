#!/usr/bin/env python3
"""Extract the reference's own fixtures into tests/golden/reference_fixtures.json.

Run in the build container (it reads /root/reference, which is not on the GPU
box). It copies DATA only: frame byte arrays from test/common/test_packet_*.h,
the checksum known-answer vectors of test/validation/api/chksum/chksum.c, the
frames of the pcap files the example tests replay, and the expectations those
tests assert (encoded below with the file:line they come from). No reference
source text is stored. It also copies the two capture files byte for byte
(data files the reference's tests replay): example/classifier/udp64.pcap ->
classifier_udp64.pcap and test/performance/udp64.pcap -> perf_udp64.pcap.

    python3 tests/golden/make_golden.py [/root/reference]
"""
from __future__ import annotations

import json
import os
import re
import struct
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_fixtures.json")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cls_testpkt  # noqa: E402  (tests/cls_testpkt.py: create_packet() restated)

ARRAY_RE = re.compile(r"static\s+(?:const\s+)?uint8_t\s+(\w+)\s*\[[^\]]*\](?:\s+ODP_ALIGNED\(\d+\))?"
                      r"\s*=\s*\{(.*?)\};", re.S)


def c_arrays(path):
    """name -> bytes for every `static [const] uint8_t name[] = {...};`"""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for name, body in ARRAY_RE.findall(txt):
        if "{" in body:      # nested (2-D / struct) arrays handled separately
            continue
        vals = [int(v, 0) for v in re.findall(r"0x[0-9A-Fa-f]+|\b\d+\b", body)]
        out[name] = bytes(vals)
    return out


def nested_rows(path, name):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    m = re.search(name + r"\s*\[[^\]]*\]\s*\[[^\]]*\][^=]*=\s*\{(.*?)\};", txt, re.S)
    rows = re.findall(r"\{([^{}]*)\}", m.group(1))
    return [bytes(int(v, 0) for v in re.findall(r"0x[0-9A-Fa-f]+", r)) for r in rows]


def udp_vectors(path):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    m = re.search(r"udp_test_vect\s*\[NUM_UDP\][^=]*=\s*\{(.*?)\};", txt, re.S)
    out = []
    for ln, body in re.findall(r"\.len\s*=\s*(\d+),\s*\.data\s*=\s*\{([^}]*)\}", m.group(1)):
        data = bytes(int(v, 0) for v in re.findall(r"0x[0-9A-Fa-f]+", body))
        out.append(data[: int(ln)])
    return out


def pcap_frames(path):
    d = open(path, "rb").read()
    frames = []
    if d[:4] == b"\x0a\x0d\x0d\x0a":                       # pcapng
        off = 0
        while off + 12 <= len(d):
            btype, blen = struct.unpack_from("<II", d, off)
            if btype == 6:                                 # enhanced packet block
                cap = struct.unpack_from("<I", d, off + 20)[0]
                frames.append(d[off + 28: off + 28 + cap])
            elif btype == 3:                               # simple packet block
                plen = struct.unpack_from("<I", d, off + 8)[0]
                frames.append(d[off + 12: off + 12 + plen])
            off += blen
    else:                                                  # classic pcap
        magic = struct.unpack_from("<I", d, 0)[0]
        e = "<" if magic in (0xA1B2C3D4, 0xA1B23C4D) else ">"
        off = 24
        while off + 16 <= len(d):
            incl = struct.unpack_from(e + "I", d, off + 8)[0]
            frames.append(d[off + 16: off + 16 + incl])
            off += 16 + incl
    return frames


def _t(term, value, mask, val_sz=None, offset=0):
    return {"term": term, "value": value, "mask": mask,
            "val_sz": len(bytes.fromhex(value)) if val_sz is None else val_sz, "offset": offset}


def _pkt(expect, mark=0, **spec):
    return {"spec": spec, "expect": expect, "mark": mark}


def _single(name, cite, terms, packets, create_fails=False, ops=None, classifier=True):
    """test_pmr() shape (odp_classification_test_pmr.c:383-458): DefaultCos set
    on a loop pktio, one CoS "PMR test cos" reached by one PMR from it."""
    return {"name": name, "cite": cite, "classifier": classifier,
            "cos": [{"name": "DefaultCos"}, {"name": "PMR test cos"}],
            "default": "DefaultCos", "error": None,
            "pmrs": [{"src": "DefaultCos", "dst": "PMR test cos", "terms": terms, "mark": None,
                      "create_fails": create_fails}],
            "ops": ops or [], "packets": packets}


def cls_validation():
    """The reference classification suite's per-packet expectations, encoded
    as data. Each scenario lists the CoS objects and PMRs in creation order
    (first match follows cos->pmr[] order), the packets as create_packet()
    parameters plus the field edits the test makes, and the CoS the test
    asserts the packet is received on (retqueue / recvpool), and for the
    marking test the odp_packet_cls_mark() value.

    Sources: test/validation/api/classification/odp_classification_test_pmr.c
    (suite "pmr"), odp_classification_tests.c (suite "classification"),
    odp_classification_common.c (create_packet, MACs, constants), and
    classification.h. On linux-generic, find_first_supported_l3_pmr() is
    ODP_PMR_UDP_SPORT and find_first_supported_proto() is UDP
    (odp_classification_common.c:544-587 against odp_cls_capability(),
    platform/linux-generic/odp_classification.c:153-201)."""
    D, T = "DefaultCos", "PMR test cos"
    L = "loop"
    S = []
    # ---- suite "pmr": one term per test via test_pmr() ---------------------
    S.append(_single("tcp_sport", "odp_classification_test_pmr.c:460-490",
                     [_t("TCP_SPORT", "0400", "ffff")],
                     [_pkt(T, mac=L, edits=[["sport", "0400"]]),
                      _pkt(D, mac=L, edits=[["sport", "0401"]])]))
    S.append(_single("udp_dport", "odp_classification_test_pmr.c:492-525",
                     [_t("UDP_DPORT", "0800", "ffff")],
                     [_pkt(T, mac=L, l4="udp", edits=[["dport", "0800"]]),
                      _pkt(D, mac=L, l4="udp", edits=[["dport", "0801"]])]))
    S.append(_single("udp_sport", "odp_classification_test_pmr.c:527-560",
                     [_t("UDP_SPORT", "0400", "ffff")],
                     [_pkt(T, mac=L, l4="udp", edits=[["sport", "0400"]]),
                      _pkt(D, mac=L, l4="udp", edits=[["sport", "0401"]])]))
    for v6 in (False, True):
        tag = "ipv6" if v6 else "ipv4"
        S.append(_single(f"{tag}_proto", "odp_classification_test_pmr.c:562-602",
                         [_t("IPPROTO", "11", "ff")],
                         [_pkt(T, mac=L, l4="udp", ipv6=v6), _pkt(D, mac=L, l4="tcp", ipv6=v6)]))
        S.append(_single(f"{tag}_dscp", "odp_classification_test_pmr.c:604-645",
                         [_t("IP_DSCP", "20", "3f")],
                         [_pkt(T, mac=L, l4="udp", ipv6=v6, dscp=0x20),
                          _pkt(D, mac=L, l4="udp", ipv6=v6, dscp=0)]))
    S.append(_single("dmac", "odp_classification_test_pmr.c:647-747",
                     [_t("DMAC", "99aabbccddee", "ffffffffffff")],
                     [_pkt(T, l4="udp", edits=[["eth_dst", "99aabbccddee"]]), _pkt(D)]))
    S.append(_single("packet_len", "odp_classification_test_pmr.c:749-780",
                     # val = 1024, mask = 0xff00 as CPU-endian (LE) uint32_t
                     [_t("LEN", "00040000", "00ff0000")],
                     [_pkt(T, mac=L, l4="udp", len=1024), _pkt(D, mac=L)]))
    S.append(_single("vlan_id_0", "odp_classification_test_pmr.c:782-815",
                     [_t("VLAN_ID_0", "0123", "0fff")],
                     [_pkt(T, mac=L, vlan=True, edits=[["vlan0_tci", "0123"]]), _pkt(D, mac=L)]))
    S.append(_single("vlan_id_x", "odp_classification_test_pmr.c:817-863",
                     [_t("VLAN_ID_X", "0345", "0fff")],
                     [_pkt(T, mac=L, vlan=True, edits=[["vlanx_tci", "0345"]]),
                      _pkt(T, mac=L, vlan=True, qinq=True, edits=[["vlanx_tci", "0345"]]),
                      _pkt(D, mac=L)]))
    S.append(_single("vlan_pcp_0", "odp_classification_test_pmr.c:865-901",
                     [_t("VLAN_PCP_0", "05", "07")],
                     # tci = 5 << ODPH_VLANHDR_PCP_SHIFT | 0x123
                     [_pkt(T, mac=L, vlan=True, edits=[["vlan0_tci", "a123"]]),
                      _pkt(D, mac=L, vlan=True)]))
    S.append(_single("eth_type_0", "odp_classification_test_pmr.c:903-931",
                     [_t("ETHTYPE_0", "86dd", "ffff")],
                     [_pkt(T, mac=L, ipv6=True), _pkt(D, mac=L)]))
    S.append(_single("eth_type_x", "odp_classification_test_pmr.c:933-979",
                     [_t("ETHTYPE_X", "0800", "ffff")],
                     [_pkt(T, mac=L, vlan=True, edits=[["vlanx_tci", "0123"]]),
                      _pkt(T, mac=L, vlan=True, qinq=True, edits=[["vlanx_tci", "0123"]]),
                      _pkt(D, mac=L)]))
    S.append(_single("pool_set", "odp_classification_test_pmr.c:981-1078",
                     [_t("IPPROTO", "11", "ff")], [_pkt(T, mac=L, l4="udp")],
                     ops=["cos_pool_set"]))
    S.append(_single("queue_set", "odp_classification_test_pmr.c:1080-1176",
                     [_t("IPPROTO", "11", "ff")], [_pkt(T, mac=L, l4="udp")],
                     ops=["cos_queue_set"]))
    addr_edits = [["ipv4_src", "0a000058"], ["ipv4_dst", "0a000063", "ipv4_csum"]]
    S.append(_single("ipv4_saddr", "odp_classification_test_pmr.c:1178-1227",
                     [_t("SIP_ADDR", "0a000058", "ffffffff")],
                     [_pkt(T, mac=L, edits=addr_edits), _pkt(D, mac=L)]))
    S.append(_single("ipv4_daddr", "odp_classification_test_pmr.c:1178-1232",
                     [_t("DIP_ADDR", "0a000063", "ffffffff")],
                     [_pkt(T, mac=L, edits=addr_edits), _pkt(D, mac=L)]))
    v6mask = "00000000000000000000ffffffffffff"
    S.append(_single("ipv6_daddr", "odp_classification_test_pmr.c:1234-1268",
                     [_t("DIP6_ADDR", "00000000000000000000ffff0a010164", v6mask)],
                     [_pkt(T, mac=L, ipv6=True,
                           edits=[["ipv6_dst", "00000000000000000000ffff0a010164"]]),
                      _pkt(D, mac=L, ipv6=True)]))
    S.append(_single("ipv6_saddr", "odp_classification_test_pmr.c:1270-1303",
                     [_t("SIP6_ADDR", "00000000000000000000ffff0a010101", v6mask)],
                     [_pkt(T, mac=L, ipv6=True,
                           edits=[["ipv6_src", "00000000000000000000ffff0a010101"]]),
                      _pkt(D, mac=L, ipv6=True)]))
    for n, nm in ((2, "tcp_dport"), (32 // 4, "tcp_dport_multi")):   # SHM_PKT_NUM_BUFS / 4
        pk = [_pkt(T, mac=L, edits=[["dport", "0800"]]) for _ in range(n)]
        pk += [_pkt(D, mac=L, edits=[["dport", "0801"]]) for _ in range(n)]
        pk += [_pkt(T, mac=L, edits=[["dport", "0800"]]) if (i % 5) < 2 else
               _pkt(D, mac=L, edits=[["dport", "0801"]]) for i in range(2 * n)]
        S.append(_single(nm, "odp_classification_test_pmr.c:201-369,1305-1313",
                         [_t("TCP_DPORT", "0800", "ffff")], pk))
    cust_edits = [["ipv4_src", "0a000858"], ["ipv4_dst", "0a000963", "ipv4_csum"]]
    S.append(_single("custom_frame", "odp_classification_test_pmr.c:1315-1371,1882-1885",
                     [_t("CUSTOM_FRAME", "0a000800", "ffffff00", offset=26)],
                     [_pkt(T, mac=L, edits=cust_edits), _pkt(D, mac=L)]))
    S.append(_single("custom_l3", "odp_classification_test_pmr.c:1315-1371,1887-1890",
                     [_t("CUSTOM_L3", "0a000900", "ffffff00", offset=16)],
                     [_pkt(T, mac=L, edits=cust_edits), _pkt(D, mac=L)]))
    for v6 in (False, True):
        tag = "ipv6" if v6 else "ipv4"
        for l4, fld in (("ah", "ah_spi"), ("esp", "esp_spi")):
            # val = odp_cpu_to_be_32(0x11223344); the miss writes val + 1 as a
            # host (LE) integer: 44332211 + 1 -> bytes 12 22 33 44
            S.append(_single(f"ipsec_spi_{l4}_{tag}", "odp_classification_test_pmr.c:1892-1982",
                             [_t("IPSEC_SPI", "11223344", "ffffffff")],
                             [_pkt(T, mac=L, l4=l4, ipv6=v6, edits=[[fld, "11223344"]]),
                              _pkt(D, mac=L, l4=l4, ipv6=v6, edits=[[fld, "12223344"]])]))
    # terms linux-generic does not advertise (odp_classification.c:153-201) and
    # rejects at create (:717-720): the reference runs these tests only when the
    # capability bit is set (ODP_TEST_INFO_CONDITIONAL, :2148-2154), so here only
    # the create failure is asserted; the frames still exercise the parser
    for nm, term, val, l4, cite in (
            ("sctp_sport", "SCTP_SPORT", "0400", "sctp", "odp_classification_test_pmr.c:1605-1657"),
            ("sctp_dport", "SCTP_DPORT", "0800", "sctp", "odp_classification_test_pmr.c:1605-1662"),
            ("icmp_type", "ICMP_TYPE", "08", "icmp", "odp_classification_test_pmr.c:1664-1697"),
            ("icmp_code", "ICMP_CODE", "01", "icmp", "odp_classification_test_pmr.c:1699-1732"),
            ("icmp_id", "ICMP_ID", "1234", "icmp", "odp_classification_test_pmr.c:1734-1767"),
            ("gtpu_teid", "GTPV1_TEID", "deadbeef", "gtp", "odp_classification_test_pmr.c:1769-1829"),
            ("igmp_grpaddr", "IGMP_GRP_ADDR", "deadbeef", "igmp",
             "odp_classification_test_pmr.c:1831-1865")):
        S.append(_single(nm, cite, [_t(term, val, "ff" * (len(val) // 2))],
                         [_pkt(D, mac=L, l4=l4)], create_fails=True))
    S.append(_single("pktin_classifier_flag", "odp_classification_test_pmr.c:105-199",
                     [_t("TCP_DPORT", "0800", "ffff")],
                     [_pkt("NOCLS", mac=L, edits=[["dport", "0800"]])], classifier=False))
    # ---- serial / parallel / marking chains (:1381-1603, :1867-1880) --------
    for nm, num_udp, marking in (("pmr_serial", 1, False), ("pmr_parallel", 4, False),
                                 ("pmr_marking", 4, True)):
        cos = [{"name": D}, {"name": "cos_ip"}] + [{"name": f"udp_{i}"} for i in range(num_udp)]
        pmrs = [{"src": D, "dst": "cos_ip", "terms": [_t("DIP_ADDR", "0a000963", "ffffffff")],
                 "mark": 1 if marking else None}]
        pmrs += [{"src": "cos_ip", "dst": f"udp_{i}",
                  "terms": [_t("UDP_DPORT", (1000 + i).to_bytes(2, "big").hex(), "ffff")],
                  "mark": 2 + i if marking else None} for i in range(num_udp)]
        pk = [_pkt("cos_ip", mark=1 if marking else 0, mac=L, l4="tcp",
                   edits=[["ipv4_dst", "0a000963", "ipv4_csum"]])]
        pk += [_pkt(f"udp_{i}", mark=2 + i if marking else 0, mac=L, l4="udp",
                    edits=[["ipv4_dst", "0a000963", "ipv4_csum"],
                           ["dport", (1000 + i).to_bytes(2, "big").hex()]])
               for i in range(num_udp)]
        pk += [_pkt(D, mac=L)]
        S.append({"name": nm, "cite": "odp_classification_test_pmr.c:1381-1603,1867-1880",
                  "classifier": True, "cos": cos, "default": D, "error": None, "pmrs": pmrs,
                  "ops": [], "packets": pk})
    # ---- suite "classification" (odp_classification_tests.c:610-1003): one
    # pktio, every CoS configured in cls_pktio_configure_common() order ------
    sp = lambda port: ["sport", port.to_bytes(2, "big").hex()]   # noqa: E731
    src = lambda a: ["ipv4_src", ip_hex(a), "ipv4_csum"]          # noqa: E731
    cos = [{"name": "DefaultCoS"}, {"name": "DropCoS", "action": "drop", "stats": True},
           {"name": "ErrorCos"}, {"name": "SrcCos"}, {"name": "DstCos"},
           {"name": "SrcCosRev"}, {"name": "DstCosRev"}, {"name": "PMR_CoS"},
           {"name": "cos_pmr_composite"}]
    u = lambda port: _t("UDP_SPORT", port.to_bytes(2, "big").hex(), "ffff")  # noqa: E731
    sip = lambda a: _t("SIP_ADDR", ip_hex(a), "ffffffff")                     # noqa: E731
    pmrs = [
        {"src": "DefaultCoS", "dst": "DropCoS", "terms": [u(4001)], "mark": None},     # :468-504
        {"src": "DefaultCoS", "dst": "SrcCos", "terms": [sip("10.0.0.5")], "mark": None},  # :334-336
        {"src": "SrcCos", "dst": "DstCos", "terms": [u(3000)], "mark": None},
        {"src": "SrcCosRev", "dst": "DstCosRev", "terms": [u(3001)], "mark": None},  # :337-339
        {"src": "DefaultCoS", "dst": "SrcCosRev", "terms": [sip("10.0.0.7")], "mark": None},
        {"src": "DefaultCoS", "dst": "PMR_CoS", "terms": [u(4000)], "mark": None},      # :711-763
        {"src": "DefaultCoS", "dst": "cos_pmr_composite",                               # :790-856
         "terms": [sip("10.0.0.6"), u(5000)], "mark": None},
    ]
    pk = [
        _pkt("DefaultCoS", l4="udp"),                                                   # :439-466
        _pkt("DropCoS", l4="udp", edits=[sp(4001)]),                                    # :506-534
        _pkt("ErrorCos", l4="udp", edits=[["ipv4_ver_ihl", "85"], ["ipv4_chksum", "0000"]]),
        _pkt("DstCos", l4="udp", edits=[src("10.0.0.5"), sp(3000)]),                    # :343-396
        _pkt("SrcCos", l4="udp", edits=[src("10.0.0.5")]),
        _pkt("DstCosRev", l4="udp", edits=[src("10.0.0.7"), sp(3001)]),
        _pkt("SrcCosRev", l4="udp", edits=[src("10.0.0.7")]),
        _pkt("PMR_CoS", l4="udp", edits=[sp(4000)]),                                    # :765-788
        _pkt("cos_pmr_composite", l4="udp", edits=[src("10.0.0.6"), sp(5000)]),         # :858-890
    ]
    S.append({"name": "cls_pktio", "cite": "odp_classification_tests.c:216-396,398-534,610-1003",
              "classifier": True, "cos": cos, "default": "DefaultCoS", "error": "ErrorCos",
              "pmrs": pmrs, "ops": [], "packets": pk,
              # test_pktio_drop_cos(): the DROP CoS counts the packet (:528-529)
              "cos_stats": {"DropCoS": 1}})
    # basic suite: cls_pmr_composite_create (odp_classification_basic.c:621-694):
    # max_terms_per_pmr (8) identical TCP_DPORT terms on one PMR
    # (val = 1024 as a host-endian uint16_t: bytes 00 04; the test asserts only
    # that the PMR is created, no packets are sent)
    S.append(_single("pmr_composite_create", "odp_classification_basic.c:621-694",
                     [_t("TCP_DPORT", "0004", "ffff")] * 8, []))
    # give every frame the seq number create_packet() would (one counter per run)
    seq = 0
    for s in S:
        for p in s["packets"]:
            seq += 1
            p["frame"] = cls_testpkt.build(p["spec"], seq=seq).hex()
    return S


def ip_hex(a):
    return bytes(int(x) for x in a.split(".")).hex()


def main():
    tc = os.path.join(REF, "test/common")
    frames = {}
    for f in ("test_packet_ipv4.h", "test_packet_ipv6.h", "test_packet_ipv4_with_crc.h",
              "test_packet_ipsec.h", "test_packet_custom.h"):
        frames.update(c_arrays(os.path.join(tc, f)))

    # parser expectations: test/validation/api/pktio/parser.c:225-500 asserts these
    # flags on each frame after a loop pktio receive with parser.layer = ALL
    parser_expect = {
        "test_packet_arp": {"has": ["eth", "arp"], "not": ["ipv4", "ipv6"]},
        "test_packet_ipv4_icmp": {"has": ["eth", "ipv4", "icmp"],
                                  "not": ["ipv6", "tcp", "udp", "sctp"]},
        "test_packet_ipv4_tcp": {"has": ["eth", "ipv4", "tcp"], "not": ["ipv6", "udp", "sctp"]},
        "test_packet_ipv4_udp": {"has": ["eth", "ipv4", "udp"], "not": ["ipv6", "tcp", "sctp"]},
        "test_packet_vlan_ipv4_udp": {"has": ["eth", "vlan", "ipv4", "udp"],
                                      "not": ["ipv6", "tcp", "sctp"]},
        "test_packet_vlan_qinq_ipv4_udp": {"has": ["eth", "vlan", "vlan_qinq", "ipv4", "udp"],
                                           "not": ["ipv6", "tcp", "sctp"]},
        "test_packet_ipv4_sctp": {"has": ["eth", "ipv4", "sctp"], "not": ["ipv6", "tcp", "udp"]},
        "test_packet_ipv6_icmp": {"has": ["eth", "ipv6", "icmp"],
                                  "not": ["ipv4", "tcp", "udp", "sctp"]},
        "test_packet_ipv6_tcp": {"has": ["eth", "ipv6", "tcp"], "not": ["ipv4", "udp", "sctp"]},
        "test_packet_ipv6_udp": {"has": ["eth", "ipv6", "udp"], "not": ["ipv4", "tcp", "sctp"]},
        "test_packet_vlan_ipv6_udp": {"has": ["eth", "vlan", "ipv6", "udp"],
                                      "not": ["ipv4", "tcp", "sctp"]},
        "test_packet_ipv6_sctp": {"has": ["eth", "ipv6", "sctp"], "not": ["ipv4", "tcp", "udp"]},
    }
    # loopback_packet() additionally asserts odp_packet_has_error() == 0 (parser.c:217)

    ck = os.path.join(REF, "test/validation/api/chksum/chksum.c")
    ck_arrays = c_arrays(ck)
    long_pad = 11            # UDP_LONG_PADDING (chksum.c:81)
    chksum_kat = {
        # chksum.c:244-256: ~odp_chksum_ones_comp16(hdr, 20) == 0
        "ip_hdr": [h.hex() for h in nested_rows(ck, "ip_hdr_test_vect")],
        # chksum.c:258-271: ~odp_chksum_ones_comp16(vect, len) == 0
        "udp": [u.hex() for u in udp_vectors(ck)],
        # chksum.c:273-312: ~ones_comp16(long) == be_to_cpu_16(0xF396)
        "udp_long": ck_arrays["udp_test_vect_long"][:-long_pad].hex(),
        "udp_long_res_cpu": 0x96F3,
    }

    pcaps = {
        "classifier_udp64": [f.hex() for f in pcap_frames(os.path.join(REF, "example/classifier/udp64.pcap"))],
        "perf_udp64": [f.hex() for f in pcap_frames(os.path.join(REF, "test/performance/udp64.pcap"))],
    }
    classifier_expect = {
        # example/classifier/odp_classifier_run.sh:17-19 and
        # platform/linux-generic/test/example/classifier/pktio_env:21-22
        "rule": {"term": "ODP_PMR_SIP_ADDR", "value": "10.10.10.0", "mask": "0xFFFFFF00",
                 "cos": "queue1"},
        "min_count": {"queue1": 100, "DefaultCos": 100},
    }
    # helper/test/chksum.c:72-118: IPv4 header of the helper test packet and the
    # checksum odph_ipv4_csum_update() must produce (:118 == 0x3965)
    helper_ipv4 = {
        "header": bytes([0x45, 0x00, 0x00, 0x34, 0x00, 0x01, 0x00, 0x00, 0x00, 0x11, 0x00,
                         0x00, 192, 168, 0, 1, 192, 168, 0, 2]).hex(),
        "csum": 0x3965,
        "note": "tot_len = 24 B user area + 8 + 20 (struct udata_struct is 24 B on LP64)",
    }

    data = {
        "generator": "tests/golden/make_golden.py",
        "reference": "Linaro/odp 1.46.0.0 @ /root/reference",
        "frames": {k: v.hex() for k, v in sorted(frames.items())},
        "parser_expect": parser_expect,
        "chksum_kat": chksum_kat,
        "pcap": pcaps,
        "classifier_expect": classifier_expect,
        "helper_ipv4": helper_ipv4,
        "cls_validation": cls_validation(),
    }
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(f"wrote {OUT}: {len(frames)} frames, "
          f"{sum(len(v) for v in pcaps.values())} pcap frames")
    import shutil
    for src, dst in (("example/classifier/udp64.pcap", "classifier_udp64.pcap"),
                     ("test/performance/udp64.pcap", "perf_udp64.pcap")):
        shutil.copyfile(os.path.join(REF, src), os.path.join(os.path.dirname(OUT), dst))


if __name__ == "__main__":
    main()
