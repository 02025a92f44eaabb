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
