"""TEST INFRASTRUCTURE — restatement of the reference classification test
suite's packet builder, so its MATCH / NO_MATCH expectations can be replayed
as fixtures (tests/golden/make_golden.py encodes the cases, this module makes
the bytes).

Follows:
  * create_packet()            test/validation/api/classification/odp_classification_common.c:296-542
  * cls_pkt_set_seq()          odp_classification_common.c:93-135 (magic + seq trailer)
  * test constants             test/validation/api/classification/classification.h:10-82
                               odp_classification_common.c:11-27
  * odph_udp_tcp_chksum(GENERATE / VERIFY)   helper/chksum.c:92-353
  * odph_ipv4_csum_update()    helper/include/odp/helper/ip.h:109-190
  * odph_sctp_chksum_set()     helper/chksum.c:380-403
  * loop pktio MAC             platform/linux-generic/pktio/loop.c:95,602-606

Payload bytes the reference leaves uninitialised (odp_packet_alloc of a pool
buffer) are zero here. The L4 checksum is generated before the seq trailer is
written, exactly as create_packet() does (:488, :539), so TCP/UDP checksums
of these frames do not verify; the reference tests run without pktin
checksum options, so nothing depends on them.
"""
from __future__ import annotations

import struct

ETH_LEN, VLAN_LEN, IPV4_LEN, IPV6_LEN = 14, 4, 20, 40
L4_HDR_LEN = {"tcp": 20, "udp": 8, "gtp": 8, "sctp": 12, "icmp": 8, "igmp": 8, "ah": 24,
              "esp": 8}
L4_PROTO = {"tcp": 6, "udp": 17, "gtp": 17, "sctp": 132, "icmp": 1, "igmp": 2, "ah": 51,
            "esp": 50}
DEFAULT_SMAC = bytes([0x07, 0x08, 0x09, 0x0a, 0x0b, 0x0c])
DEFAULT_DMAC = bytes([0x01, 0x02, 0x03, 0x04, 0x05, 0x06])
LOOP_MAC = bytes([0x02, 0xe9, 0x34, 0x80, 0x73, 0x01])
DEFAULT_SADDR, DEFAULT_DADDR = "10.0.0.1", "10.0.0.100"
DEFAULT_SPORT, DEFAULT_DPORT = 1024, 2048
MAGIC_VAL = 0xdeadbeef
DATA_MAGIC = 0x01020304
DEFAULT_TTL = 128
GTPU_UDP_PORT = 2152
IPV6_SRC = bytes(10) + b"\xff\xff" + bytes([10, 0, 0, 1])
IPV6_DST = bytes(10) + b"\xff\xff" + bytes([10, 0, 0, 100])


def ip4(s: str) -> bytes:
    """parse_ipv4_string() + odp_cpu_to_be_32: network-order address bytes."""
    return bytes(int(x) for x in s.split("/")[0].split("."))


def prefix_mask(bits: int) -> bytes:
    return ((0xFFFFFFFF << (32 - bits)) & 0xFFFFFFFF).to_bytes(4, "big")


def _fold(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def ones_sum_be(data: bytes) -> int:
    """16-bit one's-complement sum of big-endian words (odd byte padded)."""
    if len(data) & 1:
        data = data + b"\x00"
    return _fold(sum(struct.unpack(f">{len(data) // 2}H", data)))


_CRC32C = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ (0x82F63B78 if _c & 1 else 0)
    _CRC32C.append(_c)


def crc32c(data: bytes, crc: int) -> int:
    for b in data:
        crc = _CRC32C[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc


class TestPacket:
    """A frame built like create_packet(), with its layer offsets."""

    def __init__(self, l4="tcp", ipv6=False, vlan=False, qinq=False, dscp=0, length=0,
                 seq=1):
        assert not qinq or vlan
        self.l4, self.ipv6, self.vlan, self.qinq = l4, ipv6, vlan, qinq
        payload_len = 8 + length + (8 if l4 == "gtp" else 0)
        vlan_len = (2 * VLAN_LEN if qinq else VLAN_LEN) if vlan else 0
        l3_hdr = IPV6_LEN if ipv6 else IPV4_LEN
        l4_len = L4_HDR_LEN[l4] + payload_len
        l3_len = l3_hdr + l4_len
        self.l3 = ETH_LEN + vlan_len
        self.l4off = self.l3 + l3_hdr
        f = bytearray(self.l3 + l3_len)
        f[0:6] = DEFAULT_DMAC
        f[6:12] = DEFAULT_SMAC
        eth_type = 0x86DD if ipv6 else 0x0800
        if vlan:
            if qinq:
                f[12:14] = b"\x88\xa8"
                f[14:16] = b"\x00\x00"
                f[16:18] = b"\x81\x00"
                f[18:20] = b"\x00\x00"
                f[20:22] = eth_type.to_bytes(2, "big")
            else:
                f[12:14] = b"\x81\x00"
                f[14:16] = b"\x00\x00"
                f[16:18] = eth_type.to_bytes(2, "big")
        else:
            f[12:14] = eth_type.to_bytes(2, "big")
        proto = L4_PROTO[l4]
        l3 = self.l3
        if not ipv6:
            f[l3] = 0x45
            f[l3 + 1] = (dscp << 2) & 0xFF
            f[l3 + 2:l3 + 4] = l3_len.to_bytes(2, "big")
            f[l3 + 4:l3 + 6] = (seq & 0xFFFF).to_bytes(2, "big")
            f[l3 + 8] = DEFAULT_TTL
            f[l3 + 9] = proto
            f[l3 + 12:l3 + 16] = ip4(DEFAULT_SADDR)
            f[l3 + 16:l3 + 20] = ip4(DEFAULT_DADDR)
        else:
            vtf = (6 << 28) | (((dscp << 2) & 0xFF) << 20) | (seq & 0xFFFFF)
            f[l3:l3 + 4] = vtf.to_bytes(4, "big")
            f[l3 + 4:l3 + 6] = l4_len.to_bytes(2, "big")
            f[l3 + 6] = proto
            f[l3 + 7] = DEFAULT_TTL
            f[l3 + 8:l3 + 24] = IPV6_SRC
            f[l3 + 24:l3 + 40] = IPV6_DST
        self.f = f
        if not ipv6:
            self.ipv4_csum_update()
        o = self.l4off
        if l4 == "igmp":
            f[o + 4:o + 8] = MAGIC_VAL.to_bytes(4, "big")
            f[o] = 0x12
        elif l4 == "icmp":
            f[o] = 8                                        # ODPH_ICMP_ECHO
        elif l4 == "sctp":
            f[o:o + 2] = DEFAULT_SPORT.to_bytes(2, "big")
            f[o + 2:o + 4] = DEFAULT_DPORT.to_bytes(2, "big")
            self.sctp_chksum_set()
        elif l4 in ("udp", "gtp"):
            f[o:o + 2] = DEFAULT_SPORT.to_bytes(2, "big")
            dport = GTPU_UDP_PORT if l4 == "gtp" else DEFAULT_DPORT
            f[o + 2:o + 4] = dport.to_bytes(2, "big")
            f[o + 4:o + 6] = (payload_len + 8).to_bytes(2, "big")
            if l4 == "gtp":
                g = o + 8
                f[g + 4:g + 8] = MAGIC_VAL.to_bytes(4, "big")   # teid
                f[g] = 0x30                                      # GTPv1, no options
                f[g + 1] = 1                                     # echo request
                f[g + 2:g + 4] = struct.pack("<H", 8)            # plen, host order
            self.udp_tcp_chksum_generate()
        elif l4 == "ah":
            f[o] = 4                                             # next_header = ODPH_IPV4
            f[o + 1] = 24 // 4 - 2
            f[o + 4:o + 8] = struct.pack("<I", 256)              # spi, host order
            f[o + 8:o + 12] = struct.pack("<I", 1)
        elif l4 == "esp":
            f[o:o + 4] = struct.pack("<I", 256)
            f[o + 4:o + 8] = struct.pack("<I", 1)
        else:                                                    # tcp
            f[o:o + 2] = DEFAULT_SPORT.to_bytes(2, "big")
            f[o + 2:o + 4] = DEFAULT_DPORT.to_bytes(2, "big")
            f[o + 12] = 0x50                                     # hl = 5
            f[o + 13] = 0x10                                     # ack
            self.udp_tcp_chksum_generate()
        # cls_pkt_set_seq(): magic + seq at the end of the L3 payload
        f[-8:] = struct.pack(">II", DATA_MAGIC, seq)

    # ---- helper checksum routines -------------------------------------------
    def ipv4_csum_update(self):
        l3 = self.l3
        ihl = (self.f[l3] & 0xF) * 4
        self.f[l3 + 10:l3 + 12] = b"\x00\x00"
        c = (~ones_sum_be(bytes(self.f[l3:l3 + ihl]))) & 0xFFFF
        self.f[l3 + 10:l3 + 12] = c.to_bytes(2, "big")

    def sctp_chksum_set(self):
        o = self.l4off
        self.f[o + 8:o + 12] = bytes(4)
        s = (~crc32c(bytes(self.f[o:]), 0xFFFFFFFF)) & 0xFFFFFFFF
        self.f[o + 8:o + 12] = struct.pack("<I", s)

    def udp_tcp_chksum_generate(self):
        c = udp_tcp_chksum(bytes(self.f), self.l3, self.l4off, self.ipv6,
                           "tcp" if self.l4 == "tcp" else "udp", generate=True)
        off = self.l4off + (16 if self.l4 == "tcp" else 6)
        self.f[off:off + 2] = c.to_bytes(2, "big")

    # ---- field edits the tests make after create_packet() --------------------
    def edit(self, field: str, value: bytes):
        f, o, l3 = self.f, self.l4off, self.l3
        pos = {
            "eth_dst": 0, "eth_src": 6,
            "vlan0_tci": ETH_LEN,
            "vlanx_tci": ETH_LEN + (VLAN_LEN if self.qinq else 0),
            "ipv4_ver_ihl": l3, "ipv4_chksum": l3 + 10,
            "ipv4_src": l3 + 12, "ipv4_dst": l3 + 16,
            "ipv6_src": l3 + 8, "ipv6_dst": l3 + 24,
            "sport": o, "dport": o + 2,
            "icmp_type": o, "icmp_code": o + 1, "icmp_id": o + 4,
            "igmp_group": o + 4,
            "gtp_info": o + 8, "gtp_teid": o + 12,
            "ah_spi": o + 4, "esp_spi": o,
        }[field]
        f[pos:pos + len(value)] = value

    def bytes(self) -> bytes:
        return bytes(self.f)


def udp_tcp_chksum(frame: bytes, l3: int, l4: int, ipv6: bool, proto: str,
                   generate: bool = False):
    """odph_udp_tcp_chksum() over a contiguous frame (helper/chksum.c:265-353).

    UDP sums udp.length bytes (not frame_len - l4 like the platform verify);
    TCP sums l3_len - (l4 - l3). GENERATE returns the checksum to store (the
    field is zeroed first, :156-164); VERIFY returns 0 ok / 1 UDP checksum
    absent / 2 bad (:342-347)."""
    f = bytearray(frame)
    is_tcp = proto == "tcp"
    ck = l4 + (16 if is_tcp else 6)
    stored = int.from_bytes(f[ck:ck + 2], "big")
    if not generate and stored == 0 and not is_tcp:
        return 1                                                   # :152-154
    if generate:
        f[ck:ck + 2] = b"\x00\x00"
    if ipv6:
        addrs = bytes(f[l3 + 8:l3 + 40])
        p = f[l3 + 6]
        l3_len = int.from_bytes(f[l3 + 4:l3 + 6], "big") + IPV6_LEN
    else:
        addrs = bytes(f[l3 + 12:l3 + 20])
        p = f[l3 + 9]
        l3_len = int.from_bytes(f[l3 + 2:l3 + 4], "big")
    l4_len = (l3_len - (l4 - l3)) if is_tcp else int.from_bytes(f[l4 + 4:l4 + 6], "big")
    s = ones_sum_be(addrs) + l4_len + p
    s += ones_sum_be(bytes(f[l4:l4 + l4_len]))
    c = (~_fold(s)) & 0xFFFF
    if generate:
        return c
    return 0 if c == 0 else 2


def build(spec: dict, seq: int = 1) -> bytes:
    """Frame for one fixture packet spec: create_packet() parameters, then the
    edits in order; 'mac': 'loop' overwrites both MACs with the loop pktio's
    address as test_pmr() does (odp_classification_test_pmr.c:425-427)."""
    p = TestPacket(l4=spec.get("l4", "tcp"), ipv6=spec.get("ipv6", False),
                   vlan=spec.get("vlan", False), qinq=spec.get("qinq", False),
                   dscp=spec.get("dscp", 0), length=spec.get("len", 0), seq=seq)
    for field, hexval, *post in spec.get("edits", []):
        p.edit(field, bytes.fromhex(hexval))
        for step in post:
            {"ipv4_csum": p.ipv4_csum_update, "sctp_csum": p.sctp_chksum_set,
             "l4_csum": p.udp_tcp_chksum_generate}[step]()
    if spec.get("mac") == "loop":
        p.edit("eth_src", LOOP_MAC)
        p.edit("eth_dst", LOOP_MAC)
    return p.bytes()
