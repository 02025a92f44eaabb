"""Toeplitz (thash_softrss) pinned on published RSS verification vectors.

The reference's hash-queue selection (get_dest_queue -> packet_rss_hash ->
thash_softrss, /root/reference/platform/linux-generic/odp_classification.c:
372-382, 1751-1817; include/protocols/thash.h:81-99) uses the standard 40-byte
RSS key (odp_classification.c:50-58). The reference holds no hash vector of
its own (its tests assert only `!= ODP_QUEUE_INVALID`,
test/validation/api/classification/odp_classification_basic.c:815-816), so:

* the oracle's thash_softrss core is checked against the public RSS
  verification suite for that key (the table every RSS implementation is
  tested with: IPv4 / IPv4+TCP and IPv6 / IPv6+TCP hashes of five and three
  address / port tuples, words in host order: src, dst, sport << 16 | dport);
* end to end on the GPU: an IPv6 CoS hashing addresses only. The reference
  loads IPv6 addresses in host order (thash_load_ipv6_addr), so the tuple is
  exactly the published one and the queue index must equal
  (hash & (CLS_COS_QUEUE_MAX - 1)) % num_queue of the published hash.
  (IPv4 addresses and the port word are loaded raw, in network order, so
  those tuples differ from the published ones: they stay pinned by the
  oracle's literal restatement, `test_hash_queues`.)
"""
import ipaddress

import numpy as np
import pytest

import oracle
from helpers import pack
from odp_amd import _lib as L
from odp_amd import gen

# (dst, src, dport, sport, hash over addresses, hash over addresses + ports)
V4 = [
    ("161.142.100.80", "66.9.149.187", 1766, 2794, 0x323E8FC2, 0x51CCC178),
    ("65.69.140.83", "199.92.111.2", 4739, 14230, 0xD718262A, 0xC626B0EA),
    ("12.22.207.184", "24.19.198.95", 38024, 12898, 0xD2D0A5DE, 0x5C2B394A),
    ("209.142.163.6", "38.27.205.30", 2217, 48228, 0x82989176, 0xAFC7327F),
    ("202.188.127.2", "153.39.163.191", 1303, 44251, 0x5D1809C5, 0x10E828A2),
]
V6 = [
    ("3ffe:2501:200:3::1", "3ffe:2501:200:1fff::7", 1766, 2794, 0x2CC18CD5, 0x40207D3D),
    ("ff02::1", "3ffe:501:8::260:97ff:fe40:efab", 4739, 14230, 0x0F0C461C, 0xDDE51BBF),
    ("fe80::200:f8ff:fe21:67cf", "3ffe:1900:4545:3:200:f8ff:fe21:67cf", 38024, 44251,
     0x4B61E985, 0x02D1FEEF),
]


def _words(addr):
    b = ipaddress.ip_address(addr).packed
    return [int.from_bytes(b[i:i + 4], "big") for i in range(0, len(b), 4)]


@pytest.mark.parametrize("dst,src,dport,sport,h3,h4", V4)
def test_oracle_thash_ipv4_vectors(dst, src, dport, sport, h3, h4):
    t = _words(src) + _words(dst)
    assert oracle.thash(t) == h3
    assert oracle.thash(t + [(sport << 16) | dport]) == h4


@pytest.mark.parametrize("dst,src,dport,sport,h3,h4", V6)
def test_oracle_thash_ipv6_vectors(dst, src, dport, sport, h3, h4):
    t = _words(src) + _words(dst)
    assert oracle.thash(t) == h3
    assert oracle.thash(t + [(sport << 16) | dport]) == h4


def _v6_frames():
    """IPv6/UDP frames carrying the published address pairs (64 copies each,
    so every vector fills a whole wave)."""
    frames = []
    for dst, src, dport, sport, _, _ in V6:
        a = gen.ipv6_frames(1, 128, np.array([0], np.uint64), np.array([0], np.uint64),
                            gen.PROTO_UDP, np.array([sport]), np.array([dport]))
        a[0, 22:38] = np.frombuffer(ipaddress.ip_address(src).packed, np.uint8)
        a[0, 38:54] = np.frombuffer(ipaddress.ip_address(dst).packed, np.uint8)
        frames += [bytes(a[0])] * 64
    return frames


@pytest.mark.gpu
@pytest.mark.parametrize("nq", [32, 7])
def test_gpu_ipv6_hash_queue_vectors(gpu_ctx, fresh_cls, nq):
    p = fresh_cls.loop_pktio()
    d = fresh_cls.cos_create("d", num_queue=nq, hash_proto=fresh_cls.HASH_IPV6)
    assert d
    assert fresh_cls.default_cos_set(p, d) == 0
    assert fresh_cls.pktio_start(p) == 0
    frames = _v6_frames()
    buf, desc = pack(frames)
    rules = fresh_cls.pktio_rules(p)
    tbl = gpu_ctx.table(rules)
    g = gpu_ctx.classify(tbl, buf, len(frames), desc=desc)
    q = L.out_hashq(g["out"]).reshape(len(V6), 64)
    for k, (_, _, _, _, h3, _) in enumerate(V6):
        assert (q[k] == (h3 & 31) % nq).all(), (k, q[k][:4], hex(h3))
    o = oracle.classify(rules, buf, len(frames), desc=desc)
    assert np.array_equal(g["out"], o["out"])


@pytest.mark.parametrize("nq", [32, 7])
def test_oracle_ipv6_hash_queue_vectors(fresh_cls, nq):
    """The oracle's packet_rss_hash tuple loading on the same frames (CPU)."""
    p = fresh_cls.loop_pktio()
    d = fresh_cls.cos_create("d", num_queue=nq, hash_proto=fresh_cls.HASH_IPV6)
    assert d and fresh_cls.default_cos_set(p, d) == 0
    frames = _v6_frames()
    buf, desc = pack(frames)
    o = oracle.classify(fresh_cls.pktio_rules(p), buf, len(frames), desc=desc)
    q = L.out_hashq(o["out"]).reshape(len(V6), 64)
    for k, (_, _, _, _, h3, _) in enumerate(V6):
        assert (q[k] == (h3 & 31) % nq).all(), (k, q[k][:4], hex(h3))
