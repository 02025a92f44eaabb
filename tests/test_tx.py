"""Loop pktio transmit side (include/odpg_tx.h):
loopback_fix_checksums + get_dest_queue (pktio/loop.c:415-523).

CPU: the restatement (oracle/odp_oracle.c oracle_tx_prepare) is pinned
against the reference's own fixtures: the test_packet_*_crc frames and the
other golden frames whose checksums the RX verify accepts must come back
byte-identical after their checksum fields are zeroed and re-inserted (UDP,
IPv4, SCTP); the TCP insert reproduces the reference's write at l4 + 6
(odp_packet.c:1838-1840). Queue picks are checked against crc32c of the
get_dest_queue tuple built by hand (crc32c itself is pinned by the
test_oracle_golden KATs).
GPU: odpg_tx_prepare vs the oracle, bit-exact on every frame byte and the
per-packet word, over golden, mutated and IMIX frames, with parsed or given
per-packet metadata and every config / override combination."""
import numpy as np
import pytest

import oracle
import rulesets
from helpers import ALL_CHKSUM, GOLDEN, golden_frames, pack
from odp_amd import _lib as L
from odp_amd import gen

CFG_ALL = L.PKTOUT_IPV4_CHKSUM | L.PKTOUT_UDP_CHKSUM | L.PKTOUT_TCP_CHKSUM | L.PKTOUT_SCTP_CHKSUM


def _offsets(fr):
    """(l3, l4, input_flags) of one frame from the oracle parser."""
    buf, desc = pack([fr])
    o = oracle.classify(_EMPTY_RULES, buf, 1, desc=desc, opt=ALL_CHKSUM, classify=False)
    m = o["meta"][0]
    return int(m["l3_offset"]), int(m["l4_offset"]), int(m["input_flags"]), int(o["out"][0])


def _empty_rules():
    from odp_amd import _lib
    r = _lib.odpg_rules_t()
    r.default_cos = -1
    r.error_cos = -1
    return r


_EMPTY_RULES = _empty_rules()


def _zero(fr, off, n):
    b = bytearray(fr)
    b[off:off + n] = bytes(n)
    return bytes(b)


def test_tx_insert_reproduces_reference_checksums():
    """Zeroed checksum fields of the reference's checksummed frames come back
    identical (IPv4 header, UDP, SCTP)."""
    names, frames = golden_frames()
    checked = {"ipv4": 0, "udp": 0, "sctp": 0}
    for name, fr in zip(names, frames):
        l3, l4, inf, w = _offsets(fr)
        l3_ok = ((w >> 16) & 3) == L.ODPG_CHKSUM_OK
        l4_ok = ((w >> 18) & 3) == L.ODPG_CHKSUM_OK
        is_udp, is_sctp = inf >> 24 & 1, inf >> 26 & 1
        z = fr
        cfg = 0
        if l3_ok:
            z = _zero(z, l3 + 10, 2)
            cfg |= L.PKTOUT_IPV4_CHKSUM
        if l4_ok and is_udp:
            z = _zero(z, l4 + 6, 2)
            cfg |= L.PKTOUT_UDP_CHKSUM
        if l4_ok and is_sctp:
            z = _zero(z, l4 + 8, 4)
            cfg |= L.PKTOUT_SCTP_CHKSUM
        if not cfg:
            continue
        n = len(z)
        out, got = oracle.tx_prepare(np.frombuffer(z, np.uint8), 1, stride=n, pktout_cfg=cfg)
        assert bytes(got) == fr, name
        checked["ipv4"] += bool(cfg & L.PKTOUT_IPV4_CHKSUM)
        checked["udp"] += bool(cfg & L.PKTOUT_UDP_CHKSUM)
        checked["sctp"] += bool(cfg & L.PKTOUT_SCTP_CHKSUM)
        assert out[0] & L.TX_OUT_IPV4 == (L.TX_OUT_IPV4 if cfg & L.PKTOUT_IPV4_CHKSUM else 0)
    assert checked["ipv4"] >= 8 and checked["udp"] >= 8 and checked["sctp"] >= 1, checked


def test_tx_tcp_insert_writes_at_udp_offset():
    """_odp_packet_tcp_udp_chksum_insert writes the TCP checksum at
    l4 + _ODP_UDP_CSUM_OFFSET (odp_packet.c:1838-1840), summed with those two
    bytes zeroed; the TCP header's own checksum field stays as it was."""
    fr = bytes.fromhex(GOLDEN["frames"]["test_packet_ipv4_tcp"])
    l3, l4, inf, w = _offsets(fr)
    assert inf >> 25 & 1
    out, got = oracle.tx_prepare(np.frombuffer(fr, np.uint8), 1, stride=len(fr),
                                 pktout_cfg=L.PKTOUT_TCP_CHKSUM)
    got = bytes(got)
    assert out[0] & L.TX_OUT_TCP
    assert got[:l4 + 6] == fr[:l4 + 6] and got[l4 + 8:] == fr[l4 + 8:]
    # recompute: pseudo header + segment with bytes l4+6..7 zeroed
    seg = bytearray(fr[l4:])
    seg[6:8] = b"\0\0"
    tl = len(fr) - l4
    pseudo = fr[l3 + 12:l3 + 20] + bytes([0, 6]) + tl.to_bytes(2, "big")
    c = oracle.ones_comp16(pseudo + bytes(seg))
    assert got[l4 + 6:l4 + 8] == (~c & 0xFFFF).to_bytes(2, "little")


def test_tx_queue_pick_crc32c():
    """get_dest_queue (loop.c:468-523): crc32c(ports, addrs, init 0) % num_qs;
    index % num_qs without hashing."""
    fr = bytes.fromhex(GOLDEN["frames"]["test_packet_ipv4_udp"])
    l3, l4, inf, w = _offsets(fr)
    a = np.frombuffer(fr, np.uint8)
    for qs in (1, 3, 8):
        out, _ = oracle.tx_prepare(a, 1, stride=len(fr), num_qs=qs, index=5)
        assert out[0] & 0xFFFF == 5 % qs
        out, _ = oracle.tx_prepare(a, 1, stride=len(fr), num_qs=qs,
                                   hash_proto=L.HASH_IPV4_UDP | L.HASH_IPV4)
        tup = fr[l4:l4 + 4] + fr[l3 + 12:l3 + 20]
        assert out[0] & 0xFFFF == oracle.crc32c(tup, 0) % qs
        out, _ = oracle.tx_prepare(a, 1, stride=len(fr), num_qs=qs, hash_proto=L.HASH_IPV4)
        assert out[0] & 0xFFFF == oracle.crc32c(fr[l3 + 12:l3 + 20], 0) % qs
    fr6 = bytes.fromhex(GOLDEN["frames"]["test_packet_ipv6_udp"])
    l3, l4, inf, w = _offsets(fr6)
    out, _ = oracle.tx_prepare(np.frombuffer(fr6, np.uint8), 1, stride=len(fr6), num_qs=7,
                               hash_proto=L.HASH_IPV6_UDP | L.HASH_IPV6)
    assert out[0] & 0xFFFF == oracle.crc32c(fr6[l4:l4 + 4] + fr6[l3 + 8:l3 + 40], 0) % 7


def test_tx_then_rx_verifies():
    """Round trip: UDP / IPv4 checksums inserted on TX verify OK on RX."""
    n = 300
    fr = gen.c2_frames(n, seed=3).reshape(n, 64).copy()
    fr[:, 24:26] = 0                    # IPv4 header checksum
    fr[:, 40:42] = 0                    # UDP checksum
    out, got = oracle.tx_prepare(fr.reshape(-1), n, stride=64,
                                 pktout_cfg=L.PKTOUT_IPV4_CHKSUM | L.PKTOUT_UDP_CHKSUM)
    assert np.all(out & L.TX_OUT_IPV4) and np.all(out & L.TX_OUT_UDP)
    o = oracle.classify(_EMPTY_RULES, got, n, stride=64, opt=ALL_CHKSUM, classify=False)
    assert np.all((o["out"] >> 16) & 3 == L.ODPG_CHKSUM_OK)
    assert np.all((o["out"] >> 18) & 3 == L.ODPG_CHKSUM_OK)
    assert np.array_equal(got, gen.c2_frames(n, seed=3))


# ---- GPU parity --------------------------------------------------------------
def _random_meta(rng, desc):
    n = len(desc)
    meta = np.zeros(n, np.dtype(L.TX_META_FIELDS))
    ln = desc["len"].astype(np.int64)
    l3 = np.where(rng.random(n) < 0.8, 14, rng.integers(0, np.maximum(ln, 1)))
    l4 = np.where(rng.random(n) < 0.8, l3 + 20, rng.integers(0, np.maximum(ln, 1)))
    l3 = np.where(rng.random(n) < 0.05, L.OFFSET_INVALID, l3)
    l4 = np.where(rng.random(n) < 0.05, L.OFFSET_INVALID, l4)
    meta["l3_offset"] = l3
    meta["l4_offset"] = np.minimum(l4, 0xFFFF)
    meta["flags"] = rng.integers(0, 16, n) | (rng.integers(0, 16, n) << 8)
    return meta


def _corpora():
    _, gold = golden_frames()
    mut = [bytes(x) for x in rulesets.mutate_corpus(600, seed=11)]
    imix_buf, imix_desc = gen.c3_frames(2000, seed=5)
    imix = [bytes(imix_buf[d["offset"]:d["offset"] + d["len"]]) for d in imix_desc]
    return {"golden": gold, "mutated": mut, "imix": imix}


@pytest.mark.gpu
@pytest.mark.parametrize("corpus", ["golden", "mutated", "imix"])
@pytest.mark.parametrize("with_meta", [False, True])
def test_tx_gpu_parity(gpu_ctx, corpus, with_meta):
    frames = _corpora()[corpus]
    buf, desc = pack(frames)
    n = len(frames)
    rng = np.random.default_rng(len(frames) + with_meta)
    meta = _random_meta(rng, desc) if with_meta else None
    for cfg, capa, hp, qs, idx in [
            (CFG_ALL, L.PKTOUT_LOOP_CAPA, 0, 1, 0),
            (CFG_ALL, L.PKTOUT_LOOP_CAPA, L.HASH_IPV4_UDP | L.HASH_IPV4 | L.HASH_IPV6, 8, 3),
            (L.PKTOUT_UDP_CHKSUM | L.PKTOUT_TCP_CHKSUM, L.PKTOUT_LOOP_CAPA,
             L.HASH_IPV4_TCP | L.HASH_IPV6_TCP | L.HASH_IPV6, 5, 9),
            (0, L.PKTOUT_LOOP_CAPA, 0x3F, 16, 2),
            (CFG_ALL, L.PKTOUT_IPV4_CHKSUM | L.PKTOUT_SCTP_CHKSUM, L.HASH_IPV4, 3, 1)]:
        o_out, o_fr = oracle.tx_prepare(buf, n, desc=desc, meta=meta, pktout_cfg=cfg,
                                        pktout_capa=capa, hash_proto=hp, num_qs=qs, index=idx)
        g_out, g_fr = gpu_ctx.tx_prepare(buf, n, desc=desc, meta=meta, pktout_cfg=cfg,
                                         pktout_capa=capa, hash_proto=hp, num_qs=qs, index=idx)
        bad = np.nonzero(o_out != g_out)[0]
        assert len(bad) == 0, (corpus, cfg, hp, bad[:5], o_out[bad[:5]], g_out[bad[:5]])
        assert np.array_equal(o_fr, g_fr[:len(o_fr)]), (corpus, cfg, hp)
        assert np.any(o_out & 0xF0000) or cfg == 0   # some insert ran


@pytest.mark.gpu
def test_tx_gpu_stride64(gpu_ctx):
    """Fixed-stride C2 frames with zeroed checksums: every packet gets its
    IPv4 and UDP checksums back, on the GPU as in the oracle."""
    n = 64 * 300 + 7
    ref = gen.c2_frames(n, seed=9)
    fr = ref.reshape(n, 64).copy()
    fr[:, 24:26] = 0
    fr[:, 40:42] = 0
    fr = fr.reshape(-1)
    cfg = L.PKTOUT_IPV4_CHKSUM | L.PKTOUT_UDP_CHKSUM
    g_out, g_fr = gpu_ctx.tx_prepare(fr, n, stride=64, pktout_cfg=cfg,
                                     hash_proto=L.HASH_IPV4_UDP | L.HASH_IPV4, num_qs=4)
    o_out, o_fr = oracle.tx_prepare(fr, n, stride=64, pktout_cfg=cfg,
                                    hash_proto=L.HASH_IPV4_UDP | L.HASH_IPV4, num_qs=4)
    assert np.array_equal(g_out, o_out)
    assert np.array_equal(g_fr[:len(ref)], ref)
    assert np.array_equal(o_fr, ref)
    assert len(np.unique(g_out & 0xFFFF)) == 4


@pytest.mark.gpu
def test_tx_gpu_stride64_mixed_waves(gpu_ctx):
    """Stride-64 batches run the persistent kernel: tiles of plain frames
    take the register path and write whole frames back through the LDS
    transpose, tiles with any other frame the generic path per lane. Every
    third tile here mixes in mutated frames (VLAN, IPv6, SNAP, truncated,
    bad headers cut to 64 bytes); the last tile is ragged."""
    n = 64 * 97 + 33
    fr = gen.c2_frames(n, seed=21).reshape(n, 64).copy()
    fr[:, 24:26] = 0
    mut = rulesets.mutate_corpus(2000, seed=23, max_len=64)
    k = 0
    for t in range(0, (n + 63) // 64, 3):
        for j in range(t * 64, min(n, t * 64 + 64), 5):
            m = np.frombuffer(bytes(mut[k % len(mut)])[:64], np.uint8)
            fr[j, :] = 0
            fr[j, :len(m)] = m
            k += 1
    fr = fr.reshape(-1)
    for cfg, hp, qs in [(CFG_ALL, L.HASH_IPV4_UDP | L.HASH_IPV4, 4),
                        (L.PKTOUT_TCP_CHKSUM, L.HASH_IPV6 | L.HASH_IPV6_TCP, 7),
                        (0, 0, 3)]:
        g_out, g_fr = gpu_ctx.tx_prepare(fr, n, stride=64, pktout_cfg=cfg, hash_proto=hp,
                                         num_qs=qs, index=5)
        o_out, o_fr = oracle.tx_prepare(fr, n, stride=64, pktout_cfg=cfg, hash_proto=hp,
                                        num_qs=qs, index=5)
        bad = np.nonzero(o_out != g_out)[0]
        assert len(bad) == 0, (cfg, bad[:5], o_out[bad[:5]], g_out[bad[:5]])
        assert np.array_equal(o_fr, g_fr[:len(o_fr)]), cfg
