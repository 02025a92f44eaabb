"""The compiled hit-map region (TBL_XMASK, cls_compile.cpp) that the lean
descriptor kernel (classify_gf.hip) walks, checked on the CPU: a host
emulation of the kernel's classification stage over the table image
(tests/xm_emul.py), driven by the oracle's parse metadata, must give the
oracle's CoS and mark for every packet the oracle parsed without error.
Covers the AND-chain form (complex PMRs' chains as rule bits: C2x, C3, the
all-term and random mixed rule sets) and the lazy form (more chains than
rule bits), the group gates, CUSTOM_L3 / CUSTOM_FRAME guards and
unsatisfiable chains."""
import numpy as np
import pytest

import oracle
import rulesets
from helpers import ALL_CHKSUM, pack
from odp_amd import _lib as L
from odp_amd import gen, gpu
from xm_emul import XmTable, TBL_XMASK, FL_ERROR_MASK


def _check(rules, frames, opt, what, min_cos=2, want_and=None):
    """frames: list of bytes"""
    t = XmTable(gpu.compile_rules(rules))
    assert t.flags & TBL_XMASK, what
    if want_and is not None:
        assert (len(t.xflat) == 0) == want_and, (what, len(t.xflat))
    buf, desc = pack(frames)
    o = oracle.classify(rules, buf, len(frames), desc=desc, opt=opt)
    seen = set()
    checked = 0
    for i, fr in enumerate(frames):
        m = o["meta"][i]
        w = int(o["out"][i])
        if (int(m["flags"]) & FL_ERROR_MASK) or (w & L.ODPG_OUT_PARSE_ERR):
            continue
        cos, mark, matched = t.walk(np.frombuffer(fr, np.uint8), m)
        exp_cos = w & 0xFFFF
        assert cos == exp_cos, (what, i, cos, exp_cos, fr.hex())
        mv = bool(w & L.ODPG_OUT_MARK_VALID)
        assert mv == (matched and mark != 0 and cos != 0xFFFD), (what, i)
        if mv:
            assert mark == int(o["mark"][i]), (what, i)
        seen.add(cos)
        checked += 1
    assert checked > len(frames) // 4, what
    assert len(seen) >= min_cos, (what, sorted(seen))
    return t


def _frames64(buf):
    a = np.asarray(buf).reshape(-1, 64)
    return [bytes(r) for r in a]


def test_c2x_and_form(fresh_cls):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2x_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    t = _check(rules, _frames64(gen.c2x_frames(3000, seed=3)), ALL_CHKSUM, "c2x",
               min_cos=30, want_and=True)
    assert t.nw == 2 and t.nbits <= 64


def test_c3_and_form(fresh_cls):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c3_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    buf, desc = gen.c3_frames(2500, seed=9)
    frames = [bytes(buf[int(d["offset"]):int(d["offset"]) + int(d["len"])]) for d in desc]
    _check(rules, frames, ALL_CHKSUM, "c3", min_cos=10, want_and=True)


@pytest.mark.parametrize("corpus", ["mutate", "edge"])
def test_all_terms(fresh_cls, corpus):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    rulesets.all_terms_rules(fresh_cls, p, stats=False)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    t = XmTable(gpu.compile_rules(rules))
    if not t.flags & TBL_XMASK:
        pytest.skip("the all-term table is not in the hit-map form")
    fr = (rulesets.mutate_corpus(2500, seed=5) if corpus == "mutate"
          else rulesets.imix_edge_corpus(2500, seed=4))
    _check(rules, fr, ALL_CHKSUM, "all_terms " + corpus)


@pytest.mark.parametrize("seed", range(6))
def test_random_mixed(fresh_cls, seed):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    rulesets.random_mixed_rules(fresh_cls, p, seed=seed, stats=False)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    t = XmTable(gpu.compile_rules(rules))
    if not t.flags & TBL_XMASK:
        pytest.skip("not in the hit-map form")
    fr = rulesets.mutate_corpus(1500, seed=seed + 40) + rulesets.imix_edge_corpus(800, seed=seed)
    _check(rules, fr, ALL_CHKSUM, f"random {seed}", min_cos=1)


def test_wide_slots_kx(fresh_cls):
    """more than 16 key slots read: slots 16..18 stay out of the 16-word
    key vector (xm_kx) and the probes select them"""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    rulesets.wide_slots_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    t = _check(fresh_cls.pktio_rules(p), rulesets.wide_slots_corpus(3000), ALL_CHKSUM,
               "wide slots", min_cos=6)
    assert t.kx == 1


def test_key_vector_remap(fresh_cls):
    """at most 16 slots read (C2x reads L4 + 0): slots 16..18 take key-vector
    words no group reads"""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2x_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    t = XmTable(gpu.compile_rules(fresh_cls.pktio_rules(p)))
    assert t.kx == 0 and len(set(t.kpos)) == 3
    used = {int(g[2]) >> 8 for g in t.groups}
    assert all(k < 16 and k not in used for k in t.kpos)


def test_lazy_form(fresh_cls):
    """more chain bits than XM_MAX_PMR: the bits are the PMR indices and the
    complex PMRs are evaluated per level from their records"""
    c = fresh_cls
    assert c.set_limits(256, 512, 256) == 0
    p = c.loop_pktio(pktin=ALL_CHKSUM)
    T = c.Term
    default = c.cos_create("lz_default", queue=c.queue(0))
    leaves = [c.cos_create(f"lz_{k}", queue=c.queue(1 + k)) for k in range(64)]
    assert default and all(leaves)
    assert c.default_cos_set(p, default) == 0
    for k in range(128):
        # IP_DSCP + IPPROTO: two chains (IPv4 / IPv6) per PMR: 256 bits
        assert c.pmr_create([T(c.PMR_IP_DSCP, bytes([k & 63]), b"\x3f"),
                             T(c.PMR_IPPROTO, bytes([17 if k < 64 else 6]), b"\xff")],
                            default, leaves[k % 64])
    for k in range(128):
        # two single-word rules per leaf: 384 rule bits in the chain form
        assert c.pmr_create([T(c.PMR_UDP_DPORT, (k).to_bytes(2, "big"), b"\xff\xff")],
                            leaves[k % 64], leaves[(k % 64 + 1) % 64])
    assert c.pktio_start(p) == 0
    rules = c.pktio_rules(p)
    fr = rulesets.mutate_corpus(1500, seed=11) + rulesets.imix_edge_corpus(1500, seed=12)
    t = _check(rules, fr, ALL_CHKSUM, "lazy", min_cos=2, want_and=False)
    assert t.nbits == t.h["num_pmr"]
