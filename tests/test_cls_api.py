"""odp_cls_* object-model semantics (host, no GPU), modelled on the reference's
basic suite test/validation/api/classification/odp_classification_basic.c and
the data-model behaviour of platform/linux-generic/odp_classification.c."""
import ctypes as C

from odp_amd import _lib as L
from odp_amd import gen


def sip(cls, addr, mask=0xFFFFFFFF):
    return cls.Term(cls.PMR_SIP_ADDR, gen.be_bytes(gen.ip4(addr), 4), gen.be_bytes(mask, 4))


def test_capability(fresh_cls):
    c = fresh_cls.capability()
    assert (c.max_cos, c.max_pmr, c.max_pmr_per_cos, c.max_terms_per_pmr) == (64, 256, 8, 8)
    assert c.max_hash_queues == 32 and c.max_mark == 0xFFFF
    assert c.pmr_range_supported == 0


def test_handles_are_index_plus_one(fresh_cls):
    a = fresh_cls.cos_create("a", queue=fresh_cls.queue(1))
    b = fresh_cls.cos_create("b", queue=fresh_cls.queue(2))
    assert (a, b) == (1, 2)
    assert L.lib.odp_cos_to_u64(b) == 2
    p = fresh_cls.pmr_create([sip(fresh_cls, "1.2.3.4")], a, b)
    assert p == 1 and L.lib.odp_pmr_to_u64(p) == 1


def test_cos_create_param_checks(fresh_cls):
    # enqueue CoS needs a queue when num_queue == 1 (odp_classification.c:245-246)
    assert fresh_cls.cos_create("noq") is None
    # num_queue bounds (:250-251)
    assert fresh_cls.cos_create("big", num_queue=33) is None
    # drop CoS needs no queue (:239-243)
    d = fresh_cls.cos_create("drop", action=fresh_cls.COS_ACTION_DROP)
    assert d and fresh_cls.cos_queue(d) is None


def test_cos_max_entries(fresh_cls):
    made = [fresh_cls.cos_create(f"c{i}", queue=fresh_cls.queue(i)) for i in range(64)]
    assert all(made)
    assert fresh_cls.cos_create("one-too-many", queue=fresh_cls.queue(99)) is None
    assert fresh_cls.cos_destroy(made[10]) == 0
    # first free slot is reused (:276-279)
    assert fresh_cls.cos_create("again", queue=fresh_cls.queue(100)) == made[10]


def test_pmr_per_cos_limit_and_terms(fresh_cls):
    src = fresh_cls.cos_create("src", queue=fresh_cls.queue(1))
    dst = fresh_cls.cos_create("dst", queue=fresh_cls.queue(2))
    pmrs = [fresh_cls.pmr_create([sip(fresh_cls, f"10.0.0.{i}")], src, dst) for i in range(8)]
    assert all(pmrs)
    assert fresh_cls.pmr_create([sip(fresh_cls, "10.0.0.9")], src, dst) is None   # :807-808
    # bad sizes / ranges / unsupported terms (:653-726)
    other = fresh_cls.cos_create("o", queue=fresh_cls.queue(3))
    assert fresh_cls.pmr_create([fresh_cls.Term(fresh_cls.PMR_SIP_ADDR, b"\1\2\3", b"\xff\xff\xff")],
                                other, dst) is None
    assert fresh_cls.pmr_create([fresh_cls.Term(fresh_cls.PMR_ICMP_TYPE, b"\1", b"\xff")],
                                other, dst) is None
    t = sip(fresh_cls, "1.1.1.1")
    t.range_term = True
    assert fresh_cls.pmr_create([t], other, dst) is None
    assert fresh_cls.pmr_create([sip(fresh_cls, "1.1.1.1")] * 9, other, dst) is None
    # custom terms accept any size <= 16
    assert fresh_cls.pmr_create([fresh_cls.Term(fresh_cls.PMR_CUSTOM_FRAME, b"\x01" * 16,
                                                b"\xff" * 16, offset=20)], other, dst)
    # invalid CoS handles
    assert fresh_cls.pmr_create([sip(fresh_cls, "1.1.1.1")], 999, dst) is None


def test_value_masked_at_create(fresh_cls):
    p = fresh_cls.loop_pktio()
    a = fresh_cls.cos_create("a", queue=fresh_cls.queue(1))
    b = fresh_cls.cos_create("b", queue=fresh_cls.queue(2))
    assert fresh_cls.default_cos_set(p, a) == 0
    assert fresh_cls.pmr_create([fresh_cls.Term(fresh_cls.PMR_SIP_ADDR, b"\x0a\x0b\x0c\x0d",
                                                b"\xff\xff\xff\x00")], a, b)
    r = fresh_cls.pktio_rules(p)
    t = r.pmr[0].terms[0]
    assert bytes(t.value[:4]) == b"\x0a\x0b\x0c\x00"      # value &= mask (:732-733)
    assert t.val_sz == 4


def test_pmr_destroy_swaps_last_into_slot(fresh_cls):
    """odp_cls_pmr_destroy moves the last rule into the freed slot, which
    changes first-match order (odp_classification.c:757-761)."""
    p = fresh_cls.loop_pktio()
    src = fresh_cls.cos_create("src", queue=fresh_cls.queue(1))
    dsts = [fresh_cls.cos_create(f"d{i}", queue=fresh_cls.queue(10 + i)) for i in range(4)]
    assert fresh_cls.default_cos_set(p, src) == 0
    pm = [fresh_cls.pmr_create([sip(fresh_cls, f"10.0.0.{i}")], src, dsts[i]) for i in range(4)]
    assert fresh_cls.pmr_destroy(pm[1]) == 0
    r = fresh_cls.pktio_rules(p)
    ci = fresh_cls.to_index(src)
    ce = r.cos[ci]
    order = [r.rule_pmr[ce.rule_start + k] for k in range(ce.num_rule)]
    dst = [r.rule_dst[ce.rule_start + k] for k in range(ce.num_rule)]
    assert order == [0, 3, 2]
    assert dst == [fresh_cls.to_index(dsts[i]) for i in (0, 3, 2)]
    assert fresh_cls.pmr_destroy(pm[1]) == -1               # already destroyed
    # the freed PMR slot is reused first
    again = fresh_cls.pmr_create([sip(fresh_cls, "10.0.0.9")], src, dsts[1])
    assert again == pm[1]


def test_pktio_setters(fresh_cls):
    p = fresh_cls.loop_pktio()
    a = fresh_cls.cos_create("a", queue=fresh_cls.queue(1))
    assert fresh_cls.default_cos_set(p, a) == 0
    assert fresh_cls.default_cos_set(p, None) == 0          # NULL default allowed (:591)
    assert fresh_cls.error_cos_set(p, None) == -1           # error cos must be valid (:614-618)
    assert fresh_cls.error_cos_set(p, a) == 0
    assert fresh_cls.default_cos_set(p, 77) == -1
    assert fresh_cls.skip_set(p, 4) == -95                  # -ENOTSUP (:624-631)
    assert fresh_cls.headroom_set(p, 64) == 0
    r = fresh_cls.pktio_rules(p)
    assert r.default_cos == -1 and r.error_cos == fresh_cls.to_index(a)


def test_pktio_config_rejects_drop_bits(fresh_cls):
    """loop pktio capability has no drop_* bits (pktio/loop.c:664-670)."""
    p = fresh_cls.pktio_open("loop")
    assert fresh_cls.pktio_config(p, pktin=L.PKTIN_DROP_UDP_ERR) == -1
    assert fresh_cls.pktio_config(p, pktin=L.PKTIN_UDP_CHKSUM | L.PKTIN_IPV4_CHKSUM) == 0


def test_cos_queue_api(fresh_cls):
    a = fresh_cls.cos_create("a", queue=fresh_cls.queue(1))
    assert fresh_cls.cos_queue(a) == fresh_cls.queue(1)
    assert fresh_cls.cos_queue_set(a, fresh_cls.queue(5)) == 0
    assert fresh_cls.cos_queue(a) == fresh_cls.queue(5)
    assert fresh_cls.cos_num_queue(a) == 1
    h = fresh_cls.cos_create("h", num_queue=4,
                             hash_proto=fresh_cls.HASH_IPV4 | fresh_cls.HASH_IPV4_UDP)
    assert fresh_cls.cos_num_queue(h) == 4
    n, qs = fresh_cls.cos_queues(h)
    assert n == 4 and len(set(qs)) == 4 and None not in qs
    assert fresh_cls.cos_queue_set(h, fresh_cls.queue(7)) == -1   # hashing enabled (:511-514)
    assert fresh_cls.cos_destroy(h) == 0
    assert fresh_cls.cos_num_queue(h) == 0


def test_generation_bumps(fresh_cls):
    g0 = L.lib.odpg_cls_generation()
    a = fresh_cls.cos_create("a", queue=fresh_cls.queue(1))
    assert L.lib.odpg_cls_generation() > g0
    g1 = L.lib.odpg_cls_generation()
    fresh_cls.cos_destroy(a)
    assert L.lib.odpg_cls_generation() > g1


def test_raised_limits(fresh_cls):
    assert fresh_cls.set_limits(2048, 2048, 32) == 0
    c = fresh_cls.capability()
    assert (c.max_cos, c.max_pmr, c.max_pmr_per_cos) == (2048, 2048, 32)
    p = fresh_cls.loop_pktio()
    r = gen.build_c4_rules(fresh_cls, p)
    assert len(r["pmrs"]) == 1024
    # limits can only change before the first create
    assert fresh_cls.set_limits(64, 256, 8) != 0
