"""The reference classification validation suite, replayed as fixtures.

`tests/golden/make_golden.py` encodes every per-packet expectation of
test/validation/api/classification/{odp_classification_test_pmr.c,
odp_classification_tests.c, odp_classification_basic.c} as data (CoS objects
and PMRs in creation order, packets as create_packet() parameters plus the
test's field edits, the CoS the test asserts the packet is received on, and
odp_packet_cls_mark()). `tests/cls_testpkt.py` makes the frames.

Two independent routes to the rule table are checked:
  * `direct_rules` builds the odpg_rules_t straight from the fixture
    (pmr_create_term's value &= mask, odp_classification.c:728-733; rules per
    source CoS in creation order, :826-829), without odp_cls.c;
  * the odp_cls_* API (odp_cls.c) builds it from the same objects.
The oracle must meet every expectation through both (CPU tests), and every
GPU kernel strategy must produce the oracle's results through both (-m gpu).
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from cls_testpkt import udp_tcp_chksum  # noqa: F401  (re-exported for test_helper_verify)
from helpers import GOLDEN, assert_same, pack
from odp_amd import _lib as L
from odp_amd import cls as CLS

SCEN = GOLDEN["cls_validation"]
IDS = [s["name"] for s in SCEN]


def term_id(name):
    return getattr(CLS, "PMR_" + name)


def direct_rules(sc):
    """odpg_rules_t from the fixture alone. Returns (rules, keepalive, index)."""
    idx = {c["name"]: i for i, c in enumerate(sc["cos"])}
    ncos = len(sc["cos"])
    coses = (L.odpg_cos_t * ncos)()
    pmrs = [p for p in sc["pmrs"] if not p.get("create_fails")]
    parr = (L.odpg_pmr_t * max(len(pmrs), 1))()
    per_src = {i: [] for i in range(ncos)}
    for k, p in enumerate(pmrs):
        parr[k].num_terms = len(p["terms"])
        parr[k].mark = p["mark"] or 0
        for j, t in enumerate(p["terms"]):
            v, m = bytes.fromhex(t["value"]), bytes.fromhex(t["mask"])
            tt = parr[k].terms[j]
            tt.term, tt.val_sz, tt.offset = term_id(t["term"]), t["val_sz"], t["offset"]
            for b in range(t["val_sz"]):
                tt.value[b] = v[b] & m[b]
                tt.mask[b] = m[b]
        per_src[idx[p["src"]]].append((k, idx[p["dst"]]))
    slots_p, slots_d = [], []
    for i, c in enumerate(sc["cos"]):
        coses[i].valid = 1
        coses[i].action = 1 if c.get("action") == "drop" else 0
        coses[i].num_queue = 1
        coses[i].stats_enable = int(bool(c.get("stats")))
        coses[i].rule_start = len(slots_p)
        coses[i].num_rule = len(per_src[i])
        for k, d in per_src[i]:
            slots_p.append(k)
            slots_d.append(d)
    rp = (C.c_uint32 * max(len(slots_p), 1))(*slots_p)
    rd = (C.c_uint32 * max(len(slots_d), 1))(*slots_d)
    r = L.odpg_rules_t(ncos, coses, len(pmrs), parr, len(slots_p), rp, rd,
                       idx[sc["default"]] if sc["default"] else -1,
                       idx[sc["error"]] if sc["error"] else -1)
    return r, (coses, parr, rp, rd), idx


def api_rules(cls, sc):
    """The same objects through the odp_cls_* API (odp_amd/csrc/odp_cls.c)."""
    p = cls.loop_pktio(classifier=sc["classifier"])
    h = {}
    for i, c in enumerate(sc["cos"]):
        drop = c.get("action") == "drop"
        h[c["name"]] = cls.cos_create(
            c["name"], queue=None if drop else cls.queue(i),
            action=cls.COS_ACTION_DROP if drop else cls.COS_ACTION_ENQUEUE,
            stats_enable=bool(c.get("stats")))
        assert h[c["name"]], c
    for pm in sc["pmrs"]:
        terms = [cls.Term(term_id(t["term"]), bytes.fromhex(t["value"]),
                          bytes.fromhex(t["mask"]), offset=t["offset"], val_sz=t["val_sz"])
                 for t in pm["terms"]]
        r = cls.pmr_create(terms, h[pm["src"]], h[pm["dst"]], mark=pm["mark"])
        if pm.get("create_fails"):
            assert not r, f"{sc['name']}: the reference rejects this term at create"
        else:
            assert r, pm
    for op in sc["ops"]:
        tgt = h[sc["pmrs"][0]["dst"]]
        if op == "cos_pool_set":          # odp_classification_test_pmr.c:1034-1036
            assert cls.cos_pool_set(tgt, 0x7001) == 0 and cls.cos_pool(tgt) == 0x7001
        elif op == "cos_queue_set":       # :1133-1135
            assert cls.cos_queue_set(tgt, 0x7002) == 0 and cls.cos_queue(tgt) == 0x7002
    if sc["default"]:
        assert cls.default_cos_set(p, h[sc["default"]]) == 0
    if sc["error"]:
        assert cls.error_cos_set(p, h[sc["error"]]) == 0
    assert cls.pktio_start(p) == 0
    idx = {k: cls.to_index(v) for k, v in h.items()}
    return cls.pktio_rules(p), idx, p


def frames_of(sc):
    fr = [bytes.fromhex(p["frame"]) for p in sc["packets"]]
    return pack(fr)


def check_expectations(sc, res, idx, what):
    out, mark = res["out"], res["mark"]
    for i, p in enumerate(sc["packets"]):
        w = int(out[i])
        cos = w & 0xFFFF
        if p["expect"] == "NOCLS":
            assert cos == L.ODPG_COS_NOCLS, (what, i)
            continue
        exp = idx[p["expect"]]
        assert cos == exp, f"{what} pkt {i}: CoS {cos}, reference expects {p['expect']} ({exp})"
        drop = any(c["name"] == p["expect"] and c.get("action") == "drop" for c in sc["cos"])
        assert bool(w & L.ODPG_OUT_CLS_DROP) == drop, (what, i)
        got_mark = int(mark[i]) if w & L.ODPG_OUT_MARK_VALID else 0
        assert got_mark == p["mark"], f"{what} pkt {i}: mark {got_mark} != {p['mark']}"
    for name, n in sc.get("cos_stats", {}).items():
        assert int(res["stats"][4 + idx[name]]) == n, (what, name)


def test_fixture_inventory():
    """Every suite the survey names is represented."""
    names = set(IDS)
    for must in ("tcp_sport", "udp_dport", "udp_sport", "ipv4_proto", "ipv6_proto",
                 "ipv4_dscp", "ipv6_dscp", "dmac", "packet_len", "vlan_id_0", "vlan_id_x",
                 "vlan_pcp_0", "eth_type_0", "eth_type_x", "ipv4_saddr", "ipv4_daddr",
                 "ipv6_saddr", "ipv6_daddr", "custom_frame", "custom_l3",
                 "ipsec_spi_ah_ipv4", "ipsec_spi_esp_ipv6", "pmr_serial", "pmr_parallel",
                 "pmr_marking", "cls_pktio", "pktin_classifier_flag", "tcp_dport_multi"):
        assert must in names, must
    assert sum(len(s["packets"]) for s in SCEN) >= 100


@pytest.mark.parametrize("sc", SCEN, ids=IDS)
def test_oracle_direct(sc):
    """The oracle meets the reference's expectations on rules built from the
    fixture alone (no odp_cls.c involved)."""
    rules, keep, idx = direct_rules(sc)
    if not sc["packets"]:
        return
    buf, desc = frames_of(sc)
    res = oracle.classify(rules, buf, len(sc["packets"]), desc=desc,
                          classify=sc["classifier"])
    check_expectations(sc, res, idx, f"{sc['name']} direct")
    del keep


@pytest.mark.parametrize("sc", SCEN, ids=IDS)
def test_oracle_api(fresh_cls, sc):
    """The same through the odp_cls_* object model, and equal to the direct
    build packet for packet (so odp_cls.c's term storing is checked against
    the fixture, not against itself)."""
    rules, idx, _ = api_rules(fresh_cls, sc)
    if not sc["packets"]:
        return
    buf, desc = frames_of(sc)
    n = len(sc["packets"])
    res = oracle.classify(rules, buf, n, desc=desc, classify=sc["classifier"])
    check_expectations(sc, res, idx, f"{sc['name']} api")
    drules, keep, _ = direct_rules(sc)
    dres = oracle.classify(drules, buf, n, desc=desc, classify=sc["classifier"])
    assert_same({k: res[k] for k in ("out", "mark", "meta")},
                {k: dres[k] for k in ("out", "mark", "meta")}, f"{sc['name']} api vs direct")
    del keep


def test_capability_matches_create_failures(fresh_cls):
    """Terms the reference's capability leaves out are the ones pmr_create
    rejects (odp_classification.c:153-201, :717-720)."""
    capa = fresh_cls.capability()
    for sc in SCEN:
        for pm in sc["pmrs"]:
            if pm.get("create_fails"):
                t = term_id(pm["terms"][0]["term"])
                assert not (capa.supported_terms >> t) & 1, pm


@pytest.mark.gpu
def test_gpu_all_strategies(gpu_ctx, fresh_cls):
    """Every scenario through every kernel strategy (walk, evaluate-all, hash
    walk, auto), with rules from the fixture and from odp_cls.c: bit-exact
    with the oracle, and the reference's expectations met."""
    for sc in SCEN:
        if not sc["packets"]:
            continue
        fresh_cls.reset()
        arules, aidx, _ = api_rules(fresh_cls, sc)
        drules, keep, didx = direct_rules(sc)
        buf, desc = frames_of(sc)
        n = len(sc["packets"])
        for rules, idx, src in ((drules, didx, "direct"), (arules, aidx, "api")):
            o = oracle.classify(rules, buf, n, desc=desc, classify=sc["classifier"])
            tbl = gpu_ctx.table(rules)
            for mode in (1, 2, 3, 0):
                gpu_ctx.set_kernel_mode(mode)
                g = gpu_ctx.classify(tbl, buf, n, desc=desc, classify=sc["classifier"])
                assert_same(g, o, f"{sc['name']} {src} mode {mode}")
                check_expectations(sc, g, idx, f"{sc['name']} {src} mode {mode} (GPU)")
            gpu_ctx.set_kernel_mode(0)
            del tbl
        del keep


@pytest.mark.gpu
def test_gpu_scenarios_batched(gpu_ctx, fresh_cls):
    """All single-PMR scenarios' packets in one large launch per scenario
    (replicated to 4096 packets) so the tile loop, not just the first wave,
    meets the expectations."""
    for sc in SCEN:
        if not sc["packets"] or sc["name"] == "cls_pktio":
            continue
        drules, keep, idx = direct_rules(sc)
        fr = [bytes.fromhex(p["frame"]) for p in sc["packets"]]
        reps = 4096 // len(fr) + 1
        buf, desc = pack(fr * reps)
        n = len(fr) * reps
        o = oracle.classify(drules, buf, n, desc=desc, classify=sc["classifier"])
        tbl = gpu_ctx.table(drules)
        g = gpu_ctx.classify(tbl, buf, n, desc=desc, classify=sc["classifier"])
        assert_same(g, o, sc["name"])
        assert np.array_equal(g["out"][: len(fr)], g["out"][len(fr): 2 * len(fr)])
        del tbl, keep
