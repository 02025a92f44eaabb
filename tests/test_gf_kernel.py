"""The lean descriptor kernel (classify_gf.hip): descriptor (IMIX) batches
under a hybrid hash-walk table in its hit-map form (TBL_XMASK), verdict
words only, auto mode. Bit-exact against the oracle on the C3 traffic, the
IMIX edge corpus (rulesets.imix_edge_corpus: every register-parse edge and
the frames that must leave it), the mutation corpus and the golden frames,
under each RX checksum option mix; and the launch really took the kernel
(odpg_last_kernel() == 2)."""
import numpy as np
import pytest

import oracle
import rulesets
from helpers import ALL_CHKSUM, TBL_XMASK, assert_same, golden_frames, pack, table_flags
from odp_amd import _lib as L
from odp_amd import gen

OPTS = [0, L.PKTIN_IPV4_CHKSUM, L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM, L.PKTIN_TCP_CHKSUM,
        ALL_CHKSUM]


def _c3(cls, opt):
    p = cls.loop_pktio(pktin=opt)
    gen.build_c3_rules(cls, p, stats=False)
    assert cls.pktio_start(p) == 0
    return cls.pktio_rules(p)


def test_c3_table_takes_the_gf_form(fresh_cls):
    assert table_flags(_c3(fresh_cls, ALL_CHKSUM)) & TBL_XMASK


def test_edge_corpus_spans_both_parses():
    fr = rulesets.imix_edge_corpus(4096)
    lens = np.array([len(f) for f in fr])
    assert lens.min() < 64 and lens.max() > 1514 and np.any(lens == 64) and np.any(lens == 74)
    v6 = sum(1 for f in fr if f[12:14] == b"\x86\xdd")
    assert 0.2 < v6 / len(fr) < 0.45


def _verdicts(ctx, rules, buf, n, desc, opt):
    tbl = ctx.table(rules)
    g = ctx.classify(tbl, buf, n, desc=desc, opt=opt, want_mark=False, want_meta=False,
                     want_stats=False)
    assert L.lib.odpg_last_kernel() == 2, "the launch did not take the lean descriptor kernel"
    o = oracle.classify(rules, buf, n, desc=desc, opt=opt)
    return g, o


@pytest.mark.gpu
@pytest.mark.parametrize("opt", OPTS)
@pytest.mark.parametrize("corpus", ["c3", "edge", "mutate", "golden"])
def test_gf_kernel_matches_oracle(gpu_ctx, fresh_cls, opt, corpus):
    rules = _c3(fresh_cls, opt)
    if corpus == "c3":
        n = 64 * 1031 + 17
        buf, desc = gen.c3_frames(n, seed=77 + opt)
    else:
        frames = (rulesets.imix_edge_corpus(24000, seed=opt + 1) if corpus == "edge" else
                  rulesets.mutate_corpus(12000, seed=61) if corpus == "mutate" else
                  golden_frames()[1])
        buf, desc = pack(frames)
        n = len(frames)
    g, o = _verdicts(gpu_ctx, rules, buf, n, desc, opt)
    assert_same({"out": g["out"]}, {"out": o["out"]}, f"gf {corpus} opt={opt:#x}")
    if corpus == "c3":
        assert len(np.unique(o["out"] & 0xFFFF)) > 10


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097, 1 << 18])
def test_gf_kernel_batch_sizes(gpu_ctx, fresh_cls, n):
    rules = _c3(fresh_cls, ALL_CHKSUM)
    buf, desc = gen.c3_frames(n, seed=n)
    g, o = _verdicts(gpu_ctx, rules, buf, n, desc, ALL_CHKSUM)
    assert_same({"out": g["out"]}, {"out": o["out"]}, f"gf n={n}")


@pytest.mark.gpu
@pytest.mark.parametrize("corpus", ["c3", "edge"])
def test_gf_kernel_sharded_counters(gpu_ctx, fresh_cls, corpus):
    """The counted launch (sharded pktio / per-queue counters) on the lean
    descriptor kernel: two launches, one fold, against the oracle's counts."""
    from helpers import assert_counters, expected_counters
    rules = _c3(fresh_cls, ALL_CHKSUM)
    if corpus == "c3":
        n = 64 * 517 + 9
        buf, desc = gen.c3_frames(n, seed=5)
    else:
        frames = rulesets.imix_edge_corpus(20000, seed=11)
        buf, desc = pack(frames)
        n = len(frames)
    tbl = gpu_ctx.table(rules)
    o = oracle.classify(rules, buf, n, desc=desc, opt=ALL_CHKSUM)
    cnt = gpu_ctx.counters(tbl)
    for _ in range(2):
        g = gpu_ctx.classify(tbl, buf, n, desc=desc, opt=ALL_CHKSUM, want_mark=False,
                             want_meta=False, counters=cnt)
        assert L.lib.odpg_last_kernel() == 2
        assert np.array_equal(g["out"], o["out"])
    want = expected_counters(o, tbl.num_cos)
    assert_counters(cnt.fold(), {k: v * 2 for k, v in want.items()}, f"gf counters {corpus}")
    cnt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [64, 128, 256])
def test_gf_kernel_fixed_stride(gpu_ctx, fresh_cls, stride):
    """Fixed-stride batches take the same kernel (each frame's descriptor
    computed as (i * stride, stride)): edge-corpus frames cut / padded into
    stride slots, C3 rules, every checksum option mix; ragged last tile."""
    frames = rulesets.imix_edge_corpus(64 * 157 + 29, seed=stride)
    n = len(frames)
    buf = np.zeros((n, stride), np.uint8)
    for k, f in enumerate(frames):
        m = np.frombuffer(bytes(f)[:stride], np.uint8)
        buf[k, :len(m)] = m
    buf = buf.reshape(-1)
    for opt in (ALL_CHKSUM, L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM, 0):
        fresh_cls.reset()
        rules = _c3(fresh_cls, opt)
        tbl = gpu_ctx.table(rules)
        g = gpu_ctx.classify(tbl, buf, n, stride=stride, opt=opt, want_mark=False,
                             want_meta=False, want_stats=False)
        assert L.lib.odpg_last_kernel() == 2, "fixed stride did not take the lean descriptor kernel"
        o = oracle.classify(rules, buf, n, stride=stride, opt=opt)
        assert np.array_equal(g["out"], o["out"]), (stride, opt)


@pytest.mark.gpu
def test_c2x_takes_the_gf_kernel(gpu_ctx, fresh_cls):
    """The C2x rule mix (multi-word DIP6 and DMAC terms, IPPROTO / DSCP
    alternative pairs in multi-term rules, CUSTOM_FRAME) compiles to the
    hit-map form and its 64-byte batches run the lean descriptor kernel."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2x_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    assert table_flags(rules) & TBL_XMASK
    n = 64 * 500 + 3
    fr = gen.c2x_frames(n, seed=5)
    tbl = gpu_ctx.table(rules)
    g = gpu_ctx.classify(tbl, fr, n, stride=64, opt=ALL_CHKSUM, want_mark=False,
                         want_meta=False, want_stats=False)
    assert L.lib.odpg_last_kernel() == 2
    o = oracle.classify(rules, fr, n, stride=64, opt=ALL_CHKSUM)
    assert np.array_equal(g["out"], o["out"])


def _c2x(cls):
    p = cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2x_rules(cls, p)
    assert cls.pktio_start(p) == 0
    return cls.pktio_rules(p)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097, 1 << 18])
def test_gf_s64_batch_sizes(gpu_ctx, fresh_cls, n):
    """The fixed 64-byte stride instantiation (S64: coalesced tile loads
    through the LDS rows, no descriptors, no tail pass) on C2x traffic and
    the edge corpus cut to 64 bytes, ragged last tiles; verdict-only and
    counted launches."""
    from helpers import assert_counters, expected_counters
    rules = _c2x(fresh_cls)
    fr = gen.c2x_frames(n, seed=n + 3).reshape(n, 64).copy()
    edge = rulesets.imix_edge_corpus(max(1, n // 4), seed=n)
    for k, f in enumerate(edge):          # a quarter of the slots: edge frames
        b = np.frombuffer(bytes(f)[:64], np.uint8)
        fr[4 * k % n] = 0
        fr[4 * k % n, :len(b)] = b
    fr = fr.reshape(-1)
    tbl = gpu_ctx.table(rules)
    o = oracle.classify(rules, fr, n, stride=64, opt=ALL_CHKSUM)
    g = gpu_ctx.classify(tbl, fr, n, stride=64, opt=ALL_CHKSUM, want_mark=False,
                         want_meta=False, want_stats=False)
    assert L.lib.odpg_last_kernel() == 2
    assert_same({"out": g["out"]}, {"out": o["out"]}, f"s64 n={n}")
    cnt = gpu_ctx.counters(tbl)
    g = gpu_ctx.classify(tbl, fr, n, stride=64, opt=ALL_CHKSUM, want_mark=False,
                         want_meta=False, counters=cnt)
    assert L.lib.odpg_last_kernel() == 2
    assert np.array_equal(g["out"], o["out"])
    assert_counters(cnt.fold(), expected_counters(o, tbl.num_cos), f"s64 counters n={n}")
    cnt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["desc", "stride64"])
def test_gf_kernel_wide_slots(gpu_ctx, fresh_cls, layout):
    """A table whose groups read more than 16 key slots (xm_kx: slots 16..18
    selected per probe) on descriptor and fixed-stride batches."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    rulesets.wide_slots_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    assert table_flags(rules) & TBL_XMASK
    frames = rulesets.wide_slots_corpus(64 * 200 + 11, seed=21)
    n = len(frames)
    if layout == "desc":
        buf, desc = pack(frames)
        g, o = _verdicts(gpu_ctx, rules, buf, n, desc, ALL_CHKSUM)
    else:
        buf = np.zeros((n, 64), np.uint8)
        for k, f in enumerate(frames):
            b = np.frombuffer(bytes(f)[:64], np.uint8)
            buf[k, :len(b)] = b
        buf = buf.reshape(-1)
        tbl = gpu_ctx.table(rules)
        g = gpu_ctx.classify(tbl, buf, n, stride=64, opt=ALL_CHKSUM, want_mark=False,
                             want_meta=False, want_stats=False)
        assert L.lib.odpg_last_kernel() == 2
        o = oracle.classify(rules, buf, n, stride=64, opt=ALL_CHKSUM)
    assert_same({"out": g["out"]}, {"out": o["out"]}, f"wide slots {layout}")
    assert len(np.unique(o["out"] & 0xFFFF)) >= 6
