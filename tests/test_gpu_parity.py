"""GPU parity: libodpg.so's gfx950 kernels vs the CPU restatement (oracle) on
the same inputs, through the C-ABI. Bit-exact on every output: verdict word,
mark, full parser metadata (packet_parser_t) and the pktio / CoS counters."""
import numpy as np
import pytest

import oracle
import rulesets
from helpers import (ALL_CHKSUM, GOLDEN, assert_counters, assert_same, expected_counters,
                     golden_frames, pack)
from odp_amd import _lib as L
from odp_amd import gen

pytestmark = pytest.mark.gpu

OPTS = [0, L.PKTIN_IPV4_CHKSUM, L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM, ALL_CHKSUM]


def both(ctx, rules, buf, num, stride=0, desc=None, opt=0, layer=L.LAYER_ALL, classify=True):
    """Classify on the GPU with every kernel strategy (walk, evaluate-all,
    auto) and on the oracle; the strategies must agree bit for bit."""
    tbl = ctx.table(rules)
    o = oracle.classify(rules, buf, num, stride=stride, desc=desc, opt=opt, layer=layer,
                        classify=classify)
    res = {}
    for mode in (1, 2, 3, 0):
        ctx.set_kernel_mode(mode)
        res[mode] = ctx.classify(tbl, buf, num, stride=stride, desc=desc, opt=opt,
                                 layer=layer, classify=classify)
    # verdicts, marks and metadata without counters: in such launches the
    # general kernel's odd waves sum their checksum tails after the CoS walk
    for mode in (3, 0):
        ctx.set_kernel_mode(mode)
        vo = ctx.classify(tbl, buf, num, stride=stride, desc=desc, opt=opt, layer=layer,
                          classify=classify, want_stats=False)
        assert_same(res[1], vo, f"no-counter launch, mode {mode}")
    ctx.set_kernel_mode(0)
    assert_same(res[1], res[2], "walk vs evaluate-all")
    assert_same(res[1], res[3], "walk vs hash walk")
    if stride == 64 and desc is None:
        # verdict words only: auto mode may take the lean 64-byte kernel
        lean = ctx.classify(tbl, buf, num, stride=stride, opt=opt, layer=layer,
                            classify=classify, want_mark=False, want_meta=False,
                            want_stats=False)
        assert_same(res[1], lean, f"walk vs verdict-only (kernel {L.lib.odpg_last_kernel()})")
        # verdict words + pktio counters (the lean kernel's counted launch)
        lean = ctx.classify(tbl, buf, num, stride=stride, opt=opt, layer=layer,
                            classify=classify, want_mark=False, want_meta=False)
        assert_same(res[1], lean, f"walk vs verdict+stats (kernel {L.lib.odpg_last_kernel()})")
    if desc is not None:
        # verdict words only: auto mode may take the lean descriptor kernel
        vo = ctx.classify(tbl, buf, num, desc=desc, opt=opt, layer=layer, classify=classify,
                          want_mark=False, want_meta=False, want_stats=False)
        assert_same({"out": res[1]["out"]}, {"out": vo["out"]},
                    f"walk vs verdict-only (kernel {L.lib.odpg_last_kernel()})")
    # sharded counters (odpg.h): the walk and auto (lean kernel where it
    # applies), two launches each, one fold against the oracle's counts
    cnt = ctx.counters(tbl)
    want = expected_counters(o, tbl.num_cos)
    for mode in (1, 0):
        ctx.set_kernel_mode(mode)
        for _ in range(2):
            g = ctx.classify(tbl, buf, num, stride=stride, desc=desc, opt=opt, layer=layer,
                             classify=classify, want_mark=False, want_meta=False, counters=cnt)
            assert np.array_equal(g["out"], res[1]["out"]), f"counters launch, mode {mode}"
        f = cnt.fold()
        assert_counters(f, {k: v * 2 for k, v in want.items()},
                        f"mode {mode} kernel {L.lib.odpg_last_kernel()}")
    ctx.set_kernel_mode(0)
    cnt.close()
    return res[0], o


def default_only(cls, pktin=0):
    p = cls.loop_pktio(pktin=pktin)
    d = cls.cos_create("DefaultCos", queue=cls.queue(0), stats_enable=True)
    e = cls.cos_create("ErrorCos", queue=cls.queue(1), stats_enable=True)
    assert cls.default_cos_set(p, d) == 0 and cls.error_cos_set(p, e) == 0
    assert cls.pktio_start(p) == 0
    return p


@pytest.mark.parametrize("opt", OPTS)
def test_golden_frames(gpu_ctx, fresh_cls, opt):
    p = default_only(fresh_cls, pktin=opt)
    names, frames = golden_frames()
    buf, desc = pack(frames)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, len(frames), desc=desc, opt=opt)
    assert_same(g, o, f"golden opt={opt}")


@pytest.mark.parametrize("layer", [L.LAYER_NONE, L.LAYER_L2, L.LAYER_L3, L.LAYER_L4])
def test_parse_layers_no_cls(gpu_ctx, fresh_cls, layer):
    p = default_only(fresh_cls, pktin=ALL_CHKSUM)
    names, frames = golden_frames()
    buf, desc = pack(frames)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, len(frames), desc=desc,
                opt=ALL_CHKSUM, layer=layer, classify=False)
    assert_same(g, o, f"layer {layer}")


def test_example_classifier_pcap(gpu_ctx, fresh_cls):
    p = fresh_cls.loop_pktio()
    r = gen.build_c1_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    frames = [bytes.fromhex(h) for h in GOLDEN["pcap"]["classifier_udp64"]]
    buf, desc = pack(frames)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, len(frames), desc=desc)
    assert_same(g, o, "classifier pcap")
    cos = g["out"] & 0xFFFF
    assert (cos == fresh_cls.to_index(r["queue1"])).sum() == 100
    assert (cos == fresh_cls.to_index(r["default"])).sum() == 100


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_all_terms_fuzz(gpu_ctx, fresh_cls, seed):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    rulesets.all_terms_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    frames = rulesets.mutate_corpus(20000, seed=seed)
    buf, desc = pack(frames)
    for opt in (0, ALL_CHKSUM):
        g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, len(frames), desc=desc, opt=opt)
        assert_same(g, o, f"fuzz seed={seed} opt={opt}")


def test_c1_stride64(gpu_ctx, fresh_cls):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c1_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    n = 1 << 16
    fr = gen.c1_frames(n)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, n, stride=64, opt=ALL_CHKSUM)
    assert_same(g, o, "C1")


@pytest.mark.parametrize("n", [1, 63, 255, 257, 4097, 1 << 20])
def test_c2_stride64_sizes(gpu_ctx, fresh_cls, n):
    """Ragged batch sizes up to the headline 2^20 batch, bit-exact end to end."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    fr = gen.c2_frames(n)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, n, stride=64, opt=ALL_CHKSUM)
    assert_same(g, o, f"C2 n={n}")
    assert g["stats"][0] == n                        # every packet delivered


@pytest.mark.parametrize("n", [255, 1 << 16])
def test_c2x_mixed_terms(gpu_ctx, fresh_cls, n):
    """The C2x bench workload (SURVEY 8(d)'s second C2 rule mix: VLAN / QinQ
    / IPv6 / multicast frames against ETHTYPE, DMAC, IPPROTO, DSCP, VLAN,
    DIP6, CUSTOM and port terms), every kernel strategy vs the oracle."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2x_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    fr = gen.c2x_frames(n)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, n, stride=64, opt=ALL_CHKSUM)
    assert_same(g, o, f"C2x n={n}")
    assert g["stats"][0] == n
    assert n < 4096 or len(np.unique(o["out"] & 0xFFFF)) > 40


def test_c2_stride_variants(gpu_ctx, fresh_cls):
    """Same frames at strides 64 / 128 / 256 / 2048 (different kernel variants)."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    n = 5000
    fr = gen.c2_frames(n).reshape(n, 64)
    rules = fresh_cls.pktio_rules(p)
    ref = None
    for stride in (64, 128, 256, 2048):
        buf = np.zeros((n, stride), np.uint8)
        buf[:, :64] = fr
        # stride > 64 makes the frame length = stride: zero padding is summed
        g, o = both(gpu_ctx, rules, buf.reshape(-1), n, stride=stride, opt=ALL_CHKSUM)
        assert_same(g, o, f"stride {stride}")
        if ref is None:
            ref = g["out"] & 0xFFFF
        assert np.array_equal(g["out"] & 0xFFFF, ref)


def test_host_path_matches_device(gpu_ctx, fresh_cls):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    n = 300000
    fr = gen.c2_frames(n)
    rules = fresh_cls.pktio_rules(p)
    tbl = gpu_ctx.table(rules)
    d = gpu_ctx.classify(tbl, fr, n, stride=64, opt=ALL_CHKSUM)
    h = gpu_ctx.classify_host(tbl, fr, n, stride=64, opt=ALL_CHKSUM, chunk=65536,
                              want_mark=True, want_meta=True)
    assert_same(h, d, "host vs device")
    frames = rulesets.mutate_corpus(9000, seed=11)
    buf, desc = pack(frames)
    d = gpu_ctx.classify(tbl, buf, len(frames), desc=desc, opt=ALL_CHKSUM)
    h = gpu_ctx.classify_host(tbl, buf, len(frames), desc=desc, opt=ALL_CHKSUM, chunk=1000,
                              want_mark=True, want_meta=True)
    assert_same(h, d, "host vs device (desc)")


def test_cycle_is_bounded(gpu_ctx, fresh_cls):
    """A matching CoS cycle makes the reference loop forever
    (odp_classification.c:1603-1631); here it ends as ODPG_COS_LOOP."""
    p = fresh_cls.loop_pktio()
    a = fresh_cls.cos_create("a", queue=fresh_cls.queue(1))
    b = fresh_cls.cos_create("b", queue=fresh_cls.queue(2))
    fresh_cls.default_cos_set(p, a)
    any_udp = fresh_cls.Term(fresh_cls.PMR_IPPROTO, b"\x11", b"\xff")
    assert fresh_cls.pmr_create([any_udp], a, b)
    assert fresh_cls.pmr_create([any_udp], b, a)
    assert fresh_cls.pktio_start(p) == 0
    fr = gen.c2_frames(1000)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, 1000, stride=64)
    assert_same(g, o, "cycle")
    assert np.all((g["out"] & 0xFFFF) == L.ODPG_COS_LOOP)


def test_destroyed_and_invalid_cos(gpu_ctx, fresh_cls):
    """Rules to a destroyed CoS are skipped (:1610-1611); a destroyed default
    CoS is still returned (:1687-1694); no default -> discard (-1)."""
    p = fresh_cls.loop_pktio()
    d = fresh_cls.cos_create("d", queue=fresh_cls.queue(1), stats_enable=True)
    x = fresh_cls.cos_create("x", queue=fresh_cls.queue(2))
    y = fresh_cls.cos_create("y", queue=fresh_cls.queue(3))
    fresh_cls.default_cos_set(p, d)
    any_udp = fresh_cls.Term(fresh_cls.PMR_IPPROTO, b"\x11", b"\xff")
    assert fresh_cls.pmr_create([any_udp], d, x, mark=5)
    assert fresh_cls.pmr_create([any_udp], d, y, mark=6)
    assert fresh_cls.pktio_start(p) == 0
    fr = gen.c2_frames(512)
    fresh_cls.cos_destroy(x)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, 512, stride=64)
    assert_same(g, o, "dst destroyed")
    assert np.all((g["out"] & 0xFFFF) == fresh_cls.to_index(y)) and np.all(g["mark"] == 6)
    fresh_cls.cos_destroy(d)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, 512, stride=64)
    assert_same(g, o, "default destroyed")
    assert np.all((g["out"] & 0xFFFF) == fresh_cls.to_index(d))
    fresh_cls.default_cos_set(p, None)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, 512, stride=64)
    assert_same(g, o, "no default")
    assert np.all((g["out"] & 0xFFFF) == L.ODPG_COS_NONE) and g["stats"][3] == 512


def test_hash_queues(gpu_ctx, fresh_cls):
    """num_queue > 1: Toeplitz RSS -> queue index (odp_classification.c:372-382,
    :1751-1817) for IPv4/IPv6 x UDP/TCP hash protocol mixes."""
    for hp in (fresh_cls.HASH_IPV4 | fresh_cls.HASH_IPV4_UDP,
               fresh_cls.HASH_IPV4_TCP | fresh_cls.HASH_IPV6_TCP,
               fresh_cls.HASH_IPV6 | fresh_cls.HASH_IPV4 | fresh_cls.HASH_IPV6_UDP):
        fresh_cls.reset()
        p = fresh_cls.loop_pktio()
        d = fresh_cls.cos_create("d", num_queue=7, hash_proto=hp)
        assert d
        fresh_cls.default_cos_set(p, d)
        assert fresh_cls.pktio_start(p) == 0
        frames = rulesets.mutate_corpus(4000, seed=hp)
        buf, desc = pack(frames)
        g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, len(frames), desc=desc)
        assert_same(g, o, f"hash {hp}")
        q = L.out_hashq(g["out"])
        assert q.max() < 7 and len(np.unique(q)) > 1


def test_hash_queues_every_proto_mix(gpu_ctx, fresh_cls):
    """Every combination of the six odp_cls_hash_proto_t bits (v4 / v6, with
    and without UDP / TCP ports) on the mutation corpus: the queue the kernel
    picks equals the oracle's literal packet_rss_hash + thash_softrss
    (odp_classification.c:1751-1817, thash.h:81-99)."""
    frames = rulesets.mutate_corpus(1500, seed=0x7E)
    buf, desc = pack(frames)
    bits = (fresh_cls.HASH_IPV4_UDP, fresh_cls.HASH_IPV4_TCP, fresh_cls.HASH_IPV4,
            fresh_cls.HASH_IPV6_UDP, fresh_cls.HASH_IPV6_TCP, fresh_cls.HASH_IPV6)
    for m in range(1, 64):
        hp = 0
        for k, b in enumerate(bits):
            if m >> k & 1:
                hp |= b
        fresh_cls.reset()
        p = fresh_cls.loop_pktio()
        d = fresh_cls.cos_create("d", num_queue=32, hash_proto=hp)
        assert d
        fresh_cls.default_cos_set(p, d)
        assert fresh_cls.pktio_start(p) == 0
        rules = fresh_cls.pktio_rules(p)
        g = gpu_ctx.classify(gpu_ctx.table(rules), buf, len(frames), desc=desc)
        o = oracle.classify(rules, buf, len(frames), desc=desc)
        assert np.array_equal(g["out"], o["out"]), f"hash proto mix {m:#x}"


def test_pktio_recv_batch_counters(gpu_ctx, fresh_cls):
    """odpg_pktio_recv_batch updates odp_cls_cos_stats / odp_pktio_stats like
    loopback_recv (loop.c:304-374) and match_pmr_cos (:1621-1622)."""
    import ctypes as C
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    r = gen.build_c2_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    n = 100000
    fr = gen.c2_frames(n)
    out = np.zeros(n, np.uint32)
    rc = L.lib.odpg_pktio_recv_batch(p, gpu_ctx.h, fr.ctypes.data, None, 64, n, 0,
                                     out.ctypes.data, None)
    assert rc == 0
    o = oracle.classify(fresh_cls.pktio_rules(p), fr, n, stride=64, opt=ALL_CHKSUM)
    assert np.array_equal(out, o["out"])
    st = fresh_cls.pktio_stats(p)
    assert st.in_packets == n and st.in_octets == 64 * n and st.in_errors == 0
    for c in [r["default"]] + r["l1"] + r["leaves"]:
        rc, cs = fresh_cls.cos_stats(c)
        assert rc == 0 and cs.packets == o["stats"][4 + fresh_cls.to_index(c)]
    # queue counters of the leaf CoS equal the packets delivered there
    leaf = r["leaves"][3]
    rc, qs = fresh_cls.queue_stats(leaf, fresh_cls.cos_queue(leaf))
    assert rc == 0 and qs.packets == int(((out & 0xFFFF) == fresh_cls.to_index(leaf)).sum())
    # device-pointer variant adds the same counts again
    fb = gpu_ctx.buffer(fr.nbytes)
    fb.upload(fr)
    ob = gpu_ctx.buffer(4 * n)
    rc = L.lib.odpg_pktio_recv_batch(p, gpu_ctx.h, fb.ptr, None, 64, n, 1, ob.ptr, None)
    assert rc == 0
    gpu_ctx.sync()                   # the device path is asynchronous
    assert np.array_equal(ob.download(np.uint32, n), out)
    st = fresh_cls.pktio_stats(p)
    assert st.in_packets == 2 * n and st.in_octets == 128 * n
    for c in [r["default"]] + r["l1"] + r["leaves"]:
        rc, cs = fresh_cls.cos_stats(c)
        assert rc == 0 and cs.packets == 2 * o["stats"][4 + fresh_cls.to_index(c)]
    # queue counters after the device call: every queue of every CoS
    want = expected_counters(o, len(o["stats"]) - 4)["queue"]
    for c in [r["default"]] + r["l1"] + r["leaves"]:
        rc, qs = fresh_cls.queue_stats(c, fresh_cls.cos_queue(c))
        assert rc == 0 and qs.packets == 2 * want[fresh_cls.to_index(c), 0], c
    # reads fold once: a second read sees the same totals
    assert fresh_cls.pktio_stats(p).in_packets == 2 * n
    fresh_cls.pktio_stats_reset(p)
    assert fresh_cls.pktio_stats(p).in_packets == 0
    rc = L.lib.odpg_pktio_recv_batch(p, gpu_ctx.h, fb.ptr, None, 64, n, 1, ob.ptr, None)
    assert rc == 0 and fresh_cls.pktio_stats(p).in_packets == n
    del C


def test_raised_limits_1024_pmr(gpu_ctx, fresh_cls):
    assert fresh_cls.set_limits(2048, 2048, 32) == 0
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c4_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    n = 1 << 20                      # the C4 bench batch per GPU
    fr = gen.c2_frames(n)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, n, stride=64, opt=ALL_CHKSUM)
    assert_same(g, o, "C4 1024 PMR")


@pytest.mark.parametrize("opt", [0, L.PKTIN_IPV4_CHKSUM, ALL_CHKSUM])
def test_stride64_fast_path_edges(gpu_ctx, fresh_cls, opt):
    """64-byte stride: waves that take the register fast path and waves that
    fall back to the generic parser, with every edge the fast path decides."""
    p = fresh_cls.loop_pktio(pktin=opt)
    rulesets.all_terms_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    n = 64 * 300
    fr = rulesets.plain64_corpus(n)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, n, stride=64, opt=opt)
    assert_same(g, o, f"fast path opt={opt}")
    # C2 rules (TBL_SIMPLE) over the same frames
    fresh_cls.reset()
    p = fresh_cls.loop_pktio(pktin=opt)
    gen.build_c2_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, n, stride=64, opt=opt)
    assert_same(g, o, f"fast path C2 opt={opt}")


@pytest.mark.parametrize("layout", ["stride64", "desc"])
def test_simple_table_hash_groups(gpu_ctx, fresh_cls, layout):
    """TBL_SIMPLE tables: hash groups with duplicate values, linear runs,
    LEN / never / match-all rules; fast-path and generic waves."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    rulesets.simple_mixed_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    if layout == "stride64":
        n = 64 * 200
        fr = rulesets.plain64_corpus(n, seed=9)
        g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, n, stride=64, opt=ALL_CHKSUM)
    else:
        frames = rulesets.mutate_corpus(12000, seed=21)
        buf, desc = pack(frames)
        g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, len(frames), desc=desc,
                    opt=ALL_CHKSUM)
    assert_same(g, o, f"simple/hash {layout}")
    assert len(np.unique(g["out"] & 0xFFFF)) > 3


@pytest.mark.parametrize("n", [1, 257, 1 << 15, 1 << 20])
def test_c3_imix_dag(gpu_ctx, fresh_cls, n):
    """C3: IMIX 64/570/1518 B, IPv4/IPv6, UDP/TCP, checksum errors / zero /
    fragments, 256-PMR DAG with mixed term kinds, error CoS, descriptors."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c3_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    buf, desc = gen.c3_frames(n)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, n, desc=desc, opt=ALL_CHKSUM)
    assert_same(g, o, "c3")


@pytest.mark.parametrize("drop", [L.PKTIN_DROP_UDP_ERR | L.PKTIN_DROP_TCP_ERR,
                                  L.PKTIN_DROP_IPV4_ERR | L.PKTIN_DROP_UDP_ERR])
def test_c3_drop_options(gpu_ctx, fresh_cls, drop):
    """C3 traffic with pktin drop options: frames whose L4 checksum (summed
    over the long tails) fails are dropped before classification, also when
    the wave sums its tails after the CoS walk."""
    opt = ALL_CHKSUM | drop
    # the loop pktio's capability has no drop options (pktio/loop.c:650-670):
    # they reach the kernel through the batch's pktin word only
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c3_rules(fresh_cls, p, stats=False)
    assert fresh_cls.pktio_start(p) == 0
    n = 40000
    buf, desc = gen.c3_frames(n, seed=123)
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, n, desc=desc, opt=opt)
    assert_same(g, o, f"c3 drop {drop:#x}")
    assert np.any((o["out"] & 0xFFFF) == L.ODPG_COS_PDROP)


def test_c3_host_path(gpu_ctx, fresh_cls):
    """C3 through the pinned-host path (chunked H2D of variable-length frames)."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c3_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    n = 20000
    buf, desc = gen.c3_frames(n, seed=99)
    rules = fresh_cls.pktio_rules(p)
    tbl = gpu_ctx.table(rules)
    h = gpu_ctx.classify_host(tbl, buf, n, desc=desc, opt=ALL_CHKSUM, chunk=3000,
                              want_mark=True)
    o = oracle.classify(rules, buf, n, desc=desc, opt=ALL_CHKSUM)
    np.testing.assert_array_equal(h["out"], o["out"])
    np.testing.assert_array_equal(h["mark"], o["mark"])
    np.testing.assert_array_equal(h["stats"], o["stats"])


@pytest.mark.parametrize("opt", OPTS)
@pytest.mark.parametrize("variant", ["mixed", "drop_err", "no_default"])
def test_lean64_kernel(gpu_ctx, fresh_cls, opt, variant):
    """The lean 64-byte kernel (auto mode, verdict words only): fast and
    generic waves of the plain64 corpus, marks, DROP-action CoS, error CoS,
    no default CoS; verdict words bit-exact vs the oracle, and the launch
    really took the lean kernel."""
    p = fresh_cls.loop_pktio(pktin=opt)
    if variant == "mixed":
        rulesets.simple_mixed_rules(fresh_cls, p, stats=False)
    elif variant == "drop_err":
        c, T = fresh_cls, fresh_cls.Term
        d = c.cos_create("d", queue=c.queue(0))
        q1 = c.cos_create("q1", queue=c.queue(1))
        q2 = c.cos_create("q2", queue=c.queue(2))
        drop = c.cos_create("drop", action=c.COS_ACTION_DROP)
        err = c.cos_create("err", queue=c.queue(70))
        assert c.default_cos_set(p, d) == 0 and c.error_cos_set(p, err) == 0
        assert c.pmr_create([T(c.PMR_SIP_ADDR, gen.be_bytes(gen.ip4("192.168.0.0"), 4),
                               gen.be_bytes(0xFFFF8000, 4))], d, q1, mark=3)
        assert c.pmr_create([T(c.PMR_UDP_SPORT, gen.be_bytes(5, 2), b"\x00\xff")],
                            q1, drop, mark=9)
        assert c.pmr_create([T(c.PMR_TCP_DPORT, gen.be_bytes(7, 2), b"\xff\xff")], q1, q2)
    else:
        q = fresh_cls.cos_create("q", queue=fresh_cls.queue(3))
        assert q
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    n = 64 * 257 + 5
    fr = rulesets.plain64_corpus(n, seed=31)
    tbl = gpu_ctx.table(rules)
    g = gpu_ctx.classify(tbl, fr, n, stride=64, opt=opt, want_mark=False, want_meta=False,
                         want_stats=False)
    assert L.lib.odpg_last_kernel() == 1
    o = oracle.classify(rules, fr, n, stride=64, opt=opt)
    assert_same({"out": g["out"]}, {"out": o["out"]}, f"lean64 {variant} opt={opt}")
    # with the pktio counters (in_packets / octets / errors / discards)
    g = gpu_ctx.classify(tbl, fr, n, stride=64, opt=opt, want_mark=False, want_meta=False)
    assert L.lib.odpg_last_kernel() == 1
    assert_same({"out": g["out"], "stats": g["stats"]}, {"out": o["out"], "stats": o["stats"]},
                f"lean64+stats {variant} opt={opt}")


def _hashwalk_rules(c, p):
    """A TBL_HASHWALK table (exact-match values repeated across CoS) with
    marks, a DROP-action leaf, an error CoS and a leaf chain two levels deep:
    the lean kernel's walk-group form."""
    T = c.Term
    d = c.cos_create("d", queue=c.queue(0))
    err = c.cos_create("err", queue=c.queue(1))
    drop = c.cos_create("drop", action=c.COS_ACTION_DROP)
    assert c.default_cos_set(p, d) == 0 and c.error_cos_set(p, err) == 0
    l1 = [c.cos_create(f"l1_{a}", queue=c.queue(2 + a)) for a in range(4)]
    for a in range(4):
        assert c.pmr_create([T(c.PMR_SIP_ADDR, gen.be_bytes(gen.ip4("10.0.0.0") | (a << 14), 4),
                               gen.be_bytes(0xFFFFC000, 4))], d, l1[a], mark=a + 1)
    k = 0
    for a in range(4):
        for j in range(6):
            leaf = drop if (a, j) == (2, 3) else c.cos_create(f"leaf_{k}", queue=c.queue(10 + k))
            k += 1
            assert c.pmr_create([T(c.PMR_UDP_DPORT, gen.be_bytes(j + 1, 2), b"\xff\xff")],
                                l1[a], leaf, mark=100 + k if j % 2 else 0)
            if (a, j) == (1, 0):
                # one more level below this leaf
                deep = c.cos_create("deep", queue=c.queue(60))
                assert c.pmr_create([T(c.PMR_UDP_SPORT, gen.be_bytes(7, 2), b"\x00\x0f")],
                                    leaf, deep, mark=77)


@pytest.mark.parametrize("opt", [0, L.PKTIN_IPV4_CHKSUM, ALL_CHKSUM])
@pytest.mark.parametrize("variant", ["c4", "marks_drop"])
def test_lean64_hashwalk(gpu_ctx, fresh_cls, opt, variant):
    """The lean 64-byte kernel's walk-group form (TBL_LEAN64HW, auto mode,
    verdict words and pktio counters): the 1024-PMR C4 table and a small
    hash-walk table with marks / DROP / error CoS / a third level, on the
    plain64 corpus (fast and generic waves) and C2 traffic; bit-exact vs the
    oracle, and the launch really took the lean kernel."""
    if variant == "c4":
        assert fresh_cls.set_limits(2048, 2048, 32) == 0
    p = fresh_cls.loop_pktio(pktin=opt)
    if variant == "c4":
        gen.build_c4_rules(fresh_cls, p)
    else:
        _hashwalk_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    tbl = gpu_ctx.table(rules)
    n = 64 * 257 + 5
    for fr in (rulesets.plain64_corpus(n, seed=37), gen.c2_frames(n, seed=41)):
        o = oracle.classify(rules, fr, n, stride=64, opt=opt)
        g = gpu_ctx.classify(tbl, fr, n, stride=64, opt=opt, want_mark=False, want_meta=False,
                             want_stats=False)
        assert L.lib.odpg_last_kernel() == 1
        assert_same({"out": g["out"]}, {"out": o["out"]}, f"lean64 hw {variant} opt={opt}")
        g = gpu_ctx.classify(tbl, fr, n, stride=64, opt=opt, want_mark=False, want_meta=False)
        assert L.lib.odpg_last_kernel() == 1
        assert_same({"out": g["out"], "stats": g["stats"]},
                    {"out": o["out"], "stats": o["stats"]}, f"lean64 hw+stats {variant} opt={opt}")


@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_hybrid_walk_random_rules(gpu_ctx, fresh_cls, seed):
    """Random DAGs mixing single-word, IPv4/IPv6-alternative and complex PMRs
    (the hybrid hash walk's three rule forms) on the fuzz corpus: every
    kernel strategy bit-exact with the oracle."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    r = rulesets.random_mixed_rules(fresh_cls, p, seed, complex_share=0.15 + 0.1 * (seed % 4))
    assert len(r["pmrs"]) > 20
    assert fresh_cls.pktio_start(p) == 0
    frames = rulesets.mutate_corpus(20000, seed=seed)
    buf, desc = pack(frames)
    for opt in (0, ALL_CHKSUM):
        g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), buf, len(frames), desc=desc, opt=opt)
        assert_same(g, o, f"random rules seed={seed} opt={opt}")
    assert len(np.unique(g["out"] & 0xFFFF)) > 3


def test_table_larger_than_lds(gpu_ctx, fresh_cls):
    """A hash-walk table near the raised limits (16 SIP CoS x 1000 UDP_DPORT
    rules, 16016 PMRs): its CoS-keyed groups exceed a workgroup's LDS, so the
    lean kernel and the LDS-resident strategies fall back to the walk instead
    of failing the launch; every strategy stays bit-exact."""
    c, T = fresh_cls, fresh_cls.Term
    assert c.set_limits(2048, 16384, 1024) == 0
    p = c.loop_pktio(pktin=ALL_CHKSUM)
    d = c.cos_create("d", queue=c.queue(0))
    assert c.default_cos_set(p, d) == 0
    leaves = [c.cos_create(f"leaf{j}", queue=c.queue(100 + j)) for j in range(1000)]
    for a in range(16):
        l1 = c.cos_create(f"l1_{a}", queue=c.queue(10 + a))
        assert c.pmr_create([T(c.PMR_SIP_ADDR, gen.be_bytes(gen.ip4("10.0.0.0") | (a << 12), 4),
                               gen.be_bytes(0xFFFFF000, 4))], d, l1)
        for j in range(1000):
            assert c.pmr_create([T(c.PMR_UDP_DPORT, gen.be_bytes(j, 2), b"\xff\xff")], l1, leaves[j])
    assert c.pktio_start(p) == 0
    n = 64 * 300
    fr = gen.c2_frames(n).reshape(n, 64).copy()
    rng = np.random.default_rng(3)
    src = (gen.ip4("10.0.0.0") + rng.integers(0, 1 << 17, n)).astype(np.uint64)
    fr[:, 26:30] = np.stack([(src >> s) & 0xFF for s in (24, 16, 8, 0)], 1).astype(np.uint8)
    dport = rng.integers(0, 1100, n)
    fr[:, 36] = dport >> 8
    fr[:, 37] = dport & 0xFF
    fr = fr.reshape(-1)
    # checksums are not verified (pktin 0): the edited frames still parse plainly
    g, o = both(gpu_ctx, fresh_cls.pktio_rules(p), fr, n, stride=64, opt=0)
    assert_same(g, o, "16k-PMR hash walk")
    assert len(np.unique(g["out"] & 0xFFFF)) > 500
