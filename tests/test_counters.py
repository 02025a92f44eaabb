"""Sharded device counters (include/odpg.h "sharded counters").

The pktio, CoS and per-queue counters the reference keeps as atomics
(pktio/loop.c:304-374, odp_classification.c:1621-1622,1697-1698,
odp_classification_internal.h:64-78) accumulate per workgroup on the device
and are folded when read. Parity: the fold equals the oracle's counters and
the per-(CoS, queue) deliveries implied by its verdicts. Every parity case in
test_gpu_parity.py also runs through counters (both()); this file covers the
object's own contract: accumulation over launches, fold-and-clear, the lean
and general kernels, hash queues, the host-buffer path and argument errors."""
import ctypes as C

import numpy as np
import pytest

import oracle
import rulesets
from helpers import ALL_CHKSUM, assert_counters, expected_counters, pack
from odp_amd import _lib as L
from odp_amd import gen


def test_counter_words_layout():
    """ODPG_COUNTER_WORDS(num_cos) = 4 + num_cos + num_cos * COS_QUEUE_MAX."""
    assert L.COS_QUEUE_MAX == 32 and L.ABI_VERSION == 2
    assert C.sizeof(L.odpg_result_t) == 5 * C.sizeof(C.c_void_p)


@pytest.mark.gpu
def test_accumulate_and_clear(gpu_ctx, fresh_cls):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    tbl = gpu_ctx.table(rules)
    cnt = gpu_ctx.counters(tbl)
    want = None
    for k, n in enumerate((1, 63, 4097, 1 << 20)):
        fr = gen.c2_frames(n, seed=100 + k)
        o = oracle.classify(rules, fr, n, stride=64, opt=ALL_CHKSUM)
        e = expected_counters(o, tbl.num_cos)
        want = e if want is None else {x: want[x] + e[x] for x in want}
        g = gpu_ctx.classify(tbl, fr, n, stride=64, opt=ALL_CHKSUM, want_mark=False,
                             want_meta=False, counters=cnt)
        assert L.lib.odpg_last_kernel() == 1          # the lean 64-byte kernel
        assert np.array_equal(g["out"], o["out"])
    f = cnt.fold()
    assert_counters(f, want, "four launches")
    assert f["pktio"][0] == 1 + 63 + 4097 + (1 << 20)
    z = cnt.fold()                                    # the fold cleared the rows
    assert not any(np.any(z[k]) for k in z)


@pytest.mark.gpu
def test_hash_queue_columns(gpu_ctx, fresh_cls):
    """num_queue > 1 CoS: one column per hash queue (general kernel)."""
    p = fresh_cls.loop_pktio()
    d = fresh_cls.cos_create("d", num_queue=7, stats_enable=True,
                             hash_proto=fresh_cls.HASH_IPV4 | fresh_cls.HASH_IPV4_UDP)
    x = fresh_cls.cos_create("x", queue=fresh_cls.queue(3), num_queue=1)
    y = fresh_cls.cos_create("y", num_queue=3, hash_proto=fresh_cls.HASH_IPV4,
                             stats_enable=True)
    fresh_cls.default_cos_set(p, d)
    any_tcp = fresh_cls.Term(fresh_cls.PMR_IPPROTO, b"\x06", b"\xff")
    assert fresh_cls.pmr_create([any_tcp], d, x)
    assert fresh_cls.pmr_create([fresh_cls.Term(fresh_cls.PMR_UDP_DPORT, b"\x00\x07",
                                                b"\x00\x07")], d, y)
    assert fresh_cls.pktio_start(p) == 0
    frames = rulesets.mutate_corpus(6000, seed=5)
    buf, desc = pack(frames)
    rules = fresh_cls.pktio_rules(p)
    tbl = gpu_ctx.table(rules)
    cnt = gpu_ctx.counters(tbl)
    o = oracle.classify(rules, buf, len(frames), desc=desc)
    g = gpu_ctx.classify(tbl, buf, len(frames), desc=desc, counters=cnt)
    assert np.array_equal(g["out"], o["out"])
    f = cnt.fold()
    e = expected_counters(o, tbl.num_cos)
    assert_counters(f, e, "hash queues")
    di = fresh_cls.to_index(d)
    assert np.count_nonzero(f["queue"][di]) > 1 and not np.any(f["queue"][di, 7:])


@pytest.mark.gpu
def test_host_path_counters(gpu_ctx, fresh_cls):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    tbl = gpu_ctx.table(rules)
    cnt = gpu_ctx.counters(tbl)
    n = 200000
    fr = gen.c2_frames(n)
    o = oracle.classify(rules, fr, n, stride=64, opt=ALL_CHKSUM)
    out = np.zeros(n, np.uint32)
    b = L.odpg_batch_t(fr.ctypes.data, None, 64, n, ALL_CHKSUM, L.LAYER_ALL, 1)
    r = L.odpg_result_t(out.ctypes.data, None, None, None, cnt.h)
    assert L.lib.odpg_classify_host(gpu_ctx.h, tbl.h, C.byref(b), C.byref(r), 30000) == 0
    assert np.array_equal(out, o["out"])
    assert_counters(cnt.fold(), expected_counters(o, tbl.num_cos), "host path")


@pytest.mark.gpu
def test_counters_errors(gpu_ctx, fresh_cls):
    p = fresh_cls.loop_pktio()
    gen.build_c1_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    from odp_amd import gpu
    other = gpu.Context(0)
    t1 = gpu_ctx.table(fresh_cls.pktio_rules(p))
    t3 = other.table(fresh_cls.pktio_rules(p))       # same layout, other context
    cnt = gpu_ctx.counters(t1)
    fr = gen.c1_frames(256)
    fb = gpu_ctx.buffer(fr.nbytes)
    fb.upload(fr)
    ob = gpu_ctx.buffer(4 * 256)
    sb = gpu_ctx.buffer(8 * (4 + t1.num_cos))
    b = L.odpg_batch_t(fb.ptr, None, 64, 256, 0, L.LAYER_ALL, 1)
    # counters and a stats block together
    r = L.odpg_result_t(ob.ptr, None, None, sb.ptr, cnt.h)
    assert L.lib.odpg_classify(gpu_ctx.h, t1.h, C.byref(b), C.byref(r)) == -22
    # a table of another layout (an extra hash-queue CoS)
    fresh_cls.cos_create("h", num_queue=4, hash_proto=fresh_cls.HASH_IPV4)
    t2 = gpu_ctx.table(fresh_cls.pktio_rules(p))
    r = L.odpg_result_t(ob.ptr, None, None, None, cnt.h)
    assert L.lib.odpg_classify(gpu_ctx.h, t2.h, C.byref(b), C.byref(r)) == -22
    # a counters object of another context
    assert L.lib.odpg_classify(other.h, t3.h, C.byref(b), C.byref(r)) == -22
    del t3
    other.close()
    assert L.lib.odpg_classify(gpu_ctx.h, t1.h, C.byref(b), C.byref(r)) == 0
    gpu_ctx.sync()
    assert cnt.fold()["pktio"][0] == 256


@pytest.mark.gpu
def test_recv_batch_rule_changes(gpu_ctx, fresh_cls):
    """odpg_pktio_recv_batch across rule changes: the binding is recompiled
    in place (odpg_table_update) and its counters carry on; counts made
    before a CoS was destroyed never reach the CoS later created in its slot
    (the reference's cos_create zeroes its counters)."""
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    r = gen.build_c2_rules(fresh_cls, p, stats=True)
    assert fresh_cls.pktio_start(p) == 0
    n = 50000
    fr = gen.c2_frames(n, seed=9)
    fb = gpu_ctx.buffer(fr.nbytes)
    fb.upload(fr)
    ob = gpu_ctx.buffer(4 * n)
    leaf = r["leaves"][5]

    def recv():
        o = oracle.classify(fresh_cls.pktio_rules(p), fr, n, stride=64, opt=ALL_CHKSUM)
        rc = L.lib.odpg_pktio_recv_batch(p, gpu_ctx.h, fb.ptr, None, 64, n, 1, ob.ptr, None)
        assert rc == 0
        gpu_ctx.sync()
        assert np.array_equal(ob.download(np.uint32, n), o["out"])
        return o

    o1 = recv()
    # a PMR change: the CoS layout is kept
    extra = fresh_cls.pmr_create([fresh_cls.Term(fresh_cls.PMR_UDP_SPORT, b"\x00\x07",
                                                 b"\x00\xff")], r["l1"][0], leaf)
    assert extra
    o2 = recv()
    want_leaf = int(o1["stats"][4 + fresh_cls.to_index(leaf)] + o2["stats"][4 + fresh_cls.to_index(leaf)])
    rc, cs = fresh_cls.cos_stats(leaf)
    assert rc == 0 and cs.packets == want_leaf
    rc, qs = fresh_cls.queue_stats(leaf, fresh_cls.cos_queue(leaf))
    q_want = sum(int(((o["out"] & 0xFFFF) == fresh_cls.to_index(leaf)).sum()) for o in (o1, o2))
    assert rc == 0 and qs.packets == q_want
    st = fresh_cls.pktio_stats(p)
    assert st.in_packets == 2 * n
    # destroy a leaf without reading its counters, create another CoS in its
    # slot and route the same rules to it
    slot = fresh_cls.to_index(leaf)
    assert fresh_cls.pmr_destroy(extra) == 0
    o3 = recv()                                       # counts for the old leaf
    assert fresh_cls.cos_destroy(leaf) == 0
    new = fresh_cls.cos_create("new_leaf", queue=fresh_cls.queue(77), stats_enable=True)
    assert fresh_cls.to_index(new) == slot
    o4 = recv()
    rc, cs = fresh_cls.cos_stats(new)
    assert rc == 0 and cs.packets == int(o4["stats"][4 + slot])
    rc, qs = fresh_cls.queue_stats(new, fresh_cls.cos_queue(new))
    assert rc == 0 and qs.packets == int(((o4["out"] & 0xFFFF) == slot).sum())
    assert fresh_cls.pktio_stats(p).in_packets == 4 * n
    del o3
