"""Device groups (include/odpg_group.h): one batch classified by several
device contexts of one process, sharded by packet range, the rule table
compiled once and imported per member, the members' counters summed when
folded (SURVEY.md §8(e) in the C-ABI itself, not only in the
torch.distributed harness). On the one-GPU box the members share device 0,
each with its own context and stream; the verdicts and counters must equal a
single context's over the whole batch bit for bit, and the oracle's."""
import numpy as np
import pytest

import oracle
from helpers import ALL_CHKSUM, assert_counters, expected_counters
from odp_amd import _lib as L
from odp_amd import gen, gpu


@pytest.mark.parametrize("num", [0, 1, 63, 64, 65, 1000, 4096, 64 * 1031 + 17, (1 << 20) + 5])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 8])
def test_group_range_partitions_the_batch(num, n):
    """Host arithmetic (no device): the members' ranges are contiguous,
    disjoint, cover [0, num) in member order, start on 64-packet tiles, are
    of one size except the last non-empty one, and are empty only past the
    batch's end."""
    rs = [gpu.group_range(num, n, i) for i in range(n)]
    pos = 0
    for i, (lo, hi) in enumerate(rs):
        assert lo == pos and lo <= hi, (num, n, rs)
        assert lo % 64 == 0 or lo == num, (num, n, rs)
        pos = hi
    assert pos == num
    sizes = [hi - lo for lo, hi in rs if hi - lo]
    assert len(set(sizes[:-1])) <= 1 and (not sizes or sizes[-1] <= max(sizes)), rs
    # a member is empty only past the batch's end
    assert all(lo == num for lo, hi in rs if hi == lo)
    assert gpu.group_range(num, n, n) == (0, 0)


def test_group_create_fails_cleanly_without_a_device():
    import ctypes as C
    if L.lib.odpg_device_count() > 0:
        pytest.skip("a device is visible")
    h = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    assert L.lib.odpg_group_create(devs, 2, C.byref(h)) != 0
    assert L.lib.odpg_group_create(devs, 0, C.byref(h)) != 0


def _rules(cls, cfg):
    """C2 with per-CoS statistics (the general kernel's counted launch), C2x
    and C3 without (the lean descriptor kernel's)"""
    p = cls.loop_pktio(pktin=ALL_CHKSUM)
    {"c2": gen.build_c2_rules, "c3": gen.build_c3_rules,
     "c2x": gen.build_c2x_rules}[cfg](cls, p, stats=cfg == "c2")
    assert cls.pktio_start(p) == 0
    return cls.pktio_rules(p)


@pytest.mark.gpu
@pytest.mark.parametrize("members", [2, 3])
@pytest.mark.parametrize("cfg", ["c2", "c2x", "c3"])
def test_group_host_batch_matches_one_context(gpu_ctx, fresh_cls, cfg, members):
    rules = _rules(fresh_cls, cfg)
    n = 64 * 777 + 29
    if cfg == "c3":
        frames, desc = gen.c3_frames(n, seed=3)
        stride = 0
    else:
        frames = (gen.c2_frames if cfg == "c2" else gen.c2x_frames)(n, seed=3)
        desc, stride = None, 64
    o = oracle.classify(rules, frames, n, stride=stride, desc=desc, opt=ALL_CHKSUM)
    # one context, whole batch, counted
    tbl = gpu_ctx.table(rules)
    cnt = gpu_ctx.counters(tbl)
    one = gpu_ctx.classify(tbl, frames, n, stride=stride, desc=desc, opt=ALL_CHKSUM,
                           want_mark=False, want_meta=False, counters=cnt)["out"]
    one_cnt = cnt.fold()
    cnt.close()
    g = gpu.Group([0] * members)
    try:
        g.load(rules)
        for _ in range(2):
            out = g.classify_host(frames, n, stride=stride, desc=desc, opt=ALL_CHKSUM,
                                  counted=True, chunk=1 << 14)
            assert np.array_equal(out, one), cfg
            assert np.array_equal(out, o["out"]), cfg
        got = g.fold()
        for k in ("pktio", "cos", "queue"):
            assert np.array_equal(got[k], 2 * one_cnt[k]), (cfg, k)
        assert_counters(got, {k: 2 * v for k, v in expected_counters(o, tbl.num_cos).items()},
                        f"group {cfg}")
        # folded: the next fold starts from zero
        assert not any(int(x) for x in g.fold()["pktio"])
    finally:
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 100, 64 * 513 + 7])
def test_group_device_shards(gpu_ctx, fresh_cls, n):
    """Device-resident shards: member i's range in its own context's HBM,
    launched asynchronously on every member, then synced."""
    rules = _rules(fresh_cls, "c2x")
    frames = gen.c2x_frames(n, seed=n)
    o = oracle.classify(rules, frames, n, stride=64, opt=ALL_CHKSUM)
    g = gpu.Group([0, 0, 0, 0])
    try:
        g.load(rules)
        out = g.classify_shards(frames, n, 64, opt=ALL_CHKSUM, counted=True)
        assert np.array_equal(out, o["out"])
        got = g.fold()
        assert int(got["pktio"][0]) + int(got["pktio"][2]) == n
        assert_counters(got, expected_counters(o, g.num_cos), "group shards")
    finally:
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [5, 64 * 300 + 5])
def test_group_device_shards_descriptors(gpu_ctx, fresh_cls, n):
    """Device-resident C3 shards (IMIX frames behind descriptors, the
    descriptor kernel, checksum tails): each member holds the frame buffer
    and its range's descriptors; three members, counted."""
    rules = _rules(fresh_cls, "c3")
    frames, desc = gen.c3_frames(n, seed=7)
    o = oracle.classify(rules, frames, n, stride=0, desc=desc, opt=ALL_CHKSUM)
    g = gpu.Group([0, 0, 0])
    try:
        g.load(rules)
        out = g.classify_shards(frames, n, 0, opt=ALL_CHKSUM, counted=True, desc=desc)
        assert np.array_equal(out, o["out"])
        assert_counters(g.fold(), expected_counters(o, g.num_cos), "group C3 shards")
    finally:
        g.close()


@pytest.mark.gpu
def test_group_reload_keeps_counts_of_the_same_layout(gpu_ctx, fresh_cls):
    rules = _rules(fresh_cls, "c2")
    n = 5000
    frames = gen.c2_frames(n, seed=1)
    g = gpu.Group([0, 0])
    try:
        g.load(rules)
        g.classify_host(frames, n, stride=64, opt=ALL_CHKSUM, counted=True)
        g.load(rules)                      # a new generation, same CoS count
        g.classify_host(frames, n, stride=64, opt=ALL_CHKSUM, counted=True)
        assert int(g.fold()["pktio"][0]) == 2 * n
    finally:
        g.close()
