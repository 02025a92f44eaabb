"""Completion fences (odpg_fence_*, include/odpg.h): what the runtime's
receive pipeline (odp_rt.c) relies on. A fence recorded behind a launch
reports pending or done without blocking, odpg_fence_wait makes the
launch's results final, and several bursts in flight complete in launch
order with the same verdicts as one synchronous launch each (checked
against the oracle)."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import ALL_CHKSUM
from odp_amd import _lib as L
from odp_amd import gen

lib = L.lib


def test_fence_rejects_null():
    assert lib.odpg_fence_create(None, None) < 0
    assert lib.odpg_fence_query(None) < 0
    assert lib.odpg_fence_wait(None) < 0
    lib.odpg_fence_destroy(None)            # no-op


@pytest.mark.gpu
def test_fences_complete_bursts_in_order(gpu_ctx, fresh_cls):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    rules = fresh_cls.pktio_rules(p)
    tbl = gpu_ctx.table(rules)
    nb, n = 4, 4096
    frames = [gen.c2_frames(n, seed=31 + k) for k in range(nb)]
    bufs, outs, fences = [], [], []
    for k in range(nb):
        fb = gpu_ctx.buffer(frames[k].nbytes)
        fb.upload(frames[k])
        ob = gpu_ctx.buffer(4 * n)
        f = C.c_void_p()
        assert lib.odpg_fence_create(gpu_ctx.h, C.byref(f)) == 0
        bufs.append(fb)
        outs.append(ob)
        fences.append(f.value)
    try:
        # every burst launched and fenced before any is waited for
        for k in range(nb):
            gpu_ctx.classify_dev(tbl, bufs[k], n, stride=64, opt=ALL_CHKSUM, out_buf=outs[k])
            assert lib.odpg_fence_record(gpu_ctx.h, fences[k]) == 0
            assert lib.odpg_fence_query(fences[k]) in (0, 1)
        assert lib.odpg_fence_wait(fences[-1]) == 0
        # the stream completes in order: the last fence done means all are
        for k in range(nb):
            assert lib.odpg_fence_query(fences[k]) == 1
            got = outs[k].download(np.uint32, n)
            exp = oracle.classify(rules, frames[k], n, stride=64, opt=ALL_CHKSUM)["out"]
            assert np.array_equal(got, exp), f"burst {k}"
    finally:
        for f in fences:
            lib.odpg_fence_destroy(f)
