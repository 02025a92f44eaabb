"""Compiled-table images (odpg_rules_compile / odpg_table_import): the bytes
a multi-GPU job compiles once on rank 0 and broadcasts."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import ALL_CHKSUM
from odp_amd import _lib as L
from odp_amd import gen, gpu


def _c2(cls):
    p = cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c2_rules(cls, p)
    assert cls.pktio_start(p) == 0
    return cls.pktio_rules(p)


def test_compile_size_query_and_determinism(fresh_cls):
    rules = _c2(fresh_cls)
    n = C.c_size_t(0)
    assert L.lib.odpg_rules_compile(C.byref(rules), None, C.byref(n)) == -28   # -ENOSPC
    assert n.value > 16
    small = C.c_size_t(n.value - 1)
    buf = (C.c_uint8 * n.value)()
    assert L.lib.odpg_rules_compile(C.byref(rules), buf, C.byref(small)) == -28
    assert small.value == n.value
    img = gpu.compile_rules(rules)
    assert len(img) == n.value and img == gpu.compile_rules(rules)
    assert img[:4] == b"ODPT" and int.from_bytes(img[4:8], "little") == L.ABI_VERSION


@pytest.mark.gpu
def test_import_equals_create(gpu_ctx, fresh_cls):
    rules = _c2(fresh_cls)
    img = gpu.compile_rules(rules)
    n = 1 << 16
    fr = gen.c2_frames(n)
    a = gpu_ctx.classify(gpu_ctx.table(rules), fr, n, stride=64, opt=ALL_CHKSUM)
    b = gpu_ctx.classify(gpu_ctx.table(image=img), fr, n, stride=64, opt=ALL_CHKSUM)
    o = oracle.classify(rules, fr, n, stride=64, opt=ALL_CHKSUM)
    assert np.array_equal(a["out"], b["out"]) and np.array_equal(b["out"], o["out"])
    assert np.array_equal(a["stats"], b["stats"])
    # a damaged or truncated image is refused
    t = C.c_void_p()
    for bad in (b"XXXX" + img[4:], img[:-1], img[:8]):
        buf = (C.c_uint8 * len(bad)).from_buffer_copy(bad)
        assert L.lib.odpg_table_import(gpu_ctx.h, buf, len(bad), C.byref(t)) == -22
