"""Child process of tests/test_destroy_order.py: makes counted launches on
one context, then destroys the counters, the table, a forwarder, a fence and
the context in the order given on the command line (odpg.h "object
lifetimes": any order is valid). Uses the raw C-ABI, not the Python
wrappers' finalizers, so the order is exactly the one named. Exits 0 when
every step returned and the counters folded to the launches' packet count.

usage: python destroy_order_child.py cnt,tbl,fwd,fence,ctx
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from odp_amd import _lib as L  # noqa: E402
from odp_amd import cls, gen, gpu  # noqa: E402

lib = L.lib


def main():
    order = sys.argv[1].split(",")
    assert sorted(order) == sorted(["cnt", "tbl", "fwd", "fence", "ctx"]), order
    opt = L.PKTIN_IPV4_CHKSUM | L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM
    cls.reset()
    p = cls.loop_pktio(pktin=opt)
    gen.build_c2_rules(cls, p)
    assert cls.pktio_start(p) == 0
    rules = cls.pktio_rules(p)
    n = 1 << 16
    frames = gen.c2_frames(n)

    ctx = C.c_void_p()
    L.check(lib.odpg_ctx_create(0, None, C.byref(ctx)), "ctx")
    tbl = C.c_void_p()
    L.check(lib.odpg_table_create(ctx, C.byref(rules), C.byref(tbl)), "table")
    cnt = C.c_void_p()
    L.check(lib.odpg_counters_create(ctx, tbl, C.byref(cnt)), "counters")
    fence = C.c_void_p()
    L.check(lib.odpg_fence_create(ctx, C.byref(fence)), "fence")
    routes = gpu.make_routes(gen.c5_routes())
    param = gpu.make_fwd_param(L.FWD_HASH, 4)
    fwd = C.c_void_p()
    L.check(lib.odpg_fwd_create(ctx, routes, len(routes), C.byref(param), C.byref(fwd)), "fwd")

    fb = C.c_void_p()
    ob = C.c_void_p()
    L.check(lib.odpg_dev_alloc(ctx, frames.nbytes, C.byref(fb)), "alloc")
    L.check(lib.odpg_dev_alloc(ctx, 4 * n, C.byref(ob)), "alloc")
    L.check(lib.odpg_memcpy_h2d(ctx, fb, frames.ctypes.data, frames.nbytes), "h2d")
    launches = 8
    for _ in range(launches):
        b = L.odpg_batch_t(fb.value, None, 64, n, opt, L.LAYER_ALL, 1)
        r = L.odpg_result_t(ob.value, None, None, None, cnt.value)
        L.check(lib.odpg_classify(ctx, tbl, C.byref(b), C.byref(r)), "classify")
    L.check(lib.odpg_fence_record(ctx, fence), "fence record")
    words = np.zeros(L.lib.odpg_table_num_cos(tbl) * (1 + L.COS_QUEUE_MAX) + 4, np.uint64)
    L.check(lib.odpg_counters_fold(cnt, words.ctypes.data_as(C.POINTER(C.c_uint64))), "fold")
    got = int(words[0] + words[2] + words[3])       # in_packets + in_errors + in_discards
    L.check(lib.odpg_dev_free(ctx, fb), "free")
    L.check(lib.odpg_dev_free(ctx, ob), "free")

    destroy = {"cnt": lambda: lib.odpg_counters_destroy(cnt),
               "tbl": lambda: lib.odpg_table_destroy(tbl),
               "fwd": lambda: lib.odpg_fwd_destroy(fwd),
               "fence": lambda: lib.odpg_fence_destroy(fence),
               "ctx": lambda: lib.odpg_ctx_destroy(ctx)}
    for k in order:
        destroy[k]()
    cls.reset()
    print("ok", ",".join(order), got, flush=True)
    sys.exit(0 if got == launches * n else 3)


if __name__ == "__main__":
    main()
