"""Per-wave start / end times of the lean 64-byte kernel (experiment build
with the tools/exp/l64_times.patch experiment patch,
on the bench's C2 launch shape: how long after the
kernel's first wave each wave ends, by the number of tiles it ran. Shows
the tile-drain tail. s_memrealtime ticks at 100 MHz.

Usage: PATCHES=l64_times REBUILD=classify64 bash tools/exp_build.sh exp_times
       ODPG_LIB=odp_amd/lib/exp_times/libodpg.so python tools/wave_times.py [--config c2]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from odp_amd import _lib as L  # noqa: E402
from odp_amd import cls, gen, gpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c4"])
    ap.add_argument("--counted", action="store_true")
    ap.add_argument("--launches", type=int, default=30)
    a = ap.parse_args()
    opt = L.PKTIN_IPV4_CHKSUM | L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM
    cls.reset()
    if a.config == "c4":
        assert cls.set_limits(2048, 2048, 32) == 0
    p = cls.loop_pktio(pktin=opt)
    {"c1": gen.build_c1_rules, "c2": gen.build_c2_rules, "c4": gen.build_c4_rules}[a.config](cls, p)
    assert cls.pktio_start(p) == 0
    rules = cls.pktio_rules(p)
    n = 1 << 20
    frames = (gen.c1_frames if a.config == "c1" else gen.c2_frames)(n)
    ctx = gpu.Context(0)
    tbl = ctx.table(rules)
    bufs = []
    for _ in range(5):
        fb = ctx.buffer(frames.nbytes)
        fb.upload(frames)
        bufs.append(fb)
    ob = ctx.buffer(4 * n)
    cnt = ctx.counters(tbl) if a.counted else None
    for i in range(a.launches):
        b = L.odpg_batch_t(bufs[i % 5].ptr, None, 64, n, opt, L.LAYER_ALL, 1)
        r = L.odpg_result_t(ob.ptr, None, None, None, cnt.h if cnt else None)
        L.check(L.lib.odpg_classify(ctx.h, tbl.h, C.byref(b), C.byref(r)), "classify")
    ctx.sync()
    assert L.lib.odpg_last_kernel() == 1
    raw = np.zeros(2 * 65536, np.uint64)
    L.check(L.lib.odpg_diag_l64_times(raw.ctypes.data_as(C.c_void_p), 65536), "times")
    raw = raw.reshape(-1, 2)
    pro = None
    if hasattr(L.lib, "odpg_diag_l64_tpro"):          # tools/exp/l64_times_pro.patch
        pro = np.zeros(65536, np.uint64)
        L.check(L.lib.odpg_diag_l64_tpro(pro.ctypes.data_as(C.c_void_p), 65536), "tpro")
    used = raw[:, 0] != 0
    gws = np.nonzero(used)[0]
    st = raw[used, 0].astype(np.int64)
    en = (raw[used, 1] & ((1 << 48) - 1)).astype(np.int64)
    tiles = (raw[used, 1] >> 48).astype(np.int64)
    # only the last launch: the waves whose start lies within the last launch
    t0 = st.max() - 20000
    last = st >= t0
    st, en, tiles, gws = st[last], en[last], tiles[last], gws[last]
    base = st.min()
    if pro is not None:
        # the workgroup's prologue (table copy to LDS + barrier): wave start
        # to the first tile
        pr = pro[gws].astype(np.int64) - st
        prologue = {q: round(float(np.percentile(pr, q)) / 100.0, 3) for q in (0, 50, 90, 100)}
    else:
        prologue = None
    out = {"config": a.config, "counted": a.counted, "waves": int(len(st)),
           "kernel_span_us": round((en.max() - base) / 100.0, 3),
           "start_spread_us": round((st.max() - base) / 100.0, 3),
           "end_us": {q: round(float(np.percentile(en - base, q)) / 100.0, 3)
                      for q in (0, 10, 50, 90, 100)},
           "prologue_us": prologue, "by_tiles": {}}
    for k in sorted(set(tiles.tolist())):
        m = tiles == k
        out["by_tiles"][int(k)] = {"waves": int(m.sum()),
                                   "end_us_p50": round(float(np.median(en[m] - base)) / 100.0, 3),
                                   "end_us_max": round(float((en[m] - base).max()) / 100.0, 3)}
    # by XCD (workgroups go round-robin over the 8 XCDs) and by dispatch
    # order (wave index eighths)
    wpg = int(os.environ.get("ODPG_WAVES_PER_WG", "4"))
    xcd = (gws // wpg) % 8
    out["end_us_p50_by_xcd"] = [round(float(np.median(en[xcd == x] - base)) / 100.0, 3)
                                for x in range(8)]
    order = np.argsort(gws)
    eighths = [slice(len(order) * k // 8, len(order) * (k + 1) // 8) for k in range(8)]
    out["end_us_p50_by_gw_eighth"] = [round(float(np.median((en[order] - base)[e])) / 100.0, 3)
                                      for e in eighths]
    out["start_us_p50_by_gw_eighth"] = [round(float(np.median((st[order] - base)[e])) / 100.0, 3)
                                        for e in eighths]
    # busy waves over time (10 ns bins): the drain's shape
    hist = []
    for t in range(0, int(en.max() - base) + 1, 50):
        hist.append(int(((st - base) <= t).sum() - ((en - base) <= t).sum()))
    out["alive_every_0.5us"] = hist
    print(json.dumps(out))


if __name__ == "__main__":
    main()
