"""HBM streaming floor of the classifier's launch shape (diagnostic).

Times odpg_diag_stream (include/odpg.h) over rotating 64 MiB batches of 2^20
64-byte frames for each access pattern and grid size, and prints one JSON line
per variant: microseconds per launch and the GB/s of 68 B/frame.

    python tools/diag_stream.py [--npkt 1048576] [--steps 100]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from odp_amd import _lib as L  # noqa: E402
from odp_amd import gpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npkt", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--grids", default="0,1024,1280,2048,4096")
    ap.add_argument("--patterns", default="0,1,2,16,17,18")
    ap.add_argument("--fill", default="zero", choices=["zero", "c2"],
                    help="buffer contents: zeros, or the C2 bench frames")
    a = ap.parse_args()
    ctx = gpu.Context(0)
    n = a.npkt
    nbuf = max(2, -(-300 * (1 << 20) // (n * 64)))
    src = [ctx.buffer(n * 64) for _ in range(nbuf)]
    if a.fill == "c2":
        from odp_amd import gen
        fr = gen.c2_frames(n)
    for b in src:
        if a.fill == "c2":
            b.upload(fr)
        else:
            b.zero()
    outs = [ctx.buffer(4 * n) for _ in range(nbuf)]
    lib = L.lib
    for pat in [int(x) for x in a.patterns.split(",")]:
        for grid in [int(x) for x in a.grids.split(",")]:
            for i in range(10):
                L.check(lib.odpg_diag_stream(ctx.h, src[i % nbuf].ptr, n, outs[i % nbuf].ptr,
                                             pat, grid), "diag")
            ctx.sync()
            lib.odpg_event_record(ctx.h, 0)
            for i in range(a.steps):
                lib.odpg_diag_stream(ctx.h, src[i % nbuf].ptr, n, outs[i % nbuf].ptr, pat, grid)
            lib.odpg_event_record(ctx.h, 1)
            ctx.sync()
            ms = C.c_float(0)
            L.check(lib.odpg_event_elapsed_ms(ctx.h, 0, 1, C.byref(ms)), "event")
            us = ms.value * 1e3 / a.steps
            print(json.dumps({"npkt": n, "fill": a.fill, "pattern": pat, "grid": grid,
                              "us": round(us, 2),
                              "GBps": round(68 * n / (us * 1e-6) / 1e9, 1),
                              "Mpps": round(n / us, 1)}), flush=True)


if __name__ == "__main__":
    main()
