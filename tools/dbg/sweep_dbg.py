"""Debug: one validation scenario's batched launch, per-packet verdicts and
frame lengths (run once per library build, compare the outputs)."""
import json, sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
from helpers import pack
import test_cls_validation as V
from odp_amd import cls, gpu

name = sys.argv[1]
sc = [s for s in V.SCEN if s["name"] == name][0]
cls.reset()
drules, keep, idx = V.direct_rules(sc)
fr = [bytes.fromhex(p["frame"]) for p in sc["packets"]]
buf, desc = pack(fr * 40)
n = len(fr) * 40
ctx = gpu.Context(0)
for mode in (0, 1, 2, 3):
    ctx.set_kernel_mode(mode)
    tbl = ctx.table(drules)
    g = ctx.classify(tbl, buf, n, desc=desc, classify=sc["classifier"])
    print(mode, "lens", [len(f) for f in fr], "out", (g["out"][:80] & 0xffff).tolist())
m = g["meta"]
print("meta l3", [int(x) for x in m["l3_offset"][:64]])
print("meta if", [hex(int(x)) for x in m["input_flags"][40:50]])
