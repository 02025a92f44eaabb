"""Average rocprofv3 --pmc counters per kernel over all dispatches.

Usage: python tools/pmc_summary.py gpurun_out/pmc_c2 [--write c2]
  (reads p*/run_counter_collection.csv; --write stores the classify kernel's
  HBM bytes per launch in profiles/pmc_traffic_<cfg>.json for bench.py)
FETCH_SIZE is reported in KiB and doubled for gfx950 as the microarch guide's
HBM section prescribes; WRITE_SIZE in KiB as is.
"""
import collections
import csv
import glob
import json
import sys


def kernel_fingerprint():
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from kernel_fingerprint import fingerprint
    return fingerprint()


def summarize(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")
                    + glob.glob(f"{d}/pmc_*/run_counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if "classify_kernel" in k:
                k = "odpg_classify_kernel"
            per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            acc[k][c].append(v)
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    return out


if __name__ == "__main__":
    s = summarize(sys.argv[1])
    # the timed kernel: the odpg_* kernel with the most dispatches (the lean
    # odpg_cls64_kernel for C1/C2/C4, odpg_classify_kernel for C3,
    # odpg_l3fwd_kernel for C5, odpg_tx_kernel for tx), counter folds and
    # runtime copies excluded
    skip = ("rocclr", "stats_reduce", "stats_fold")
    kname = max((n for n in s if "odpg_" in n and
                 not any(x in n for x in skip)),
                key=lambda n: s[n]["dispatches"], default="odpg_classify_kernel")
    k = s.get(kname, {})
    if "FETCH_SIZE" in k:
        k["hbm_read_bytes"] = k["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in k:
        k["hbm_write_bytes"] = k["WRITE_SIZE"] * 1024
    w = k.get("SQ_WAVES")
    if w:
        for c in list(k):
            if c.startswith("SQ_INSTS") or c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE") \
                    or c == "SQ_WAVE_CYCLES":
                k[c + "/wave"] = k[c] / w
    print(json.dumps(s, indent=1, sort_keys=True))
    if "--write" in sys.argv:
        cfg = sys.argv[sys.argv.index("--write") + 1]
        rec = {"config": cfg, "kernel": kname,
               "dispatches": k["dispatches"],
               "fetch_size_kib_raw": k.get("FETCH_SIZE"), "write_size_kib": k.get("WRITE_SIZE"),
               "hbm_read_bytes": k.get("hbm_read_bytes"),
               "hbm_write_bytes": k.get("hbm_write_bytes"),
               "bytes_per_launch": round(k.get("hbm_read_bytes", 0) + k.get("hbm_write_bytes", 0)),
               "correction": "FETCH_SIZE x 2 on gfx950 (MI355X_MICROARCH.md HBM section), KiB",
               # the kernel sources the counters were collected on: bench.py
               # reports the figure as stale once they differ
               "kernel_sources_sha256": kernel_fingerprint()}
        with open(f"profiles/pmc_traffic_{cfg}.json", "w") as fh:
            json.dump(rec, fh, indent=1)
