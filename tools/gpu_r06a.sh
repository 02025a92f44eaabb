#!/bin/bash
# Round-6 baseline on a fresh box: default / C2x / C3 / C4 bench lines (no CPU leg).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06a}
mkdir -p $OUT
for cfg in ${CFGS:-c2 c2x c3 c4}; do
  timeout -k 10 300 python bench.py --no-cpu --config $cfg --runs 3 > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || exit $?
  python - "$OUT/bench_$cfg.json" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(d["config"]["workload"][:20], d["value"], d["roofline"]["kernel_ms"], d.get("with_pktio_counters",{}).get("kernel_ms"))
PY
done
