#!/bin/bash
# TCC read-request sizes per launch (calibrates FETCH_SIZE on each access
# pattern): 32 B, 64 B and all EA read requests, plus the 128 B (bubble) count.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in ${CFGS:-c2 c3}; do
  rm -rf gpurun_out/pmc_${cfg}_rq
  CFG=$cfg TAG=_rq GROUPS_="TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_BUBBLE_sum" BENCH_ARGS="--no-stats ${BENCH_X:-}" bash tools/pmc.sh || exit 3
  python3 tools/pmc_summary.py gpurun_out/pmc_${cfg}_rq > gpurun_out/pmc_${cfg}_rq.json || exit 3
  python3 - "$cfg" <<'PY'
import json, sys
cfg = sys.argv[1]
d = json.load(open(f"gpurun_out/pmc_{cfg}_rq.json"))
k = max((n for n in d if "odpg_" in n and "fold" not in n), key=lambda n: d[n]["dispatches"])
v = d[k]
print(cfg, k[:40], {c: round(x) for c, x in v.items()})
PY
done
echo rdreq-done
