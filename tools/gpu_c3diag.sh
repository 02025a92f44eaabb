#!/bin/bash
# C3 stage breakdown + HBM reads of the load-only and parse-only floors and
# the no-tail experiment build (any failure ends the script).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/c3_breakdown.sh || exit 3
CFG=c3 VARIANTS="base exp_notail" STEPS=50 BENCH_EXTRA=--no-stats bash tools/ab.sh || exit 3
for d in none parse full; do
  CFG=c3 TAG=_f$d GROUPS_="FETCH_SIZE" BENCH_ARGS="--no-stats --diag $d" bash tools/pmc.sh || exit 3
  python3 tools/pmc_summary.py gpurun_out/pmc_c3_f$d | python3 -c "import json,sys;d=json.load(sys.stdin);[print('$d',k,v['FETCH_SIZE']*2048/1e6,'MB') for k,v in d.items() if 'FETCH_SIZE' in v]" || exit 3
done
echo c3diag-done
