#!/bin/bash
# Round-5 session at: counted lean launches with 4 copies of the LDS
# histogram (tools/exp/l64_hist4.patch): fewer lanes of one add at one
# address.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05at
ODPG_LIB=$PWD/odp_amd/lib/exp_h4/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_counters.py tests/test_mask_groups.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05at/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05at/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in c2 c1; do
    CFG=$c TAG=_at$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_h4" bash tools/ab.sh || exit $?
  done
done
