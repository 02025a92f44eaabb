#!/bin/bash
# Round-5 session av: counted lean launches with per-bin ballot counts for
# the first L64_HROUNDS distinct bins of a wave (tools/exp/l64_hballot.patch).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05av
ODPG_LIB=$PWD/odp_amd/lib/exp_hb4/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_counters.py tests/test_mask_groups.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05av/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05av/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in c1 c2; do
    CFG=$c TAG=_av$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_hb4 exp_hb16" bash tools/ab.sh || exit $?
  done
done
