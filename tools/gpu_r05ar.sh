#!/bin/bash
# Round-5 session ar: the hit-map groups' descriptors read from an LDS copy
# (uniform ds_read + readfirstlane) instead of scalar loads
# (tools/exp/probe_lds.patch): scalar and LDS loads share one counter, so a
# scalar load in the probe loop holds up every LDS wait behind it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ar
ODPG_LIB=$PWD/odp_amd/lib/exp_plds/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_counters.py -m gpu > gpurun_out/r05ar/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05ar/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  CFG=c2x TAG=_ar$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_plds" bash tools/ab.sh || exit $?
  CFG=c3 TAG=_ar$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_plds" bash tools/ab.sh || exit $?
done
