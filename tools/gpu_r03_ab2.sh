#!/bin/bash
# Counted launches: all-wave flush (C4 default, C2 experiment) vs last-wave flush.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_cls_validation.py -m gpu > gpurun_out/pytest_cnt.log 2>&1
rc=$?; echo "parity tests: $rc"; tail -2 gpurun_out/pytest_cnt.log; [ $rc -eq 0 ] || exit $rc
ODPG_LIB=$PWD/odp_amd/lib/exp_mgbar/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -m gpu -k "counter or c2 or stride64" > gpurun_out/pytest_mgbar.log 2>&1
rc=$?; echo "mgbar tests: $rc"; tail -2 gpurun_out/pytest_mgbar.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for r in 1 2; do
  CFG=c4 TAG=_$r BENCH_EXTRA="--no-cpu" VARIANTS="base exp_hwlast" bash tools/ab.sh || exit $?
  CFG=c2 TAG=_$r BENCH_EXTRA="--no-cpu" VARIANTS="base exp_mgbar" bash tools/ab.sh || exit $?
done
