#!/bin/bash
# TX: persistent coalesced kernel (3 / 4 waves per SIMD) vs one-pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_tx.py tests/test_odp_rt.py tests/test_rt_verdict.py -m gpu > gpurun_out/pytest_tx.log 2>&1
rc=$?; echo "tx tests: $rc"; tail -2 gpurun_out/pytest_tx.log; [ $rc -eq 0 ] || exit $rc
CFG=tx BENCH_EXTRA="--no-cpu" VARIANTS="base exp_txp4 exp_txone base exp_txp4 exp_txone" bash tools/ab.sh || exit $?
