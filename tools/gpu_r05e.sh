#!/bin/bash
# Round-5 session e: hit mask folded into the OR / AND words, own last units
# by word compares: parity, then C2x / C3 against the previous commit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05e
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_helper_chksum.py -m gpu > gpurun_out/r05e/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -3 gpurun_out/r05e/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in c2x c3; do
    CFG=$c TAG=_e$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_prev" bash tools/ab.sh || exit $?
  done
done
