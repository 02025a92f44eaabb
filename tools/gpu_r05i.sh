#!/bin/bash
# Round-5 session i: issue priority experiments on the lean kernel (C2 / C1),
# against the base build (counter row written to LDS behind the first tile).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05i
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_counters.py -m gpu > gpurun_out/r05i/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/r05i/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for c in c2 c1; do
    CFG=$c TAG=_i$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_pleft exp_pslot" bash tools/ab.sh || exit $?
  done
done
