#!/bin/bash
# Tiles handed out inside the workgroup (LDS counter) for the CoS-keyed lean
# kernel (C4): parity tests, then C4 / C2 / C1 A/B against the previous
# commit's library (exp_prev).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_counters.py tests/test_group.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in c4 c2 c1; do
  CFG=$c VARIANTS="base exp_prev base exp_prev" TAG=r06r bash tools/ab.sh || exit $?
done
