#!/bin/bash
# Counted lean-kernel launches at 7 / 8 waves per SIMD (exp_cnt7 / exp_cnt8)
# against the shipped 6 (C2, C1); the descriptor kernel's probe address as
# one shift-add (base vs exp_prev) on C2x with the gf tests.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06s; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
CFG=c2x VARIANTS="base exp_prev base exp_prev" TAG=r06s bash tools/ab.sh || exit $?
for c in c2 c1; do
  CFG=$c VARIANTS="exp_prev exp_cnt7 exp_cnt8 exp_prev exp_cnt7 exp_cnt8" TAG=r06s bash tools/ab.sh || exit $?
done
