#!/bin/bash
# An A/B session on one GPU box: the parity tests named in TESTS against the
# base library, then tools/ab.sh over the experiment builds named in
# VARIANTS (built beforehand with tools/exp_build.sh) for each config in
# CFGS, REPEAT times, interleaved. Example:
#   CFGS="c2 c4" VARIANTS="base exp_x" REPEAT=2 bash tools/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${TESTS:-tests/test_gpu_parity.py} -m gpu > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq 1 ${REPEAT:-2}); do
  for c in ${CFGS:-c2}; do
    CFG=$c TAG=_$r BENCH_EXTRA="${BENCH_EXTRA:---no-cpu}" VARIANTS="${VARIANTS:-base}" bash tools/ab.sh || exit $?
  done
done
