#!/bin/bash
# Round-5 session h: the lean kernel's tiles from per-queue counters (dynamic
# distribution) against the static round robin (exp_prev): parity, then C2
# / C1 / C4 A/B, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05h
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_counters.py tests/test_bench_cls.py tests/test_walk_groups.py -m gpu > gpurun_out/r05h/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -3 gpurun_out/r05h/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for c in c2 c1 c4; do
    CFG=$c TAG=_h$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_prev" bash tools/ab.sh || exit $?
  done
done
