#!/bin/bash
# Round-5 session c: direct-indexed branch-free hit-map probes in the
# descriptor kernel: parity, then C2x / C3 A/B over probe batching and
# occupancy.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_cls_validation.py tests/test_destroy_order.py -m gpu > gpurun_out/r05c/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -3 gpurun_out/r05c/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in c2x c3; do
    CFG=$c TAG=_c$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_p4 exp_w4 exp_nogen" bash tools/ab.sh || exit $?
  done
done
