#!/bin/bash
# Device groups, runtime device list, other_configs bench test; then the C2x
# part-removal A/B (experiment builds).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_group.py tests/test_odp_rt.py tests/test_dist.py -m gpu > gpurun_out/r06e_pytest.log 2>&1
rc=$?; echo "tests: $rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r06e_pytest.log | tail -25; [ $rc -eq 0 ] || exit $rc
CFG=c2x VARIANTS="base exp_gf_noprobe exp_gf_nowalk exp_gf_noparse exp_s64w5 base exp_gf_noprobe exp_gf_nowalk exp_gf_noparse exp_s64w5" TAG=r06d BENCH_EXTRA=--no-stats bash tools/ab.sh
