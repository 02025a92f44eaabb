#!/bin/bash
# Round-5 session aa: C2x (2-word hit maps): line-shaped window loads
# (tools/exp/xw_all.patch) at 5 and 4 waves/SIMD, and 4 waves alone.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05aa
ODPG_LIB=$PWD/odp_amd/lib/exp_xw4/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py -m gpu > gpurun_out/r05aa/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/r05aa/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  CFG=c2x TAG=_aa$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_w4 exp_xw4 exp_xw5" bash tools/ab.sh || exit $?
done
