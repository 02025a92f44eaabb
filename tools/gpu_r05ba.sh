#!/bin/bash
# Round-5 session ba: C2x with the line-shaped window and tail loads at 4
# waves per SIMD (tools/exp/xw_all.patch, -DGF_WAVES=4), against the base
# and the base at 4 waves.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ba
ODPG_LIB=$PWD/odp_amd/lib/exp_xw4/libodpg.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_counters.py -m gpu > gpurun_out/r05ba/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05ba/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  CFG=c2x TAG=_ba$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_xw4 exp_w4" bash tools/ab.sh || exit $?
done
