#!/bin/bash
# Round-5 session aw: lean kernel with two tiles in flight per wave
# (tools/exp/l64_pf2.patch) at 8 and 6 waves per SIMD, against the base at
# 8 and at 6 (occupancy control).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05aw
ODPG_LIB=$PWD/odp_amd/lib/exp_pf2/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_counters.py tests/test_mask_groups.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05aw/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05aw/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in c1 c2 c4; do
    CFG=$c TAG=_aw$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_pf2 exp_pf2w6 exp_w6" bash tools/ab.sh || exit $?
  done
done
