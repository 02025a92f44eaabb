#!/bin/bash
# Round-5 session ai: C4 (CoS-keyed cuckoo lean kernel) workgroup size: the
# LDS table copy per workgroup and the rows set the waves per CU
# (1024 threads: one workgroup, 4 waves per SIMD).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ai
ODPG_LIB=$PWD/odp_amd/lib/exp_hw640/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_counters.py tests/test_mask_groups.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05ai/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/r05ai/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  CFG=c4 TAG=_ai$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_hw512 exp_hw640 exp_hw768" bash tools/ab.sh || exit $?
done
