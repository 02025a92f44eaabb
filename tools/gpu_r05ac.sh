#!/bin/bash
# Round-5 session ac: counted lean launches with the histogram add issued one
# tile late (tools/exp/l64_cnt_defer.patch): counter tests of the build, then
# C2 / C4 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ac
ODPG_LIB=$PWD/odp_amd/lib/exp_cdefer/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_counters.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05ac/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/r05ac/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in c2 c4; do
    CFG=$c TAG=_ac$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_cdefer" bash tools/ab.sh || exit $?
  done
done
