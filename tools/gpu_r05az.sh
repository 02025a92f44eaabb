#!/bin/bash
# Round-5 session az: nontemporal verdict stores in the lean kernel
# (tools/exp/l64_ntstore.patch).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05az
ODPG_LIB=$PWD/odp_amd/lib/exp_nts/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_counters.py tests/test_mask_groups.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05az/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05az/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for c in c1 c2 c4; do
    CFG=$c TAG=_az$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_nts" bash tools/ab.sh || exit $?
  done
done
