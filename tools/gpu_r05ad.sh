#!/bin/bash
# Round-5 session ad: each frame's last tail unit in the line shape
# (tools/exp/own_xp.patch): descriptor-kernel tests of the build, C3 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ad
ODPG_LIB=$PWD/odp_amd/lib/exp_ownxp/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py -m gpu > gpurun_out/r05ad/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/r05ad/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  CFG=c3 TAG=_ad$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_ownxp" bash tools/ab.sh || exit $?
done
