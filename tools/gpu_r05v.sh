#!/bin/bash
# Round-5 session v: line-shaped tail loads (SEG_XPOSE) on C3: parity of the
# experiment build (descriptor-kernel tests), then A/B against the base.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05v
ODPG_LIB=$PWD/odp_amd/lib/exp_xp/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py -m gpu > gpurun_out/r05v/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/r05v/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  CFG=c3 TAG=_v$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_xp" bash tools/ab.sh || exit $?
done
