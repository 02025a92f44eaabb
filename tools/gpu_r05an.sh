#!/bin/bash
# Round-5 session an: the verdict store deferred past the next tile's probes
# (tools/exp/gf_late_store.patch): the probes' indexed key reads wait for
# every vector memory operation in flight.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05an
ODPG_LIB=$PWD/odp_amd/lib/exp_lstore/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py -m gpu > gpurun_out/r05an/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05an/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  CFG=c2x TAG=_an$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_lstore" bash tools/ab.sh || exit $?
  CFG=c3 TAG=_an$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_lstore" bash tools/ab.sh || exit $?
done
