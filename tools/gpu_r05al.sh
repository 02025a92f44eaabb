#!/bin/bash
# Round-5 session al: C2x hit-map probes per iteration (GF_PROBES chain-free
# groups, GF_CPROBES chain groups, tools/exp/gf_cprobes.patch): the probes
# are 15 of C2x's 40 us (session ak).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05al
ODPG_LIB=$PWD/odp_amd/lib/exp_u3c4/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py -m gpu > gpurun_out/r05al/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05al/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  CFG=c2x TAG=_al$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_u3 exp_u4 exp_u6 exp_u3c4 exp_u6c4" bash tools/ab.sh || exit $?
done
