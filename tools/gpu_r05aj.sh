#!/bin/bash
# Round-5 session aj: (1) C4 lean-kernel workgroup size (LDS table copy per
# workgroup); (2) descriptor-kernel probes with a branch-free key select and
# the chain words in the group's scalar loads (tools/exp/probe_sel.patch) on
# C2x / C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05aj
for v in exp_hw640 exp_psel; do
  ODPG_LIB=$PWD/odp_amd/lib/$v/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_counters.py tests/test_mask_groups.py tests/test_gf_kernel.py -m gpu > gpurun_out/r05aj/pytest_$v.log 2>&1
  rc=$?; echo "tests $v: $rc"; tail -1 gpurun_out/r05aj/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  CFG=c4 TAG=_aj$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_hw512 exp_hw640 exp_hw768" bash tools/ab.sh || exit $?
  CFG=c2x TAG=_aj$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_psel" bash tools/ab.sh || exit $?
  CFG=c3 TAG=_aj$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_psel" bash tools/ab.sh || exit $?
done
