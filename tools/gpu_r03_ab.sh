#!/bin/bash
# Counted launches: C2 at 7 waves per SIMD; C4 counted at 256-thread workgroups.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  CFG=c2 TAG=_$r BENCH_EXTRA="--no-cpu" VARIANTS="base exp_cnt7" bash tools/ab.sh || exit $?
  CFG=c4 TAG=_$r BENCH_EXTRA="--no-cpu" VARIANTS="base exp_cntfirst exp_cntfirst7" bash tools/ab.sh || exit $?
done
