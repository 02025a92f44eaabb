#!/bin/bash
# C2 / C1 resident-grid sweep of the lean kernel (workgroups per launch).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for g in 1280 1536 1792 2048; do
    ODPG_L64_GRID=$g CFG=c2 TAG=_g${g}_$r BENCH_EXTRA="--no-cpu --no-stats" VARIANTS="exp_grid" bash tools/ab.sh || exit $?
  done
done
for g in 1536 2048; do
  ODPG_L64_GRID=$g CFG=c1 TAG=_g$g BENCH_EXTRA="--no-cpu --no-stats" VARIANTS="exp_grid" bash tools/ab.sh || exit $?
done
