#!/bin/bash
# C1 / C2 lean-kernel grid: 7 vs 8 workgroups per CU.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for c in c1 c2; do
    for g in 1792 2048; do
      ODPG_L64_GRID=$g CFG=$c TAG=_g${g}_$r BENCH_EXTRA="--no-cpu --no-stats" VARIANTS="exp_grid" bash tools/ab.sh || exit $?
    done
  done
done
