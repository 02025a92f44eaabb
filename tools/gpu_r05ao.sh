#!/bin/bash
# Round-5 session ao: C2's grid: all 8 workgroups per CU (8192 waves, 2 tiles
# each) and a balanced grid (every wave the same number of tiles), against
# the shipped 7 per CU (a third of the waves take a third tile).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2 3; do
  CFG=c2 TAG=_ao$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_g8 exp_gbal" bash tools/ab.sh || exit $?
done
