#!/bin/bash
# Round-5 session t: the descriptor kernel's wide (8-word hit map) launches
# at 5 waves/SIMD (40 B/lane spill) against 4 on C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  CFG=c3 TAG=_t$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_w5" bash tools/ab.sh || exit $?
done
