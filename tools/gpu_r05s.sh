#!/bin/bash
# Round-5 session s: tail passes in flight per wave (SEG_PASSES 2 / 3 / 4) on C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  CFG=c3 TAG=_s$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_np3 exp_np4" bash tools/ab.sh || exit $?
done
