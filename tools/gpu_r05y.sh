#!/bin/bash
# Round-5 session y: nontemporal tail-pass loads (tools/exp/seg_nt.patch) on C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  CFG=c3 TAG=_y$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_segnt" bash tools/ab.sh || exit $?
done
