#!/bin/bash
# Round-5 session ab (diagnostic): where the counted lean launch's extra time
# goes on C2 / C4: no histogram adds, no flush, no row read
# (tools/exp/l64_diag_*.patch; results wrong by design, timing only).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  for c in c2 c4; do
    CFG=$c TAG=_ab$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_noadd exp_noflush exp_norow" bash tools/ab.sh || exit $?
  done
done
