#!/bin/bash
# Round-5 session z: nontemporal own-unit loads (tools/exp/own_nt.patch) on C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  CFG=c3 TAG=_z$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_ownnt" bash tools/ab.sh || exit $?
done
