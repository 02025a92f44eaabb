#!/bin/bash
# Round-5 session ak (diagnostic): where C2x's time goes: no hit-map probes,
# no walk (tools/exp/gf_diag_*.patch; results wrong by design), plus the
# parse-only floor (bench --diag parse).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  CFG=c2x TAG=_ak$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_noprobe exp_nowalk" bash tools/ab.sh || exit $?
  CFG=c2x DIAG=parse TAG=_ak$r BENCH_EXTRA=--no-cpu VARIANTS="base" bash tools/ab.sh || exit $?
  CFG=c2x DIAG=none TAG=_ak$r BENCH_EXTRA=--no-cpu VARIANTS="base" bash tools/ab.sh || exit $?
done
