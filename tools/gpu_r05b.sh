#!/bin/bash
# Round-5 session b: the descriptor kernel without its generic parse
# (experiment builds, GF_EXP_NOGEN: C2x / C3 traffic is all register-parse
# frames, so results stay exact) at several occupancies.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  for c in c3 c2x; do
    CFG=$c TAG=_b$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_nogen exp_nogen5 exp_nogen6 exp_nogen4" bash tools/ab.sh || exit $?
  done
done
