#!/bin/bash
# Round-5 session ay: the final tree's GPU suite, smoke() and the default
# bench line (what the driver runs at round end).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=r05ay bash tools/gpu_full_tests.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r05ay/bench.json 2> gpurun_out/r05ay/bench.err
rc=$?; echo "bench: $rc"; cat gpurun_out/r05ay/bench.json; exit $rc
