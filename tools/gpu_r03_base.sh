#!/bin/bash
# Round-3 session: the new / changed GPU tests, then bench line and
# rocprofv3 kernel stats for C2 (headline), A/B of the C2 tile staging,
# bench, stats and HBM counters for C3 (IMIX), A/B of the C4 workgroup size
# and of the persistent l3fwd kernel (C5).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${FIRST:-tests/test_thash_vectors.py tests/test_l3fwd.py tests/test_gpu_parity.py} -m gpu > gpurun_out/pytest_first.log 2>&1
rc=$?; echo "first tests: $rc"; tail -5 gpurun_out/pytest_first.log; [ $rc -eq 0 ] || exit $rc
STEPS="bench prof" TAG=_c2 bash tools/gpu_round.sh || exit $?
CFG=c2 BENCH_EXTRA="--no-stats" VARIANTS="base exp_nocoal base exp_nocoal" bash tools/ab.sh || exit $?
CFG=c5 BENCH_EXTRA="--no-stats" VARIANTS="base exp_fwdold base exp_fwdold" bash tools/ab.sh || exit $?
CFG=c5 TAG=_lpm BENCH_EXTRA="--no-stats --fwd-mode lpm" VARIANTS="base exp_fwdold" bash tools/ab.sh || exit $?
CFG=c4 BENCH_EXTRA="--no-stats" VARIANTS="base exp_hw512 exp_hw768 exp_hw1024 base" bash tools/ab.sh || exit $?
STEPS="bench prof pmc" TAG=_c3 BENCH_ARGS="--config c3" bash tools/gpu_round.sh || exit $?
