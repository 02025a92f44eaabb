#!/bin/bash
# Branch-free register parse + multi-queue loop pktio: gf / parity / runtime
# tests, then C2x / C3 A/B against the previous commit's library (exp_prev).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_odp_rt.py tests/test_rt_verdict.py -m gpu > gpurun_out/r06h_pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -3 gpurun_out/r06h_pytest.log; [ $rc -eq 0 ] || exit $rc
CFG=c2x VARIANTS="base exp_prev base exp_prev" TAG=${TAG:-r06h} bash tools/ab.sh || exit $?
CFG=c3 VARIANTS="base exp_prev base exp_prev" TAG=${TAG:-r06h} bash tools/ab.sh
