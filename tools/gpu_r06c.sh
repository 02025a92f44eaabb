#!/bin/bash
# Probe rework (key-vector remap, VALU hit test, guard-split loops, b128
# entries) + S64: gf parity tests, then C2x / C3 A/B against the round-5
# library (exp_old) and S64 at 5 waves (exp_s64w5).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_xmask_emul.py -m gpu > gpurun_out/r06c_pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -3 gpurun_out/r06c_pytest.log; [ $rc -eq 0 ] || exit $rc
CFG=c2x VARIANTS="base exp_old exp_s64w5 base exp_old exp_s64w5" TAG=r06c bash tools/ab.sh || exit $?
CFG=c3 VARIANTS="base exp_old base exp_old" TAG=r06c bash tools/ab.sh
