#!/bin/bash
# S64 descriptor-kernel instantiation: parity tests, then C2x A/B (base = S64,
# exp_nos64 = the old stride path, exp_s64w6 = S64 at 6 waves per SIMD).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py -m gpu -k "gf or c2x or xm or mixed" > gpurun_out/r06b_pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -3 gpurun_out/r06b_pytest.log; [ $rc -eq 0 ] || exit $rc
CFG=c2x VARIANTS="base exp_nos64 exp_s64w6 base exp_nos64 exp_s64w6" TAG=r06b bash tools/ab.sh
