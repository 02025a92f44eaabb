#!/bin/bash
# Round-5 session ah: the dword at byte 64 taken from the early tail pass
# instead of its own lane-per-frame load (tools/exp/x64_tail.patch, on top
# of own_xp): descriptor-kernel tests of the build, C3 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ah
ODPG_LIB=$PWD/odp_amd/lib/exp_x64/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05ah/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/r05ah/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  CFG=c3 TAG=_ah$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_ownxp exp_x64" bash tools/ab.sh || exit $?
done
