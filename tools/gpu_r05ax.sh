#!/bin/bash
# Round-5 session ax: C3's dword at byte 64 taken from the early tail pass's
# loads instead of a lane-per-frame load (tools/exp/gf_x64.patch).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ax
ODPG_LIB=$PWD/odp_amd/lib/exp_x64/libodpg.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_counters.py tests/test_packet_parse.py tests/test_mask_groups.py -m gpu > gpurun_out/r05ax/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 gpurun_out/r05ax/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for c in c3 c2x; do
    CFG=$c TAG=_ax$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_x64" bash tools/ab.sh || exit $?
  done
done
