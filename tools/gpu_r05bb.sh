#!/bin/bash
# Round-5 session bb: per-dispatch GPU clock of the C3 launches under the
# profiler (GRBM_GUI_ACTIVE / GRBM_COUNT per dispatch against its duration),
# to see whether the drift of C3's traced launch times is clock.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bb
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT/grbm_c3 -o run \
  -- python3 bench.py --no-cpu --no-stats --config c3 --steps 100 --warmup 10 --runs 1 > $OUT/grbm_c3.log 2>&1
rc=$?; echo "grbm c3: $rc"; ls -R $OUT | head; exit $rc
