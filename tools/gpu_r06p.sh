#!/bin/bash
# C3 under the kernel trace: the record's command (10 warmup launches) and
# one with 300 warmup launches, to see whether the mid-trace slowdown is a
# transient of the run's first milliseconds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06p; mkdir -p $OUT
for w in 10 300; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3_w$w -o run \
    -- python3 bench.py --no-cpu --config c3 --others none --steps 100 --warmup $w --runs 1 > $OUT/prof_c3_w$w.log 2>&1 || exit $?
done
