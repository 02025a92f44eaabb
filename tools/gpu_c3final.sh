#!/bin/bash
# C3 bench line (CPU baseline included) and its rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c3 --steps 100 --warmup 10 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 3
cat gpurun_out/bench_c3.json
rm -rf gpurun_out/prof
STEPS="prof" BENCH_ARGS="--config c3" bash tools/gpu_round.sh || exit $?
echo c3final-done
