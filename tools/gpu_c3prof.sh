#!/bin/bash
# C3 measurement session: bench line (with CPU baseline), parse-only floor,
# rocprofv3 kernel stats, HBM PMC passes. Each GPU step time-limited; stop on
# the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c3 --steps 100 --warmup 10 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
cat gpurun_out/bench_c3.json
timeout -k 10 300 python bench.py --config c3 --no-cpu --no-stats --diag parse --steps 50 --warmup 5 > gpurun_out/c3_diag_parse.json 2>&1 || exit $?
tail -1 gpurun_out/c3_diag_parse.json
STEPS="prof" BENCH_ARGS="--config c3" bash tools/gpu_round.sh || exit $?
CFG=c3 GROUPS_="FETCH_SIZE WRITE_SIZE" bash tools/pmc.sh || exit $?
echo done
