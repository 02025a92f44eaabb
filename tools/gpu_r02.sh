#!/bin/bash
# Round-2 measurement session: parity tests + smoke, the C2 bench line (CPU
# baseline included), rocprofv3 kernel stats and HBM PMC passes for C2 and C3.
# Every GPU step is time-limited; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
STEPS="tests bench prof" bash tools/gpu_round.sh || exit $?
STEPS="pmc" BENCH_ARGS="--no-stats" bash tools/gpu_round.sh || exit $?
mkdir -p gpurun_out/c2pmc && mv gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/c2pmc/ || exit 5
mv gpurun_out/prof gpurun_out/prof_c2 || exit 5
timeout -k 10 300 python bench.py --config c3 --steps 100 --warmup 10 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
cat gpurun_out/bench_c3.json
STEPS="prof" BENCH_ARGS="--config c3" bash tools/gpu_round.sh || exit $?
mv gpurun_out/prof gpurun_out/prof_c3 || exit 5
STEPS="pmc" BENCH_ARGS="--config c3 --no-stats" bash tools/gpu_round.sh || exit $?
mkdir -p gpurun_out/c3pmc && mv gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/c3pmc/ || exit 5
echo r02-done
