#!/bin/bash
# Round-end style session: GPU parity tests + smoke + default bench (C2), then
# the C3 measurement set (bench with CPU baseline, rocprofv3 stats, HBM PMC).
# Each GPU step is time-limited; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
STEPS="tests bench" bash tools/gpu_round.sh || exit $?
bash tools/gpu_c3prof.sh || exit $?
echo final-done
