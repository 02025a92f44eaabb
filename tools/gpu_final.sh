#!/bin/bash
# Round-end style session: GPU parity tests + smoke + default bench (C2), the
# C3 measurement set (bench with CPU baseline, parse floor, rocprofv3 stats,
# HBM PMC) and the C3 SQ instruction counters. Each GPU step is time-limited;
# stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
STEPS="tests bench" bash tools/gpu_round.sh || exit $?
bash tools/gpu_c3prof.sh || exit $?
CFG=c3 TAG=_sq BENCH_ARGS="--no-stats" GROUPS_="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH" bash tools/pmc.sh || exit $?
echo final-done
