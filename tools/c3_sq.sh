set -u
export TMPDIR=/tmp
bash tools/c3_breakdown.sh || exit 3
SQ1="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH"
SQ2="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS"
CFG=c3 TAG=_sq GROUPS_="$SQ1 $SQ2" BENCH_ARGS="--no-stats" bash tools/pmc.sh || exit 3
python3 tools/pmc_summary.py gpurun_out/pmc_c3_sq > gpurun_out/pmc_c3_sq_summary.json || exit 3
CFG=c3 TAG=_sqparse GROUPS_="$SQ1 $SQ2" BENCH_ARGS="--no-stats --diag parse" bash tools/pmc.sh || exit 3
python3 tools/pmc_summary.py gpurun_out/pmc_c3_sqparse > gpurun_out/pmc_c3_sqparse_summary.json || exit 3
