# C3 SQ instruction / wait counters, full launch and the parse-only diag
# (one rocprofv3 --pmc pass per counter group). Usage: TAG=_x bash tools/c3_sq.sh
set -u
export TMPDIR=/tmp
SQ1="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH"
SQ2="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS"
for d in ${DIAGS:-full parse}; do
  CFG=c3 TAG=_sq$d${TAG:-} GROUPS_="$SQ1 $SQ2" BENCH_ARGS="--no-stats --diag $d" bash tools/pmc.sh || exit 3
  python3 tools/pmc_summary.py gpurun_out/pmc_c3_sq$d${TAG:-} > gpurun_out/pmc_c3_sq$d${TAG:-}_summary.json || exit 3
done
