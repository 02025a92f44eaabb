#!/bin/bash
# HBM traffic and SQ instruction/wait counters for one bench config, one
# rocprofv3 --pmc pass per counter group (no tracing domains combined).
# Usage: CFG=c2 bash tools/pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG="${CFG:-c2}"
OUT=gpurun_out/pmc_$CFG${TAG:-}
mkdir -p $OUT
GROUPS_="${GROUPS_:-FETCH_SIZE WRITE_SIZE SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS}"
i=0
for g in $GROUPS_; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc ${g//,/ } --output-format csv -d $OUT/p$i -o run \
    -- python3 bench.py --no-cpu --config $CFG --steps 20 --warmup 2 ${BENCH_ARGS:-} > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc $g: $rc" | tee -a $OUT/status.txt
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
