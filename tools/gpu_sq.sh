#!/bin/bash
# SQ instruction / wait counters (and optionally FETCH/WRITE) for bench
# configs, one rocprofv3 --pmc pass per group, then one bench line each.
# Usage: CFGS="c2x c3" TAG=_r04a bash tools/gpu_sq.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for CFG in ${CFGS:-c2x}; do
  OUT=gpurun_out/sq_$CFG${TAG:-}
  mkdir -p $OUT
  GROUPS_="${GROUPS_:-SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS SQ_WAVES,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE}"
  i=0
  for g in $GROUPS_; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc ${g//,/ } --output-format csv -d $OUT/p$i -o run \
      -- python3 bench.py --no-cpu --no-stats --config $CFG --steps 20 --warmup 2 ${BENCH_ARGS:-} > $OUT/p$i.log 2>&1
    rc=$?; echo "pmc $CFG $g: $rc" | tee -a $OUT/status.txt
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
  done
  python tools/pmc_summary.py $OUT > $OUT/summary.json 2>&1
  timeout -k 10 300 python bench.py --no-cpu --config $CFG > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench $CFG: $rc"; cat $OUT/bench.json
  [ $rc -eq 0 ] || exit $rc
done
