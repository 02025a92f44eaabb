#!/bin/bash
# Round-6 record: GPU suite + smoke; per config the HBM counters (FETCH_SIZE /
# WRITE_SIZE passes -> profiles/pmc_traffic_<cfg>.json on these sources),
# rocprofv3 kernel stats and the bench line; SQ instruction counters of the
# descriptor kernel (C2x, C3) and the CoS-keyed lean kernel (C4);
# odp_pktio_perf through the runtime (1 + 1, -c 4, -c 8, -p workers). Each GPU
# step has its own time limit; the first failure / fault / timeout ends the
# script. CFGS selects configs, SKIP_TESTS / EXTRAS=0 skip parts.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06final}
mkdir -p $OUT
exec 3>&1
step() {
  local n=$1; shift
  "$@"; local rc=$?
  echo "$n: $rc" >> $OUT/status.txt; echo "$n: $rc" >&3
  [ $rc -eq 0 ] || exit $rc
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -o log_cli=false > $OUT/pytest_gpu.log 2>&1
  tail -2 $OUT/pytest_gpu.log
  step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
fi
for cfg in ${CFGS:-c2 c1 c2x c3 c4 c5 tx}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    step "pmc $cfg $c" timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$cfg/pmc_$c -o run \
      -- python3 bench.py --no-cpu --no-stats --config $cfg --others none --steps 20 --warmup 2 --runs 1 > $OUT/pmc_${cfg}_$c.log 2>&1
  done
  python tools/pmc_summary.py $OUT/pmc_$cfg --write $cfg > $OUT/pmc_${cfg}_summary.json && \
    cp profiles/pmc_traffic_$cfg.json $OUT/
  step "stats $cfg" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$cfg -o run \
    -- python3 bench.py --no-cpu --config $cfg --others none --steps 100 --warmup 300 --runs 1 > $OUT/prof_$cfg.log 2>&1
  extra=""; [ $cfg = c2 ] || [ $cfg = c3 ] && extra="--e2e"
  step "bench $cfg" timeout -k 10 600 python bench.py --config $cfg --others none $extra > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err
  cat $OUT/bench_$cfg.json | cut -c1-400
done
if [ "${EXTRAS:-1}" = 1 ]; then
  C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  C2="SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
  for cfg in c2x c3 c4; do
    step "sq $cfg" timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $OUT/sq_$cfg/p1 -o run \
      -- python3 bench.py --no-cpu --no-stats --config $cfg --others none --steps 20 --warmup 2 --runs 1 > $OUT/sq_${cfg}_1.log 2>&1
    step "sq2 $cfg" timeout -k 10 120 rocprofv3 --pmc $C2 --output-format csv -d $OUT/sq_$cfg/p2 -o run \
      -- python3 bench.py --no-cpu --no-stats --config $cfg --others none --steps 20 --warmup 2 --runs 1 > $OUT/sq_${cfg}_2.log 2>&1
    python tools/pmc_summary.py $OUT/sq_$cfg > $OUT/sq_${cfg}_summary.json
  done
  step "bench c5 lpm" timeout -k 10 600 python bench.py --config c5 --fwd-mode lpm > $OUT/bench_c5lpm.json 2> $OUT/bench_c5lpm.err
  step "bench default" timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
  cat $OUT/bench_default.json
  step "odp_bench_cls_gpu" timeout -k 10 300 odp_amd/lib/odp_bench_cls_gpu > $OUT/odp_bench_cls_gpu.txt 2>&1
  for a in "" "-c 8"; do
    tag=$(echo "x$a" | tr -d ' -')
    step "pktio_perf $a" env ODP_RT_PROF=1 timeout -k 10 240 oracle/_ref/odp_pktio_perf -v $a > $OUT/pktio_perf_$tag.txt 2>&1
    grep -E "Maximum|odp_rt:" $OUT/pktio_perf_$tag.txt | tail -3
  done
fi
echo done | tee -a $OUT/status.txt
