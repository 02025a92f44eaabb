#!/bin/bash
# Round-3 record: GPU suite + smoke; per config the HBM counters (FETCH_SIZE /
# WRITE_SIZE passes -> profiles/pmc_traffic_<cfg>.json on these sources),
# rocprofv3 kernel stats and the bench line. Each GPU step has its own time
# limit; the first failure / fault / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT
exec 3>&1   # the script's stdout, for status lines (a step's own output may be redirected)
step() {  # name, then the command; stops the script on any failure
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
      -- python3 bench.py --no-cpu --no-stats --config $cfg --steps 20 --warmup 2 > $OUT/pmc_${cfg}_$c.log 2>&1
  done
  python tools/pmc_summary.py $OUT/pmc_$cfg --write $cfg > $OUT/pmc_${cfg}_summary.json && \
    cp profiles/pmc_traffic_$cfg.json $OUT/
  step "stats $cfg" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$cfg -o run \
    -- python3 bench.py --no-cpu --config $cfg --steps 100 --warmup 10 > $OUT/prof_$cfg.log 2>&1
  extra=""; [ $cfg = c2 ] || [ $cfg = c3 ] && extra="--e2e"
  step "bench $cfg" timeout -k 10 600 python bench.py --config $cfg $extra > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err
  cat $OUT/bench_$cfg.json
done
if [ -z "${CFGS:-}" ]; then
  step "bench c5 lpm" timeout -k 10 600 python bench.py --config c5 --fwd-mode lpm > $OUT/bench_c5lpm.json 2> $OUT/bench_c5lpm.err
  step "bench default" timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
  cat $OUT/bench_default.json
  step "odp_bench_cls_gpu" timeout -k 10 300 odp_amd/lib/odp_bench_cls_gpu > $OUT/odp_bench_cls_gpu.txt 2>&1
fi
echo done | tee -a $OUT/status.txt
