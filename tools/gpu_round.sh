#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats and HBM
# counters. Every GPU step has its own time limit; a fault / abort / timeout
# stops the script (no further GPU work in this call).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-tests bench prof pmc}"
BENCH_ARGS="${BENCH_ARGS:-}"
T="${TAG:-}"   # suffix of the output files (several configs in one call)

gate() {  # $1 = exit status; 0/1 (test failures) continue, anything else stops
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "GPU step ended with status $rc: stopping" | tee -a $OUT/status.txt
    exit "$rc"
  fi
}

for s in $STEPS; do
  case $s in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
    rc=$?; echo "pytest gpu: $rc" | tee -a $OUT/status.txt; tail -5 $OUT/pytest_gpu.log; gate $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
    rc=$?; echo "smoke: $rc" | tee -a $OUT/status.txt; tail -3 $OUT/smoke.log; gate $rc ;;
  bench)
    timeout -k 10 600 python bench.py $BENCH_ARGS > $OUT/bench$T.json 2> $OUT/bench$T.err
    rc=$?; echo "bench: $rc" | tee -a $OUT/status.txt; cat $OUT/bench$T.json; tail -3 $OUT/bench$T.err; gate $rc ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$T -o run \
      -- python3 bench.py --no-cpu --steps 100 --warmup 10 $BENCH_ARGS > $OUT/prof$T.log 2>&1
    rc=$?; echo "rocprof stats: $rc" | tee -a $OUT/status.txt; tail -3 $OUT/prof$T.log; gate $rc ;;
  pmc)
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc${T}_$c -o run \
        -- python3 bench.py --no-cpu --steps 20 --warmup 2 $BENCH_ARGS > $OUT/pmc${T}_$c.log 2>&1
      rc=$?; echo "rocprof pmc $c: $rc" | tee -a $OUT/status.txt; tail -2 $OUT/pmc${T}_$c.log; gate $rc
    done ;;
  esac
done
echo "done" | tee -a $OUT/status.txt
