#!/bin/bash
# Round-5 session g: the whole GPU suite on the cleaned kernels (experiment
# switches out of the shipped sources), then bench lines for C2, C2x, C3, C4.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests -m gpu > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "all gpu tests: $rc"; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c2x c3 c4; do
  timeout -k 10 300 python bench.py --no-cpu --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $c: $rc"; tail -3 $OUT/bench_$c.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/bench_$c.json'));c=d.get('with_pktio_counters') or {};print('$c', d['value'], d['roofline']['kernel_ms'], 'counted', c.get('kernel_ms'))"
done
