#!/bin/bash
# Round-5 session j: runtime queues as handle rings (lock-free empty checks,
# loop ring popped as handles): runtime GPU tests, then odp_pktio_perf at
# the default, -c 4 and -c 8 worker counts.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_odp_rt.py tests/test_rt_verdict.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "" "-c 4" "-c 8"; do
  tag=$(echo "x$a" | tr -d ' -')
  timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  rc=$?; echo "odp_pktio_perf $a: $rc"; grep -E "Maximum|Result|workers" $OUT/pktio_perf_$tag.txt | tail -4
  [ $rc -eq 0 ] || exit $rc
done
