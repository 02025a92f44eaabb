#!/bin/bash
# Round-5 session aq (record, runtime): the runtime GPU tests and
# odp_pktio_perf at every worker count on the committed sources.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05aq
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_odp_rt.py tests/test_rt_verdict.py tests/test_packet_parse.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "" "-c 4" "-c 6" "-c 8" "-c 12" "-c 8 -t 2" "-p"; do
  tag=$(echo "x$a" | tr -d ' -')
  ODP_RT_PROF=1 timeout -k 10 150 oracle/_ref/odp_pktio_perf -v $a > $OUT/pktio_perf_$tag.txt 2>&1
  rc=$?; echo "odp_pktio_perf $a: $rc $(grep -E 'Maximum' $OUT/pktio_perf_$tag.txt)"
  [ $rc -eq 0 ] || exit $rc
done
