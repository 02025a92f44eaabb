#!/bin/bash
# Round-4 session K: the runtime's receive pipeline (bursts in flight per
# pktio): runtime / verdict / pktio tests, odp_pktio_perf with the receive
# profile.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
step "pytest rt" timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_odp_rt.py tests/test_rt_verdict.py tests/test_pcap.py tests/test_packet_parse.py > $OUT/pytest.log 2>&1
tail -3 $OUT/pytest.log
for a in "" "-c 4" "-p" "-c 8"; do
  tag=$(echo "x$a" | tr -d ' -')
  step "pktio_perf $a" env ODP_RT_PROF=1 timeout -k 10 240 oracle/_ref/odp_pktio_perf -v $a > $OUT/pktio_perf_$tag.txt 2>&1
  grep -E "Maximum|odp_rt:" $OUT/pktio_perf_$tag.txt | tail -4
done
