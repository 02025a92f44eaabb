#!/bin/bash
# Round-5 session o: odp_pktio_perf -c 4 / -c 8 with the delivery profile
# split (binding release, queue appends).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05o
mkdir -p $OUT
for a in "-c 4" "-c 8"; do
  tag=$(echo "x$a" | tr -d ' -')
  ODP_RT_PROF=1 timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  rc=$?; echo "odp_pktio_perf $a: $rc"; head -1 $OUT/pktio_perf_$tag.txt; grep -E "Maximum" $OUT/pktio_perf_$tag.txt
  [ $rc -eq 0 ] || exit $rc
done
