#!/bin/bash
# Round-5 session p (experiment): which part of the delivery loop costs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05p
mkdir -p $OUT
for x in 5 6 7 8; do
  ODP_RT_EXP=$x ODP_RT_PROF=1 timeout -k 10 240 oracle/_ref/odp_pktio_perf -c 4 > $OUT/pktio_perf_$x.txt 2>&1
  rc=$?; echo "exp $x: $rc"; head -1 $OUT/pktio_perf_$x.txt; grep -E "Maximum" $OUT/pktio_perf_$x.txt
  [ $rc -eq 0 ] || exit $rc
done
