#!/bin/bash
# Round-5 session am: the runtime under more workers than one L3 holds and in
# plain-queue mode with several workers (chunked delivery, placement
# fallback), each run under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05am
mkdir -p $OUT
for a in "-c 12" "-c 15" "-c 8"; do
  tag=$(echo "x$a" | tr -d ' -')
  ODP_RT_PROF=1 timeout -k 10 150 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  rc=$?; echo "odp_pktio_perf $a: $rc $(grep -E 'Maximum' $OUT/pktio_perf_$tag.txt)"
  [ $rc -eq 0 ] || exit $rc
done
