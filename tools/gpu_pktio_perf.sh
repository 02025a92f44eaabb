#!/bin/bash
# test/performance/odp_pktio_perf (reference source, unmodified) on the loop
# device through the GPU receive path: the maximum lossless rate search,
# scheduler and plain-queue input, 1 and 2 RX workers.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for a in "" "-p" "-c 4"; do
  tag=$(echo "x$a" | tr -d ' -')
  timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  rc=$?; echo "odp_pktio_perf $a: $rc"; grep -E "Maximum|Result|Starting|workers" $OUT/pktio_perf_$tag.txt | tail -5
  [ $rc -eq 0 ] || exit $rc
done
