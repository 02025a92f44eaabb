#!/bin/bash
# Round-5 session ap: receive delivery chunk size (RX_CHUNK 64 / 128 / 256)
# on odp_pktio_perf -c 4 / -c 8 (the library picked by LD_LIBRARY_PATH over
# the binary's RUNPATH).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ap
mkdir -p $OUT
for rep in 1 2; do for v in base exp_ch64 exp_ch256; do
  lib=""; [ $v = base ] || lib=$PWD/odp_amd/lib/$v
  for a in "-c 4" "-c 8"; do
    tag=$(echo "x$a" | tr -d ' -')
    LD_LIBRARY_PATH=$lib timeout -k 10 150 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_${v}_${tag}_$rep.txt 2>&1
    rc=$?; echo "$v odp_pktio_perf $a: $rc $(grep -E 'Maximum' $OUT/pktio_perf_${v}_${tag}_$rep.txt)"
    [ $rc -eq 0 ] || exit $rc
  done
done; done
