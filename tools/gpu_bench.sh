#!/bin/bash
# Bench lines for several configs (CFGS, default "c2 c3"), each with the
# end-to-end host path (--e2e) and the CPU baseline, then the ODP-facing
# example bench (odp_bench_cls_gpu: recv_batch vs raw odpg_classify over
# rotating HBM buffers). Every step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for c in ${CFGS:-c2 c3}; do
  timeout -k 10 400 python bench.py --config $c ${BENCH_ARGS---e2e} > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  rc=$?; echo "bench $c: $rc"; cat $OUT/bench_$c.json; tail -3 $OUT/bench_$c.err
  [ $rc -eq 0 ] || exit $rc
done
if [ -z "${NO_EXAMPLE:-}" ]; then
  timeout -k 10 300 odp_amd/lib/odp_bench_cls_gpu > $OUT/odp_bench_cls_gpu.txt 2>&1
  rc=$?; echo "odp_bench_cls_gpu: $rc"; tail -6 $OUT/odp_bench_cls_gpu.txt
  exit $rc
fi
