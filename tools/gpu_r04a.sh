#!/bin/bash
# Round-4 session A: parity of the chain-bit hit map + tag-shifted register
# parse (gf kernel), SQ counters of C2x on HEAD~ (lib/base) and on the new
# build, bench lines for c2x / c3 on both. First failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_gf_kernel.py tests/test_gpu_parity.py -k "gf or c2x or c3" \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
tail -3 $OUT/pytest.log
for v in new base; do
  lib=""; [ $v = base ] && lib=odp_amd/lib/base/libodpg.so
  for cfg in c2x c3; do
    step "bench $cfg $v" env ODPG_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --config $cfg > $OUT/bench_${cfg}_$v.json 2> $OUT/bench_${cfg}_$v.err
    cat $OUT/bench_${cfg}_$v.json
  done
done
step "sq base" env ODPG_LIB=odp_amd/lib/base/libodpg.so CFGS=c2x TAG=_base bash tools/gpu_sq.sh
step "sq new" env CFGS=c2x TAG=_new bash tools/gpu_sq.sh
