#!/bin/bash
# Round-4 session F: gf kernel with the window shift inside the fast branch
# (no spills at 5 waves): parity, then C3 / C2x at 4 vs 5 waves per SIMD vs
# round 3's library, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
soft() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -le 1 ] || exit $rc; }
soft pytest timeout -k 10 600 python -u -m pytest tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_counters.py \
  tests/test_rt_verdict.py -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
b() {  # tag, env..., then bench args after --
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_$tag.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'], 'counted', c.get('value'), c.get('kernel_ms'))"
}
L=odp_amd/lib
for r in 1 2; do
  b c3_w4_$r X=1 -- --config c3
  b c3_w5_$r ODPG_LIB=$L/exp_w5/libodpg.so -- --config c3
  b c3_base_$r ODPG_LIB=$L/base/libodpg.so -- --config c3
  b c2x_$r X=1 -- --config c2x
  b c2x_w5_$r ODPG_LIB=$L/exp_w5/libodpg.so -- --config c2x
done
b c3_lazy X=1 ODPG_XM_LAZY=1 -- --config c3
b c3_w5_lazy ODPG_XM_LAZY=1 ODPG_LIB=$L/exp_w5/libodpg.so -- --config c3
