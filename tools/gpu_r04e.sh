#!/bin/bash
# Round-4 session E: age-aware tile counts per CU workgroup slot on C2 / C1
# (ODPG_L64_SLOTS), verdict-only and counted; C3 / C2x on the current gf
# kernel vs round 3's library; parity of the lean and gf kernels.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04e
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
soft() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -le 1 ] || exit $rc; }
soft pytest timeout -k 10 600 python -u -m pytest tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_counters.py \
  -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
b() {  # tag, env..., then bench args after --
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_$tag.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'], 'counted', c.get('value'), c.get('kernel_ms'))"
}
L=odp_amd/lib
b c2 X=1 -- --config c2
for v in 3,3,2,2,2,2,2 3,3,3,2,2,2,1 4,3,3,2,2,1,1 3,3,3,3,2,1,1 4,4,2,2,2,1,1; do
  b c2_s$v ODPG_L64_SLOTS=$v -- --config c2 --no-stats
done
for v in 3,3,3,3,2,2 4,3,3,2,2,2 3,3,3,3,3,1; do
  b c2cnt_s$v ODPG_L64_SLOTS=$v -- --config c2
done
b c1 X=1 -- --config c1 --no-stats
for v in 3,2,2,2,2,2,2,1 3,3,2,2,2,2,1,1 3,3,3,2,2,1,1,1; do
  b c1_s$v ODPG_L64_SLOTS=$v -- --config c1 --no-stats
done
step "wave_times s" env ODPG_LIB=$L/exp_times/libodpg.so ODPG_L64_SLOTS=3,3,3,2,2,2,1 timeout -k 10 120 python tools/wave_times.py --config c2 > $OUT/wave_times_s.json 2> $OUT/wave_times_s.err
cut -c1-700 $OUT/wave_times_s.json
b c3 X=1 -- --config c3
b c3_base ODPG_LIB=$L/base/libodpg.so -- --config c3
b c2x X=1 -- --config c2x
