#!/bin/bash
# Round-4 session C: gf kernel occupancy / probe A/B on C3, lean-kernel wave
# end times (C2 verdict-only vs counted), counted-occupancy A/B, C4 wall vs
# event gap, odp_pktio_perf through the zero-copy receive path, C3 SQ counters.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
soft() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -le 1 ] || exit $rc; }
soft pytest timeout -k 10 600 python -u -m pytest tests/test_gf_kernel.py tests/test_gpu_parity.py tests/test_counters.py \
  tests/test_rt_verdict.py tests/test_odp_rt.py tests/test_dist.py -m gpu -q --maxfail=5 --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
b() {  # tag, env..., then bench args after --
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_$tag.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'], 'enq', d.get('host_enqueue_ms_per_step'), 'counted', c.get('value'), c.get('kernel_ms'))"
}
L=odp_amd/lib
b c3 X=1 -- --config c3
b c3_g8_5 ODPG_LIB=$L/exp_g8_5/libodpg.so -- --config c3
b c3_nocond ODPG_LIB=$L/exp_nocond/libodpg.so -- --config c3
b c3_lazy ODPG_XM_LAZY=1 -- --config c3
b c3_base ODPG_LIB=$L/base/libodpg.so -- --config c3
b c2x X=1 -- --config c2x
b c2 X=1 -- --config c2
b c2_cnt7 ODPG_LIB=$L/exp_cnt7/libodpg.so -- --config c2
b c2_cnt8 ODPG_LIB=$L/exp_cnt8/libodpg.so -- --config c2
b c4 X=1 -- --config c4
b c4_base ODPG_LIB=$L/base/libodpg.so -- --config c4
for m in "" "--counted"; do
  step "wave_times c2 $m" env ODPG_LIB=$L/exp_times/libodpg.so timeout -k 10 120 python tools/wave_times.py --config c2 $m > $OUT/wave_times_c2$m.json 2> $OUT/wave_times_c2$m.err
  cut -c1-400 $OUT/wave_times_c2$m.json
done
for a in "" "-p" "-c 4"; do
  tag=$(echo "x$a" | tr -d ' -')
  step "pktio_perf $a" timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  grep -E "Maximum|Result" $OUT/pktio_perf_$tag.txt | tail -3
done
step "sq c3" env CFGS=c3 TAG=_r04c bash tools/gpu_sq.sh
