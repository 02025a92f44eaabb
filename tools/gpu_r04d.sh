#!/bin/bash
# Round-4 session D: lean-kernel grid sweep on C2 (the drain after the last
# loads), wave end-time profiles, odp_pktio_perf through the zero-copy
# receive path, C3 SQ counters.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04d
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
L=odp_amd/lib
for g in 1024 1280 1536 1792 2048; do
  step "c2 grid $g" env ODPG_LIB=$L/exp_gridenv/libodpg.so ODPG_L64_GRID=$g timeout -k 10 300 python bench.py --no-cpu --config c2 \
    > $OUT/bench_c2_g$g.json 2> $OUT/bench_c2_g$g.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_c2_g$g.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('grid $g', d['value'], d['roofline']['kernel_ms'], 'counted', c.get('kernel_ms'))"
  step "wave_times $g" env ODPG_LIB=$L/exp_gridenv/libodpg.so ODPG_L64_GRID=$g timeout -k 10 120 python tools/wave_times.py --config c2 \
    > $OUT/wave_times_c2_g$g.json 2> $OUT/wave_times_c2_g$g.err
  cut -c1-600 $OUT/wave_times_c2_g$g.json
done
for a in "" "-p" "-c 4"; do
  tag=$(echo "x$a" | tr -d ' -')
  step "pktio_perf $a" timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  grep -E "Maximum|Result" $OUT/pktio_perf_$tag.txt | tail -3
done
step "sq c3" env CFGS=c3 TAG=_r04d bash tools/gpu_sq.sh
