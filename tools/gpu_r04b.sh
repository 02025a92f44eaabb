#!/bin/bash
# Round-4 session B: the whole GPU suite on the key-vector gf kernel, the
# plain-store counter flush and the zero-copy receive path; bench lines
# (c2x, c3 chain vs lazy form vs 4 waves, c2 / c4 counted) and the
# reference odp_pktio_perf through the runtime.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
soft() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -le 1 ] || exit $rc; }
soft pytest timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
tail -3 $OUT/pytest.log
b() {  # tag, env..., then bench args after --
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.load(open('$OUT/bench_$tag.json'));c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'], 'counted', c.get('value'), c.get('kernel_ms'))"
}
b c2x X=1 -- --config c2x
b c3 X=1 -- --config c3
b c3_lazy ODPG_XM_LAZY=1 -- --config c3
b c3_w4 ODPG_LIB=odp_amd/lib/exp_w4/libodpg.so -- --config c3
b c2x_w4 ODPG_LIB=odp_amd/lib/exp_w4/libodpg.so -- --config c2x
b c2 X=1 -- --config c2
b c2_base ODPG_LIB=odp_amd/lib/base/libodpg.so -- --config c2
b c4 X=1 -- --config c4
b c4_base ODPG_LIB=odp_amd/lib/base/libodpg.so -- --config c4
for a in "" "-p" "-c 4"; do
  tag=$(echo "x$a" | tr -d ' -')
  step "pktio_perf $a" timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  grep -E "Maximum|Result" $OUT/pktio_perf_$tag.txt | tail -3
done
