#!/bin/bash
# Round-4 session H: C3 stage isolation (hit map / tails / walk compiled out)
# of round 3's gf kernel against this round's, 4 vs 5 waves; odp_pktio_perf
# with the pooled packet allocator.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04h
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
b() {
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu --runs 3 "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_$tag.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], 'counted', c.get('kernel_ms'))"
}
L=odp_amd/lib
for a in "" "-c 4"; do
  tag=$(echo "x$a" | tr -d ' -')
  step "pktio_perf $a" timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  grep -E "Maximum|Result" $OUT/pktio_perf_$tag.txt | tail -3
done
for v in base r3_nohm r3_notail r3_nowalk cur_w4 cur_nohm cur_notail cur_nowalk; do
  b c3_$v ODPG_LIB=$L/$v/libodpg.so -- --config c3
done
b c3_cur X=1 -- --config c3
b c2x_cur X=1 -- --config c2x
