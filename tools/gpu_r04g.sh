#!/bin/bash
# Round-4 session G: C3 bisect of the gf kernel against round 3's library
# (commits of this round, the tag-shift code compiled out, 4 vs 5 waves).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04g
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
b() {
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu --runs 3 "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_$tag.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], 'counted', c.get('kernel_ms'))"
}
L=odp_amd/lib
for r in 1 2; do
  for v in base exp_1bf84c4 exp_ecfc2e4 exp_notag5 exp_notag4 exp_w5; do
    b c3_${v}_$r ODPG_LIB=$L/$v/libodpg.so -- --config c3
  done
  b c3_cur_$r X=1 -- --config c3
  for v in exp_ecfc2e4 exp_notag5 exp_w5; do
    b c2x_${v}_$r ODPG_LIB=$L/$v/libodpg.so -- --config c2x
  done
  b c2x_cur_$r X=1 -- --config c2x
done
