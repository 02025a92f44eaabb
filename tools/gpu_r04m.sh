#!/bin/bash
# Round-4 session M: paired chain-free group probes (C3, C2x); counted gf
# launches with the histogram adds / the flush compiled out (C2x, C3).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04m
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
  for cfg in c3 c2x; do
    b ${cfg}_main_$r X=1 -- --config $cfg
    for v in y_pair y_nobin y_noflush; do
      b ${cfg}_${v}_$r ODPG_LIB=$L/$v/libodpg.so -- --config $cfg
    done
  done
done
