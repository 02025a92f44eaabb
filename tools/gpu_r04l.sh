#!/bin/bash
# Round-4 session L: C3 tail-pass owners from an LDS mark map (main) vs the
# bpermute search (x_nomarks); cost split (owner search / own units / pass
# attribution compiled out); counted launches with the load-free flush.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04l
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
  b c3_main_$r X=1 -- --config c3
  for v in x_nomarks x_notailw x_no_owner x_no_own x_no_scan x_nt; do
    b c3_${v}_$r ODPG_LIB=$L/$v/libodpg.so -- --config c3
  done
done
# counted launches: the flush's identity-column loop without loads
b c2 X=1 -- --config c2
b c2x X=1 -- --config c2x
b c4 X=1 -- --config c4
step "pytest counters" timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_counters.py tests/test_gf_kernel.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
