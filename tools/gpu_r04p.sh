#!/bin/bash
# Round-4 session P: new gf defaults (paired probes, mark map, masked last
# units) vs the tail pass after the walk (z_e2): time and HBM traffic on
# C3; C2x verdict-only / counted at 4 and 5 waves.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04p
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
b() {
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu --runs 3 "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_$tag.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], 'counted', c.get('kernel_ms'))"
}
step "pytest gf" timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gf_kernel.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
L=odp_amd/lib
for v in main z_e2; do
  lib=$L/$v/libodpg.so; [ $v = main ] && lib=$L/libodpg.so
  for c in FETCH_SIZE WRITE_SIZE; do
    step "pmc $v $c" env ODPG_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$v/pmc_$c -o run \
      -- python3 bench.py --no-cpu --no-stats --config c3 --steps 20 --warmup 2 --runs 1 > $OUT/pmc_${v}_$c.log 2>&1
  done
  python tools/pmc_summary.py $OUT/pmc_$v > $OUT/pmc_${v}_summary.json
  grep -A3 clsgf $OUT/pmc_${v}_summary.json | head -8
done
for r in 1 2; do
  b c3_main_$r X=1 -- --config c3
  b c3_z_e2_$r ODPG_LIB=$L/z_e2/libodpg.so -- --config c3
  b c2x_main_$r X=1 -- --config c2x
  b c2x_w_v4_$r ODPG_LIB=$L/w_v4/libodpg.so -- --config c2x
  b c2x_w_c5_$r ODPG_LIB=$L/w_c5/libodpg.so -- --config c2x
done
