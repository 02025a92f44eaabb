#!/bin/bash
# Round-4 session I: hit map with the chain-free groups in a loop of their
# own and (wide maps) the zero entry on a miss; gf parity; odp_pktio_perf
# with the receive-burst profile.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
b() {
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu --runs 3 "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_$tag.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], 'counted', c.get('kernel_ms'))"
}
step "pytest gf" timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gf_kernel.py tests/test_xmask_emul.py > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
L=odp_amd/lib
for a in "" "-c 4"; do
  tag=$(echo "x$a" | tr -d ' -')
  step "pktio_perf $a" env ODP_RT_PROF=1 timeout -k 10 240 oracle/_ref/odp_pktio_perf -v $a > $OUT/pktio_perf_$tag.txt 2>&1
  grep -E "Maximum|odp_rt:" $OUT/pktio_perf_$tag.txt | tail -4
done
for r in 1 2; do
  b c3_new_$r X=1 -- --config c3
  b c3_z16_$r ODPG_LIB=$L/new_z16/libodpg.so -- --config c3
  b c3_w4_$r ODPG_LIB=$L/new_w4/libodpg.so -- --config c3
  b c3_old_$r ODPG_LIB=$L/exp_ecfc2e4/libodpg.so -- --config c3
  b c2x_new_$r X=1 -- --config c2x
  b c2x_z2_$r ODPG_LIB=$L/new_z2/libodpg.so -- --config c2x
done
