#!/bin/bash
# Round-4 session J: new gf defaults (zero entry, 4 waves for wide / counted
# launches): parity, C3 / C2x bench lines, SQ instruction counts of C3 with
# the tails / hit map / walk compiled out; odp_pktio_perf receive profile.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
step() { local n=$1; shift; "$@"; local rc=$?; echo "$n: $rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
b() {
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  step "bench $tag" env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu --runs 3 "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  python -c "import json;d=json.loads([l for l in open('$OUT/bench_$tag.json') if l.strip()][0]);c=d.get('with_pktio_counters') or {};print('$tag', d['value'], d['roofline']['kernel_ms'], 'counted', c.get('kernel_ms'))"
}
step "pytest gf" timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gf_kernel.py tests/test_xmask_emul.py tests/test_counters.py > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
for a in "" "-c 4"; do
  tag=$(echo "x$a" | tr -d ' -')
  step "pktio_perf $a" env ODP_RT_PROF=1 timeout -k 10 240 oracle/_ref/odp_pktio_perf -v $a > $OUT/pktio_perf_$tag.txt 2>&1
  grep -E "Maximum|odp_rt:" $OUT/pktio_perf_$tag.txt | tail -4
done
b c3 X=1 -- --config c3
b c2x X=1 -- --config c2x
L=odp_amd/lib
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"
for v in main x_nt x_nh x_nw; do
  lib=$L/$v/libodpg.so; [ $v = main ] && lib=$L/libodpg.so
  step "sq $v" env ODPG_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $OUT/sq_$v -o run \
      -- python3 bench.py --no-cpu --no-stats --config c3 --steps 20 --warmup 2 --runs 1 > $OUT/sq_$v.log 2>&1
  python tools/pmc_summary.py $OUT/sq_$v > $OUT/sq_$v.json 2>&1
  python -c "
import json;d=json.load(open('$OUT/sq_$v.json'))
for k,x in d.items():
  if 'clsgf' in k: print('$v', k[:30], {a.split('/')[0][8:]:round(b) for a,b in x.items() if a.endswith('/wave')})"
done
