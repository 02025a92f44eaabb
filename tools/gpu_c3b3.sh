#!/bin/bash
# C3 stage costs of the current kernel: full / no tails / no complex rules,
# parse-only floors; plus SQ instruction counts of the full launch.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in "full base" "full exp_notail" "full exp_noxlist" "parse base" "parse exp_notail"; do
  set -- $cfg; d=$1; v=$2
  if [ "$v" = base ]; then lib=""; else lib="$PWD/odp_amd/lib/$v/libodpg.so"; fi
  ODPG_LIB="$lib" timeout -k 10 200 python bench.py --config c3 --no-cpu --no-stats --diag $d --steps 100 --warmup 10 > gpurun_out/b3_${d}_$v.json 2>gpurun_out/b3_${d}_$v.err || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/b3_${d}_$v.json'));print('$d $v', d['value'], d['roofline']['kernel_ms'])"
done
CFG=c3 TAG=_q GROUPS_="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_VMEM_RD,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES SQ_WAVES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS,SQ_WAVE_CYCLES" BENCH_ARGS="--no-stats" bash tools/pmc.sh || exit 3
python3 tools/pmc_summary.py gpurun_out/pmc_c3_q | python3 -c "
import json,sys;d=json.load(sys.stdin)['odpg_classify_kernel']
print(' '.join('%s=%.0f'%(k.replace('SQ_INSTS_','').replace('SQ_',''),v) for k,v in d.items() if k.endswith('/wave')))"
echo b3-done
