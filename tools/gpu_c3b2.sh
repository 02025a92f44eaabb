#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for d in full parse parse-nochk; do
  for v in base exp_notail exp_seg3; do
    if [ "$v" = base ]; then lib=""; else lib="$PWD/odp_amd/lib/$v/libodpg.so"; fi
    ODPG_LIB="$lib" timeout -k 10 200 python bench.py --config c3 --no-cpu --no-stats --diag $d --steps 100 --warmup 10 > gpurun_out/b2_${d}_$v.json 2>gpurun_out/b2_${d}_$v.err || exit 3
    python3 -c "import json;d=json.load(open('gpurun_out/b2_${d}_$v.json'));print('$d $v', d['value'], d['roofline']['kernel_ms'])"
  done
done
G="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA"
CFG=c3 TAG=_w GROUPS_="$G" BENCH_ARGS="--no-stats" bash tools/pmc.sh || exit 3
python3 tools/pmc_summary.py gpurun_out/pmc_c3_w | python3 -c "
import json,sys;d=json.load(sys.stdin)['odpg_classify_kernel']
print(' '.join('%s=%.0f'%(k.replace('SQ_',''),v) for k,v in d.items() if k.endswith('/wave') or k=='SQ_BUSY_CYCLES'))"
echo b2-done
