#!/bin/bash
# VALU / SALU per wave of each C3 stage: diag floors and the no-tail build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
G="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
run() { # tag lib diag
  ODPG_LIB="$2" CFG=c3 TAG=_v$1 GROUPS_="$G" BENCH_ARGS="--no-stats --diag $3" bash tools/pmc.sh || exit 3
  python3 tools/pmc_summary.py gpurun_out/pmc_c3_v$1 | python3 -c "
import json,sys;d=json.load(sys.stdin)['odpg_classify_kernel']
print('$1', ' '.join('%s=%.0f'%(k.replace('SQ_INSTS_','').replace('SQ_',''),v) for k,v in d.items() if k.endswith('/wave')))" || exit 3
}
run full "" full
run notail "$PWD/odp_amd/lib/exp_notail/libodpg.so" full
run parse "" parse
run nochk "" parse-nochk
run l3 "" l3
run none "" none
echo c3valu-done
