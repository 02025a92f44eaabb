#!/bin/bash
# GPU parity, C3 bench, and the C3 launch's HBM read / write bytes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_c3quick.sh || exit 3
rm -rf gpurun_out/pmc_c3_t
CFG=c3 TAG=_t GROUPS_="FETCH_SIZE WRITE_SIZE" BENCH_ARGS="--no-stats" bash tools/pmc.sh || exit 3
python3 tools/pmc_summary.py gpurun_out/pmc_c3_t | python3 -c "
import json,sys;d=json.load(sys.stdin)['odpg_classify_kernel']
print('c3 read MB', d['FETCH_SIZE']*2048/1e6, 'write MB', d['WRITE_SIZE']*1024/1e6)"
