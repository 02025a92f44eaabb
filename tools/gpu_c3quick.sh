#!/bin/bash
# GPU parity tests, then the C3 bench (no CPU baseline) and its SQ VALU count.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --no-cpu --steps 100 --warmup 10 > gpurun_out/c3q.json 2> gpurun_out/c3q.err || exit 3
python3 -c "import json;d=json.load(open('gpurun_out/c3q.json'));print('c3', d['value'], d['roofline']['kernel_ms'], d['with_pktio_counters']['kernel_ms'])"
for v in ${VARIANTS:-}; do
  ODPG_LIB=$PWD/odp_amd/lib/$v/libodpg.so timeout -k 10 300 python bench.py --config c3 --no-cpu --no-stats --steps 100 --warmup 10 > gpurun_out/c3q_$v.json 2> gpurun_out/c3q_$v.err || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/c3q_$v.json'));print('$v', d['value'], d['roofline']['kernel_ms'])"
done
if [ -n "${SQ:-}" ]; then
  CFG=c3 TAG=_q GROUPS_="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_VMEM_RD,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES" BENCH_ARGS="--no-stats" bash tools/pmc.sh || exit 3
  python3 tools/pmc_summary.py gpurun_out/pmc_c3_q | python3 -c "
import json,sys;d=json.load(sys.stdin)['odpg_classify_kernel']
print(' '.join('%s=%.0f'%(k.replace('SQ_INSTS_','').replace('SQ_',''),v) for k,v in d.items() if k.endswith('/wave')))"
fi
echo quick-done
