#!/bin/bash
# GPU parity tests, then the C2 bench (verdict-only and counted launches).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --steps 300 --warmup 20 > gpurun_out/c2q.json 2> gpurun_out/c2q.err || exit 3
python3 -c "import json;d=json.load(open('gpurun_out/c2q.json'));print('c2', d['value'], d['roofline']['kernel_ms'], 'counted', d['with_pktio_counters']['kernel_ms'])"
done
echo quick-done
