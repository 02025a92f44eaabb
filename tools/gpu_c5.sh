#!/bin/bash
# GPU parity suite, then the C5 bench lines (hash and LPM) with the CPU baseline.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for m in hash lpm; do
  timeout -k 10 300 python bench.py --config c5 --fwd-mode $m --steps 50 --warmup 5 > gpurun_out/c5_$m.json 2> gpurun_out/c5_$m.err || exit $?
  cat gpurun_out/c5_$m.json
done
