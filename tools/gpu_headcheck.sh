#!/bin/bash
# Check of the committed tree as the driver runs it at round end: the GPU
# suite, smoke() and the default bench line, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06head}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest: $rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke: $rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?; echo "bench: $rc"; cut -c1-300 $OUT/bench_default.json
