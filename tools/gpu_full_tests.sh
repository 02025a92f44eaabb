#!/bin/bash
# The whole GPU test suite and smoke(), outputs under gpurun_out/<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "gpu tests: $rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke: $rc"; tail -3 $OUT/smoke.log; exit $rc
