#!/bin/bash
# The GPU tests named in FIRST (default: the runtime / boundary tests) verbosely,
# then the whole GPU suite unless ONLY_FIRST is set.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${FIRST:-tests/test_rt_verdict.py tests/test_packet_parse.py tests/test_odp_rt.py tests/test_dist.py \
  tests/test_hash_result.py} -m gpu > $OUT/pytest_new.log 2>&1
rc=$?; echo "first tests: $rc"; tail -25 $OUT/pytest_new.log
[ $rc -eq 0 ] || exit $rc
[ -z "${ONLY_FIRST:-}" ] || exit 0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests -m gpu > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "all gpu tests: $rc"; tail -5 $OUT/pytest_gpu.log
exit $rc
