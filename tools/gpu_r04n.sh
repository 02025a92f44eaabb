#!/bin/bash
# Round-4 session N: which tail-pass change breaks the C3 gf parity (mark
# map / whole-word last units), each variant through the gf parity test.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
L=odp_amd/lib
for v in x_nomarks x_notailw main; do
  lib=$L/$v/libodpg.so; [ $v = main ] && lib=$L/libodpg.so
  ODPG_LIB=$lib timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gf_kernel.py > $OUT/pytest_$v.log 2>&1
  echo "$v: $?"; tail -1 $OUT/pytest_$v.log
done
