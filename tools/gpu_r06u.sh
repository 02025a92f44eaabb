#!/bin/bash
# odp_pktio_perf (-c 8, and 1 + 1) with the runtime's spin waits yielding
# after 2^15 pauses (base) against pause-only waits (exp_spin), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06u; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_odp_rt.py tests/test_rt_verdict.py tests/test_group.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "runtime tests: $rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base exp_spin; do
    lp=""; [ $v = base ] || lp=$PWD/odp_amd/lib/$v
    for a in "-c 8" ""; do
      tag=$(echo "x$a" | tr -d ' -')
      LD_LIBRARY_PATH=$lp timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pp_${v}_${tag}_$r.txt 2>&1 || exit $?
      echo "$v $a round $r: $(grep Maximum $OUT/pp_${v}_${tag}_$r.txt)"
    done
  done
done
