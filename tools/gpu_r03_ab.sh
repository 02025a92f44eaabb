#!/bin/bash
# C3 early tails (tails before the next windows): parity, A/B, HBM counters.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py -m gpu > gpurun_out/pytest_first.log 2>&1
rc=$?; echo "first tests: $rc"; tail -3 gpurun_out/pytest_first.log; [ $rc -eq 0 ] || exit $rc
CFG=c3 BENCH_EXTRA="--no-cpu" VARIANTS="base exp_noearly base exp_noearly" bash tools/ab.sh || exit $?
for v in base; do
  lib=""; [ $v = base ] || lib=$PWD/odp_amd/lib/$v/libodpg.so
  for c in FETCH_SIZE WRITE_SIZE; do
    ODPG_LIB="$lib" timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc3b_$v/pmc_$c -o run \
      -- python3 bench.py --no-cpu --no-stats --config c3 --steps 20 --warmup 2 > gpurun_out/pmc3b_${v}_$c.log 2>&1
    rc=$?; echo "pmc $v $c: $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
