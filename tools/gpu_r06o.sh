#!/bin/bash
# C3 register-spill fix (parse_fast_gf in its pre-e990c72 form, exp_prs) and
# the branch-free CoS-keyed walk of the lean kernel (exp_hwbf): parity tests on
# each variant library, A/B against the record library (base), C3 HBM
# counters of exp_prs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06o; mkdir -p $OUT
ODPG_LIB=$PWD/odp_amd/lib/exp_prs/libodpg.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py tests/test_gpu_parity.py -m gpu > $OUT/pytest_prs.log 2>&1
rc=$?; echo "tests prs: $rc"; tail -2 $OUT/pytest_prs.log; [ $rc -eq 0 ] || exit $rc
ODPG_LIB=$PWD/odp_amd/lib/exp_hwbf/libodpg.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_counters.py -m gpu > $OUT/pytest_hwbf.log 2>&1
rc=$?; echo "tests hwbf: $rc"; tail -2 $OUT/pytest_hwbf.log; [ $rc -eq 0 ] || exit $rc
CFG=c4 VARIANTS="base exp_hwbf base exp_hwbf" TAG=r06o bash tools/ab.sh || exit $?
CFG=c3 VARIANTS="base exp_prs base exp_prs" TAG=r06o bash tools/ab.sh || exit $?
CFG=c2x VARIANTS="base exp_prs base exp_prs" TAG=r06o bash tools/ab.sh || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  ODPG_LIB=$PWD/odp_amd/lib/exp_prs/libodpg.so timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_c3/pmc_$c -o run \
    -- python3 bench.py --no-cpu --no-stats --config c3 --others none --steps 20 --warmup 2 --runs 1 > $OUT/pmc_c3_$c.log 2>&1 || exit $?
done
python tools/pmc_summary.py $OUT/pmc_c3 > $OUT/pmc_c3_summary.json; tail -8 $OUT/pmc_c3_summary.json
