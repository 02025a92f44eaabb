set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
ODPG_LIB=$PWD/odp_amd/lib/exp_p1w4/libodpg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gf_kernel.py -m gpu > gpurun_out/pytest_sweep.log 2>&1; echo "sweep tests: $?"; tail -2 gpurun_out/pytest_sweep.log
CFG=c3 BENCH_EXTRA="--no-stats" VARIANTS="base exp_p1w5 exp_p1w4 exp_p0w5 base" bash tools/ab.sh
