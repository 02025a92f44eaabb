set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
FIRST="tests/test_gf_kernel.py tests/test_gpu_parity.py" ONLY_FIRST=1 bash tools/gpu_tests.sh && \
CFG=c3 BENCH_EXTRA="--no-stats" VARIANTS="base exp_b512 exp_pipe0 exp_w4 base" bash tools/ab.sh
