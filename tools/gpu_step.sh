set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
FIRST="tests/test_gf_kernel.py" ONLY_FIRST=1 bash tools/gpu_tests.sh && \
CFG=c3 BENCH_EXTRA=--no-stats VARIANTS="base exp_notail exp_nohm exp_w6" bash tools/ab.sh
