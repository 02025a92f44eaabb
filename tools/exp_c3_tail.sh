# C3 occupancy x tail variant A/B (experiment builds under odp_amd/lib/exp_*)
set -u
export TMPDIR=/tmp
CFG=c3 VARIANTS="base exp_g5 exp_g5c exp_g5s8" STEPS=50 BENCH_EXTRA=--no-stats bash tools/ab.sh || exit 3
CFG=c3 TAG=r2 VARIANTS="base exp_g5 exp_g5c exp_g5s8" STEPS=50 BENCH_EXTRA=--no-stats bash tools/ab.sh || exit 3
