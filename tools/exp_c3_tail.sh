# C3 tail reduction A/B: balanced segmented (base) vs per-frame passes
# (exp_coop) vs no tail sums at all (exp_notail, wrong verdicts: cost only)
set -u
export TMPDIR=/tmp
CFG=c3 DIAG=parse VARIANTS="base exp_coop exp_notail" STEPS=50 BENCH_EXTRA=--no-stats bash tools/ab.sh || exit 3
CFG=c3 DIAG=parse-nochk VARIANTS="base" STEPS=50 BENCH_EXTRA=--no-stats bash tools/ab.sh || exit 3
