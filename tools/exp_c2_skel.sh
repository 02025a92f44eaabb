# C2 counted-launch experiment: per-CoS delivery histogram layouts
# (experiment builds under odp_amd/lib/exp_*)
set -u
export TMPDIR=/tmp
VARIANTS="base exp_nf exp_bnone exp_both" STEPS=300 bash tools/ab.sh || exit 3
TAG=r2 VARIANTS="base exp_nf exp_bnone exp_both" STEPS=300 bash tools/ab.sh || exit 3
