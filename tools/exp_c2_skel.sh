# C2 counted-launch experiment: per-CoS delivery histogram layouts
# (experiment builds under odp_amd/lib/exp_*)
set -u
export TMPDIR=/tmp
VARIANTS="base exp_s8 exp_s64 exp_nodlv" STEPS=300 bash tools/ab.sh || exit 3
TAG=r2 VARIANTS="base exp_s8 exp_s64 exp_nodlv" STEPS=300 bash tools/ab.sh || exit 3
