# C2 lean-kernel ablations (experiment builds under odp_amd/lib/exp_*)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lean_parity.log 2>&1; rc=$?; tail -3 gpurun_out/lean_parity.log; [ $rc -eq 0 ] || exit 3
VARIANTS="base exp_nomatch exp_skel" STEPS=200 bash tools/ab.sh || exit 3
TAG=r2 VARIANTS="base exp_nomatch exp_skel" STEPS=200 bash tools/ab.sh || exit 3
CFG=c4 VARIANTS="base" STEPS=200 bash tools/ab.sh || exit 3
CFG=c1 VARIANTS="base" STEPS=200 bash tools/ab.sh || exit 3
