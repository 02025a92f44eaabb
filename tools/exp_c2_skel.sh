# C2 lean-kernel experiments (experiment builds under odp_amd/lib/exp_*)
set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "lean64 or stride64 or c2 or c1 or raised" > gpurun_out/lean_parity.log 2>&1; rc=$?; tail -3 gpurun_out/lean_parity.log; [ $rc -eq 0 ] || exit 3
VARIANTS="base exp_w8 exp_skel" STEPS=200 bash tools/ab.sh || exit 3
for g in 1024 1536 2048; do ODPG_L64_GRID=$g TAG=g$g VARIANTS="exp_g exp_w8 exp_skel" STEPS=200 bash tools/ab.sh || exit 3; done
CFG=c4 VARIANTS="base exp_w8" STEPS=200 bash tools/ab.sh || exit 3
