#!/bin/bash
# Round-5 session a: C3 breakdown (experiment builds), SQ counters of the C4
# lean kernel, and the counted wave-times run that
# segfaulted in round 4 (r04c), under faulthandler.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05a
ODPG_LIB=$PWD/odp_amd/lib/exp_times/libodpg.so timeout -k 10 120 python -X faulthandler tools/wave_times.py --counted \
  > gpurun_out/r05a/wave_times_counted.json 2> gpurun_out/r05a/wave_times_counted.err
echo "wave_times counted: $?"; tail -25 gpurun_out/r05a/wave_times_counted.err
for r in 1 2; do
  CFG=c3 TAG=_$r BENCH_EXTRA=--no-cpu VARIANTS="base exp_nohmwalk exp_notail exp_bare exp_sweep exp_w5" bash tools/ab.sh || exit $?
done
CFGS=c4 TAG=_r05a bash tools/gpu_sq.sh || exit $?
