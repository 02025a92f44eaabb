#!/bin/bash
# Where C4's time goes: per-wave start / prologue-end / end stamps
# (tools/exp/l64_times_pro.patch) for C4 and C2, verdict-only and counted.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06q; mkdir -p $OUT
for c in c4 c2; do
  for k in "" "--counted"; do
    w=4; [ $c = c4 ] && w=16
    ODPG_WAVES_PER_WG=$w ODPG_LIB=$PWD/odp_amd/lib/exp_tpro/libodpg.so timeout -k 10 120 \
      python tools/wave_times.py --config $c $k > $OUT/times_$c$k.json 2> $OUT/times_$c$k.err || exit $?
    python3 -c "import json;d=json.load(open('$OUT/times_$c$k.json'));print('$c$k', d['kernel_span_us'], d['prologue_us'], d['end_us'], d['by_tiles'])"
  done
done
