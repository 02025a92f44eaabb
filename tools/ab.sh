#!/bin/bash
# A/B experiment builds (odp_amd/lib/exp_*/libodpg.so, see the Makefile's
# OUT/EXTRA) on one bench config: prints value and kernel time per variant.
# Usage: CFG=c3 DIAG=parse VARIANTS="base exp_notail" bash tools/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CFG="${CFG:-c2}"; DIAG="${DIAG:-full}"; VARIANTS="${VARIANTS:-base}"
STEPS="${STEPS:-50}"
for v in $VARIANTS; do
  if [ "$v" = base ]; then lib=""; else lib="$PWD/odp_amd/lib/$v/libodpg.so"; fi
  ODPG_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu --config $CFG --diag $DIAG \
    --steps $STEPS --warmup 5 ${BENCH_EXTRA:-} > gpurun_out/ab_${CFG}_${DIAG}${TAG:-}_$v.json 2> gpurun_out/ab_${CFG}_${DIAG}${TAG:-}_$v.err \
    || { tail -3 gpurun_out/ab_${CFG}_${DIAG}${TAG:-}_$v.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab_${CFG}_${DIAG}${TAG:-}_$v.json'));c=d.get('with_pktio_counters') or {};print('$CFG $DIAG${TAG:-} $v', d['value'], d['roofline']['kernel_ms'], 'counted', c.get('value'), c.get('kernel_ms'))"
done
