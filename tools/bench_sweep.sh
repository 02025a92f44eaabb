#!/bin/bash
# Short benches of every single-GPU config plus the diagnostic floors of C2
# (parse-only, loads+stores only). Each GPU step has its own time limit; any
# failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CFGS="${CFGS:-c1 c2 c4}"
DIAGS="${DIAGS:-parse none}"
for c in $CFGS; do
  timeout -k 10 240 python bench.py --no-cpu --config $c --steps 100 --warmup 10 \
    > gpurun_out/b_$c.json 2> gpurun_out/b_$c.err || { tail -5 gpurun_out/b_$c.err; exit 3; }
done
for d in $DIAGS; do
  timeout -k 10 240 python bench.py --no-cpu --config c2 --diag $d --steps 100 --warmup 10 \
    > gpurun_out/b_c2_$d.json 2> gpurun_out/b_c2_$d.err || { tail -5 gpurun_out/b_c2_$d.err; exit 3; }
done
for f in gpurun_out/b_*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', d['value'], 'Mpps', d['roofline']['kernel_ms'], 'ms', d['roofline']['frac'])"
done
