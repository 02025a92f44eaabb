#!/bin/bash
# Bench lines of the other configs (no CPU baseline): C1, C4, C5 hash / LPM, TX.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in "c1" "c4" "c5 --fwd-mode hash" "c5 --fwd-mode lpm" "tx"; do
  set -- $c; tag=$(echo "$c" | tr -d ' -' )
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps 100 --warmup 10 > gpurun_out/o_$tag.json 2> gpurun_out/o_$tag.err || { tail -3 gpurun_out/o_$tag.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/o_$tag.json'));print('$tag', d['value'], d['unit'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
echo others-done
