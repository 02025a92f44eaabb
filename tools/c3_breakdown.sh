#!/bin/bash
# C3 stage breakdown: kernel strategies and diagnostic floors (one short
# bench per line; any failure ends the script).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu --no-stats --config c3 --steps 50 --warmup 5 "$@" \
    > gpurun_out/c3b_$tag.json 2> gpurun_out/c3b_$tag.err || { tail -5 gpurun_out/c3b_$tag.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/c3b_$tag.json'));print('$tag', d['value'], 'Mpps', d['roofline']['kernel_ms'], 'ms')"
}
run walk --kernel-mode 1
run evalall --kernel-mode 2
run parse --diag parse
run nochk --diag parse-nochk
run l3 --diag l3
run none --diag none
