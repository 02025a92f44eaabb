#!/bin/bash
# C3 kernel time vs launch grid (ODPG_GRID_CAP lifts the resident-grid clamp).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for g in ${GRIDS:-default 1024 1366 2048 4096}; do
  if [ "$g" = default ]; then e=""; else e="ODPG_GRID_CAP=$g"; fi
  env $e timeout -k 10 200 python bench.py --config c3 --no-cpu --no-stats --steps 100 --warmup 10 > gpurun_out/grid_$g.json 2>gpurun_out/grid_$g.err || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/grid_$g.json'));print('grid $g', d['value'], d['roofline']['kernel_ms'])"
done
echo grid-done
