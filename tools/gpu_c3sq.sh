#!/bin/bash
# C3 SQ counters (full launch and parse-only) + the TCC request-size counters
# this rocprofv3 lists (for calibrating FETCH_SIZE on the C3 access pattern).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_L.txt 2>&1 || exit 3
grep -oE "TCC_EA0_RD[A-Z0-9_]*|TCC_BUBBLE[A-Z0-9_]*|TCC_REQ[A-Z0-9_]*" gpurun_out/rocprof_L.txt | sort -u > gpurun_out/tcc_rd_counters.txt
cat gpurun_out/tcc_rd_counters.txt
bash tools/c3_sq.sh || exit 3
echo c3sq-done
