#!/bin/bash
# Round-4 sessions K + L in one call.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r04k.sh && bash tools/gpu_r04l.sh
