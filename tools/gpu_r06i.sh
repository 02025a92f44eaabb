#!/bin/bash
# SQ counters of the current descriptor kernel (C2x, C3) and the counted
# S64 launch at 6 waves (exp_s64c6) against 5.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFGS="c2x c3" TAG=_r06i GROUPS_="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS" bash tools/gpu_sq.sh || exit $?
CFG=c2x VARIANTS="base exp_s64c6 base exp_s64c6" TAG=r06i bash tools/ab.sh
