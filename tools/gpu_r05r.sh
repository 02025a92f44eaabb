#!/bin/bash
# Round-5 session r: SQ counters + FETCH/WRITE of the shipped kernels (after
# the experiment strip) for C2x, C3 (descriptor kernel) and C4 (lean kernel,
# CoS-keyed cuckoo), one --pmc pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFGS="c2x c3 c4" TAG=_r05r \
GROUPS_="FETCH_SIZE WRITE_SIZE SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS SQ_WAVES,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE" \
  bash tools/gpu_sq.sh
