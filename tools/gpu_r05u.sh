#!/bin/bash
# Round-5 session u: L2 request-size mix (FETCH_SIZE's 64-B tally), TA / TCP
# stalls and L2 hit rates of the descriptor kernel (C3) against the lean
# kernel (C2), one --pmc pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFGS="c3 c2" TAG=_r05u BENCH_ARGS=--no-stats \
GROUPS_="TCC_EA0_RDREQ,TCC_EA0_RDREQ_128B,TCC_EA0_RDREQ_64B,TCC_EA0_RDREQ_32B TA_TA_BUSY,TA_ADDR_STALLED_BY_TC_CYCLES,TCP_TCC_READ_REQ,TCP_TCC_READ_REQ_LATENCY,TCP_PENDING_STALL_CYCLES,TCP_TCP_TA_DATA_STALL_CYCLES TCC_HIT,TCC_MISS,TCC_REQ,TCC_READ FETCH_SIZE" \
  bash tools/gpu_sq.sh
