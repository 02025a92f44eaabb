#!/bin/bash
# Round-5 session ag: C3 counters with nontemporal tail loads (descriptor-kernel GPU
# tests, then C3's request-size / TA / TCP / L2 counters and SQ counters.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ag
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gf_kernel.py -m gpu > gpurun_out/r05ag/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 gpurun_out/r05ag/pytest.log; [ $rc -eq 0 ] || exit $rc
CFGS="c3" TAG=_r05ag BENCH_ARGS=--no-stats \
GROUPS_="TCC_EA0_RDREQ,TCC_EA0_RDREQ_128B,TCC_EA0_RDREQ_64B,TCC_EA0_RDREQ_32B TA_TA_BUSY,TA_ADDR_STALLED_BY_TC_CYCLES,TCP_TCC_READ_REQ,TCP_TCC_READ_REQ_LATENCY,TCP_PENDING_STALL_CYCLES,TCP_TCP_TA_DATA_STALL_CYCLES TCC_HIT,TCC_MISS,TCC_REQ,TCC_READ FETCH_SIZE WRITE_SIZE SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS SQ_WAVES,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE" \
  bash tools/gpu_sq.sh
