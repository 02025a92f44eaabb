#!/bin/bash
# Round-5 session n: odp_pktio_perf, lock-free pktio counts and started flag, adaptive mutexes: CPU
# share, then worker splits (-t = transmit workers) and the receive-stage
# profile (ODP_RT_PROF=1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05n
mkdir -p $OUT
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; grep Cpus_allowed_list /proc/self/status; lscpu | grep -E "Model name|Thread|Core|Socket|NUMA node"; } > $OUT/cpu.txt 2>&1
cat $OUT/cpu.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_odp_rt.py tests/test_rt_verdict.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "tests: $rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "-c 4" "-c 6" "-c 8" "-c 8 -t 2" "-c 8 -p"; do
  tag=$(echo "x$a" | tr -d ' -')
  ODP_RT_PROF=1 timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  rc=$?; echo "odp_pktio_perf $a: $rc"; grep -E "Maximum|workers" $OUT/pktio_perf_$tag.txt | tail -3
  [ $rc -eq 0 ] || exit $rc
done
