#!/bin/bash
# Round-5 session k: where odp_pktio_perf -c 8 loses its rate: the box's CPU
# share, then worker splits (-t = transmit workers) and the receive-stage
# profile (ODP_RT_PROF=1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05k
mkdir -p $OUT
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; grep Cpus_allowed_list /proc/self/status; lscpu | grep -E "Model name|Thread|Core|Socket|NUMA node"; } > $OUT/cpu.txt 2>&1
cat $OUT/cpu.txt
for a in "-c 6" "-c 8 -t 2" "-c 8 -t 6" "-c 8"; do
  tag=$(echo "x$a" | tr -d ' -')
  ODP_RT_PROF=1 timeout -k 10 240 oracle/_ref/odp_pktio_perf $a > $OUT/pktio_perf_$tag.txt 2>&1
  rc=$?; echo "odp_pktio_perf $a: $rc"; grep -E "Maximum|workers" $OUT/pktio_perf_$tag.txt | tail -3
  [ $rc -eq 0 ] || exit $rc
done
