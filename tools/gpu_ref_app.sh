# The reference's example/classifier (oracle/_ref, built unmodified against
# include/ by oracle/ref_apps.mk) on udp64.pcap with its run-script rule
set -u
mkdir -p gpurun_out
python - <<'PY'
import sys
sys.path[:0] = ["tests"]
from helpers import GOLDEN
from test_odp_rt import write_pcap
write_pcap("gpurun_out/udp64.pcap", [bytes.fromhex(h) for h in GOLDEN["pcap"]["classifier_udp64"]])
PY
timeout -k 10 90 ./oracle/_ref/odp_classifier -t 2 -i pcap:in=gpurun_out/udp64.pcap -m 0 \
  -p "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1" -P -C "queue1:100" -C "DefaultCos:100" \
  > gpurun_out/ref_odp_classifier.txt 2>&1
rc=$?; echo "exit status $rc" >> gpurun_out/ref_odp_classifier.txt; tail -n 25 gpurun_out/ref_odp_classifier.txt; exit $rc
