"""test/performance's classifier cases on the library
(examples/odp_bench_cls_gpu.c): odp_bench_pktio_sp's
cls_pmr_create timing over the odp_cls_* API, the per-generation rule-table
rebuild, and device-resident odpg_pktio_recv_batch throughput with every
verdict checked."""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
EXAMPLE = os.path.join(os.path.dirname(HERE), "odp_amd", "lib", "odp_bench_cls_gpu")


def test_bench_example_builds():
    assert os.access(EXAMPLE, os.X_OK)


def test_bench_example_rejects_bad_args():
    r = subprocess.run([EXAMPLE, "-n", "0"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "must be > 0" in r.stderr


@pytest.mark.gpu
def test_bench_example_run():
    batch, steps = 1 << 16, 10
    r = subprocess.run([EXAMPLE, "-n", "32", "-r", "50", "-b", str(batch), "-s", str(steps)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    assert re.search(r"odp_cls_pmr_create\(\)\s+1600 calls", out), out
    assert re.search(r"odp_cls_pmr_destroy\(\)\s+1600 calls", out), out
    assert "0 verdicts off" in out, out
    # 20 rebuild + 20 same-rule one-packet batches, 5 warmup + `steps` timed
    m = re.search(r"in_packets (\d+), in_octets (\d+)", out)
    n = 40 + (5 + steps) * batch
    assert m and int(m.group(1)) == n and int(m.group(2)) == 64 * n, out
