"""The host runtime (odp_amd/csrc/odp_rt.c, odp_cls.c, pcap.c) under
ThreadSanitizer and AddressSanitizer + UBSan, no GPU: tests/c/Makefile's
"san" targets build the runtime's C test programs (odp_rt_host.c: barrier,
thread ids, shm, pools, queue registry and rings, scheduler under
contention; odp_rt_loop.c: the loop pktio in DIRECT / SCHED / QUEUE / pcap
input modes and the chunked, ordered hand-over between four receiving
threads) with the device entry points replaced by tests/c/gpu_stub.c
(classification through the CPU oracle, fences complete on record). The
device groups (group.cpp: groups of 1, 3 and 5 contexts, host batches and
per-member shards, against one context) run the same way. The
reference's CI runs its suites under ASan + UBSan the same way
(.github/workflows/ci-pipeline.yml:399-412). A sanitizer report, a failed
check or a nonzero exit fails the test."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CDIR = os.path.join(HERE, "c")
REPORTS = ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "runtime error:",
           "ERROR: LeakSanitizer")


@pytest.fixture(scope="module")
def san_build():
    r = subprocess.run(["make", "-s", "-C", CDIR, "san"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("prog", ["odp_rt_host", "odp_rt_loop", "odp_rt_loop:0,0,0", "group_host"])
@pytest.mark.parametrize("san", ["tsan", "asan"])
def test_runtime_under_sanitizer(san_build, prog, san):
    """odp_rt_loop:0,0,0 runs with three device contexts (ODPG_DEVICES):
    receive bursts spread over them. group_host: device groups of 1, 3 and 5
    contexts (group.cpp, one host thread per member) against one context"""
    env = dict(os.environ)
    prog, _, devs = prog.partition(":")
    if devs:
        env["ODPG_DEVICES"] = devs
    env["TSAN_OPTIONS"] = "halt_on_error=1 second_deadlock_stack=1"
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1"
    r = subprocess.run(["timeout", "-k", "10", "540", os.path.join(CDIR, f"{prog}.{san}")],
                       capture_output=True, text=True, env=env, cwd=CDIR)
    out = r.stdout + r.stderr
    assert not [x for x in REPORTS if x in out], out[-6000:]
    assert r.returncode == 0 and "PASS" in r.stdout, out[-4000:]
    if prog == "odp_rt_loop":
        assert "F sched, 4 threads: 200000 packets, each once and in order per thread" in r.stdout
        assert "B sched+cls: 300 packets, 150 to net10, 150 to default" in r.stdout
        assert "G sched hash=1: 300 packets" in r.stdout
    if prog == "group_host":
        assert "verdicts and counters equal one context's" in r.stdout
