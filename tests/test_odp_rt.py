"""The ODP runtime subset (include/odp_api.h, odp/rt.h, odp/helper/odph_api.h)
and the drop-in check of SURVEY §8(f) rank 4: the reference's own
example/classifier source, compiled unmodified against these headers and
linked to libodpg.so (oracle/ref_apps.mk), classifies
example/classifier/udp64.pcap with the reference run script's rule and
passes its own CI packet-count check (odp_classifier_run.sh:17-19,
pktio_env: 100 packets to queue1, 100 to DefaultCos); the reference's
test/performance/odp_bench_pktio_sp.c (with test/common/bench_common.c and
export_results.c) builds the same way and runs all its cases; and the loop
device (tests/c/odp_rt_loop.c) sends packets back through the GPU
classifier in DIRECT, SCHED and QUEUE input modes."""
import ctypes as C
import os
import re
import struct
import subprocess

import pytest

from helpers import GOLDEN, make_c_tests as _make_c
from odp_amd import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF_APP = os.path.join(ROOT, "oracle", "_ref", "odp_classifier")
REF_SRC = "/root/reference/example/classifier/odp_classifier.c"
REF_BENCH = os.path.join(ROOT, "oracle", "_ref", "odp_bench_pktio_sp")
REF_PERF = os.path.join(ROOT, "oracle", "_ref", "odp_pktio_perf")
LOOP_TEST = os.path.join(HERE, "c", "odp_rt_loop")
PROTO = re.compile(r"^[A-Za-z_][\w \*]*?\b((?:odph|odp)_\w+)\s*\(", re.M)


def _declared(path):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"^#.*$", "", txt, flags=re.M)
    txt = re.sub(r"static inline[^{]*\{[^}]*\}", "", txt, flags=re.S)
    txt = re.sub(r"typedef[^;]*;", "", txt, flags=re.S)
    return {m.group(1) for m in PROTO.finditer(txt)}


def test_runtime_symbols_exported():
    names = _declared(os.path.join(ROOT, "include", "odp", "rt.h")) | \
        _declared(os.path.join(ROOT, "include", "odp", "helper", "odph_api.h"))
    assert {"odp_schedule_multi", "odp_pool_create", "odph_thread_create",
            "odp_packet_l3_ptr"} <= names and len(names) > 60
    nm = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    assert not sorted(names - exported), sorted(names - exported)


@pytest.mark.skipif(not os.path.exists(REF_SRC), reason="reference sources not present")
def test_reference_classifier_builds_unmodified():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-f", "ref_apps.mk"],
                   check=True, capture_output=True)
    for app in (REF_APP, REF_BENCH, REF_PERF):
        assert os.access(app, os.X_OK), app
        out = subprocess.run(["ldd", app], capture_output=True, text=True).stdout
        assert "libodpg.so" in out, app


def test_loop_test_program_builds():
    _make_c()
    assert os.access(LOOP_TEST, os.X_OK)


def test_pktio_lookup_modes_and_capabilities():
    """No GPU needed: name rules and the mode checks of the queue accessors
    (odp_packet_io.c:406-410, 798-829, 2364-2503)."""
    from odp_amd import cls
    lib = C.CDLL(L.LIB_PATH)
    cls.reset()

    class PktioParam(C.Structure):
        _fields_ = [("in_mode", C.c_int), ("out_mode", C.c_int), ("rest", C.c_uint8 * 64)]
    lib.odp_pktio_open.restype = C.c_void_p
    lib.odp_pktio_lookup.restype = C.c_void_p
    pp = PktioParam()
    lib.odp_pktio_param_init(C.byref(pp))
    assert (pp.in_mode, pp.out_mode) == (0, 0)            # DIRECT / DIRECT
    a = lib.odp_pktio_open(b"loop", None, C.byref(pp))
    assert a
    assert not lib.odp_pktio_open(b"loop", None, C.byref(pp))     # already opened
    assert lib.odp_pktio_lookup(b"loop") == a and not lib.odp_pktio_lookup(b"loop3")
    pp.in_mode, pp.out_mode = 2, 1                        # SCHED / QUEUE
    b = lib.odp_pktio_open(b"loop3", None, C.byref(pp))
    assert b and lib.odp_pktio_lookup(b"loop3") == b
    for h in (a, b):
        assert lib.odp_pktin_queue_config(C.c_void_p(h), None) == 0
        assert lib.odp_pktout_queue_config(C.c_void_p(h), None) == 0
    qs = (C.c_void_p * 4)()
    pq = (C.c_uint64 * 8)()
    assert lib.odp_pktin_queue(C.c_void_p(a), pq, 4) == 1
    assert lib.odp_pktin_event_queue(C.c_void_p(a), qs, 4) == -1
    assert lib.odp_pktout_queue(C.c_void_p(a), pq, 4) == 1
    assert lib.odp_pktout_event_queue(C.c_void_p(a), qs, 4) == -1
    assert lib.odp_pktin_queue(C.c_void_p(b), pq, 4) == -1
    assert lib.odp_pktin_event_queue(C.c_void_p(b), qs, 4) == 1 and qs[0]
    assert lib.odp_pktout_queue(C.c_void_p(b), pq, 4) == -1
    assert lib.odp_pktout_event_queue(C.c_void_p(b), qs, 4) == 1 and qs[0]
    # up to 16 output queues per loop pktio (loop.c's max_output_queues):
    # more is refused
    pq2 = (C.c_uint8 * 512)()
    lib.odp_pktout_queue_param_init(pq2)
    struct.pack_into("<I", pq2, 4, 17)                    # num_queues (after op_mode)
    assert lib.odp_pktout_queue_config(C.c_void_p(a), pq2) == -1
    assert lib.odp_pktio_close(C.c_void_p(a)) == 0 and lib.odp_pktio_close(C.c_void_p(b)) == 0
    assert not lib.odp_pktio_lookup(b"loop")
    # capabilities the reference bench sizes itself by
    pc = (C.c_uint32 * 64)()
    assert lib.odp_pool_capability(pc) == 0 and pc[0] > 0
    sc = (C.c_uint32 * 9)()
    assert lib.odp_schedule_capability(sc) == 0 and sc[3] > 1000    # max_queues
    cls.reset()


def test_host_side_runtime_pieces():
    lib = C.CDLL(L.LIB_PATH)
    # helper parsers (helper/eth.c, helper/ip.c)
    ip = C.c_uint32()
    assert lib.odph_ipv4_addr_parse(C.byref(ip), b"10.10.10.7") == 0 and ip.value == 0x0A0A0A07
    assert lib.odph_ipv4_addr_parse(C.byref(ip), b"10.10.10.256") == -1
    mac = (C.c_uint8 * 6)()
    assert lib.odph_eth_addr_parse(mac, b"02:e9:34:80:73:01") == 0
    assert bytes(mac) == bytes.fromhex("02e934807301")
    # a packet pool, packets and a plain queue (no GPU involved)

    class PoolParam(C.Structure):
        _fields_ = [("type", C.c_int), ("buf", C.c_uint32 * 3), ("pkt", C.c_uint32 * 7),
                    ("reserved", C.c_uint64 * 8)]
    pp = PoolParam()
    lib.odp_pool_param_init(C.byref(pp))
    pp.pkt[0] = 2                                     # num
    lib.odp_pool_create.restype = C.c_void_p
    pool = lib.odp_pool_create(b"p", C.byref(pp))
    assert pool
    lib.odp_packet_alloc.restype = C.c_void_p
    a = lib.odp_packet_alloc(C.c_void_p(pool), 64)
    b = lib.odp_packet_alloc(C.c_void_p(pool), 64)
    assert a and b and not lib.odp_packet_alloc(C.c_void_p(pool), 64)   # pool of 2
    lib.odp_queue_create.restype = C.c_void_p
    lib.odp_queue_deq.restype = C.c_void_p
    q = lib.odp_queue_create(b"q", None)
    assert lib.odp_queue_enq(C.c_void_p(q), C.c_void_p(a)) == 0
    assert lib.odp_queue_enq(C.c_void_p(q), C.c_void_p(b)) == 0
    assert lib.odp_queue_deq(C.c_void_p(q)) == a and lib.odp_queue_deq(C.c_void_p(q)) == b
    assert not lib.odp_queue_deq(C.c_void_p(q))
    lib.odp_packet_free(C.c_void_p(a))
    lib.odp_packet_free(C.c_void_p(b))
    assert lib.odp_queue_destroy(C.c_void_p(q)) == 0
    assert lib.odp_pool_destroy(C.c_void_p(pool)) == 0


@pytest.mark.gpu
def test_loop_device_through_gpu_classifier():
    assert os.access(LOOP_TEST, os.X_OK), "make -C tests/c (built by __graft_entry__.build)"
    r = subprocess.run(["timeout", "-k", "10", "100", LOOP_TEST], capture_output=True, text=True)
    assert r.returncode == 0 and "PASS" in r.stdout, (r.stdout[-3000:], r.stderr[-2000:])
    assert "A direct: received 300" in r.stdout and "C queue: 300 packets" in r.stdout
    assert "D pcap loops=3: 40 packets" in r.stdout
    assert "E pcap small pool: 20 packets" in r.stdout
    for m in ("direct hash=1", "sched hash=1", "direct hash=0"):
        assert f"G {m}: 300 packets" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
def test_loop_device_over_several_device_contexts():
    """ODPG_DEVICES=0,0,0: the runtime opens three device contexts (here all
    on the one GPU) and spreads receive bursts over them (odp_rt.c
    slot_get); every check of the loop program holds, including the
    4-thread ordered delivery."""
    r = subprocess.run(["timeout", "-k", "10", "100", LOOP_TEST], capture_output=True, text=True,
                       env=dict(os.environ, ODPG_DEVICES="0,0,0"))
    assert r.returncode == 0 and "PASS" in r.stdout, (r.stdout[-3000:], r.stderr[-2000:])
    assert "F sched, 4 threads: 200000 packets, each once and in order per thread" in r.stdout


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_BENCH), reason="reference bench not built here")
def test_reference_bench_pktio_sp_runs_every_case():
    r = subprocess.run(["timeout", "-k", "10", "100", REF_BENCH, "-r", "20"],
                       capture_output=True, text=True)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    cases = re.findall(r"^\[(\d\d)\] (\w+)(.*)$", r.stdout, re.M)
    assert [int(c[0]) for c in cases] == list(range(1, 11)), r.stdout[-3000:]
    assert not [c for c in cases if "n/a" in c[2]], r.stdout[-3000:]   # cls_pmr_create ran
    assert "odp_cls_pmr_create()" in r.stdout and "odp_pktin_queue_stats()" in r.stdout


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_PERF), reason="reference pktio perf test not built here")
def test_reference_pktio_perf_passes_at_fixed_rate():
    """test/performance/odp_pktio_perf.c, unmodified: one TX and one RX
    worker on the loop device, 100 ms at 1 Mpps, every packet transmitted
    must come back through the GPU receive path (scheduler input)."""
    r = subprocess.run(["timeout", "-k", "10", "100", REF_PERF, "-r", "1000000"],
                       capture_output=True, text=True)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    assert "Result: PASSED" in r.stdout, r.stdout[-3000:]
    tx = int(re.search(r"TxPkts: (\d+)", r.stdout).group(1))
    rx = int(re.search(r"RxPkts: (\d+)", r.stdout).group(1))
    assert tx >= 99000 and rx >= tx, r.stdout[-2000:]


def write_pcap(path, frames):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for k, fr in enumerate(frames):
            f.write(struct.pack("<IIII", k, 0, len(fr), len(fr)))
            f.write(fr)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_APP), reason="reference example not built here")
def test_reference_classifier_runs_and_passes_its_ci_check(tmp_path):
    frames = [bytes.fromhex(h) for h in GOLDEN["pcap"]["classifier_udp64"]]
    cap = tmp_path / "udp64.pcap"
    write_pcap(cap, frames)
    cmd = [REF_APP, "-t", "1", "-i", f"pcap:in={cap}", "-m", "0", "-p",
           "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1", "-P", "-C", "queue1:100",
           "-C", "DefaultCos:100"]
    r = subprocess.run(["timeout", "-k", "10", "90"] + cmd, capture_output=True, text=True)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    # the statistics table's last row: queue1 and DefaultCos got 100 each
    rows = [ln for ln in r.stdout.splitlines() if re.match(r"^\d+\s+\d+\s*\|", ln)]
    assert rows, r.stdout[-2000:]
    counts = [int(x.split()[0]) for x in rows[-1].split("|")[:-1]]
    assert counts[:2] == [100, 100], rows[-1]


def test_host_runtime_under_contention():
    """tests/c/odp_rt_host.c, no GPU: the barrier re-entered 40000 times by
    8 threads with a shared count checked between phases, thread ids under
    concurrent init_local / term_local, named shm reserve / lookup / free
    (a second free fails cleanly), 2^21 queue create / destroy cycles (more
    than the registry's slots: destroyed slots are reused and stale handles
    refused) and scheduled queues created / destroyed under 4 schedulers."""
    _make_c()
    r = subprocess.run(["timeout", "-k", "10", "240", os.path.join(HERE, "c", "odp_rt_host")],
                       capture_output=True, text=True)
    assert r.returncode == 0 and "PASS" in r.stdout, (r.stdout[-3000:], r.stderr[-2000:])
