"""The ODP runtime subset (include/odp_api.h, odp/rt.h, odp/helper/odph_api.h)
and the drop-in check of SURVEY §8(f) rank 4: the reference's own
example/classifier source, compiled unmodified against these headers and
linked to libodpg.so (oracle/ref_apps.mk), classifies
example/classifier/udp64.pcap with the reference run script's rule and
passes its own CI packet-count check (odp_classifier_run.sh:17-19,
pktio_env: 100 packets to queue1, 100 to DefaultCos)."""
import ctypes as C
import os
import re
import struct
import subprocess

import pytest

from helpers import GOLDEN
from odp_amd import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF_APP = os.path.join(ROOT, "oracle", "_ref", "odp_classifier")
REF_SRC = "/root/reference/example/classifier/odp_classifier.c"
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
    assert os.access(REF_APP, os.X_OK)
    out = subprocess.run(["ldd", REF_APP], capture_output=True, text=True).stdout
    assert "libodpg.so" in out


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
