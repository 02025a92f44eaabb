"""Capture reader (include/odpg_pcap.h) and the example/classifier run on
the library (examples/odp_classifier_gpu.c), SURVEY.md §8(f) rank 4.

The captures are the reference's own data files, kept as fixtures:
tests/golden/classifier_udp64.pcap = example/classifier/udp64.pcap (pcapng)
and tests/golden/perf_udp64.pcap = test/performance/udp64.pcap (classic
pcap). Their frames must equal the ones tests/golden/make_golden.py
extracted into reference_fixtures.json; the example must reproduce
odp_classifier_run.sh's 100 / 100 split (pktio_env:21-22)."""
import ctypes as C
import os
import struct
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN
from odp_amd import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
EXAMPLE = os.path.join(os.path.dirname(HERE), "odp_amd", "lib", "odp_classifier_gpu")


def read(path, align=64):
    cap = L.odpg_capture_t()
    rc = L.lib.odpg_pcap_read(path.encode(), align, C.byref(cap))
    if rc:
        return rc, None
    try:
        buf = np.ctypeslib.as_array((C.c_uint8 * cap.bytes).from_address(cap.frames)).copy()
        desc = np.ctypeslib.as_array((C.c_uint32 * (2 * cap.num)).from_address(cap.desc))
        desc = desc.reshape(-1, 2).copy()
    finally:
        L.lib.odpg_pcap_free(C.byref(cap))
    frames = [bytes(buf[o:o + n]) for o, n in desc]
    assert all(o % align == 0 for o, _ in desc)
    return 0, frames


@pytest.mark.parametrize("name,key", [("classifier_udp64.pcap", "classifier_udp64"),
                                      ("perf_udp64.pcap", "perf_udp64")])
def test_reference_captures(name, key):
    rc, frames = read(os.path.join(GOLD, name))
    assert rc == 0
    assert [f.hex() for f in frames] == GOLDEN["pcap"][key]


def _classic(frames, endian="<", nsec=False, link=1):
    magic = 0xA1B23C4D if nsec else 0xA1B2C3D4
    out = struct.pack(endian + "IHHiIII", magic, 2, 4, 0, 0, 65535, link)
    for i, f in enumerate(frames):
        out += struct.pack(endian + "IIII", i, 0, len(f), len(f)) + f
    return out


def _pcapng(frames, endian="<", simple=False):
    def block(t, body):
        body += bytes(-len(body) % 4)
        n = len(body) + 12
        return struct.pack(endian + "II", t, n) + body + struct.pack(endian + "I", n)
    out = block(0x0A0D0D0A, struct.pack(endian + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    out += block(1, struct.pack(endian + "HHI", 1, 0, 0))
    for f in frames:
        if simple:
            out += block(3, struct.pack(endian + "I", len(f)) + f)
        else:
            out += block(6, struct.pack(endian + "IIIII", 0, 0, 0, len(f), len(f)) + f)
    return out


@pytest.mark.parametrize("kind", ["le", "be", "nsec", "ng", "ng_be", "ng_simple"])
def test_formats(tmp_path, kind):
    frames = [bytes.fromhex(h) for h in GOLDEN["pcap"]["classifier_udp64"][:7]] + [b"\x01" * 3]
    data = {"le": lambda: _classic(frames), "be": lambda: _classic(frames, ">"),
            "nsec": lambda: _classic(frames, nsec=True), "ng": lambda: _pcapng(frames),
            "ng_be": lambda: _pcapng(frames, ">"),
            "ng_simple": lambda: _pcapng(frames, simple=True)}[kind]()
    p = tmp_path / "x.pcap"
    p.write_bytes(data)
    for align in (1, 16, 64):
        rc, got = read(str(p), align)
        assert rc == 0 and got == frames


def test_errors(tmp_path):
    assert read(str(tmp_path / "missing.pcap"))[0] == -2             # -ENOENT
    bad = tmp_path / "bad.pcap"
    bad.write_bytes(b"not a capture file")
    assert read(str(bad))[0] == -22                                   # -EINVAL
    frames = [b"\xaa" * 60]
    bad.write_bytes(_classic(frames)[:-5])                            # truncated record
    assert read(str(bad))[0] == -22
    bad.write_bytes(_classic(frames, link=101))                       # not Ethernet
    assert read(str(bad))[0] == -22
    ok = tmp_path / "ok.pcap"
    ok.write_bytes(_classic(frames))
    cap = L.odpg_capture_t()
    assert L.lib.odpg_pcap_read(str(ok).encode(), 3, C.byref(cap)) == -22   # align


def test_example_builds():
    assert os.access(EXAMPLE, os.X_OK)


def _run(*args):
    return subprocess.run([EXAMPLE, *args], capture_output=True, text=True, timeout=120)


@pytest.mark.gpu
def test_example_classifier_run():
    """odp_classifier_run.sh:17-19 on the library: SIP 10.10.10.0/24 ->
    queue1, 100 packets each way (pktio_env:21-22)."""
    pcap = os.path.join(GOLD, "classifier_udp64.pcap")
    r = _run("-i", pcap, "-m", "0", "-p", "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1",
             "-P", "-C", "queue1:100", "-C", "DefaultCos:100")
    assert r.returncode == 0, r.stdout + r.stderr
    counts = dict(line.split()[:2] for line in r.stdout.splitlines()[1:])
    assert counts == {"DefaultCos": "100", "queue1": "100"}
    r = _run("-i", pcap, "-p", "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1",
             "-C", "queue1:101")
    assert r.returncode == 1 and "verification failed" in r.stderr
    # a chained policy (src CoS named) and a port rule
    r = _run("-i", pcap, "-p", "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1",
             "-p", "ODP_PMR_UDP_DPORT:0:0:queue1:queue2", "-C", "queue2:100")
    assert r.returncode == 0, r.stdout + r.stderr
