"""The receive verdict on the runtime's own packets:
tests/c/odp_rt_verdict.c sends a corpus through a loop pktio with the pktin
IPv4/UDP/TCP/SCTP checksum checks on, receives it through the GPU classifier
into CoS queues (plain and hash queues), and reads every packet back through
the ODP accessors an application uses. Every value must equal what the
reference's accessors would return for the oracle's parse result of that
frame (include/odp/api/plat/packet_inlines.h:334-417,617,
packet_flag_inlines.h:62-288, odp_packet.c:2077-2118), every packet must be
on the queue get_dest_queue names, and odp_cls_hash_result(cos, pkt) must
name that same queue (odp_classification.c:384-414). The pktio, CoS and
per-queue counters must equal the oracle's.

Corpus: the C3 traffic's special frames (bad IPv4 header / L4 checksums,
UDP checksum 0, IPv4 fragments) plus ordinary IMIX frames, the mutation
corpus (truncation, VLAN / QinQ / SNAP, IPv6 extension headers, random
bytes) and the 64-byte edge corpus."""
import os
import struct
import subprocess
from collections import defaultdict

import numpy as np
import pytest

import oracle
import rulesets
from helpers import ALL_CHKSUM, IFL, make_c_tests
from odp_amd import _lib as L
from odp_amd import gen

HERE = os.path.dirname(os.path.abspath(__file__))
PROG = os.path.join(HERE, "c", "odp_rt_verdict")
OPT = ALL_CHKSUM


def verdict_rules(cls, p):
    """The rule set odp_rt_verdict.c builds, in the same creation order."""
    T = cls.Term
    d = cls.cos_create("dflt", num_queue=4, hash_proto=0x3f, stats_enable=True)
    e = cls.cos_create("err", queue=cls.queue(1), stats_enable=True)
    u = cls.cos_create("udp", queue=cls.queue(2), stats_enable=True)
    t = cls.cos_create("tcp", num_queue=3, hash_proto=2 | 16, stats_enable=True)
    dr = cls.cos_create("drop", action=cls.COS_ACTION_DROP, stats_enable=True)
    v = cls.cos_create("v6udp", queue=cls.queue(5), stats_enable=True)
    assert all((d, e, u, t, dr, v))
    assert cls.pmr_create([T(cls.PMR_IPPROTO, b"\x11", b"\xff")], d, u, mark=0x77)
    assert cls.pmr_create([T(cls.PMR_IPPROTO, b"\x06", b"\xff")], d, t, mark=0x1234)
    assert cls.pmr_create([T(cls.PMR_ETHTYPE_0, b"\x08\x06", b"\xff\xff")], d, dr, mark=0)
    assert cls.pmr_create([T(cls.PMR_UDP_DPORT, b"\x00\x3f", b"\xff\xff")], u, v, mark=9)
    assert cls.default_cos_set(p, d) == 0 and cls.error_cos_set(p, e) == 0
    return {"nq": [4, 1, 1, 3, 1, 1]}


def corpus():
    buf, desc = gen.c3_frames(30000)
    r = gen.xorshift64(gen.C_SEED ^ 0x5A5A3C3, 30000)
    special = ((r >> np.uint64(24)) % np.uint64(1000)).astype(np.int64)
    pick = np.concatenate([np.nonzero(special < 20)[0], np.arange(1200)])
    frames = [bytes(buf[int(desc["offset"][i]):int(desc["offset"][i]) + int(desc["len"][i])])
              for i in pick]
    frames += rulesets.mutate_corpus(2500, seed=41)
    p64 = rulesets.plain64_corpus(512, seed=43).reshape(-1, 64)
    frames += [bytes(x) for x in p64]
    return frames


def _flag_all(m):
    inf, fl = int(m["input_flags"]), int(m["flags"])
    b = lambda n: (inf >> IFL[n]) & 1  # noqa: E731
    bits = [int((fl & 0xFE000000) != 0), (fl >> 25) & 1, (fl >> 26) & 1,
            ((fl >> 28) | (fl >> 29)) & 1, b("l2"), b("l3"), b("l4"), b("eth"),
            b("eth_bcast"), b("eth_mcast"), b("jumbo"), b("vlan"), b("vlan_qinq"), b("arp"),
            b("ipv4"), b("ipv6"), b("ip_bcast"), b("ip_mcast"), b("ipfrag"), b("ipopt"),
            b("ipsec"), b("udp"), b("tcp"), b("sctp"), b("icmp")]
    return sum(v << k for k, v in enumerate(bits))


def _status(m, done, err):
    """odp_packet_chksum_status_t: UNKNOWN 0, BAD 1, OK 2"""
    if not (int(m["input_flags"]) >> done) & 1:
        return 0
    return 1 if (int(m["flags"]) >> err) & 1 else 2


def _types(m):
    inf = int(m["input_flags"])
    b = lambda n: (inf >> IFL[n]) & 1  # noqa: E731
    l2 = 1 if b("eth") else 0
    l3 = 0x0800 if b("ipv4") else 0x86DD if b("ipv6") else 0x0806 if b("arp") else 0xFFFF
    if b("tcp"):
        l4 = 6
    elif b("udp"):
        l4 = 17
    elif b("sctp"):
        l4 = 132
    elif b("ipsec_ah"):
        l4 = 51
    elif b("ipsec_esp"):
        l4 = 50
    elif b("icmp") and b("ipv4"):
        l4 = 1
    elif b("icmp") and b("ipv6"):
        l4 = 58
    elif b("no_next_hdr"):
        l4 = 59
    else:
        l4 = 255
    return l2, l3, l4


def test_verdict_program_builds():
    make_c_tests()
    assert os.access(PROG, os.X_OK)


@pytest.mark.gpu
def test_accessors_and_hash_result_on_received_packets(fresh_cls, tmp_path):
    assert os.access(PROG, os.X_OK), "make -C tests/c (built by __graft_entry__.build)"
    frames = corpus()
    # the oracle's verdicts under the same rules and pktin options
    p = fresh_cls.loop_pktio(pktin=OPT)
    spec = verdict_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    from helpers import pack
    buf, desc = pack(frames)
    o = oracle.classify(fresh_cls.pktio_rules(p), buf, len(frames), desc=desc, opt=OPT)

    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(struct.pack("<IIQ", 0x56524454, len(frames), OPT))
        for fr in frames:
            f.write(struct.pack("<I", len(fr)) + fr)
    outp = tmp_path / "out.txt"
    r = subprocess.run(["timeout", "-k", "10", "100", PROG, str(inp), str(outp)],
                       capture_output=True, text=True)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])

    qmap, rows, cos_pk, qs = {}, [], {}, {}
    for ln in open(outp):
        f = ln.split()
        if f[0] == "Q":
            qmap[(int(f[2]), int(f[3]))] = int(f[1])
        elif f[0] == "P":
            rows.append([int(x) for x in f[1:]])
        elif f[0] == "S":
            stats = [int(x) for x in f[1:]]
        elif f[0] == "C":
            cos_pk[int(f[1])] = int(f[2])
        elif f[0] == "QS":
            qs[int(f[1])] = (int(f[2]), int(f[3]))

    out = o["out"]
    cos = out & 0xFFFF
    hq = (out >> 24) & 31
    delivered = (cos < 6) & ((out & L.ODPG_OUT_CLS_DROP) == 0)
    want = {}
    for i in np.nonzero(delivered)[0]:
        c = int(cos[i])
        want[int(i)] = qmap[(c, int(hq[i]) % spec["nq"][c])]
    seen = defaultdict(int)
    bad = []
    for row in rows:
        (k, qid, l3s, l4s, mark, fall, l2o, l3o, l4o, l2t, l3t, l4t, ci, hqid, inp_ok,
         inf, fl) = row
        assert k >= 0, "a received packet that was never sent"
        seen[k] += 1
        m = o["meta"][k]
        exp = (want.get(k), _status(m, 32, 27), _status(m, 33, 31),
               int(m["cls_mark"]) if (int(m["input_flags"]) >> 1) & 1 else 0, _flag_all(m),
               int(m["l2_offset"]), int(m["l3_offset"]), int(m["l4_offset"])) + _types(m) + (
               int(cos[k]), want.get(k), 1, int(m["input_flags"]), int(m["flags"]))
        got = (qid, l3s, l4s, mark, fall, l2o, l3o, l4o, l2t, l3t, l4t, ci, hqid, inp_ok, inf, fl)
        if got != exp:
            bad.append((k, got, exp))
    assert not bad, f"{len(bad)} packets differ, first: {bad[:3]}"
    assert dict(seen) == {k: 1 for k in want}, "received set != the oracle's delivered set"
    # coverage: the corpus exercises every status, marks, both hash CoS
    st = {(r[2], r[3]) for r in rows}
    assert {(1, 0), (2, 2), (2, 1), (0, 0)} <= st, st
    assert {r[4] for r in rows} >= {0x77, 0x1234, 9, 0}
    assert len({r[1] for r in rows}) == sum(spec["nq"][c] for c in (0, 1, 2, 3, 5))
    # counters: pktio, CoS, per queue
    assert stats == [int(x) for x in o["stats"][:4]], (stats, o["stats"][:4])
    for c in range(6):
        assert cos_pk[c] == int(o["stats"][4 + c]), (c, cos_pk[c], o["stats"][4 + c])
    per_q = defaultdict(int)
    for qid in want.values():
        per_q[qid] += 1
    assert all(qs[q] == (per_q[q], 0) for q in qs), (qs, dict(per_q))
