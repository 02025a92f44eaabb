"""odp_cls_hash_result (classification.h:769, odp_classification.c:384-414):
the queue of a CoS a packet goes to, from the packet's parse result. Its
device-batch form odpg_cls_hash_result (an odpg_packet_t: frame + odpg_meta_t)
is checked here against the hash queue the classifier itself picks (the
verdict word's ODPG_OUT_HASHQ, oracle on CPU, the device kernels under
-m gpu) for every hash protocol mix over IPv4/IPv6 x UDP/TCP/other frames;
odp_cls_hash_result on the runtime's own packets is checked per received
packet by tests/c/odp_rt_verdict.c (tests/test_rt_verdict.py)."""
import ctypes as C

import numpy as np
import pytest

import oracle
import rulesets
from helpers import pack
from odp_amd import _lib as L

HPS = ["HASH_IPV4 | HASH_IPV4_UDP", "HASH_IPV4_TCP | HASH_IPV6_TCP",
       "HASH_IPV6 | HASH_IPV4 | HASH_IPV6_UDP", "HASH_IPV4_UDP | HASH_IPV6_UDP"]


def _setup(cls, hp_expr, nq=7):
    hp = eval(hp_expr, {}, {k: getattr(cls, k) for k in dir(cls) if k.startswith("HASH_")})
    p = cls.loop_pktio()
    d = cls.cos_create("d", num_queue=nq, hash_proto=hp)
    assert d and cls.default_cos_set(p, d) == 0 and cls.pktio_start(p) == 0
    return p, d


def _check(cls, cos, buf, desc, out, meta, nq):
    n, queues = cls.cos_queues(cos)
    assert n == nq
    checked = 0
    for i in range(len(desc)):
        off, ln = int(desc[i]["offset"]), int(desc[i]["len"])
        frame = (C.c_uint8 * ln).from_buffer_copy(bytes(buf[off:off + ln]))
        pk = L.odpg_packet_t(C.cast(frame, C.c_void_p), ln, 0)
        C.memmove(C.byref(pk.meta), meta[i:i + 1].ctypes.data, C.sizeof(L.odpg_meta_t))
        q = L.lib.odpg_cls_hash_result(cos, C.byref(pk))
        if L.out_cos(out[i]) >= 0xFFF0:      # parse drop: no CoS, no queue
            continue
        assert q == queues[L.out_hashq(out[i])], (i, q, L.out_hashq(out[i]))
        checked += 1
    return checked


@pytest.mark.parametrize("hp", HPS)
def test_hash_result_matches_classifier_queue(fresh_cls, hp):
    p, d = _setup(fresh_cls, hp)
    frames = rulesets.mutate_corpus(1500, seed=len(hp))
    buf, desc = pack(frames)
    o = oracle.classify(fresh_cls.pktio_rules(p), buf, len(frames), desc=desc)
    assert _check(fresh_cls, d, buf, desc, o["out"], o["meta"], 7) > 1000
    assert len(np.unique(L.out_hashq(o["out"]))) > 1


def test_hash_result_single_queue_and_errors(fresh_cls):
    p = fresh_cls.loop_pktio()
    q = fresh_cls.queue(5)
    d = fresh_cls.cos_create("single", queue=q)
    pk = L.odpg_packet_t(None, 0, 0)
    assert L.lib.odpg_cls_hash_result(d, C.byref(pk)) == q     # num_queue 1: its queue
    assert L.lib.odpg_cls_hash_result(None, C.byref(pk)) is None
    h = fresh_cls.cos_create("h", num_queue=4, hash_proto=fresh_cls.HASH_IPV4)
    assert L.lib.odpg_cls_hash_result(h, None) is None         # no packet
    # the runtime form refuses anything that is not one of its packets
    assert L.lib.odp_cls_hash_result(d, None) is None
    assert L.lib.odp_cls_hash_result(d, C.byref(pk)) is None
    # the hash queues are real runtime queues: named, plain by default
    n, hq = fresh_cls.cos_queues(h)
    assert n == 4 and len(set(hq)) == 4 and all(hq)
    info = (C.c_uint8 * 256)()
    for k, x in enumerate(hq):
        assert L.lib.odp_queue_info(C.c_void_p(x), info) == 0
        name = C.cast(C.c_void_p.from_buffer(info, 0).value, C.c_char_p).value
        assert name == b"_odp_cos_hq_1_%d" % k
    assert fresh_cls.cos_destroy(h) == 0                       # destroys its queues
    assert all(L.lib.odp_queue_info(C.c_void_p(x), info) == -1 for x in hq)
    del p


@pytest.mark.gpu
def test_hash_result_matches_device_queue(gpu_ctx, fresh_cls):
    p, d = _setup(fresh_cls, HPS[2], nq=5)
    frames = rulesets.mutate_corpus(3000, seed=3)
    buf, desc = pack(frames)
    g = gpu_ctx.classify(gpu_ctx.table(fresh_cls.pktio_rules(p)), buf, len(frames), desc=desc)
    assert _check(fresh_cls, d, buf, desc, g["out"], g["meta"], 5) > 2000
