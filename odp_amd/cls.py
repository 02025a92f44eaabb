"""Python mirror of the ODP classification API served by ``libodpg.so``.

Every function calls the C implementation in ``odp_amd/csrc/odp_cls.c``
(names and semantics of ``include/odp/api/spec/classification.h:697-1073``);
this module only marshals arguments so tests read like the reference's
CUnit suites (``test/validation/api/classification/``).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from . import _lib as L

lib = L.lib

# odp_cls_pmr_term_t
(PMR_LEN, PMR_ETHTYPE_0, PMR_ETHTYPE_X, PMR_VLAN_ID_0, PMR_VLAN_ID_X, PMR_VLAN_PCP_0, PMR_DMAC,
 PMR_IPPROTO, PMR_IP_DSCP, PMR_UDP_DPORT, PMR_TCP_DPORT, PMR_UDP_SPORT, PMR_TCP_SPORT,
 PMR_SIP_ADDR, PMR_DIP_ADDR, PMR_SIP6_ADDR, PMR_DIP6_ADDR, PMR_IPSEC_SPI, PMR_LD_VNI,
 PMR_CUSTOM_FRAME, PMR_CUSTOM_L3, PMR_IGMP_GRP_ADDR, PMR_ICMP_ID, PMR_ICMP_TYPE, PMR_ICMP_CODE,
 PMR_SCTP_SPORT, PMR_SCTP_DPORT, PMR_GTPV1_TEID) = range(28)
PMR_INNER_HDR_OFF = 32

COS_ACTION_ENQUEUE, COS_ACTION_DROP = 0, 1
COS_INVALID = None

# hash_proto bits (odp_pktin_hash_proto_t)
HASH_IPV4_UDP, HASH_IPV4_TCP, HASH_IPV4, HASH_IPV6_UDP, HASH_IPV6_TCP, HASH_IPV6 = (
    1, 2, 4, 8, 16, 32)


@dataclass
class Term:
    """odp_pmr_param_t: value/mask are the raw bytes (network order except LEN)."""
    term: int
    value: bytes
    mask: bytes
    offset: int = 0
    val_sz: int | None = None
    range_term: bool = False


def _h(x):
    """ctypes returns c_void_p handles as int or None."""
    return x


def reset():
    lib.odpg_cls_reset()


def set_limits(max_cos, max_pmr, max_pmr_per_cos):
    return lib.odpg_cls_set_limits(max_cos, max_pmr, max_pmr_per_cos)


def capability():
    capa = L.odp_cls_capability_t()
    L.check(lib.odp_cls_capability(C.byref(capa)), "odp_cls_capability")
    return capa


def cos_param(queue=None, action=COS_ACTION_ENQUEUE, num_queue=1, hash_proto=0,
              stats_enable=False, pool=None):
    p = L.odp_cls_cos_param_t()
    lib.odp_cls_cos_param_init(C.byref(p))
    p.action = action
    p.stats_enable = int(bool(stats_enable))
    p.num_queue = num_queue
    if num_queue > 1:
        p.h.hash_proto = hash_proto
    else:
        p.queue = queue
    p.pool = pool
    return p


def cos_create(name, queue=None, **kw):
    p = cos_param(queue=queue, **kw)
    return lib.odp_cls_cos_create(name.encode() if name else None, C.byref(p))


def cos_destroy(cos):
    return lib.odp_cos_destroy(cos)


def cos_queue(cos):
    return lib.odp_cos_queue(cos)


def cos_queue_set(cos, queue):
    return lib.odp_cos_queue_set(cos, queue)


def cos_num_queue(cos):
    return lib.odp_cls_cos_num_queue(cos)


def cos_queues(cos, num=32):
    arr = (C.c_void_p * max(num, 1))()
    n = lib.odp_cls_cos_queues(cos, arr, num)
    return n, [arr[i] for i in range(min(n, num))]


def cos_pool(cos):
    return lib.odp_cls_cos_pool(cos)


def cos_pool_set(cos, pool):
    return lib.odp_cls_cos_pool_set(cos, pool)


def _params(terms):
    arr = (L.odp_pmr_param_t * max(len(terms), 1))()
    keep = []
    for i, t in enumerate(terms):
        lib.odp_cls_pmr_param_init(C.byref(arr[i]))
        v = C.create_string_buffer(bytes(t.value), max(len(t.value), 1))
        m = C.create_string_buffer(bytes(t.mask), max(len(t.mask), 1))
        keep += [v, m]
        arr[i].term = t.term
        arr[i].range_term = int(t.range_term)
        arr[i].value = C.cast(v, C.c_void_p)
        arr[i].mask = C.cast(m, C.c_void_p)
        arr[i].val_sz = len(t.value) if t.val_sz is None else t.val_sz
        arr[i].offset = t.offset
    return arr, keep


def pmr_create(terms, src, dst, mark=None):
    """odp_cls_pmr_create (mark None) or odp_cls_pmr_create_opt."""
    arr, keep = _params(terms)
    if mark is None:
        return lib.odp_cls_pmr_create(arr, len(terms), src, dst)
    opt = L.odp_pmr_create_opt_t()
    lib.odp_cls_pmr_create_opt_init(C.byref(opt))
    opt.terms = arr
    opt.num_terms = len(terms)
    opt.mark = mark
    r = lib.odp_cls_pmr_create_opt(C.byref(opt), src, dst)
    del keep
    return r


def pmr_destroy(pmr):
    return lib.odp_cls_pmr_destroy(pmr)


def cos_stats(cos):
    st = L.odp_cls_cos_stats_t()
    rc = lib.odp_cls_cos_stats(cos, C.byref(st))
    return rc, st


def queue_stats(cos, queue):
    st = L.odp_cls_cos_stats_t()
    rc = lib.odp_cls_queue_stats(cos, queue, C.byref(st))
    return rc, st


def to_index(handle):
    """odp_cos_t / odp_pmr_t handle -> table index (handles are index + 1)."""
    return int(handle) - 1


# ---- loop pktio ------------------------------------------------------------
def pktio_open(name="loop"):
    return lib.odp_pktio_open(name.encode(), None, None)


def pktio_close(pktio):
    return lib.odp_pktio_close(pktio)


def pktio_config(pktio, pktin=0, layer=L.LAYER_ALL):
    cfg = L.odp_pktio_config_t()
    lib.odp_pktio_config_init(C.byref(cfg))
    cfg.pktin = pktin
    cfg.layer = layer
    return lib.odp_pktio_config(pktio, C.byref(cfg))


def pktin_queue_config(pktio, classifier_enable=True):
    p = L.odp_pktin_queue_param_t()
    lib.odp_pktin_queue_param_init(C.byref(p))
    p.classifier_enable = int(bool(classifier_enable))
    return lib.odp_pktin_queue_config(pktio, C.byref(p))


def pktio_start(pktio):
    return lib.odp_pktio_start(pktio)


def pktio_stop(pktio):
    return lib.odp_pktio_stop(pktio)


def pktio_stats(pktio):
    st = L.odp_pktio_stats_t()
    L.check(lib.odp_pktio_stats(pktio, C.byref(st)), "odp_pktio_stats")
    return st


def pktio_stats_reset(pktio):
    return lib.odp_pktio_stats_reset(pktio)


def default_cos_set(pktio, cos):
    return lib.odp_pktio_default_cos_set(pktio, cos)


def error_cos_set(pktio, cos):
    return lib.odp_pktio_error_cos_set(pktio, cos)


def skip_set(pktio, off):
    return lib.odp_pktio_skip_set(pktio, off)


def headroom_set(pktio, hr):
    return lib.odp_pktio_headroom_set(pktio, hr)


def pktio_rules(pktio):
    """odpg_rules_t snapshot of the pktio's classifier (C-owned arrays)."""
    r = L.odpg_rules_t()
    L.check(lib.odpg_pktio_rules(pktio, C.byref(r)), "odpg_pktio_rules")
    return r


def loop_pktio(pktin=0, classifier=True):
    """Open + configure + queue-config a loop pktio (not started)."""
    p = pktio_open("loop")
    assert p, "odp_pktio_open(loop) failed"
    assert pktio_config(p, pktin=pktin) == 0
    assert pktin_queue_config(p, classifier_enable=classifier) == 0
    return p


def queue(n):
    """A distinct application queue handle (the classifier only stores them)."""
    return 0x1000 + n
