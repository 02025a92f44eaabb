"""Thin Python driver for the odpg.h C-ABI (device buffers, tables, launches).

All compute happens in ``libodpg.so``'s gfx950 kernels; this module moves
numpy arrays in and out of HBM through the library's own helpers.
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from . import _lib as L

lib = L.lib


class DeviceBuffer:
    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        L.check(lib.odpg_dev_alloc(ctx.h, max(self.nbytes, 16), C.byref(p)), "odpg_dev_alloc")
        self.ptr = p.value

    def upload(self, arr):
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        L.check(lib.odpg_memcpy_h2d(self.ctx.h, self.ptr, a.ctypes.data, a.nbytes), "h2d")

    def download(self, dtype, count):
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            L.check(lib.odpg_memcpy_d2h(self.ctx.h, out.ctypes.data, self.ptr, out.nbytes),
                    "d2h")
        return out

    def zero(self):
        L.check(lib.odpg_memset_dev(self.ctx.h, self.ptr, 0, self.nbytes), "memset")

    def free(self):
        if self.ptr:
            if self.ctx.h:
                lib.odpg_dev_free(self.ctx.h, self.ptr)
            self.ptr = None

    def __del__(self):
        if sys.is_finalizing():   # the HIP runtime may be torn down already
            return
        try:
            self.free()
        except Exception:
            pass


def compile_rules(rules):
    """Compiled-table image of `rules` (host only, odpg_rules_compile): the
    bytes a multi-GPU job compiles once and broadcasts."""
    n = C.c_size_t(0)
    rc = lib.odpg_rules_compile(C.byref(rules), None, C.byref(n))
    if rc not in (0, -28):                 # -ENOSPC: size query
        L.check(rc, "odpg_rules_compile")
    buf = (C.c_uint8 * n.value)()
    L.check(lib.odpg_rules_compile(C.byref(rules), buf, C.byref(n)), "odpg_rules_compile")
    return bytes(buf)


class Table:
    def __init__(self, ctx, rules=None, image=None):
        t = C.c_void_p()
        if image is not None:
            b = (C.c_uint8 * len(image)).from_buffer_copy(image)
            L.check(lib.odpg_table_import(ctx.h, b, len(image), C.byref(t)), "odpg_table_import")
        else:
            L.check(lib.odpg_table_create(ctx.h, C.byref(rules), C.byref(t)),
                    "odpg_table_create")
        self.h = t.value
        self.num_cos = lib.odpg_table_num_cos(self.h)
        self.has_cycle = bool(lib.odpg_table_has_cycle(self.h))

    def __del__(self):
        if sys.is_finalizing():   # the HIP runtime may be torn down already
            return
        try:
            if self.h:
                lib.odpg_table_destroy(self.h)
                self.h = None
        except Exception:
            pass


class Counters:
    """Sharded device counters of one table layout (odpg.h "sharded
    counters"): launches add into per-workgroup rows; fold() sums them."""

    def __init__(self, ctx, table):
        h = C.c_void_p()
        L.check(lib.odpg_counters_create(ctx.h, table.h, C.byref(h)), "odpg_counters_create")
        self.h = h.value
        self.ctx = ctx
        self.num_cos = table.num_cos
        self.words = 4 + self.num_cos + self.num_cos * L.COS_QUEUE_MAX

    def fold(self):
        """Counts since the last fold: {"pktio": [in_packets, in_octets,
        in_errors, in_discards], "cos": per-CoS packets, "queue": [num_cos,
        COS_QUEUE_MAX] delivered packets}."""
        w = np.zeros(self.words, np.uint64)
        L.check(lib.odpg_counters_fold(self.h, w.ctypes.data_as(C.POINTER(C.c_uint64))),
                "odpg_counters_fold")
        n = self.num_cos
        return {"pktio": w[:4], "cos": w[4:4 + n],
                "queue": w[4 + n:].reshape(n, L.COS_QUEUE_MAX)}

    def close(self):
        if self.h:
            # valid after the context's destroy too: the counters hold a
            # reference to it (odpg.h "object lifetimes")
            lib.odpg_counters_destroy(self.h)
            self.h = None

    def __del__(self):
        if sys.is_finalizing():   # the HIP runtime may be torn down already
            return
        try:
            self.close()
        except Exception:
            pass


class Context:
    def __init__(self, device=0, stream=None):
        n = lib.odpg_device_count()
        if n <= 0:
            raise RuntimeError("no HIP device visible (odpg_device_count() == 0)")
        h = C.c_void_p()
        L.check(lib.odpg_ctx_create(device, stream, C.byref(h)), "odpg_ctx_create")
        self.h = h.value
        self.device = device

    def close(self):
        if self.h:
            lib.odpg_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        if sys.is_finalizing():   # the HIP runtime may be torn down already
            return
        try:
            self.close()
        except Exception:
            pass

    def set_kernel_mode(self, mode):
        """0 auto, 1 wave-cooperative walk, 2 evaluate-all, 3 hash walk (same results)."""
        L.check(lib.odpg_ctx_set_kernel_mode(self.h, mode), "odpg_ctx_set_kernel_mode")

    def sync(self):
        L.check(lib.odpg_ctx_sync(self.h), "odpg_ctx_sync")

    def buffer(self, nbytes):
        return DeviceBuffer(self, nbytes)

    def table(self, rules=None, image=None):
        return Table(self, rules, image)

    def counters(self, table):
        return Counters(self, table)

    def classify_dev(self, table, frames_buf, num, stride=0, desc_buf=None, opt=0,
                     layer=L.LAYER_ALL, classify=True, out_buf=None, mark_buf=None,
                     meta_buf=None, stats_buf=None, counters=None):
        b = L.odpg_batch_t(frames_buf.ptr, desc_buf.ptr if desc_buf else None, stride, num,
                           opt, layer, int(bool(classify)))
        r = L.odpg_result_t(out_buf.ptr if out_buf else None,
                            mark_buf.ptr if mark_buf else None,
                            meta_buf.ptr if meta_buf else None,
                            stats_buf.ptr if stats_buf else None,
                            counters.h if counters else None)
        L.check(lib.odpg_classify(self.h, table.h, C.byref(b), C.byref(r)), "odpg_classify")

    def classify(self, table, frames, num, stride=0, desc=None, opt=0, layer=L.LAYER_ALL,
                 classify=True, want_mark=True, want_meta=True, want_stats=True,
                 counters=None):
        """Upload host arrays, classify on the GPU, download results. With
        `counters` the launch adds into those (want_stats is ignored)."""
        if counters is not None:
            want_stats = False
        meta_dt, desc_dt = L.np_dtypes()
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        fb = self.buffer(frames.nbytes + 64)
        fb.upload(frames)
        db = None
        if desc is not None:
            desc = np.ascontiguousarray(desc, dtype=desc_dt)
            db = self.buffer(desc.nbytes)
            db.upload(desc)
        ob = self.buffer(4 * num)
        mb = self.buffer(2 * num) if want_mark else None
        eb = self.buffer(24 * num) if want_meta else None
        nst = 4 + table.num_cos
        sb = self.buffer(8 * nst) if want_stats else None
        if sb:
            sb.zero()
        self.classify_dev(table, fb, num, stride, db, opt, layer, classify, ob, mb, eb, sb,
                          counters)
        self.sync()
        res = {"out": ob.download(np.uint32, num)}
        if mb:
            res["mark"] = mb.download(np.uint16, num)
        if eb:
            res["meta"] = eb.download(meta_dt, num)
        if sb:
            res["stats"] = sb.download(np.uint64, nst)
        for b in (fb, db, ob, mb, eb, sb):
            if b:
                b.free()
        return res

    def tx_prepare(self, frames, num, stride=0, desc=None, meta=None, pktout_cfg=0,
                   pktout_capa=L.PKTOUT_LOOP_CAPA, hash_proto=0, num_qs=1, index=0):
        """loopback_send()'s checksum insertion + loop queue pick on the GPU
        (include/odpg_tx.h). Returns (out words, rewritten frames)."""
        _, desc_dt = L.np_dtypes()
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        fb = self.buffer(frames.nbytes + 64)
        fb.upload(frames)
        db = mb = None
        if desc is not None:
            desc = np.ascontiguousarray(desc, dtype=desc_dt)
            db = self.buffer(desc.nbytes)
            db.upload(desc)
        if meta is not None:
            meta = np.ascontiguousarray(meta, dtype=np.dtype(L.TX_META_FIELDS))
            mb = self.buffer(meta.nbytes)
            mb.upload(meta)
        ob = self.buffer(4 * num)
        b = L.odpg_tx_batch_t(fb.ptr, db.ptr if db else None, stride, num,
                              mb.ptr if mb else None)
        c = L.odpg_tx_cfg_t(pktout_cfg, pktout_capa, hash_proto, num_qs, index, 0)
        L.check(lib.odpg_tx_prepare(self.h, C.byref(b), C.byref(c), ob.ptr), "odpg_tx_prepare")
        self.sync()
        out = ob.download(np.uint32, num)
        fr = fb.download(np.uint8, frames.nbytes)
        for x in (fb, db, mb, ob):
            if x:
                x.free()
        return out, fr

    def classify_host(self, table, frames, num, stride=0, desc=None, opt=0,
                      layer=L.LAYER_ALL, classify=True, chunk=0, want_mark=False,
                      want_meta=False, want_stats=True):
        meta_dt, desc_dt = L.np_dtypes()
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        dptr = None
        if desc is not None:
            desc = np.ascontiguousarray(desc, dtype=desc_dt)
            dptr = desc.ctypes.data
        out = np.zeros(num, np.uint32)
        mark = np.zeros(num, np.uint16) if want_mark else None
        meta = np.zeros(num, meta_dt) if want_meta else None
        stats = np.zeros(4 + table.num_cos, np.uint64) if want_stats else None
        b = L.odpg_batch_t(frames.ctypes.data, dptr, stride, num, opt, layer,
                           int(bool(classify)))
        r = L.odpg_result_t(out.ctypes.data, mark.ctypes.data if mark is not None else None,
                            meta.ctypes.data if meta is not None else None,
                            stats.ctypes.data if stats is not None else None)
        L.check(lib.odpg_classify_host(self.h, table.h, C.byref(b), C.byref(r), chunk),
                "odpg_classify_host")
        res = {"out": out}
        if mark is not None:
            res["mark"] = mark
        if meta is not None:
            res["meta"] = meta
        if stats is not None:
            res["stats"] = stats
        return res


def group_range(num, n, member):
    """odpg_group_range: member's packet range [lo, hi) of a num-packet batch
    over n members (host arithmetic, no device)."""
    lo, hi = C.c_uint32(), C.c_uint32()
    lib.odpg_group_range(num, n, member, C.byref(lo), C.byref(hi))
    return lo.value, hi.value


class Group:
    """Several device contexts classifying one batch by packet range
    (include/odpg_group.h): the table compiled once and imported per member,
    per-member counters summed when folded."""

    def __init__(self, devices):
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        L.check(lib.odpg_group_create(devs, len(devices), C.byref(h)), "odpg_group_create")
        self.h = h.value
        self.n = len(devices)
        self.num_cos = 0

    def close(self):
        if self.h:
            lib.odpg_group_destroy(self.h)
            self.h = None

    def __del__(self):
        if sys.is_finalizing():   # the HIP runtime may be torn down already
            return
        try:
            self.close()
        except Exception:
            pass

    def load(self, rules):
        L.check(lib.odpg_group_load(self.h, C.byref(rules)), "odpg_group_load")
        self.num_cos = lib.odpg_table_num_cos(lib.odpg_group_table(self.h, 0))

    def ctx_handle(self, member):
        return lib.odpg_group_ctx(self.h, member)

    def classify_host(self, frames, num, stride=0, desc=None, opt=0, layer=L.LAYER_ALL,
                      counted=False, chunk=0):
        """Host arrays in, verdict words out (odpg_group_classify_host)."""
        _, desc_dt = L.np_dtypes()
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        dptr = None
        if desc is not None:
            desc = np.ascontiguousarray(desc, dtype=desc_dt)
            dptr = desc.ctypes.data
        out = np.zeros(num, np.uint32)
        b = L.odpg_batch_t(frames.ctypes.data, dptr, stride, num, opt, layer, 1)
        r = L.odpg_result_t(out.ctypes.data, None, None, None, None)
        L.check(lib.odpg_group_classify_host(self.h, C.byref(b), C.byref(r), int(counted), chunk),
                "odpg_group_classify_host")
        return out

    def classify_shards(self, frames, num, stride, opt=0, counted=False, desc=None):
        """Device-resident shards: member i's range uploaded to its own HBM
        (fixed stride: its frames; with descriptors: the whole frame buffer
        and its range's descriptors, offsets relative to that buffer), all
        members launched (odpg_group_classify), synced, verdicts gathered."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        B = (L.odpg_batch_t * self.n)()
        R = (L.odpg_result_t * self.n)()
        bufs = []
        for i in range(self.n):
            lo, hi = group_range(num, self.n, i)
            ctx = _CtxView(self.ctx_handle(i))
            db = None
            if desc is None:
                fb = DeviceBuffer(ctx, max(16, (hi - lo) * stride))
                if hi > lo:
                    fb.upload(frames[lo * stride:hi * stride])
            else:
                fb = DeviceBuffer(ctx, max(16, frames.nbytes))
                fb.upload(frames)
                d = np.ascontiguousarray(desc[lo:hi])
                db = DeviceBuffer(ctx, max(16, d.nbytes))
                if hi > lo:
                    db.upload(d)
            ob = DeviceBuffer(ctx, max(16, 4 * (hi - lo)))
            B[i] = L.odpg_batch_t(fb.ptr, db.ptr if db else None, 0 if db else stride, hi - lo,
                                  opt, L.LAYER_ALL, 1)
            R[i] = L.odpg_result_t(ob.ptr, None, None, None, None)
            bufs.append((lo, hi, fb, ob, db))
        L.check(lib.odpg_group_classify(self.h, B, R, int(counted)), "odpg_group_classify")
        L.check(lib.odpg_group_sync(self.h), "odpg_group_sync")
        out = np.zeros(num, np.uint32)
        for lo, hi, fb, ob, db in bufs:
            if hi > lo:
                out[lo:hi] = ob.download(np.uint32, hi - lo)
            fb.free()
            ob.free()
            if db:
                db.free()
        return out

    def fold(self):
        w = np.zeros(4 + self.num_cos + self.num_cos * L.COS_QUEUE_MAX, np.uint64)
        L.check(lib.odpg_group_counters_fold(self.h, w.ctypes.data_as(C.POINTER(C.c_uint64))),
                "odpg_group_counters_fold")
        n = self.num_cos
        return {"pktio": w[:4], "cos": w[4:4 + n],
                "queue": w[4 + n:].reshape(n, L.COS_QUEUE_MAX)}


class _CtxView:
    """A member context of a Group, for DeviceBuffer (not owned)."""

    def __init__(self, h):
        self.h = h


class Forwarder:
    """example/l3fwd forwarding table on the device (include/odpg_fwd.h)."""

    def __init__(self, ctx, routes, mode=L.FWD_HASH, port_mac=None, dest_mac=None, num_ports=4):
        self.ctx = ctx
        self.routes = make_routes(routes)
        self.param = make_fwd_param(mode, num_ports, port_mac, dest_mac)
        h = C.c_void_p()
        L.check(lib.odpg_fwd_create(ctx.h, self.routes, len(self.routes), C.byref(self.param),
                                    C.byref(h)), "odpg_fwd_create")
        self.h = h.value

    def __del__(self):
        if sys.is_finalizing():   # the HIP runtime may be torn down already
            return
        try:
            if self.h:
                lib.odpg_fwd_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def run_dev(self, frames_buf, stride, num, out_buf, src_port=0, error_check=False):
        b = L.odpg_fwd_batch_t(frames_buf.ptr, stride, num, src_port, int(bool(error_check)))
        L.check(lib.odpg_l3fwd(self.ctx.h, self.h, C.byref(b), out_buf.ptr), "odpg_l3fwd")

    def run(self, frames, stride, num, src_port=0, error_check=False):
        """Upload, forward, download: returns (out_port int32[num], frames)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        fb = self.ctx.buffer(frames.nbytes + 64)
        fb.upload(frames)
        ob = self.ctx.buffer(4 * num)
        self.run_dev(fb, stride, num, ob, src_port, error_check)
        self.ctx.sync()
        out = ob.download(np.int32, num)
        fr = fb.download(np.uint8, frames.nbytes)
        fb.free()
        ob.free()
        return out, fr


def make_routes(routes):
    """[(addr, depth, oif_id, src_mac, dst_mac), ...] -> ctypes odpg_route_t array."""
    arr = (L.odpg_route_t * len(routes))()
    for k, (addr, depth, oif, smac, dmac) in enumerate(routes):
        arr[k].addr, arr[k].depth, arr[k].oif_id = addr, depth, oif
        for j in range(6):
            arr[k].src_mac[j] = smac[j]
            arr[k].dst_mac[j] = dmac[j]
    return arr


def make_fwd_param(mode, num_ports, port_mac=None, dest_mac=None):
    p = L.odpg_fwd_param_t()
    p.mode, p.num_ports = mode, num_ports
    for i in range(L.FWD_MAX_PORTS):
        pm = port_mac[i] if port_mac and i < len(port_mac) else [0x02, 0, 0, 0xAA, 0, i]
        dm = dest_mac[i] if dest_mac and i < len(dest_mac) else [0x02, 0, 0, 0xBB, 0, i]
        for j in range(6):
            p.port_mac[i][j] = pm[j]
            p.dest_mac[i][j] = dm[j]
    return p
