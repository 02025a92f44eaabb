"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU restatement
(``oracle/build/libodp_oracle.so``, built from ``oracle/odp_oracle.c``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module; the product (``odp_amd``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libodp_oracle.so")


def build():
    subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)


def _load():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    lib.oracle_classify.restype = i32
    lib.oracle_classify.argtypes = [vp, vp, vp, u32, u32, u64, i32, i32, vp, vp, vp, vp]
    lib.oracle_classify_mt.restype = i32
    lib.oracle_classify_mt.argtypes = [vp, vp, vp, u32, u32, u64, i32, i32, vp, i32, u32]
    lib.oracle_chksum_ones_comp16.restype = C.c_uint16
    lib.oracle_chksum_ones_comp16.argtypes = [vp, u32]
    lib.oracle_crc32c.restype = u32
    lib.oracle_crc32c.argtypes = [vp, u32, u32]
    lib.oracle_thash.restype = u32
    lib.oracle_thash.argtypes = [vp, u32]
    return lib


lib = _load()

META_DT = np.dtype([("input_flags", "<u8"), ("flags", "<u4"), ("l2_offset", "<u2"),
                    ("l3_offset", "<u2"), ("l4_offset", "<u2"), ("cls_mark", "<u2"),
                    ("reserved", "<u4")])
DESC_DT = np.dtype([("offset", "<u4"), ("len", "<u4")])


def classify(rules, frames, num, stride=0, desc=None, opt=0, layer=4, classify=True,
             num_cos=None):
    """Run the CPU restatement. `rules` is an odpg_rules_t (ctypes struct)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    dptr = None
    if desc is not None:
        desc = np.ascontiguousarray(desc, dtype=DESC_DT)
        dptr = desc.ctypes.data
    out = np.zeros(num, np.uint32)
    mark = np.zeros(num, np.uint16)
    meta = np.zeros(num, META_DT)
    ncos = rules.num_cos if num_cos is None else num_cos
    stats = np.zeros(4 + ncos, np.uint64)
    lib.oracle_classify(C.byref(rules), frames.ctypes.data, dptr, stride, num, opt, layer,
                        int(bool(classify)), out.ctypes.data, mark.ctypes.data,
                        meta.ctypes.data, stats.ctypes.data)
    return {"out": out, "mark": mark, "meta": meta, "stats": stats}


def classify_mt(rules, frames, num, stride=0, desc=None, opt=0, layer=4, classify=True,
                nthreads=1, reps=1):
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    dptr = None
    if desc is not None:
        desc = np.ascontiguousarray(desc, dtype=DESC_DT)
        dptr = desc.ctypes.data
    out = np.zeros(num, np.uint32)
    n = lib.oracle_classify_mt(C.byref(rules), frames.ctypes.data, dptr, stride, num, opt,
                               layer, int(bool(classify)), out.ctypes.data, nthreads, reps)
    return out, n


def ones_comp16(data: bytes) -> int:
    b = np.frombuffer(bytes(data), np.uint8)
    return lib.oracle_chksum_ones_comp16(b.ctypes.data if len(b) else None, len(b))


def crc32c(data: bytes, init=0xFFFFFFFF) -> int:
    b = np.frombuffer(bytes(data), np.uint8)
    return lib.oracle_crc32c(b.ctypes.data if len(b) else None, len(b), init)


def thash(words) -> int:
    a = np.ascontiguousarray(words, dtype=np.uint32)
    return lib.oracle_thash(a.ctypes.data, len(a))
