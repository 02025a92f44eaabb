"""The odp_cls API boundary is ABI-equal to the reference: every struct the
API passes has the reference's x86-64 layout, field by field and bit by bit,
and the enum / constant values match.

Expected layouts: tests/golden/ref_abi_layout.json, computed from the
reference header text by tests/golden/make_abi_layout.py (the reference
headers need configure-generated files, so they are parsed, not compiled).
Actual layouts: a probe compiled with gcc against include/odp_cls.h."""
import ctypes as C
import json
import os
import subprocess

import pytest

from odp_amd import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = json.load(open(os.path.join(HERE, "golden", "ref_abi_layout.json")))


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    lines = ['#include <stdio.h>', '#include <string.h>', '#include <stddef.h>',
             '#include "odp_cls.h"',
             'static int bitpos(const unsigned char *p, size_t n, int *w)',
             '{ int first = -1, cnt = 0; for (size_t i = 0; i < n * 8; i++)',
             '  if (p[i / 8] >> (i % 8) & 1) { if (first < 0) first = (int)i; cnt++; }',
             '  *w = cnt; return first; }',
             'int main(void) {', 'int w;']
    for t, v in REF["types"].items():
        lines.append(f'printf("T {t} %zu %zu\\n", sizeof({t}), _Alignof({t}));')
        for path, _, _ in v["fields"]:
            lines.append(f'printf("F {t} {path} %zu %zu\\n", offsetof({t}, {path}), '
                         f'sizeof((({t} *)0)->{path}));')
        for path, _, _ in v["bits"]:
            lines.append(f'{{ {t} x; memset(&x, 0, sizeof x); x.{path} = 1; '
                         f'int p = bitpos((const unsigned char *)&x, sizeof x, &w); '
                         f'memset(&x, 0, sizeof x); x.{path} = ~0ull; '
                         f'bitpos((const unsigned char *)&x, sizeof x, &w); '
                         f'printf("B {t} {path} %d %d\\n", p, w); }}')
    for n in REF["enums"]:
        lines.append(f'printf("E {n} %lld\\n", (long long){n});')
    for n in REF["defines"]:
        lines.append(f'printf("D {n} %lld\\n", (long long)({n}));')
    lines += ['return 0; }']
    d = tmp_path_factory.mktemp("abi")
    src, exe = d / "probe.c", d / "probe"
    src.write_text("\n".join(lines) + "\n")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wno-overflow", "-I", os.path.join(ROOT, "include"),
                    str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    got = {"T": {}, "F": {}, "B": {}, "E": {}, "D": {}}
    for ln in out.splitlines():
        k, *rest = ln.split()
        if k == "T":
            got["T"][rest[0]] = (int(rest[1]), int(rest[2]))
        elif k in ("F", "B"):
            got[k][(rest[0], rest[1])] = (int(rest[2]), int(rest[3]))
        else:
            got[k][rest[0]] = int(rest[1])
    return got


@pytest.mark.parametrize("t", sorted(REF["types"]))
def test_struct_layout(probe, t):
    want = REF["types"][t]
    assert probe["T"][t] == (want["size"], want["align"]), t
    for path, off, size in want["fields"]:
        assert probe["F"][(t, path)] == (off, size), (t, path)
    for path, bit, width in want["bits"]:
        assert probe["B"][(t, path)] == (bit, width), (t, path)


def test_enums_and_constants(probe):
    for n, v in REF["enums"].items():
        assert probe["E"][n] == v, n
    for n, v in REF["defines"].items():
        assert probe["D"][n] == v, n


def test_ctypes_mirrors_match():
    """odp_amd/_lib.py's ctypes mirrors have the C sizes (Python host side)."""
    for t in ("odp_cls_cos_param_t", "odp_cls_capability_t", "odp_pktio_config_t",
              "odp_pktin_queue_param_t", "odp_queue_param_t", "odp_pmr_param_t",
              "odp_pmr_create_opt_t", "odp_pktio_stats_t", "odp_cls_cos_stats_t"):
        assert C.sizeof(getattr(L, t)) == REF["types"][t]["size"], t
    assert L.odp_cls_cos_param_t.pool.offset == 80 and L.odp_pktio_config_t.pause_rx.offset == 48
