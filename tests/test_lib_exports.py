"""The C-ABI library loads and exports every function include/*.h declares
(no compute calls: this runs on CPU-only hosts)."""
import os
import re
import subprocess

from odp_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROTO = re.compile(r"^[A-Za-z_][\w \*]*?\b((?:odpg|odp)_\w+)\s*\(", re.M)


def declared():
    names = set()
    for h in sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h")):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = re.sub(r"^#.*$", "", txt, flags=re.M)
        txt = re.sub(r"typedef[^;]*;", "", txt, flags=re.S)
        for m in PROTO.finditer(txt):
            names.add(m.group(1))
    return names


def test_headers_declare_something():
    d = declared()
    assert "odpg_classify" in d and "odp_cls_cos_create" in d and "odpg_l3fwd" in d
    assert len(d) > 60


def test_every_declared_symbol_exported():
    nm = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    missing = sorted(declared() - exported)
    assert not missing, missing


def test_every_declared_symbol_bound():
    assert declared() <= set(L.SIGNATURES), sorted(declared() - set(L.SIGNATURES))


def test_library_is_gfx950():
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        return
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", L.LIB_PATH], capture_output=True,
                         text=True).stdout if os.path.exists("/opt/rocm/bin/roc-obj-ls") else ""
    if out:
        assert "gfx950" in out


def test_abi_version_without_gpu():
    assert L.lib.odpg_abi_version() == L.ABI_VERSION == 2
    assert b"gfx950" in L.lib.odpg_build_info()
