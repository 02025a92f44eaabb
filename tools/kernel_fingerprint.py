"""Fingerprint of the device code's sources: sha256 over the HIP kernels,
their headers, the table compiler and the build flags (odp_amd/csrc). PMC
summaries record it (tools/pmc_summary.py --write) and bench.py compares it
with the tree it runs from, so a traffic figure measured on other kernels is
reported as stale. Host-only sources (odp_cls.c, odp_rt.c, pcap.c) are left
out: they do not change what the kernels read and write."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fingerprint(root=ROOT):
    c = os.path.join(root, "odp_amd", "csrc")
    files = sorted(glob.glob(os.path.join(c, "*.hip")) + glob.glob(os.path.join(c, "*.h")) +
                   [os.path.join(c, "cls_compile.cpp"), os.path.join(c, "Makefile")])
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()


if __name__ == "__main__":
    print(fingerprint())
