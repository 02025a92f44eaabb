#!/bin/bash
# Register / spill counts per classify-kernel instantiation (gfx950 ISA of
# classify.hip, or the file given): name  sgpr  sgpr_spill  vgpr
set -u
SRC="$(realpath "${1:-$(dirname "$0")/../odp_amd/csrc/classify.hip}")"
T=$(mktemp -d)
(cd $T && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --save-temps ${KFLAGS:-} -c "$SRC" -o k.o 2>/dev/null)
grep -E "^\s+\.(name|sgpr_count|sgpr_spill_count|vgpr_count|vgpr_spill_count):" $T/*gfx950.s | paste - - - - - |
  awk '{print $2, "sgpr="$4, "sspill="$6, "vgpr="$8, "vspill="$10}' | c++filt | sed 's/(.*)//'
rm -rf $T
