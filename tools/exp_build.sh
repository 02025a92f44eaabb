#!/bin/bash
# Experiment build of libodpg.so into odp_amd/lib/<name>: the base build's
# objects, with the sources named in REBUILD (default classify_gf) compiled
# again under the given -D flags and with the experiment patches named in
# PATCHES (tools/exp/<patch>.patch, applied to a scratch copy of the
# sources; the shipped kernels carry no experiment switches).
# Usage: bash tools/exp_build.sh exp_x "-DFOO -DBAR=2"
#        PATCHES="l64_times" REBUILD=classify64 bash tools/exp_build.sh exp_times
set -eu
root="$(cd "$(dirname "$0")/.." && pwd)"
name=$1; flags=${2:-}
src="$root/odp_amd/csrc_$name"
rm -rf "$src" && cp -a "$root/odp_amd/csrc" "$src"
trap 'rm -rf "$src"' EXIT
for p in ${PATCHES:-}; do
	patch -s -d "$src" -p0 < "$root/tools/exp/$p.patch"
done
mkdir -p "$root/odp_amd/lib/$name"
for o in "$root"/odp_amd/lib/*.o; do cp -p "$o" "$root/odp_amd/lib/$name/"; done
for s in ${REBUILD:-classify_gf}; do rm -f "$root/odp_amd/lib/$name/$s.o"; done
# patched sources are newer than the copied objects of the files they touch
make -s -C "$src" OUT="../lib/$name" EXTRA="$flags" "../lib/$name/libodpg.so"
rm -f "$root/odp_amd/lib/$name"/*.o
