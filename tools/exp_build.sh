#!/bin/bash
# Experiment build of libodpg.so into odp_amd/lib/<name>: the base build's
# objects, with the sources named in REBUILD (default classify_gf) compiled
# again under the given -D flags. Usage: bash tools/exp_build.sh exp_x "-DFOO -DBAR=2"
set -eu
cd "$(dirname "$0")/../odp_amd/csrc"
name=$1; flags=${2:-}
mkdir -p ../lib/$name
for o in ../lib/*.o; do cp -p "$o" ../lib/$name/; done
for s in ${REBUILD:-classify_gf}; do rm -f ../lib/$name/$s.o; done
make -s OUT=../lib/$name EXTRA="$flags" ../lib/$name/libodpg.so
rm -f ../lib/$name/*.o
