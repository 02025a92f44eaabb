#!/bin/bash
# Where C2x's instructions go: SQ instruction counters of experiment builds
# that each leave out one part of the tile (results wrong by design).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06j
mkdir -p $OUT
for v in base exp_gf_noprobe exp_gf_nowalk exp_gf_noparse exp_gf_noshift exp_gf_noplain; do
  lib=""; [ $v = base ] || lib="$PWD/odp_amd/lib/$v/libodpg.so"
  ODPG_LIB="$lib" timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH \
    --output-format csv -d $OUT/$v/p1 -o run -- python3 bench.py --no-cpu --no-stats --config c2x --steps 20 --warmup 2 --runs 1 > $OUT/$v.log 2>&1 || exit $?
  python tools/pmc_summary.py $OUT/$v > $OUT/$v.json 2>&1
  ODPG_LIB="$lib" timeout -k 10 120 python bench.py --no-cpu --no-stats --config c2x --runs 3 --others none > $OUT/$v.bench 2>/dev/null || exit $?
  python - $OUT/$v.json $OUT/$v.bench $v <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); b=json.load(open(sys.argv[2]))
k=[x for x in d if "clsgf" in x][0]; v=d[k]; t=16384
print(sys.argv[3], "us", round(b["roofline"]["kernel_ms"]*1000,2), " ".join(f"{c[9:]}={v[c]/t:.0f}" for c in ("SQ_INSTS_VALU","SQ_INSTS_SALU","SQ_INSTS_LDS","SQ_INSTS_BRANCH")))
PY
done
