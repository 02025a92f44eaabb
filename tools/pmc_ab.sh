cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in base exp_nokeys; do
  if [ $v = base ]; then lib=""; else lib="$PWD/odp_amd/lib/$v/libodpg.so"; fi
  ODPG_LIB="$lib" timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcab_$v -o run -- python3 bench.py --no-cpu --no-stats --config c3 --steps 20 --warmup 2 > gpurun_out/pmcab_$v.log 2>&1 || exit $?
  ODPG_LIB="$lib" timeout -k 10 120 python bench.py --no-cpu --no-stats --config c3 --steps 50 --warmup 5 > gpurun_out/ab_$v.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', d['value'], d['roofline']['kernel_ms'])"
done
