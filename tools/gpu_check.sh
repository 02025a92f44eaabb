# GPU check: the gpu test suite, the C2 bench line and the recv_batch bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu ${BENCH_EXTRA:-} > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -n 5 gpurun_out/bench_c2.err; exit 3; }
cat gpurun_out/bench_c2.json
timeout -k 10 120 ./odp_amd/lib/odp_bench_cls_gpu > gpurun_out/bench_cls_gpu.txt 2>&1 || { tail -n 5 gpurun_out/bench_cls_gpu.txt; exit 4; }
tail -n 6 gpurun_out/bench_cls_gpu.txt
