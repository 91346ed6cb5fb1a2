set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02a_pytest_gpu.log; exit 1; }
tail -5 gpurun_out/r02a_pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/r02a_bench_tri.json 2> gpurun_out/r02a_bench_tri.err || exit 1
cat gpurun_out/r02a_bench_tri.json
timeout -k 10 300 python -u bench.py --nq 4 --batch 12500 --steps 1 --warmup 1 --no-cpu > gpurun_out/r02a_bench_ur5.json 2> gpurun_out/r02a_bench_ur5.err || exit 1
cat gpurun_out/r02a_bench_ur5.json
