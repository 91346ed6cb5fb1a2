set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probes/mfma_f64_layout > gpurun_out/r02b_mfma_probe.log 2>&1; cat gpurun_out/r02b_mfma_probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "parity or ragged or properties" > gpurun_out/r02b_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r02b_pytest_gpu.log; exit 1; }
tail -15 gpurun_out/r02b_pytest_gpu.log
VBOC_LIB= timeout -k 10 200 python -u tools/scratch/ur5_bisect.py tools/scratch/ref_tri_96.npz tri_mfma > gpurun_out/r02b_tri96.log 2>&1; cat gpurun_out/r02b_tri96.log
for f in mfma valu; do
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --factor $f > gpurun_out/r02b_bench_tri_$f.json 2> gpurun_out/r02b_bench_tri_$f.err || exit 1
cat gpurun_out/r02b_bench_tri_$f.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['solver'])"
done
