set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or ragged or properties" > gpurun_out/r02c_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r02c_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02c_pytest_gpu.log
VBOC_LIB= timeout -k 10 200 python -u tools/scratch/ur5_bisect.py tools/scratch/ref_tri_96.npz tri_mfma > gpurun_out/r02c_tri96.log 2>&1; cat gpurun_out/r02c_tri96.log
VBOC_LIB=vboc_amd/libvboc_amd_prof.so timeout -k 10 400 python -u tools/scratch/phase_ab.py 3 16384 0 > gpurun_out/r02c_phase_ab.log 2>&1; cat gpurun_out/r02c_phase_ab.log
for f in mfma valu; do
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --factor $f > gpurun_out/r02c_bench_tri_$f.json 2> gpurun_out/r02c_bench_tri_$f.err || exit 1
cat gpurun_out/r02c_bench_tri_$f.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['solver'])"
done
