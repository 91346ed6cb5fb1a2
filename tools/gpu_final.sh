# Round-end evidence (on the box via gpurun): GPU test suite, smoke(), the driver's bench command with its
# rocprofv3 kernel stats, and the double pendulum's configs[1] first-solve line.
# usage: bash tools/gpu_final.sh <out-subdir>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo pytest_ok &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke_ok &&
timeout -k 10 420 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
timeout -k 10 120 python bench.py --workload first-solve --nq 2 --batch 10000 --steps 1 --warmup 1 > $O/bench_double_10k.json 2> $O/bench_double_10k.err && echo double_ok &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err && echo prof_ok
