# One GPU round: GPU test suite, default bench line, rocprofv3 kernel stats of the bench command.
# usage (on the box via gpurun): bash tools/gpu_round.sh <out-subdir>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-round}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo pytest_ok &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err && echo prof_ok
