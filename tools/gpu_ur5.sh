# UR5 arm on the GPU: its test module, then a bench line at batch $2 (default 4096).
# usage (on the box via gpurun): bash tools/gpu_ur5.sh <out-subdir> [batch]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ur5}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ur5.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_ur5.log 2>&1 && echo pytest_ur5_ok &&
VBOC_PROGRESS=1 timeout -k 10 500 python -u bench.py --nq 4 --batch ${2:-100000} --warmup 0 --cpu-seconds 15 > $O/bench_ur5.json 2> $O/bench_ur5.err && cat $O/bench_ur5.json
