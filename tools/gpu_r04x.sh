# Round-4 final evidence on the final tree: GPU suite, smoke, the driver's bench command (with the CPU baseline) and
# the rocprofv3 --kernel-trace --stats run of it.  usage: bash tools/gpu_r04x.sh <out-subdir>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04x}; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc: $(tail -1 $O/pytest_gpu.log)"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python3 bench.py --steps 20 --warmup 5 --progress 30 > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_prof.json 2> $O/bench_prof.err; echo "prof exit $?"
