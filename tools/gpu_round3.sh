# Round-3 GPU evidence on the box (gpurun): kernel time of the product vs the round-2 build, per-phase cycles of a
# profiling build, the GPU test suite, smoke(), and the UR5 merit reproducer.
# usage: bash tools/gpu_round3.sh <out-subdir> <prof variant>
set -o pipefail
R=$GRAFT_REPO_ROOT; S=${1:-r03}; O=$R/gpurun_out/$S; mkdir -p $O
bash $R/tools/ring_depth.sh $S base -- $2 || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke_ok || exit 1
bash $R/tools/ur5_merit_repro.sh run $S/ur5_merit
