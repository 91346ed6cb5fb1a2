# Resident-problem sweep of k_dg at the driver's launch shape (bench.py --steps 20 --warmup 5, no CPU leg): the
# default sizes the resident set to the 256 MiB MALL (1 324 groups for the triple's data generation); round 1's
# sweep that chose it was of k_wave.  usage: bash tools/gpu_r04y.sh <out-subdir>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04y}; mkdir -p $O
cd $R
for g in ${GROUPS_LIST:-1664 2048 1024 1324}; do
  timeout -k 10 420 python3 bench.py --steps 20 --warmup 5 --no-cpu --progress 30 --wave-groups $g > $O/bench_g$g.json 2> $O/bench_g$g.err
  rc=$?; echo "groups $g exit $rc: $(grep -o '"value": [0-9.]*' $O/bench_g$g.json | head -1)"; [ $rc -eq 0 ] || exit $rc
done
