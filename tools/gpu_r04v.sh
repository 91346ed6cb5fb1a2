# Round-4 call V: the driver's bench command with restart jobs before parked resumes (--spec-first 1) beside the
# default, same box (the tail A/B at the driver's 400k launch and at its 100k warmup round)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04v}; mkdir -p $O
cd $R
timeout -k 10 420 python3 bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_default.json 2> $O/bench_default.err; rc=$?; echo "default exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python3 bench.py --steps 20 --warmup 5 --no-cpu --progress 30 --spec-first 1 > $O/bench_spec_first.json 2> $O/bench_spec_first.err; rc=$?; echo "spec_first exit $rc"
