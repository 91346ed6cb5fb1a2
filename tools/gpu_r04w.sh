# Round-4 call W: the critical-path rule for speculative restarts (dg_spec_crit): results unchanged (GPU test), the
# 60k / 100k launches and the driver's bench command with it on and off, same box
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04w}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_dg_device.py -m gpu -v --timeout 240 --timeout-method thread -k "change_nothing" > $O/pytest_spec.log 2>&1
rc=$?; echo "pytest exit $rc: $(tail -1 $O/pytest_spec.log)"; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 60000 --spec-crit 0 1 --save $O/s60k > $O/probe_60k.jsonl 2> $O/probe_60k.err; rc=$?; echo "60k exit $rc"; cat $O/probe_60k.jsonl | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 100000 --spec-crit 0 1 --save $O/s100k > $O/probe_100k.jsonl 2> $O/probe_100k.err; rc=$?; echo "100k exit $rc"; cat $O/probe_100k.jsonl | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 420 python3 bench.py --steps 20 --warmup 5 --no-cpu --progress 30 --spec-crit 1 > $O/bench_crit.json 2> $O/bench_crit.err; rc=$?; echo "bench crit exit $rc"
timeout -k 10 420 python3 bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_default.json 2> $O/bench_default.err; echo "bench default exit $?"
