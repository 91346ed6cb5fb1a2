# A/B of the dg-loop's early speculation threshold (bench.py --spec-early, solver option dg_spec_early) at the driver's
# command shape, one box, one process per setting.  usage (on the box via gpurun): bash tools/spec_early_ab.sh <out> <values...>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-spec_early}; mkdir -p $O; shift
for v in "$@"; do
  se=${v%%:*}; me=0; [ "$se" != "$v" ] && me=${v#*:}
  timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu --spec-early $se --spec-min-ext $me > $O/bench_se${v/:/_}.json 2> $O/bench_se${v/:/_}.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/bench_se${v/:/_}.json')); l=d['loop']; print('spec_early $v', d['value'], l['tail'], l['speculative_restarts']['run_by_other_waves'], l['speculative_restarts']['used'], l['configs2_round']['solves_per_s'])"
done
