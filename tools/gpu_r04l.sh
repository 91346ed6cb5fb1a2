# Round-4 evidence, part 2 (on the box via gpurun): bash tools/gpu_r04l.sh <out-subdir>
#  1. lockstep record of the six triple fixture problems the widened fixture classified 'value' (tools/lockstep_probe.py)
#  2. the driver's bench command (with the CPU baseline), the double pendulum's configs[1] lines (dg-loop and first
#     solve, 10k problems), and the rocprofv3 --kernel-trace --stats run of the driver's command
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04l}; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/lockstep_probe.py $O/lockstep.json 151 242 1464 988 197 79 > $O/lockstep.log 2>&1; rc=$?; echo "lockstep exit $rc"; cat $O/lockstep.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python3 bench.py --steps 20 --warmup 5 --progress 30 > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --nq 2 --batch 10000 --steps 1 --warmup 1 > $O/bench_double_dg_loop_10k.json 2> $O/bench_double_dg_loop_10k.err; rc=$?; echo "double dg exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --workload first-solve --nq 2 --batch 10000 --steps 1 --warmup 1 > $O/bench_double_first_solve_10k.json 2> $O/bench_double_first_solve_10k.err; rc=$?; echo "double fs exit $rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_prof.json 2> $O/bench_prof.err; echo "prof exit $?"
