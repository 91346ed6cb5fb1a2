# Round-4 call U: does the UR5 product's result depend on what ran before it?  ur5_trunc.py with and without a
# triple first-solve batch in the same process before (uninitialised-register test)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04u}; mkdir -p $O
cd $R
timeout -k 10 150 python3 -u tools/ur5_trunc.py $O/trunc_plain > $O/trunc_plain.jsonl 2> $O/trunc_plain.err; rc=$?; echo "plain exit $rc: $(head -1 $O/trunc_plain.jsonl | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/ur5_trunc.py $O/trunc_pre --pre > $O/trunc_pre.jsonl 2> $O/trunc_pre.err; rc=$?; echo "pre exit $rc: $(head -1 $O/trunc_pre.jsonl | cut -c1-150)"
