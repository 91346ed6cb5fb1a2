# Round-4 call M (on the box via gpurun): bash tools/gpu_r04m.sh <out-subdir>
# k_dg launch-tail A/B: restart jobs before parked resumes once the new problems run out (dg_spec_first 0 / 1) at
# 60k and 100k problems (configs[2]'s round), and the resident-problem count around the MALL budget (1 200 / 1 450)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04m}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 60000 --groups 0 --spec-first 0 1 --save $O/s60k > $O/probe_60k.jsonl 2> $O/probe_60k.err; rc=$?; echo "60k exit $rc"; cat $O/probe_60k.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 100000 --groups 0 --spec-first 0 1 --save $O/s100k > $O/probe_100k.jsonl 2> $O/probe_100k.err; rc=$?; echo "100k exit $rc"; cat $O/probe_100k.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 60000 --groups 1200 1450 > $O/probe_groups.jsonl 2> $O/probe_groups.err; rc=$?; echo "groups exit $rc"; cat $O/probe_groups.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 $R/tools/dg_probe.py --nq 2 --B 10000 --groups 0 --spec-first 0 1 --save $O/s10k_dbl > $O/probe_dbl10k.jsonl 2> $O/probe_dbl10k.err; rc=$?; echo "double 10k exit $rc"; cat $O/probe_dbl10k.jsonl
