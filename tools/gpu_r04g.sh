# Round-4 call G (on the box via gpurun): bash tools/gpu_r04g.sh <out-subdir>
#  1. Safe-MPC GPU tests (the network row now in the oracle's arithmetic order)
#  2. UR5 bisect, third step: the SGPR-base DMA on one ring at a time (-DVBOC_SBASE_MASK=1 factor, 2 vector,
#     4 forward, 8 costate), truncated solves
#  3. k_dg at 60k problems, eager window 0 / 2 with the per-problem count of solves taken from other waves
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04g}; mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_safempc.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_mpc.log 2>&1
rc=$?; echo "pytest_mpc exit $rc"; [ $rc -le 1 ] || exit $rc
for v in sbm1 sbm2 sbm4 sbm8; do
  VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_$v.so timeout -k 10 150 python3 -u $R/tools/ur5_trunc.py $O/trunc_$v > $O/trunc_$v.jsonl 2> $O/trunc_$v.err
  rc=$?; echo "$v trunc exit $rc: $(head -1 $O/trunc_$v.jsonl | cut -c1-120)"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 60000 --groups 0 --park 1 --window 0 2 --save $O/stats60k > $O/probe_window.jsonl 2> $O/probe_window.err && cat $O/probe_window.jsonl
