# Round-4 call F (on the box via gpurun): bash tools/gpu_r04f.sh <out-subdir>
#  1. UR5 bisect, second step: the product twice (run-to-run determinism) and the -DVBOC_DBG_CHECK builds of the
#     two failing variants (every landed ring window compared with a direct global read; printf on a mismatch)
#  2. k_dg at 60k problems: the eager speculation window 0 / 1 / 2 / 3 (dg_spec_window), parked first solves on
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04f}; mkdir -p $O
cd $R
for v in product product2 sbase_dbg wbun_dbg; do
  case $v in product*) L=$R/vboc_amd/libvboc_amd.so;; *) L=$R/vboc_amd/variants/libvboc_amd_$v.so;; esac
  VBOC_LIB=$L timeout -k 10 150 python3 -u $R/tools/ur5_trunc.py $O/trunc_$v > $O/trunc_$v.jsonl 2> $O/trunc_$v.err
  rc=$?; echo "$v trunc exit $rc: $(grep -c '^tag' $O/trunc_$v.jsonl) mismatch lines"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 python3 $R/tools/dg_probe.py --B 60000 --groups 0 --park 1 --window 0 1 2 3 --save $O/stats60k > $O/probe_window.jsonl 2> $O/probe_window.err && cat $O/probe_window.jsonl
