# Round-4 call R: UR5 vector-pass dumps of the product form and the vector-ring SGPR-base form (-DVBOC_VEC_DUMP
# builds in tools/ur5_variants/); the truncated solves of both to check the dump builds keep their behaviour.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04r}; mkdir -p $O
cd $R
for v in dump_prod dump_sbm2; do
  VBOC_LIB=$R/tools/ur5_variants/libvboc_amd_$v.so timeout -k 10 120 python3 -u tools/ur5_vecdump.py $O/vec_$v.npz > $O/vec_$v.log 2>&1; rc=$?; echo "$v dump exit $rc: $(tail -1 $O/vec_$v.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
  VBOC_LIB=$R/tools/ur5_variants/libvboc_amd_$v.so timeout -k 10 150 python3 -u tools/ur5_trunc.py $O/trunc_$v > $O/trunc_$v.jsonl 2> $O/trunc_$v.err; rc=$?; echo "$v trunc exit $rc: $(head -1 $O/trunc_$v.jsonl | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
done
