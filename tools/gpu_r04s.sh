# Round-4 call S: UR5 bisect - LDS filled with zeros / NaN before the first job (-DVBOC_LDS_ZERO / -DVBOC_LDS_NAN),
# product form and vector-ring SGPR-base form: an uninitialised LDS read would show as a changed digest / NaN.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04s}; mkdir -p $O
cd $R
for v in prodzero sbm2zero prodnan sbm2nan; do
  VBOC_LIB=$R/tools/ur5_variants/libvboc_amd_$v.so timeout -k 10 150 python3 -u tools/ur5_trunc.py $O/trunc_$v > $O/trunc_$v.jsonl 2> $O/trunc_$v.err; rc=$?
  echo "$v exit $rc: $(head -1 $O/trunc_$v.jsonl | cut -c1-150) | $(tail -1 $O/trunc_$v.jsonl | cut -c40-170)"; [ $rc -eq 0 ] || exit $rc
done
