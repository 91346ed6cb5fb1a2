# Round-4 call Q (on the box via gpurun): UR5 bisect, fifth step - the SGPR-base DMA on the vector ring (sbm2) and
# on the vector + forward rings (sbm6) with the stage base computed at the DMA (no hoisted / spilled base:
# -DVBOC_SBASE_NOHOIST).  Builds in tools/ur5_variants/ (copied there for this call).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04q}; mkdir -p $O
cd $R
for v in sbm2 sbm2nh sbm6nh; do
  VBOC_LIB=$R/tools/ur5_variants/libvboc_amd_$v.so timeout -k 10 150 python3 -u $R/tools/ur5_trunc.py $O/trunc_$v > $O/trunc_$v.jsonl 2> $O/trunc_$v.err
  rc=$?; echo "$v trunc exit $rc: $(tail -1 $O/trunc_$v.jsonl | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
done
