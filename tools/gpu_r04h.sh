# Round-4 call H (on the box via gpurun): bash tools/gpu_r04h.sh <out-subdir>
# UR5 bisect, fourth step: the vector-ring SGPR-base DMA (sbm2) and the unmasked write-back (wbun) with
#   pre / post / both: 16 extra wait states before the DMA block / after the load (before m0 is restored)
#   acq: an agent-scope acquire fence (vector L1 invalidate) before every ring's first DMA
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04h}; mkdir -p $O
cd $R
for v in sbm2 sbm2pre sbm2post sbm2both sbm2acq wbun wbunacq; do
  VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_$v.so timeout -k 10 150 python3 -u $R/tools/ur5_trunc.py $O/trunc_$v > $O/trunc_$v.jsonl 2> $O/trunc_$v.err
  rc=$?; echo "$v trunc exit $rc: $(tail -1 $O/trunc_$v.jsonl | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
done
