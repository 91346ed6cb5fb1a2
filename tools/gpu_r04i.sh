# Round-4 call I (on the box via gpurun): bash tools/gpu_r04i.sh <out-subdir>
#  1. tools/probes/dma_forms: VADDR vs SADDR LDS-DMA on every UR5 stage window (hardware semantics of the two forms)
#  2. the vector-ring SGPR-base build with every guard at once (drain, L1 invalidate, wait states before / after)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04i}; mkdir -p $O
cd $R
timeout -k 10 60 $R/tools/probes/dma_forms > $O/dma_forms.jsonl 2> $O/dma_forms.err; rc=$?; echo "dma_forms exit $rc"; cat $O/dma_forms.jsonl; [ $rc -eq 0 ] || exit $rc
for v in sbm2all; do
  VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_$v.so timeout -k 10 150 python3 -u $R/tools/ur5_trunc.py $O/trunc_$v > $O/trunc_$v.jsonl 2> $O/trunc_$v.err
  rc=$?; echo "$v trunc exit $rc: $(head -1 $O/trunc_$v.jsonl | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 150 python3 -u $R/tools/ur5_trunc.py $O/trunc_product > $O/trunc_product.jsonl 2> $O/trunc_product.err; echo "product $(tail -1 $O/trunc_product.jsonl | cut -c1-160)"
