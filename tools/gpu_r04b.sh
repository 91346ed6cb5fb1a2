# Round-4 UR5 k_wave<4> bisect (verdict r03 item 1), on the box via gpurun: bash tools/gpu_r04b.sh <out-subdir> [variants]
# For the product build and each measurement variant (vboc_amd/variants/libvboc_amd_<name>.so, tools/build_variants.sh):
#   trunc_<v>.jsonl / .npz  truncated solves (tools/ur5_trunc.py): the first cut whose digest differs from the
#                           product's locates the diverging pass
#   parity_<v>.log          tests/test_ur5.py::test_ur5_parity_with_oracle[wave-96]
# Variants: sbase = SGPR-base ring DMAs (round 3: 24 % status agreement), wbun = the chains' unmasked factor
# write-back for the arm (round 3: 41 %), *_drain = the same with every counted ring wait drained (vmcnt(0)),
# *_dbg = the same with every landed ring window compared against a direct global read (printf on a mismatch).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04b}; mkdir -p $O; shift
VARS=${@:-sbase sbase_drain wbun wbun_drain sbase_dbg wbun_dbg}
for v in product $VARS; do
  if [ $v = product ]; then L=$R/vboc_amd/libvboc_amd.so; else L=$R/vboc_amd/variants/libvboc_amd_$v.so; fi
  VBOC_LIB=$L timeout -k 10 150 python3 -u $R/tools/ur5_trunc.py $O/trunc_$v > $O/trunc_$v.jsonl 2> $O/trunc_$v.err || { echo "$v trunc failed $?"; exit 1; }
  VBOC_LIB=$L timeout -k 10 200 python3 -u -m pytest "$R/tests/test_ur5.py::test_ur5_parity_with_oracle[wave-96]" -q \
    --timeout 180 --timeout-method thread > $O/parity_$v.log 2>&1
  rc=$?
  echo "$v parity exit $rc: $(tail -1 $O/parity_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
