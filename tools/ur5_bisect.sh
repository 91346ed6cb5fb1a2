set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03z_ur5bisect; mkdir -p $O
for v in base h1 h2 shfl vaddr product; do
  if [ $v = product ]; then L=$R/vboc_amd/libvboc_amd.so; else L=$R/vboc_amd/variants/libvboc_amd_$v.so; fi
  VBOC_LIB=$L timeout -k 10 240 python -u -m pytest "tests/test_ur5.py::test_ur5_parity_with_oracle" -q --timeout 200 --timeout-method thread > $O/$v.log 2>&1
  echo "$v exit $? $(tail -1 $O/$v.log)"
done
