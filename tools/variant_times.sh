# Kernel time and result digest of tools/pass_probe.py for the product library and named variants
# (vboc_amd/variants/libvboc_amd_<name>.so), one process each (on the box via gpurun).
# usage: bash tools/variant_times.sh <out-subdir> <nq> <B> [variant names...]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-vt}; mkdir -p $O; NQ=$2; B=$3; shift 3
for v in product "$@"; do
  if [ "$v" = "product" ]; then L=$R/vboc_amd/libvboc_amd.so; else L=$R/vboc_amd/variants/libvboc_amd_$v.so; fi
  VBOC_LIB=$L timeout -k 10 120 python3 $R/tools/pass_probe.py $NQ $B > $O/time_$v.json 2> $O/time_$v.err || exit 1
  echo "$v $(cat $O/time_$v.json)"
done
