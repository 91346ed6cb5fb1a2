# Ring-depth A/B (on the box via gpurun): kernel time of the product build and the deeper-prefetch variants
# (tools/build_variants.sh), then the per-phase cycles at 64 resident problems (latency) and at the MALL budget
# of the profiling builds.
# usage: bash tools/ring_depth.sh <out-subdir> <variant...> -- <prof variant...>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ring}; mkdir -p $O; shift
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; shift
bash $R/tools/variant_times.sh ${O#$R/gpurun_out/} 3 16384 "${V[@]}" || exit 1
for p in "$@"; do
  VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_$p.so timeout -k 10 120 python3 $R/tools/gpu_perf.py 3 1024 0 dg 0 wave64,wave1408 \
    > $O/phases_$p.log 2>&1 || exit 1
  cat $O/phases_$p.log
done
