# Code size (bytes) of the wave-solver kernels in a built solver library (CPU only): the instruction-cache footprint
# of k_dg / k_wave.  usage: bash tools/kernel_sizes.sh [lib.so ...]
B=/opt/rocm/lib/llvm/bin
for L in "${@:-vboc_amd/libvboc_amd.so}"; do
  T=$(mktemp -d)
  $B/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$L" $T/stripped.so &&
  $B/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --output=$T/co.o &&
  echo "$L" && $B/llvm-readelf -sW $T/co.o | awk '$4=="FUNC" && ($8 ~ /k_dg|k_wave|k_ft/) {print "  " $3, $8}' | sort -u -k2
  rm -rf $T
done
