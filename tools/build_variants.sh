# Measurement builds of the solver library (CPU container; the .so files travel to the GPU box with gpurun):
# vboc_amd/variants/libvboc_amd_<name>.so for each "<name>:<flags>" argument, built in parallel (at most 4 at once).
# Default: the pass-repeat builds rep1..rep8 (-DVBOC_REPEAT=p, coop.h) used by tools/pass_split.sh.
# usage: bash tools/build_variants.sh ["name:-DFLAG=1 -DOTHER" ...]
set -e
cd "$(dirname "$0")/.."
mkdir -p vboc_amd/variants
if [ $# -eq 0 ]; then set -- $(for p in 1 2 3 4 5 6 7 8; do echo "rep$p:-DVBOC_REPEAT=$p"; done); fi
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 -shared $flags vboc_amd/csrc/vboc_solver.hip \
        -o vboc_amd/variants/libvboc_amd_$name.so &
  pids+=($!)
  if [ ${#pids[@]} -ge 4 ]; then wait ${pids[0]}; pids=("${pids[@]:1}"); fi
done
for p in "${pids[@]}"; do wait $p; done
ls -la vboc_amd/variants
