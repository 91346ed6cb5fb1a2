# Register / scratch / LDS usage of the wave-solver kernels (hipcc kernel-resource-usage remarks), CPU only.
# The counted LDS-DMA ring waits tolerate no scratch spills inside the solver's loops, so
# every change to coop.h / dg.h is checked with this before it goes to the GPU.
# usage: bash tools/resource_usage.sh [extra hipcc flags]   -> prints one line per kernel of interest
cd "$(dirname "$0")/.."
hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 -shared "$@" -Rpass-analysis=kernel-resource-usage \
      vboc_amd/csrc/vboc_solver.hip -o /tmp/vboc_resource_probe.so 2> /tmp/vboc_resource.txt
python3 - <<'EOF'
import re
cur, rows = None, {}
for line in open("/tmp/vboc_resource.txt"):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([^:]+): (\S+) \[", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = m.group(2)
for fn, r in rows.items():
    if "k_wave" in fn or "k_dg" in fn or "k_ft" in fn:
        print(fn[:60], {k: r.get(k) for k in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
                                              "SGPRs Spill", "VGPRs Spill", "LDS Size [bytes/block]")})
EOF
