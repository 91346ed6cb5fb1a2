"""Check the counted-wait invariant of the wave solver's LDS-DMA rings: no scratch
(spill) STORE may sit between a ring DMA (global_load_lds_dwordx4) and the next hand-counted
`s_waitcnt vmcnt(N)` - a store can complete before an older load and let the wait pass early.  (A spill
LOAD there only over-waits: loads complete in order.)
Compiles the device code to assembly (hipcc -S, gfx950, -O3) and scans every k_wave / k_dg / k_ts / k_tt instantiation.
usage: python tools/check_ring_waits.py [extra hipcc flags, e.g. -DVBOC_COMPACT=3]   (exit status 1 on a violation)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "vboc_amd", "csrc", "vboc_solver.hip")


def main():
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "dev.s")
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-std=c++17", "-O3", "-S", "--cuda-device-only",
                               *sys.argv[1:], SRC, "-o", asm])
        lines = open(asm).read().split("\n")
    bad_total = 0
    starts = [k for k, l in enumerate(lines) if re.match(r"^_ZN4vboc(6k_wave|4k_dg|4k_ts|4k_tt)I.*:", l)]
    for i in starts:
        end = next(j for j in range(i, len(lines)) if lines[j].startswith(".Lfunc_end"))
        body = lines[i:end]
        name = body[0].split(":")[0]
        scratch = [k for k, l in enumerate(body) if re.search(r"scratch_store", l)]
        dma = [k for k, l in enumerate(body) if "global_load_lds" in l]
        waits = [k for k, l in enumerate(body)
                 if re.search(r"^\s*s_waitcnt vmcnt\(\d+\)\s*$", l) and ";;#ASMSTART" in body[k - 1]]
        bad = [k for k in scratch if any(d < k for d in dma) and
               not any(max(d for d in dma if d < k) < w < k for w in waits) and any(w > k for w in waits)]
        bad_total += len(bad)
        print(f"{name}: {len(scratch)} scratch stores, {len(dma)} ring DMAs, {len(bad)} inside a DMA->wait window")
        for k in bad:
            print("   ", body[k].strip())
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
