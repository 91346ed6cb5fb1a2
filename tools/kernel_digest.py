"""Per-kernel ISA digests of a built solver library (CPU only): the gfx950 code object is unbundled from the .so and
disassembled without addresses or raw bytes, and each kernel's instruction text is hashed - two builds whose digest
of a kernel is equal run the same instructions for it (used to check that a source change leaves k_dg / k_wave
untouched).  usage: python tools/kernel_digest.py lib_a.so [lib_b.so] [--match k_dg]"""
import hashlib
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def digests(lib, match=None):
    with tempfile.TemporaryDirectory() as T:
        fb, co = os.path.join(T, "fb.bin"), os.path.join(T, "co.o")
        subprocess.check_call([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(T, "s.so")])
        subprocess.check_call([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        txt = subprocess.run([f"{B}/llvm-objdump", "-d", "--no-show-raw-insn", "--no-leading-addr", co],
                             capture_output=True, text=True, check=True).stdout
    out, name, body = {}, None, []
    for line in txt.splitlines():
        m = re.match(r"^([0-9a-f]+ )?<(.+)>:$", line.strip())
        if m:
            if name:
                out[name] = body
            name, body = m.group(2), []
        elif name and line.strip():
            body.append(re.sub(r"\s*//.*$", "", line.strip()))
    if name:
        out[name] = body
    res = {}
    for k, v in out.items():
        if match and match not in k:
            continue
        res[k] = (len(v), hashlib.sha1("\n".join(v).encode()).hexdigest()[:12])
    return res


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args = [a for a in args if a != match]
    ds = [digests(a, match) for a in args]
    names = sorted(set().union(*ds))
    for n in names:
        row = [d.get(n, (0, "-")) for d in ds]
        same = "" if len(ds) < 2 else ("  same" if len({r[1] for r in row}) == 1 else "  DIFFERENT")
        print(f"{n[:90]:90s} " + " ".join(f"{c:6d} {h}" for c, h in row) + same)
