"""Per-kernel resources (VGPRs, AGPRs, scratch, static LDS) read from a built
object's gfx950 code object -- no recompilation.
  python tools/kernel_meta.py consensus-entropy_amd/build/ce_kernels.o [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"


def meta(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    out = []
    for b in re.split(r"\n  - \.agpr_count:", notes)[1:]:
        g = lambda k: re.search(r"\n    \." + k + r":\s+(\S+)", b).group(1)
        name = subprocess.run(["c++filt", g("name")], capture_output=True, text=True).stdout.strip()
        out.append((name, int(g("vgpr_count")), int(b.split()[0]), int(g("private_segment_fixed_size")),
                    int(g("group_segment_fixed_size")), int(g("sgpr_count"))))
    return out


if __name__ == "__main__":
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, v, a, scr, lds, s in meta(sys.argv[1]):
        if flt in name:
            print(f"{v:4d}v {a:3d}a {s:3d}s scr={scr:5d} lds={lds:6d}  {name[:160]}")
