"""Kernel instantiations per code object of the built library: every kernel
descriptor should live in exactly ONE translation unit's code object
(VERDICT r02 item 6).  Prints per-object kernel counts and code sizes and any
kernel found in more than one object.
  python tools/kernel_dups.py [consensus-entropy_amd/build]"""
import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
        if os.path.getsize(fat) == 0:
            return [], 0
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "-W", co], capture_output=True, text=True).stdout
        return sorted({m.group(1) for m in re.finditer(r"\s(\S+)\.kd$", syms, re.M)}), os.path.getsize(co)


def main(build):
    where = collections.defaultdict(list)
    for obj in sorted(glob.glob(os.path.join(build, "*.o"))):
        ks, size = kernels(obj)
        print(f"{os.path.basename(obj):28s} {len(ks):4d} kernels  {size / 2**20:6.2f} MiB code object")
        for k in ks:
            where[k].append(os.path.basename(obj))
    dups = {k: v for k, v in where.items() if len(v) > 1}
    print(f"{len(where)} distinct kernels, {len(dups)} in more than one object")
    for k, v in sorted(dups.items()):
        print("  DUP", k[:120], v)
    return 1 if dups else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "consensus-entropy_amd/build"))
