"""First-call latency of the library in a fresh process:
dlopen (ce_amd.load()), the first select_mc on a 1608-item pool (module load
+ launch + sync), the first C4-shaped streaming call, and a warm call --
each in its own subprocess per library build.
  python tools/first_call.py [lib.so ...]   (default: the in-tree build)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, time, json
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch
torch.cuda.init(); torch.zeros(1, device="cuda"); torch.cuda.synchronize()
import ce_amd, ce_amd.ops as ops
t0 = time.perf_counter(); ce_amd.load(); t_load = time.perf_counter() - t0
P = torch.rand((4, 1608, 4), device="cuda", dtype=torch.float64)
Q = torch.rand((1 << 20, 16, 4), device="cuda", dtype=torch.float32)
torch.cuda.synchronize()
def tcall(fn):
    t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); return time.perf_counter() - t0
first = tcall(lambda: ops.select_mc(P, 10, "MNC"))
first_stream = tcall(lambda: ops.select_mc(Q, 10, "NMC"))
warm = min(tcall(lambda: ops.select_mc(P, 10, "MNC")) for _ in range(20))
print(json.dumps({"lib": os.path.basename(os.environ.get("CE_AMD_LIB", "libce_amd.so")),
                  "lib_MiB": os.path.getsize(ce_amd._lib.LIB_PATH) / 2**20,
                  "load_ms": t_load * 1e3, "first_select_mc_ms": first * 1e3,
                  "first_stream_call_ms": first_stream * 1e3, "warm_select_mc_ms": warm * 1e3}))
'''.replace("ROOT", repr(ROOT))


def main(libs):
    for lib in libs or [None]:
        env = dict(os.environ)
        if lib:
            env["CE_AMD_LIB"] = os.path.abspath(lib)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(out.stderr[-2000:], file=sys.stderr)
            sys.exit(out.returncode)
        print(out.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
