#!/usr/bin/env python3
"""Print the constants of glibc's table-driven f64 log (sysdeps/ieee754/dbl-64/
e_log.c + e_log_data.c, glibc >= 2.28, from ARM's optimized-routines) as they
sit in this image's libm (glibc 2.35): struct log_data = {ln2hi, ln2lo,
poly[5], poly1[11], tab[128] {invc, logc}, tab2[128] {chi, clo}}.

Used once to write consensus-entropy_amd/csrc/ce_glibc_log.hpp; the CPU test
tests/test_glibc_log.py re-checks the restatement against libm's log itself.
Reads the data only (locates ln2hi, ln2lo by value); runs nothing from libm.
"""
import struct
import sys

import numpy as np

LIBM = "/lib/x86_64-linux-gnu/libm.so.6"


def find(path=LIBM):
    data = open(path, "rb").read()
    key = struct.pack("<dd", float.fromhex("0x1.62e42fefa3800p-1"), float.fromhex("0x1.ef35793c76730p-45"))
    at = data.find(key)
    while at >= 0:
        v = np.frombuffer(data[at:at + 8 * (2 + 5 + 11 + 512)], dtype="<f8")
        # log_data (not pow's log table): poly1[0] == -0.5 and tab[0].invc ~ 1/0.69
        if v[7] == -0.5 and 1.44 < v[18] < 1.46:
            return v
        at = data.find(key, at + 1)
    raise SystemExit("log_data not found in " + path)


def main():
    v = find(sys.argv[1] if len(sys.argv) > 1 else LIBM)
    h = lambda x: float(x).hex()
    print("// ln2hi, ln2lo")
    print(f"#define CE_GLIBC_LOG_LN2 {h(v[0])}, {h(v[1])}")
    print("#define CE_GLIBC_LOG_A " + ", ".join(h(x) for x in v[2:7]))
    print("#define CE_GLIBC_LOG_B " + ", ".join(h(x) for x in v[7:18]))
    print("#define CE_GLIBC_LOG_TAB \\")
    tab = v[18:18 + 256]
    for i in range(0, 256, 4):
        end = ", \\" if i + 4 < 256 else ""
        print("    " + ", ".join(h(x) for x in tab[i:i + 4]) + end)


if __name__ == "__main__":
    main()
