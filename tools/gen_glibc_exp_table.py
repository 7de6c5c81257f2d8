#!/usr/bin/env python3
"""Print the constants of glibc's table-driven f64 exp (sysdeps/ieee754/dbl-64/
e_exp.c + e_exp_data.c, glibc >= 2.28, from ARM's optimized-routines) as they
sit in this image's libm (glibc 2.35): struct exp_data = {invln2N, shift,
negln2hiN, negln2loN, poly[4], exp2_shift, exp2_poly[5], tab[2 * 128]}.

Used once to write consensus-entropy_amd/csrc/ce_glibc_exp.hpp; the CPU test
tests/test_glibc_log.py::test_restated_exp_matches_libm re-checks the
restatement against libm's exp itself.  Reads the data only (locates invln2N,
shift by value); runs nothing from libm.
"""
import struct
import sys

import numpy as np

LIBM = "/lib/x86_64-linux-gnu/libm.so.6"


def find(path=LIBM):
    data = open(path, "rb").read()
    key = struct.pack("<dd", float.fromhex("0x1.71547652b82fep7"), float.fromhex("0x1.8p52"))
    at = data.find(key)
    while at >= 0:
        v = np.frombuffer(data[at:at + 8 * (14 + 256)], dtype="<f8")
        t = np.frombuffer(data[at + 8 * 14:at + 8 * (14 + 256)], dtype="<u8")
        # exp_data: negln2hiN = -ln2/128 (hi part), tab[1] = bits(1.0) (2^(0/128), tail 0)
        if v[2] == float.fromhex("-0x1.62e42fefa0000p-8") and t[0] == 0 and t[1] == 0x3FF0000000000000:
            return v[:14], t
        at = data.find(key, at + 1)
    raise SystemExit("exp_data not found in " + path)


def main():
    v, t = find(sys.argv[1] if len(sys.argv) > 1 else LIBM)
    h = lambda x: float(x).hex()
    print("// invln2N, shift, negln2hiN, negln2loN")
    print(f"#define CE_GLIBC_EXP_K {h(v[0])}, {h(v[1])}, {h(v[2])}, {h(v[3])}")
    print("// poly[4] = C2..C5")
    print("#define CE_GLIBC_EXP_C " + ", ".join(h(x) for x in v[4:8]))
    print("// tab[2 * 128]: {tail bits, sbits base} per k % 128")
    print("#define CE_GLIBC_EXP_TAB \\")
    for i in range(0, 256, 4):
        end = ", \\" if i + 4 < 256 else ""
        print("    " + ", ".join(f"0x{int(x):016x}ull" for x in t[i:i + 4]) + end)


if __name__ == "__main__":
    main()
