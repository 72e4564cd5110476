#!/usr/bin/env python3
"""Read glibc's powf tables out of the system libm (the third-party arithmetic the reference's powf calls,
raytracing.c:153,155) and print them as the C literals in raytracingc_amd/csrc/rtc_math.h.

glibc 2.35 powf = ARM optimized-routines powf (sysdeps/ieee754/flt-32/e_powf.c, e_powf_log2_data.c,
e_exp2f_data.c).  The data symbols are private, so they are located by content:
  * __exp2f_data.tab[32] = asuint64(2^(i/32)) - (i << 47) is computable; it is followed by shift_scaled and
    the three exp2 polynomial coefficients;
  * __powf_log2_data.tab[16] = {1/c, log2 c} pairs (log2 c == -log2(1/c) to ~1e-9) followed by the five log2
    polynomial coefficients; the last such 16-entry table in libm is powf's (log2f's comes first and is
    followed by a 4-term polynomial).
tools/check_devmath.cpp then checks the restatement against libm's powf bit for bit.
"""
import decimal
import math
import struct
import sys

LIBM = sys.argv[1] if len(sys.argv) > 1 else "/lib/x86_64-linux-gnu/libm.so.6"


def main():
    data = open(LIBM, "rb").read()
    decimal.getcontext().prec = 60
    tab = []
    for i in range(32):
        v = float(decimal.Decimal(2) ** (decimal.Decimal(i) / 32))
        tab.append((struct.unpack("<Q", struct.pack("<d", v))[0] - (i << 47)) % 2**64)
    off = data.find(b"".join(struct.pack("<Q", t) for t in tab))
    if off < 0:
        sys.exit("exp2f table not found")
    shift_scaled, c0, c1, c2 = struct.unpack("<4d", data[off + 256:off + 288])
    assert shift_scaled == float.fromhex("0x1.8p52") / 32, shift_scaled

    n = len(data) // 8
    vals = struct.unpack("<%dd" % n, data[:n * 8])

    def pair_ok(i):
        invc, logc = vals[i], vals[i + 1]
        return (invc == invc and logc == logc and 0.5 < invc < 2.1
                and abs(logc + math.log2(invc)) < 1e-5)

    tables = [i for i in range(n - 40) if all(pair_ok(i + 2 * k) for k in range(16)) and not pair_ok(i + 32)
              and not (i >= 2 and pair_ok(i - 2))]
    if not tables:
        sys.exit("log2 tables not found")
    t = tables[-1]  # powf's
    log2tab = [(vals[t + 2 * k], vals[t + 2 * k + 1]) for k in range(16)]
    poly = vals[t + 32:t + 37]
    print("constexpr double kLog2Tab[16][2] = {")
    for a, b in log2tab:
        print(f"    {{{a.hex()}, {b.hex()}}},")
    print("};")
    print("constexpr double kLog2Poly[5] = {" + ", ".join(p.hex() for p in poly) + "};")
    print("constexpr unsigned long long kExp2Tab[32] = {")
    for i in range(0, 32, 4):
        print("    " + ", ".join("0x%016xull" % v for v in tab[i:i + 4]) + ",")
    print("};")
    print("constexpr double kExp2Poly[3] = {" + ", ".join(c.hex() for c in (c0, c1, c2)) + "};")


if __name__ == "__main__":
    main()
