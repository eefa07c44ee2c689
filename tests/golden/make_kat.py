"""Generate tests/golden/kat_vectors.json — hand-derived known-answer vectors.

These vectors are computed from first principles, with exact rational
arithmetic, from a reading of the reference source — NOT from either oracle
implementation (oracle/sml_oracle.c, oracle/oracle.py np_*), so they pin both
restatements and the HIP path to one independent derivation:

  exponent  ppp.cc:141-154   max |x| by float '>' from 0 (NaN never wins),
                             e = int8(((bits(max) & 0x7f800000) >> 23) - 126)
  scale     ppp.cc:257-258   float( double(INT32_MAX) / float(W * 2^e) )
  quantize  ppp.cc:103       htonl( x86_cvttss2si64( roundf( float(x*s) ) ) )
  dequant   ppp.cc:240-241   float( float(int32 ntohl(q)) / s )   (single rounding)
  loopback  dummy_backend.cc:78-82   q * W mod 2^32

(ppp.cc = client_lib/src/prepostprocessors/cpu_exponent_quantizer_ppp.cc.)
The reference cannot be compiled in this image (glog is absent), so these
are the strongest bit-level pins available; see DESIGN.md §3.

Run: python tests/golden/make_kat.py   (rewrites kat_vectors.json)
"""
from __future__ import annotations

import json
import math
import os
import struct
from fractions import Fraction

INT32_MAX = 2147483647


def f32_bits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


def bits_f32(b: int) -> float:
    return struct.unpack("<f", struct.pack("<I", b & 0xFFFFFFFF))[0]


def round_to_f32(v) -> float:
    """Correctly round an exact value (Fraction / int / exact float) to binary32, RNE,
    with gradual underflow and overflow to inf."""
    if isinstance(v, float):
        if math.isnan(v) or math.isinf(v):
            return v
        v = Fraction(v)
    if v == 0:
        return 0.0
    sign = -1.0 if v < 0 else 1.0
    a = abs(v)
    # exponent k with 2^k <= a < 2^(k+1)
    k = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** k > a:
        k -= 1
    k = max(k, -126)                     # subnormal range shares the 2^-149 quantum
    q = Fraction(2) ** (k - 23)          # quantum at this binade
    m = a / q
    n = m.numerator // m.denominator
    r = m - n
    if r > Fraction(1, 2) or (r == Fraction(1, 2) and n % 2 == 1):
        n += 1
    val = Fraction(n) * q
    if val >= Fraction(2) ** 128:
        return sign * math.inf
    return sign * float(val)


def exponent(xs) -> int:
    cur = 0.0
    for x in xs:
        v = abs(x)
        if v > cur:                      # NaN compares false
            cur = v
    e = ((f32_bits(cur) & 0x7F800000) >> 23) - 126
    return ((e + 128) & 0xFF) - 128      # stored through int8_t*


def scale(W: int, e: int) -> float:
    p2 = Fraction(2) ** e                # powf(2, e): exact for every int8 e
    denom = round_to_f32(Fraction(W) * p2)   # float multiply
    if math.isinf(denom):
        q = 0.0
    else:
        q = INT32_MAX / float(Fraction(denom))   # IEEE double division (Python float)
    return round_to_f32(q)


def roundf_half_away(v: float) -> float:
    if math.isnan(v) or math.isinf(v):
        return v
    t = math.trunc(v)
    if abs(v - t) >= 0.5:
        t += 1 if v > 0 else -1
    return float(t)


def x86_f2u32(r: float) -> int:
    if math.isnan(r) or abs(r) >= 2.0 ** 63:
        return 0
    return int(r) & 0xFFFFFFFF


def bswap(w: int) -> int:
    return int.from_bytes((w & 0xFFFFFFFF).to_bytes(4, "little"), "big")


def quantize(x: float, s: float) -> int:
    if math.isnan(x) or math.isinf(x) or math.isinf(s):
        prod = x * s                     # IEEE specials: inf*0 = NaN, etc.
        if not (math.isnan(prod) or math.isinf(prod)):
            prod = round_to_f32(prod)
    else:
        prod = round_to_f32(Fraction(x) * Fraction(s))
    return bswap(x86_f2u32(roundf_half_away(prod)))


def dequantize(be_word: int, s: float) -> float:
    q = bswap(be_word)
    q = q - (1 << 32) if q >= (1 << 31) else q
    qf = round_to_f32(q)                 # int -> float, RNE
    if math.isinf(s):
        return 0.0 if (qf >= 0 or qf == 0) else -0.0
    if s == 0.0:
        return math.nan if qf == 0 else math.copysign(math.inf, qf)
    return round_to_f32(Fraction(qf) / Fraction(s))


def f32(x: float) -> float:
    return bits_f32(f32_bits(x)) if not math.isnan(x) else x


def case(name, xs, P, W, global_exps=None):
    xs = [f32(float(v)) for v in xs]
    n = len(xs)
    B = -(-n // P)
    exps, payload, out = [], [], []
    for k in range(B):
        blk = xs[k * P:(k + 1) * P]
        e_loc = exponent(blk)
        e = global_exps[k] if global_exps is not None else e_loc
        exps.append(e_loc)
        s = scale(W, e)
        words = [quantize(x, s) for x in blk] + [0] * (P - len(blk))
        payload += words
        agg = [bswap((bswap(w) * W) & 0xFFFFFFFF) for w in words]   # loopback x W
        out += [dequantize(w, s) for w in agg[:len(blk)]]
    return {
        "name": name, "P": P, "W": W,
        "x_bits": [f"{f32_bits(v):08x}" if not math.isnan(v) else "7fc00000" for v in xs],
        "global_exps": global_exps,
        "exps": exps,
        "payload_be": [f"{w:08x}" for w in payload],
        "loopback_out_bits": [("nan" if math.isnan(v) else f"{f32_bits(v):08x}") for v in out],
    }


def main():
    P = 64
    cases = []
    # ties: block max 1.0 -> e = 1, s = 2^30; x = (k + 1/2) / 2^30 -> x*s = k + 1/2 exactly
    ties = [1.0] + [(k + 0.5) / 2 ** 30 for k in (0, 1, 2, -1, -2, 3, -3, 100, -101)]
    cases.append(case("ties_half_away", ties + [0.0] * (P - len(ties)), P, 1))
    cases.append(case("all_zero_block", [0.0] * P + [1.5] * P, P, 1))
    cases.append(case("tiny_block_e_minus102", [1e-31, -2e-32, 3e-31] + [0.0] * (P - 3), P, 1))
    cases.append(case("block_max_e_minus96_97", [2.0 ** -98, 2.0 ** -99] + [2.0 ** -97] * (P - 2)
                      + [2.0 ** -98] + [2.0 ** -100] * (P - 1), P, 1))
    cases.append(case("denormals", [bits_f32(0x00000001), bits_f32(0x007fffff), -bits_f32(0x00400000)]
                      + [bits_f32(0x00000100 + i) for i in range(P - 3)], P, 1))
    cases.append(case("nan_skipped_in_max", [math.nan, 0.25, -0.5, math.nan] + [0.125] * (P - 4), P, 1))
    cases.append(case("inf_block", [math.inf, 1.0, -2.0] + [0.0] * (P - 3), P, 1))
    cases.append(case("huge_e128_wraps", [3.0e38, -1.0e38, 7.0] + [1.0] * (P - 3), P, 1))
    cases.append(case("e127_W3_scale_overflow", [1.5e38, 0.0, -1.0e38] + [1e37] * (P - 3), P, 3))
    cases.append(case("W3_nonpow2_scale", [0.1 * (i - 31) for i in range(P)], P, 3))
    cases.append(case("W8_pattern", [float(i) * (-1) ** i for i in range(2 * P + 5)], P, 8))
    cases.append(case("partial_last_block", [math.sin(i) for i in range(P + 7)], P, 2))
    cases.append(case("global_exps_smaller_wraps", [float(2 ** 20 + i) for i in range(P)], P, 1, global_exps=[-8]))
    cases.append(case("global_exps_larger", [0.001 * i for i in range(P)], P, 1, global_exps=[5]))
    cases.append(case("W65535", [math.cos(i) * 3 for i in range(P)], P, 65535))
    cases.append(case("P256_mixed", [((-1) ** i) * (i % 17) * 0.37 for i in range(300)], 256, 2))
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat_vectors.json")
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_kat.py", "cases": cases}, f, indent=0)
    print(f"wrote {len(cases)} cases to {path}")


if __name__ == "__main__":
    main()
