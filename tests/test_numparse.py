"""Spark 2.2.2 Cast(StringType -> DoubleType) = java.lang.Double.parseDouble, correctly rounded
for every input (ColumnProfiler.scala:427-445 casts Integral / Fractional-typed string columns
this way; `item > 3` on a string column, CheckTest.scala:196, casts the same way).

The library's parser (deequ_amd/csrc/dq_numparse.h) runs on the device in dq_cast_utf8 and in the
predicate IR's DQ_P_CAST_DOUBLE; `dq_diag_parse_double` is the host build of the same source.  It
is checked here on CPU, bit for bit, against the oracle's `java_parse_double` (Java's grammar,
values from Python's correctly rounded float() / float.fromhex) on: random decimals of 1-60
digits over the whole exponent range, exact halfway points between adjacent doubles (and one
digit either side of them), subnormals, the overflow boundary, hexadecimal literals and
malformed strings.  The device side of the same code is checked in test_gpu_cast_full.py."""
import ctypes
import math
import random
import struct
from decimal import Decimal, getcontext

import pytest

from deequ_amd import _lib as L
import pyoracle as O


def lib_parse(s: str):
    b = s.encode("utf-8")
    out = ctypes.c_double()
    ok = ctypes.c_int32()
    L.check(L.lib().dq_diag_parse_double(b, len(b), ctypes.byref(out), ctypes.byref(ok)))
    return out.value if ok.value else None


def bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def same(a, b):
    if a is None or b is None:
        return a is None and b is None
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b)
    return bits(a) == bits(b)


def check_all(strings):
    bad = []
    for s in strings:
        want = O.java_parse_double(s)
        got = lib_parse(s)
        if not same(got, want):
            bad.append((s, got, want))
    assert not bad, bad[:5]


def random_decimal(rng: random.Random) -> str:
    nd = rng.choice([1, 2, 5, 9, 15, 17, 19, 20, 21, 25, 30, 40, 60])
    digits = "".join(rng.choice("0123456789") for _ in range(nd))
    if rng.random() < 0.3:
        digits = "0" * rng.randint(1, 5) + digits
    if rng.random() < 0.6:
        k = rng.randint(0, len(digits))
        digits = digits[:k] + "." + digits[k:]
        if digits == ".":
            digits = "0."
    s = rng.choice(["", "", "-", "+"]) + digits
    if rng.random() < 0.7:
        s += rng.choice("eE") + rng.choice(["", "-", "+"]) + str(rng.randint(0, 360))
    if rng.random() < 0.1:
        s += rng.choice("fFdD")
    if rng.random() < 0.05:
        s = " \t" + s + " \n"
    return s


def test_random_decimals():
    rng = random.Random(1234)
    check_all(random_decimal(rng) for _ in range(60000))


def halfway_strings(rng: random.Random, n: int):
    out = []
    for _ in range(n):
        e = rng.choice([rng.randint(-1074, 1023), rng.randint(-1074, -1000), rng.randint(40, 80),
                        rng.randint(-80, -40), rng.randint(1000, 1023)])
        m = rng.randint(1 << 52, (1 << 53) - 1) if e > -1022 else rng.randint(1, (1 << 52) - 1)
        sh = e - 52 if e > -1022 else -1074
        # halfway between m * 2^sh and (m + 1) * 2^sh: (2m + 1) * 2^(sh - 1)
        getcontext().prec = 2000
        h = Decimal(2 * m + 1) * (Decimal(2) ** (sh - 1))
        s = format(h, "e") if rng.random() < 0.5 else format(h, "f")
        out.append(s)
        mant, _, ex = format(h, "e").partition("e")
        out.append(mant.rstrip("0") + "1e" + ex if "." in mant else mant + ".1e" + ex)  # just above
        dig = mant.replace(".", "")
        if len(dig) > 1:  # just below: decrement the last digit
            k = len(dig.rstrip("0")) - 1
            low = dig[:k] + str(int(dig[k]) - 1) + "9" * 5
            out.append(low[0] + "." + low[1:] + "e" + ex)
    return out


def test_halfway_points():
    rng = random.Random(99)
    check_all(halfway_strings(rng, 3000))


@pytest.mark.parametrize("s", [
    "0", "-0", "0.0", "-0.0e10", "1", "1.", ".5", "-.5e-3", "1e308", "1.7976931348623157e308",
    "1.7976931348623158e308", "1.7976931348623159e308", "1.797693134862315807937289714053e308",
    "1e309", "-1e309", "4.9e-324", "2.4703282292062327e-324", "2.4703282292062328e-324",
    "2.47032822920623272088e-324", "2e-324", "1e-400", "2.2250738585072011e-308",
    "2.2250738585072012e-308", "2.2250738585072014e-308", "9007199254740993", "9007199254740992.5",
    "123456789012345678901234567890", "0.1", "0.30000000000000004", "3.141592653589793238462643383279",
    "1e22", "1e23", "8.41e21", "NaN", "-NaN", "Infinity", "-Infinity", "+Infinity", "1d", "2.5F",
    "0x1p0", "0x1.8p1", "-0X1.FFFFFFFFFFFFFp1023", "0x1.fffffffffffff8p1023", "0x1p-1074", "0x1p-1075",
    "0x1.0000000000001p-1075", "0x.8p1", "0x1.00000000000008p0", "0x1.00000000000018p0", "0x10p-4d",
    "1" + "0" * 400 + "e-400", "0." + "0" * 400 + "1e400", "1e-99999999999", "1e99999999999",
    "", " ", "e5", "1e", "1e+", ".", "-", "+.", "1.2.3", "1e5.5", "0x", "0x1", "0xp1", "0x1.8",
    "nan", "inf", "Infinityx", "1_000", "١٢", "12abc", "--1", "1e-5f5",
])
def test_known_cases(s):
    check_all([s])


def test_long_digit_strings():
    rng = random.Random(5)
    strings = []
    for _ in range(300):
        n = rng.randint(700, 1200)
        d = "".join(rng.choice("0123456789") for _ in range(n))
        strings.append(d[0] + "." + d[1:] + "e" + str(rng.randint(-330, 300)))
    # halfway points spelled with trailing zeros past 800 digits, and one nonzero digit far out
    getcontext().prec = 2000
    h = Decimal(2 * ((1 << 52) + 12345) + 1) * (Decimal(2) ** -1075)
    hs = format(h, "e")
    mant, _, ex = hs.partition("e")
    strings.append(mant + "0" * 900 + "e" + ex)
    strings.append(mant + "0" * 900 + "1e" + ex)
    check_all(strings)
