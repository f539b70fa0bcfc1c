"""Java `toString` of the values Spark casts to strings.

Histogram groups `col.cast(StringType)` (Histogram.scala:63); Spark 2.2's Cast renders
integers in decimal, booleans as true/false and floats with Java's `Float.toString` /
`Double.toString`: the shortest digits that round-trip (the JDK 19+ rule, which agrees with
older JDKs except for a few rare values), plain notation for 1e-3 <= |x| < 1e7, else
computerized scientific notation `d.dddE±n`.
"""
from __future__ import annotations

import math

import numpy as np


def _shortest_digits(x: float, single: bool):
    """(digits, exponent10 of the first digit) of |x|'s shortest round-trip representation."""
    s = np.format_float_scientific(np.float32(x) if single else np.float64(x), unique=True,
                                   trim="-", exp_digits=1)
    mant, exp = s.split("e")
    digits = mant.replace(".", "").lstrip("-").rstrip("0") or "0"
    if len(digits) == 1:
        # Java picks, among the decimals of length <= 2 that round to x, the one closest to x
        # (so Double.MIN_VALUE is 4.9E-324, not 5E-324)
        s2 = np.format_float_scientific(np.float32(x) if single else np.float64(x), precision=1,
                                        unique=False, exp_digits=1)
        mant2, exp2 = s2.split("e")
        digits2 = mant2.replace(".", "").lstrip("-").rstrip("0") or "0"
        return digits2, int(exp2)
    return digits, int(exp)


def _java_fp_to_string(x: float, single: bool) -> str:
    if x != x:
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    a = abs(x)
    digits, e = _shortest_digits(a, single)
    if 1e-3 <= a < 1e7:
        point = e + 1  # digits before the decimal point
        if point <= 0:
            return sign + "0." + "0" * (-point) + digits
        if point >= len(digits):
            return sign + digits + "0" * (point - len(digits)) + ".0"
        return sign + digits[:point] + "." + digits[point:]
    return sign + digits[0] + "." + (digits[1:] or "0") + "E" + str(e)


def java_double_to_string(x: float) -> str:
    return _java_fp_to_string(float(x), single=False)


def java_float_to_string(x: float) -> str:
    return _java_fp_to_string(float(x), single=True)


def spark_cast_to_string(value, dtype: str) -> str:
    """`CAST(value AS STRING)` for a non-NULL value of the given column type."""
    if dtype == "string":
        return value
    if dtype == "bool":
        return "true" if value else "false"
    if dtype == "float64":
        return java_double_to_string(value)
    if dtype == "float32":
        return java_float_to_string(value)
    return str(int(value))
