"""ColumnProfilerRunner on a C5-shaped table vs the oracle's restatement of ColumnProfiler.profile.

C5: 100 columns -- 40 int64, 30 fp64, 10 low- and 10 high-cardinality utf8, 10
bool -- 5 % NULL each.  Here at 20k rows so the pure-Python oracle (O.column_profiles, pinned by
every ColumnProfilerTest.scala known answer in test_oracle_golden.py) finishes in seconds.  A
few columns of each family are made low-cardinality or numeric-looking so that every branch of
the three passes runs in ONE wide plan: pass-1 DataType + HLL + Completeness on 100 columns,
pass-2 Integral -> LongType and Fractional -> DoubleType casts of string columns, pass-3
histograms of int / double (Java toString, -0.0, NaN, 1.0E7) / string / bool columns.

Bar: counts, completeness, approxNumDistinct, data types, type counts, Min / Max, integral Sum /
Mean and histograms bit-exact; fp64 Sum / Mean / StdDev within 1e-12 of the exact value.
"""
import math
from fractions import Fraction

import numpy as np
import pytest

import pyoracle as O
from deequ_amd.profiles import ColumnProfilerRunner, NumericColumnProfile
from helpers import oracle_table, product_table

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12
N = 20000


def _nulls(rng, vals, frac=0.05):
    keep = rng.random(len(vals)) >= frac
    return [v if k else None for v, k in zip(vals, keep)]


def c5_spec(n=N, seed=5):
    rng = np.random.default_rng(seed)
    spec = {}
    for k in range(40):
        if k < 3:  # low cardinality: histograms of a long column (incl. 2147483647, negatives)
            pool = np.array([0, 1, -7, 42, 2147483647, -2 ** 40, 10 ** 12] + list(range(100, 130)))
            vals = rng.choice(pool, n)
        else:
            vals = rng.integers(-10 ** 6, 10 ** 9, n)
        spec["l%02d" % k] = ["int64", _nulls(rng, [int(x) for x in vals])]
    for k in range(30):
        if k == 0:  # Java Double.toString cuts and -0.0 / 0.0 as separate groups
            pool = [0.0, -0.0, 1e7, 9999999.5, 1e-3, 9.5e-4, 123.25, -2.5, 1e21, 3.0]
            vals = [pool[i] for i in rng.integers(0, len(pool), n)]
        elif k == 1:  # NaN and infinities (NaN-safe min / max, NaN sums, "NaN" in the histogram)
            pool = [1.5, float("nan"), float("inf"), -float("inf"), 2.0]
            vals = [pool[i] for i in rng.integers(0, len(pool), n)]
        else:
            vals = [float(x) for x in rng.normal(1000.0, 100.0, n)]
        spec["d%02d" % k] = ["float64", _nulls(rng, vals)]
    for k in range(10):  # low cardinality: "cat_NN" (String), one integral-looking column
        if k == 9:
            vals = [str(int(x)) for x in rng.integers(0, 60, n)]
        else:
            vals = ["cat_%02d" % x for x in rng.integers(0, 100, n)]
        spec["s%02d" % k] = ["string", _nulls(rng, vals)]
    for k in range(10):  # high cardinality: 16 digits (Integral -> LongType cast)
        ids = rng.integers(0, 10 ** 15, n)
        if k == 8:  # fractional-looking -> DoubleType cast
            vals = ["%d.%02d" % (x % 10 ** 9, x % 100) for x in ids]
        elif k == 9:  # mostly numbers, a few words -> String (no cast)
            vals = ["%016d" % x if x % 97 else "n/a" for x in ids]
        else:
            vals = ["%016d" % x for x in ids]
        spec["u%02d" % k] = ["string", _nulls(rng, vals)]
    for k in range(10):
        vals = [bool(x) for x in rng.integers(0, 2, n)]
        if k == 9:
            vals = [True] * n  # one group
        spec["b%02d" % k] = ["bool", _nulls(rng, vals)]
    return spec


def _same_float(a, b):
    if a is None or b is None:
        return a is None and b is None
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b)
    return a == b


def _exact(vals):
    fr = [Fraction(float(v)) for v in vals]
    n = len(fr)
    s1 = sum(fr)
    m2 = sum(x * x for x in fr) - s1 * s1 / n
    return float(s1), float(s1 / n), math.sqrt(float(m2 / n))


def _close(got, want):
    return abs(got - want) <= REL_TOL * max(1.0, abs(want))


def test_c5_shaped_profile_matches_oracle(gpu):
    spec = c5_spec()
    assert len(spec) == 100
    profiles = ColumnProfilerRunner().onData(product_table(spec)).run()
    want = O.column_profiles(oracle_table(spec))
    assert profiles.numRecords == want["__numRecords__"] == N
    assert list(profiles.profiles) == list(spec)
    n_hist = n_numeric_str = 0
    for name, p in profiles.profiles.items():
        w = want[name]
        assert p.completeness == w["completeness"], name
        assert p.approximateNumDistinctValues == w["approx"], name
        assert p.dataType == w["dataType"], name
        assert p.isDataTypeInferred == w["inferred"], name
        assert p.typeCounts == w["typeCounts"], name
        assert isinstance(p, NumericColumnProfile) == ("mean" in w), name
        if isinstance(p, NumericColumnProfile):
            n_numeric_str += spec[name][0] == "string"
            assert _same_float(p.minimum, w["minimum"]), (name, p.minimum, w["minimum"])
            assert _same_float(p.maximum, w["maximum"]), (name, p.maximum, w["maximum"])
            vals = w["numeric_values"]
            if any(isinstance(v, float) and not math.isfinite(v) for v in vals):
                for f in ("sum", "mean", "stdDev"):
                    assert _same_float(getattr(p, f), w[f]) or (math.isnan(getattr(p, f)) and math.isnan(w[f])), \
                        (name, f, getattr(p, f), w[f])
            elif all(isinstance(v, int) for v in vals):  # integral: Sum / Mean exact
                assert p.sum == w["sum"] and p.mean == w["mean"], name
                assert _close(p.stdDev, _exact(vals)[2]), (name, p.stdDev)
            else:
                s, m, sd = _exact(vals)
                assert _close(p.sum, s) and _close(p.mean, m) and _close(p.stdDev, sd), (name, p.sum, s, p.stdDev, sd)
        if w["histogram"] is None:
            assert p.histogram is None, name
        else:
            n_hist += 1
            assert p.histogram is not None, name
            assert p.histogram.numberOfBins == len(w["histogram"]), name
            assert {k: (v.absolute, v.ratio) for k, v in p.histogram.values.items()} == w["histogram"], name
    # the shape exercised every branch
    assert n_hist >= 3 + 2 + 10 + 10
    assert n_numeric_str >= 9 + 1
