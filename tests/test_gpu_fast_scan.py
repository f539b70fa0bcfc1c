"""The specialised 8-byte value scan (deequ_amd/csrc/dq_scan_fast.hip) against the oracle.

That kernel runs every int64 / fp64 column task with no `where` and at most one inline
`column CMP literal` predicate -- the C2 headline shape -- and neutralises NULL rows by giving
them the wave's shift value (the first valid value it saw) instead of masking each statistic.
These cases target what that design could get wrong:

* every comparison operator, as the host rewrites it to `<` / `==` (+ negation), with int and
  fractional literals, literals at the int64 / fp64 edges (the `<=` -> `< l+1` rewrite must
  fall back to the general kernel at INT64_MAX / +inf);
* NULL-heavy chunks where a wave finds no valid value to stand in (the masked loop), all-NULL
  columns, no validity bitmap at all;
* int64 wraparound of the stand-in correction, NaN / +-Inf / -0.0, ragged sizes around the
  2048-row iteration;
* the HLL rank marker (a hash whose top word of x << 9 is zero, 1 in 2^32), whose workgroup
  re-ranks its registers: fixture values from tests/golden/hll_rare_values.json;
* fast kernel == general kernel (DQ_SCAN_FAST=0) on the same plan.

Bar: bit-exact counts / Compliance / Min / Max / integral Sum / HLL registers; fp64 Sum / Mean /
StdDev within 1e-12 of the exact value (north_star)."""
import json
import math
import os
import struct

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from helpers import oracle_table, product_table
from test_gpu_parity import _check_state

pytestmark = pytest.mark.gpu

OPS = ["<", "<=", ">", ">=", "=", "!="]


def _suite(col, preds=()):
    out = [d.Size(), d.Completeness(col), d.Sum(col), d.Mean(col), d.StandardDeviation(col),
           d.Minimum(col), d.Maximum(col), d.ApproxCountDistinct(col)]
    out += [d.Compliance("p%d" % k, p) for k, p in enumerate(preds)]
    return out


def _check_each_alone(spec, col, preds):
    """One predicate per plan (the fast kernel takes at most one), stats + HLL alongside."""
    ot, pt = oracle_table(spec), product_table(spec)
    for p in list(preds) + [None]:
        an = _suite(col, [p] if p else [])
        st = d.run_scan(an, pt)
        for a in an:
            _check_state(a, st[a], ot)


def _c2_like_int(rng, n, null_frac):
    v = rng.integers(-2 ** 30, 2 ** 32, n).tolist()
    return [None if rng.random() < null_frac else x for x in v]


def _c2_like_float(rng, n, null_frac):
    v = rng.uniform(0, 1e6, n).tolist()
    return [None if rng.random() < null_frac else x for x in v]


@pytest.mark.parametrize("n", [1, 63, 2047, 2048, 2049, 4096 + 17, 40000])
@pytest.mark.parametrize("null_frac", [0.0, 0.05, 0.6])
def test_int64_operators(gpu, n, null_frac):
    rng = np.random.default_rng(n * 7 + int(null_frac * 100))
    spec = {"x": ["int64", _c2_like_int(rng, n, null_frac)]}
    lits = ["0", "12345678", "-7", "4294967295", "3.5", "-0.5", "1e9"]
    preds = ["x %s %s" % (op, lit) for op in OPS for lit in lits[:3]] + \
            ["x %s %s" % (op, lit) for op in ("<=", ">", "!=") for lit in lits[3:]]
    _check_each_alone(spec, "x", preds)


@pytest.mark.parametrize("n", [1, 2047, 2049, 40000])
@pytest.mark.parametrize("null_frac", [0.0, 0.05, 0.6])
def test_float64_operators(gpu, n, null_frac):
    rng = np.random.default_rng(n * 11 + int(null_frac * 100))
    spec = {"f": ["float64", _c2_like_float(rng, n, null_frac)]}
    preds = ["f %s %s" % (op, lit) for op in OPS for lit in ("5e5", "0", "250000.5")]
    _check_each_alone(spec, "f", preds)


def test_literal_edges_fall_back_or_agree(gpu):
    """`<=` at INT64_MAX / +inf cannot become `< l+1`: those plans take the general kernel."""
    rng = np.random.default_rng(3)
    big = [int(x) for x in rng.integers(-2 ** 63, 2 ** 63 - 1, 5000, endpoint=True)] + [2 ** 63 - 1, -(2 ** 63)]
    spec = {"x": ["int64", big], "f": ["float64", [float(v) for v in big[:-2]] + [math.inf, -math.inf]]}
    ot, pt = oracle_table(spec), product_table(spec)
    preds = ["x <= 9223372036854775807", "x > 9223372036854775807", "x < -9223372036854775808",
             "x = -9223372036854775808", "x >= -9223372036854775808"]
    fpreds = ["f <= 1e400", "f > -1e400", "f = 1e400", "f < 1e308"]
    for col, ps in (("x", preds), ("f", fpreds)):
        for p in ps:
            a = d.Compliance("p0", p)
            st = d.run_scan(_suite(col, [p]), pt)
            _check_state(a, st[a], ot)


@pytest.mark.parametrize("dtype", ["int64", "float64"])
@pytest.mark.parametrize("null_frac", [0.99, 0.997, 1.0])
def test_null_heavy_masked_loop(gpu, dtype, null_frac):
    """Waves whose probe rows are all NULL have no stand-in value: the masked loop runs."""
    rng = np.random.default_rng(int(null_frac * 1000))
    n = 200_000
    if dtype == "int64":
        vals = _c2_like_int(rng, n, null_frac)
        preds = ["x >= 0", "x < 100000"]
    else:
        vals = _c2_like_float(rng, n, null_frac)
        preds = ["x > 5e5", "x = 0"]
    spec = {"x": [dtype, vals]}
    _check_each_alone(spec, "x", preds)


def test_null_prefix_then_values(gpu):
    """The first thousands of rows NULL (every wave of the first blocks masked), then values."""
    rng = np.random.default_rng(21)
    n = 120_000
    vals = [None] * 30_000 + [int(x) for x in rng.integers(-1000, 1000, n - 30_000)]
    _check_each_alone({"x": ["int64", vals]}, "x", ["x > 0", "x = 5"])
    fvals = [None] * 30_000 + [float(x) for x in rng.normal(0, 1, n - 30_000)]
    _check_each_alone({"x": ["float64", fvals]}, "x", ["x <= 0.25"])


def test_no_validity_bitmap(gpu):
    rng = np.random.default_rng(5)
    iv = rng.integers(-2 ** 40, 2 ** 40, 70_001)
    fv = rng.normal(1e3, 1e2, 70_001)
    t = d.Table({"i": d.Column.from_numpy(iv), "f": d.Column.from_numpy(fv)})
    assert t.columns["i"].validity is None
    ot = oracle_table({"i": ["int64", iv.tolist()], "f": ["float64", fv.tolist()]})
    for col, p in (("i", "i >= 0"), ("f", "f < 1000")):
        an = _suite(col, [p])
        st = d.run_scan(an, t)
        for a in an:
            _check_state(a, st[a], ot)


def test_int64_wraparound_with_nulls(gpu):
    """Σ_sel x = Σ xm - n_unsel * c must wrap exactly like Spark's LongType sum."""
    rng = np.random.default_rng(9)
    n = 50_000
    vals = [int(x) for x in rng.integers(2 ** 62, 2 ** 63 - 1, n)]
    vals = [None if rng.random() < 0.3 else v for v in vals]
    _check_each_alone({"x": ["int64", vals]}, "x", ["x > 6917529027641081856"])


def test_float_specials_in_main_loop(gpu):
    rng = np.random.default_rng(12)
    n = 100_000
    v = rng.uniform(-1e3, 1e3, n)
    v[5_000] = np.nan
    v[60_001], v[60_002] = np.inf, -np.inf
    v[70_000] = -0.0
    vals = [None if rng.random() < 0.05 else float(x) for x in v]
    vals[5_000] = float("nan")
    ot, pt = oracle_table({"f": ["float64", vals]}), product_table({"f": ["float64", vals]})
    for p in ("f > 0", "f <= 0", "f = 0", "f != 0"):
        an = [d.Minimum("f"), d.Maximum("f"), d.ApproxCountDistinct("f"), d.Completeness("f"),
              d.Compliance(p, p)]
        st = d.run_scan(an, pt)
        for a in an:
            if not isinstance(a, d.Maximum):  # NaN wins max: checked below (NaN != NaN)
                _check_state(a, st[a], ot)
        assert math.isnan(st[d.Maximum("f")].maxValue)


def test_hll_rank_marker_reranked(gpu):
    """Values whose hash has w_hi == 0 (rank >= 33): the workgroup re-ranks that register over
    its rows, with and without statistics / NULLs, the rare rows inside the main loop."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "hll_rare_values.json")) as f:
        fx = json.load(f)
    rare = [e["value"] for e in fx["int64"]]
    rng = np.random.default_rng(44)
    n = 300_000
    base = [int(x) for x in rng.integers(-2 ** 62, 2 ** 62, n)]
    for k, v in enumerate(rare * 3):
        base[(k * 40_009 + 1_234) % n] = v
    for null_frac in (0.0, 0.1):
        vals = [None if (null_frac and rng.random() < null_frac and x not in rare) else x for x in base]
        f64 = [None if x is None else struct.unpack("<d", struct.pack("<q", x))[0] for x in vals]
        spec = {"i": ["int64", vals], "f": ["float64", f64]}
        ot, pt = oracle_table(spec), product_table(spec)
        # (the fp64 column holds the same bit patterns: huge magnitudes, so no sums on it)
        for an in ([d.ApproxCountDistinct("i"), d.ApproxCountDistinct("f")],
                   _suite("i", ["i >= 0"]),
                   [d.Completeness("f"), d.Minimum("f"), d.Maximum("f"), d.ApproxCountDistinct("f"),
                    d.Compliance("p0", "f > 0")]):
            st = d.run_scan(an, pt)
            for a in an:
                _check_state(a, st[a], ot)


def test_fast_equals_general_kernel(gpu, monkeypatch):
    """The same plans through dq_scan_values_kernel (DQ_SCAN_FAST=0): integer results and HLL
    registers identical, fp64 within the 1e-12 bar of each other."""
    rng = np.random.default_rng(31)
    n = 250_003
    spec = {"i": ["int64", _c2_like_int(rng, n, 0.05)], "f": ["float64", _c2_like_float(rng, n, 0.05)]}
    pt = product_table(spec).to_device(0)
    an = _suite("i", ["i >= 0"]) + _suite("f", ["f > 5e5"])
    fast = d.run_scan(an, pt)
    monkeypatch.setenv("DQ_SCAN_FAST", "0")
    general = d.run_scan(an, pt)
    monkeypatch.delenv("DQ_SCAN_FAST")
    for a in an:
        g, e = fast[a], general[a]
        if isinstance(a, (d.Sum, d.Mean)) and a.column == "f":
            assert abs(g.sum_value - e.sum_value) <= 1e-12 * abs(e.sum_value), a
        elif isinstance(a, d.StandardDeviation):
            assert g.n == e.n
            assert abs(g.avg - e.avg) <= 1e-12 * abs(e.avg), a
            assert abs(g.m2 - e.m2) <= 1e-12 * abs(e.m2), a
        else:
            assert g == e, (a, g, e)
