"""GPU path vs the oracle on seeded inputs: every scan-shareable analyzer, every column type,
ragged sizes around the 2048-row chunk and 16-byte vector boundaries, NULL fractions 0 / 0.3 /
1, `where` filters, inline and generic Compliance predicates.

Bar (BASELINE.json north_star): bit-exact for counts, Compliance, Min/Max, integral Sum/Mean
and HLL registers; relative error <= 1e-12 against the EXACT value for fp64 Sum/Mean/StdDev
(the oracle's sequential Spark-order sum is itself ~sqrt(n) ulps off the exact value)."""
import math
from fractions import Fraction

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from helpers import oracle_table, product_table, random_table

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12  # fp64 Sum/Mean/StdDev vs exact (north_star tolerance)

NUMERIC = ["c_int8", "c_int16", "c_int32", "c_int64", "c_float32", "c_float64"]
WHERES = [None, "c_int32 > 0", "c_string != 'k1'", "c_float64 < 1000 OR c_bool"]
PREDICATES = ["c_int64 >= 0", "COALESCE(c_float64, 0.0) > 1000", "c_int8 IS NULL",
              "c_int16 < 3.5", "c_float32 >= 1000", "c_int32 > 5 AND c_float64 < 1000",
              "c_string IN ('k1', 'k2')", "c_bool", "c_int64 BETWEEN -100 AND 2000000000",
              "c_int8 = 7", "TRUE"]


CORR_PAIRS = [("c_int64", "c_float64"), ("c_int32", "c_float32"), ("c_float64", "c_int8"),
              ("c_int16", "c_int16")]


def _analyzers():
    out = []
    for w in WHERES:
        out.append(d.Size(w))
        for c in NUMERIC:
            out += [d.Completeness(c, w), d.Sum(c, w), d.Mean(c, w), d.StandardDeviation(c, w),
                    d.Minimum(c, w), d.Maximum(c, w), d.ApproxCountDistinct(c, w)]
        out += [d.Completeness("c_string", w), d.Completeness("c_bool", w),
                d.ApproxCountDistinct("c_string", w), d.ApproxCountDistinct("c_bool", w)]
        for k, p in enumerate(PREDICATES):
            out.append(d.Compliance("p%d" % k, p, w))
        out += [d.MinLength("c_string", w), d.MaxLength("c_string", w)]
        for x, y in CORR_PAIRS:
            out.append(d.Correlation(x, y, w))
    return out


def _selected(ot, column, where):
    w = O._where_mask(ot, where)
    return [v for v, keep in zip(ot[column].values, w) if keep is True and v is not None]


def _exact_moments(vals):
    fr = [Fraction(float(v)) for v in vals]
    n = len(fr)
    s1 = sum(fr)
    s2 = sum(x * x for x in fr)
    return n, s1 / n, s2 - s1 * s1 / n


def _check_state(a, got, ot):
    name = type(a).__name__
    where = a.where
    if name in ("Size", "Completeness", "Compliance"):
        exp = {"Size": lambda: O.size_state(ot, where),
               "Completeness": lambda: O.completeness_state(ot, a.column, where),
               "Compliance": lambda: O.compliance_state(ot, a.predicate, where)}[name]()
        if exp is None:
            assert got is None, (a, got)
        elif name == "Size":
            assert got == d.NumMatches(exp.num_matches), (a, got, exp)
        else:
            assert got == d.NumMatchesAndCount(exp.num_matches, exp.count), (a, got, exp)
        return
    if name in ("MinLength", "MaxLength"):
        exp = (O.min_length_state if name == "MinLength" else O.max_length_state)(ot, a.column, where)
        if exp is None:
            assert got is None, (a, got)
        else:
            assert got == (d.MinState(exp.min_value) if name == "MinLength" else d.MaxState(exp.max_value)), (a, got)
        return
    if name == "Correlation":
        _check_correlation(a, got, ot)
        return
    if name == "ApproxCountDistinct":
        exp = O.approx_count_distinct_state(ot, a.column, where)
        assert got is not None and list(got.words) == list(exp.words), a
        return
    vals = _selected(ot, a.column, where)
    dtype = ot[a.column].dtype
    if not vals:
        assert got is None, (a, got)
        return
    integral = dtype.startswith("int")
    if name in ("Sum", "Mean"):
        s = got.sum_value
        if integral:
            assert s == O._spark_sum(dtype, vals), a  # exact int64 sum, one cast
        else:
            exact = math.fsum(float(v) for v in vals)
            assert abs(s - exact) <= REL_TOL * abs(exact) + 1e-300, (a, s, exact)
        if name == "Mean":
            assert got.count == len(vals), a
    elif name == "StandardDeviation":
        n, mean, m2 = _exact_moments(vals)
        assert got.n == float(n), a
        assert abs(got.avg - float(mean)) <= REL_TOL * abs(float(mean)) + 1e-300, (a, got.avg, float(mean))
        assert abs(got.m2 - float(m2)) <= REL_TOL * abs(float(m2)) + 1e-9, (a, got.m2, float(m2))
    elif name == "Minimum":
        _same_double(got.minValue, O.min_state(ot, a.column, where).min_value, a)
    elif name == "Maximum":
        _same_double(got.maxValue, O.max_state(ot, a.column, where).max_value, a)


def _same_double(got, want, a):
    """Bit-exact double equality where NaN equals NaN (a selected NaN wins Maximum)."""
    if want != want:
        assert got != got, (a, got, want)
    else:
        assert got == want, (a, got, want)


def _check_correlation(a, got, ot):
    """Bit-exact n; xAvg, yAvg, ck, xMk, yMk within 1e-12 of the exact (rational) values, ck on
    the scale sqrt(xMk * yMk) (it may cancel to ~0)."""
    w = O._where_mask(ot, a.where)
    pairs = [(Fraction(float(x)), Fraction(float(y))) for x, y, keep in
             zip(ot[a.firstColumn].values, ot[a.secondColumn].values, w)
             if keep is True and x is not None and y is not None]
    if not pairs:
        assert got is None, (a, got)
        return
    n = len(pairs)
    sx = sum(p[0] for p in pairs)
    sy = sum(p[1] for p in pairs)
    xmk = sum(p[0] * p[0] for p in pairs) - sx * sx / n
    ymk = sum(p[1] * p[1] for p in pairs) - sy * sy / n
    ck = sum(p[0] * p[1] for p in pairs) - sx * sy / n
    assert got.n == float(n), a
    for g, e in ((got.xAvg, sx / n), (got.yAvg, sy / n), (got.xMk, xmk), (got.yMk, ymk)):
        assert abs(g - float(e)) <= REL_TOL * abs(float(e)) + 1e-9, (a, g, float(e))
    scale = math.sqrt(float(xmk) * float(ymk))
    assert abs(got.ck - float(ck)) <= REL_TOL * scale + 1e-9, (a, got.ck, float(ck))


@pytest.mark.parametrize("n", [0, 1, 5, 17, 2047, 2048, 2049, 9000])
@pytest.mark.parametrize("null_frac", [0.0, 0.3, 1.0])
def test_scan_parity_vs_oracle(gpu, n, null_frac):
    rng = np.random.default_rng(1000 + n + int(null_frac * 10))
    spec = random_table(rng, n, null_frac)
    spec["c_bool"][1] = [None if v is None else v for v in spec["c_bool"][1]]
    if null_frac == 1.0:  # keep the filter columns populated so `where` selects something
        spec2 = random_table(rng, n, 0.0)
        for k in ("c_int32", "c_string", "c_bool"):
            spec[k] = spec2[k]
    ot, pt = oracle_table(spec), product_table(spec)
    analyzers = _analyzers()
    states = d.run_scan(analyzers, pt)
    for a in analyzers:
        _check_state(a, states[a], ot)


def test_device_resident_and_host_batches_agree(gpu):
    rng = np.random.default_rng(5)
    spec = random_table(rng, 50001, 0.1)
    pt = product_table(spec)
    analyzers = _analyzers()
    host = d.run_scan(analyzers, pt)
    dev = d.run_scan(analyzers, pt.to_device(0))
    for a in analyzers:
        assert host[a] == dev[a], a


def test_deterministic_bitwise(gpu):
    rng = np.random.default_rng(6)
    pt = product_table(random_table(rng, 30011, 0.05)).to_device(0)
    analyzers = _analyzers()
    first = d.run_scan(analyzers, pt)
    for _ in range(2):
        again = d.run_scan(analyzers, pt)
        for a in analyzers:
            assert first[a] == again[a], a


def test_sliced_arrow_columns(gpu):
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(8)
    n = 10007
    ints = pa.array([None if rng.random() < 0.2 else int(x) for x in rng.integers(-50, 50, n)], pa.int64())
    flts = pa.array([None if rng.random() < 0.2 else float(x) for x in rng.normal(0, 1, n)], pa.float64())
    strs = pa.array([None if rng.random() < 0.2 else "s%d" % x for x in rng.integers(0, 9, n)], pa.string())
    tbl = pa.table({"i": ints, "f": flts, "s": strs})
    analyzers = [d.Size(), d.Completeness("i"), d.Sum("i"), d.Mean("f"), d.StandardDeviation("f"),
                 d.Minimum("i"), d.Maximum("f"), d.ApproxCountDistinct("s"), d.ApproxCountDistinct("i"),
                 d.Compliance("c", "i > 3"), d.Compliance("s", "s = 's3'"), d.Size("s != 's1'")]
    for off, length in [(0, n), (3, 5000), (13, 8001), (1, 1), (4097, 3000)]:
        sl = tbl.slice(off, length)
        got = d.run_scan(analyzers, d.Table.from_arrow(sl))
        want = d.run_scan(analyzers, d.Table.from_arrow(pa.table({k: pa.array(sl[k].to_pylist(), sl[k].type) for k in ("i", "f", "s")})))
        for a in analyzers:
            assert got[a] == want[a], (off, a)
        ot = oracle_table({"i": ["int64", sl["i"].to_pylist()], "f": ["float64", sl["f"].to_pylist()],
                           "s": ["string", sl["s"].to_pylist()]})
        for a in analyzers:
            _check_state(a, got[a], ot)


def test_special_float_values(gpu):
    vals = [1.0, float("nan"), -3.5, float("inf"), 2.0, None, -0.5]
    ot = oracle_table({"f": ["float64", vals]})
    pt = product_table({"f": ["float64", vals]})
    st = d.run_scan([d.Minimum("f"), d.Maximum("f"), d.Sum("f"), d.Compliance("nan", "f > 1.5"),
                     d.ApproxCountDistinct("f")], pt)
    assert st[d.Minimum("f")].minValue == -3.5          # NaN never wins min (NaN-safe order)
    assert math.isnan(st[d.Maximum("f")].maxValue)       # NaN always wins max
    assert math.isnan(st[d.Sum("f")].sum_value)
    assert st[d.Compliance("nan", "f > 1.5")] == d.NumMatchesAndCount(3, 7)  # NaN > 1.5, inf, 2.0
    assert list(st[d.ApproxCountDistinct("f")].words) == list(
        O.approx_count_distinct_state(ot, "f").words)
    only_nan = d.run_scan([d.Minimum("f")], product_table({"f": ["float64", [float("nan"), None]]}))
    assert math.isnan(only_nan[d.Minimum("f")].minValue)


@pytest.mark.parametrize("ftype", ["float64", "float32"])
def test_special_float_values_in_main_loop(gpu, ftype):
    """NaN / ±Inf far from the ragged tail, where the scan tests a lane's Σd once per
    iteration: a selected NaN wins max; +Inf with -Inf (Σd NaN, no NaN value) must not; a NaN
    on a row the `where` filter drops must not either."""
    n = 300_000
    rng = np.random.default_rng(11)
    base = rng.uniform(-1e3, 1e3, n).astype(np.float32 if ftype == "float32" else np.float64)
    g = np.ones(n, dtype=np.int64)

    def run(vals, gs, where=None):
        pt = product_table({"f": [ftype, [float(v) for v in vals]], "g": ["int64", gs.tolist()]})
        return d.run_scan([d.Minimum("f", where), d.Maximum("f", where), d.Sum("f", where)], pt), where

    v = base.copy()
    v[123_457] = np.nan
    st, w = run(v, g)
    assert math.isnan(st[d.Maximum("f", w)].maxValue)
    assert st[d.Minimum("f", w)].minValue == float(np.nanmin(v))
    assert math.isnan(st[d.Sum("f", w)].sum_value)

    v = base.copy()
    v[200_001], v[200_002] = np.inf, -np.inf  # same lane, same iteration
    st, w = run(v, g)
    assert st[d.Maximum("f", w)].maxValue == math.inf
    assert st[d.Minimum("f", w)].minValue == -math.inf
    assert math.isnan(st[d.Sum("f", w)].sum_value)

    v = base.copy()
    v[77_777] = np.nan
    gs = g.copy()
    gs[77_777] = 0
    st, w = run(v, gs, "g > 0")
    keep = np.arange(n) != 77_777
    assert st[d.Maximum("f", w)].maxValue == float(v[keep].max())
    assert st[d.Minimum("f", w)].minValue == float(v[keep].min())
    assert not math.isnan(st[d.Sum("f", w)].sum_value)


def test_int64_extremes_and_wraparound(gpu):
    big = [2 ** 63 - 1, 2 ** 63 - 1, -(2 ** 63), 5, None]
    pt = product_table({"x": ["int64", big]})
    st = d.run_scan([d.Sum("x"), d.Minimum("x"), d.Maximum("x"), d.Compliance("p", "x > 3.5")], pt)
    assert st[d.Sum("x")].sum_value == float(O._wrap64(sum(v for v in big if v is not None)))
    assert st[d.Minimum("x")].minValue == float(-(2 ** 63))
    assert st[d.Maximum("x")].maxValue == float(2 ** 63 - 1)
    assert st[d.Compliance("p", "x > 3.5")] == d.NumMatchesAndCount(3, 5)


def test_large_batch_properties(gpu):
    """Size-independent properties at 8M rows (device resident): counts exact, int sum
    exact, fp64 sum within 1e-12 of math.fsum, min/max exact, merge-of-halves == whole."""
    import torch
    n = 8_000_000
    rng = np.random.default_rng(42)
    iv = rng.integers(-2 ** 30, 2 ** 32, n, dtype=np.int64)
    fv = rng.uniform(0, 1e6, n)
    valid = rng.random(n) >= 0.05
    t = d.Table({"i": d.Column.from_numpy(iv, valid), "f": d.Column.from_numpy(fv, valid)})
    tdev = t.to_device(0)
    an = [d.Size(), d.Completeness("i"), d.Sum("i"), d.Sum("f"), d.Minimum("f"), d.Maximum("i"),
          d.Mean("f"), d.Compliance("ci", "i >= 0"), d.Compliance("cf", "f > 5e5")]
    st = d.run_scan(an, tdev)
    assert st[d.Size()] == d.NumMatches(n)
    assert st[d.Completeness("i")] == d.NumMatchesAndCount(int(valid.sum()), n)
    assert st[d.Sum("i")].sum_value == float(int(iv[valid].sum()))
    exact = math.fsum(fv[valid].tolist())
    assert abs(st[d.Sum("f")].sum_value - exact) <= REL_TOL * exact
    assert st[d.Minimum("f")].minValue == fv[valid].min()
    assert st[d.Maximum("i")].maxValue == float(iv[valid].max())
    assert st[d.Compliance("ci", "i >= 0")] == d.NumMatchesAndCount(int((iv[valid] >= 0).sum()), n)
    assert st[d.Compliance("cf", "f > 5e5")] == d.NumMatchesAndCount(int((fv[valid] > 5e5).sum()), n)
    half = n // 2 + 123
    parts = d.PartitionedTable([
        d.Table({"i": d.Column.from_numpy(iv[:half], valid[:half]), "f": d.Column.from_numpy(fv[:half], valid[:half])}),
        d.Table({"i": d.Column.from_numpy(iv[half:], valid[half:]), "f": d.Column.from_numpy(fv[half:], valid[half:])}),
    ])
    st2 = d.run_scan(an, parts)
    for a in an:
        if isinstance(a, (d.Sum, d.Mean)) and a.column == "f":
            assert abs(st2[a].sum_value - exact) <= REL_TOL * exact
        else:
            assert st2[a] == st[a], a
    del tdev
    torch.cuda.empty_cache()


def test_string_lengths_unicode(gpu):
    """MinLength/MaxLength count characters the way Spark 2.2.2's UTF8String.numChars does
    (multi-byte sequences are one character each), against the oracle."""
    vals = ["", "a", "é", "€uro", "日本語テキスト", "😀😀", "x" * 300, None, "mixé€😀", "ab"]
    spec = {"s": ["string", vals * 37], "i": ["int32", list(range(len(vals) * 37))]}
    ot, pt = oracle_table(spec), product_table(spec)
    for w in (None, "i > 100", "i < 0"):
        for a in (d.MinLength("s", w), d.MaxLength("s", w)):
            _check_state(a, d.run_scan([a], pt)[a], ot)
    ctx = d.AnalysisRunner.onData(pt).addAnalyzers([d.MaxLength("s"), d.MinLength("s")]).run()
    assert ctx.metric(d.MaxLength("s")).value.get() == 300.0
    assert ctx.metric(d.MinLength("s")).value.get() == 0.0


def test_correlation_state_merge_equals_union(gpu):
    """CorrelationState.sum of two batches' states equals the state of their union (within the
    fp64 bar), and batch-split invariance of the plan."""
    rng = np.random.default_rng(77)
    spec = random_table(rng, 20000, 0.1, ["int64", "float64"])
    pt = product_table(spec)
    a = d.Correlation("c_int64", "c_float64")
    whole = d.run_scan([a], pt)[a]
    half = 20000 // 2
    parts = [d.Table.from_pydict({k: (v[0], v[1][s:e]) for k, v in spec.items()}) for s, e in ((0, half), (half, 20000))]
    merged = d.run_scan([a], parts[0])[a].sum(d.run_scan([a], parts[1])[a])
    for g, e in zip(merged.fields(), whole.fields()):
        assert abs(g - e) <= 1e-12 * max(1.0, abs(e)), (merged, whole)
    batched = d.run_scan([a], d.PartitionedTable(parts))[a]
    for g, e in zip(batched.fields(), whole.fields()):
        assert abs(g - e) <= 1e-12 * max(1.0, abs(e)), (batched, whole)
    r = a.computeMetricFrom(whole).value.get()
    assert -1.0 <= r <= 1.0


def test_hll_rare_rank_branches(gpu):
    """Hashes whose rank is not decided by the high word (1 in 2^23 rows) or exceeds 32
    (1 in 2^32): the device's wave-uniform rare branch must give the oracle's registers."""
    import json
    import os
    import struct
    with open(os.path.join(os.path.dirname(__file__), "golden", "hll_rare_values.json")) as f:
        fx = json.load(f)
    i64 = [e["value"] for e in fx["int64"]]
    i32 = [e["value"] for e in fx["int32"]]
    f64 = [struct.unpack("<d", struct.pack("<q", v))[0] for v in i64]  # same bit patterns
    # rare rows among ordinary ones, at several lane positions and inside the vector main loop
    rng = np.random.default_rng(11)
    def spread(vals, ordinary):
        out = list(ordinary)
        for k, v in enumerate(vals):
            out[(k * 977 + 5) % len(out)] = v
        return out
    n = 5000
    cols = {"a": ["int64", spread(i64, [int(x) for x in rng.integers(-2**62, 2**62, n)])],
            "b": ["int32", spread(i32, [int(x) for x in rng.integers(-2**31, 2**31, n)])],
            "c": ["float64", spread(f64, [float(x) for x in rng.normal(0, 1e6, n)])]}
    ot = oracle_table(cols)
    st = d.run_scan([d.ApproxCountDistinct(c) for c in cols], product_table(cols))
    for c in cols:
        assert list(st[d.ApproxCountDistinct(c)].words) == list(O.approx_count_distinct_state(ot, c).words), c


def test_pooled_plan_reuse_equals_fresh_plan(gpu, monkeypatch):
    """A finished plan goes back to the pool and the next run of the same analyzers over the same
    schema resets and reuses it: every state equals a fresh plan's, across tables of different
    sizes and NULL fractions (host and device batches), and the pool holds the plan afterwards."""
    from deequ_amd import engine
    engine.clear_plan_cache()
    rng = np.random.default_rng(77)
    analyzers = _analyzers()
    tables = [product_table(random_table(rng, n, f)) for n, f in ((9000, 0.1), (17, 0.0), (40001, 0.5))]
    tables[1] = tables[1].to_device(0)
    pooled = [d.run_scan(analyzers, t) for t in tables]
    assert sum(len(v) for v in engine._PLAN_POOL.values()) == 1
    monkeypatch.setenv("DEEQU_AMD_PLAN_CACHE", "0")
    for t, got in zip(tables, pooled):
        fresh = d.run_scan(analyzers, t)
        for a in analyzers:
            assert got[a] == fresh[a], a
