"""Parity cases the round-1 review found uncovered (VERDICT r1 "What's weak" 1):

* the predicate strings deequ's Check DSL emits for isContainedIn, backtick-quoted, exactly as
  Check.scala:908-912 and :936-940 build them (quotes escaped the Scala way, bounds printed by
  Double.toString), run on the GPU against the oracle;
* Spark 2.2's implicit string -> double cast in comparisons (PromoteStrings), e.g. `item > 3`
  on a string column (CheckTest.scala:193) and `unique < 4` (AnalyzerTests.scala:551-558), on
  the device through DQ_P_CAST_DOUBLE, correctly rounded for every input (no fall-back);
* FloatType comparisons with integer literals above 2^24 (float vs int -> FloatType);
* fp64 sums of values of opposite sign near DBL_MAX, in both scan kernels;
* runOnAggregatedStates over loaders holding GPU-computed partition states
  (AnalysisRunner.scala:385-460) == the metrics of the whole table;
* failure scoping as AnalysisTest.scala:206-280 injects it: an aggregation failure fails every
  scan-shareable analyzer of the run, an extraction failure only its own.
"""
import math

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd.metrics import Failure
from helpers import known_answers, oracle_table, product_table
from test_gpu_parity import _check_state

pytestmark = pytest.mark.gpu


def _java_double_str(v: float) -> str:
    return O.java_double_to_string(float(v))


def _contained_in_values(column, allowed):
    values = ",".join("'%s'" % a.replace("'", "''") for a in allowed)
    return "`%s` IS NULL OR `%s` IN (%s)" % (column, column, values)


def _contained_in_range(column, lo, hi, incl_lo=True, incl_hi=True):
    return "`%s` IS NULL OR (`%s` %s %s AND `%s` %s %s)" % (
        column, column, ">=" if incl_lo else ">", _java_double_str(lo), column, "<=" if incl_hi else "<",
        _java_double_str(hi))


def test_is_contained_in_predicates(gpu):
    rng = np.random.default_rng(17)
    n = 20011
    cats = ["a", "b", "c", "it's", "ab", "", "z"]
    spec = {
        "s": ["string", [None if rng.random() < 0.1 else cats[i] for i in rng.integers(0, len(cats), n)]],
        "i": ["int64", [None if rng.random() < 0.1 else int(x) for x in rng.integers(-50, 50, n)]],
        "f": ["float64", [None if rng.random() < 0.1 else float(x) for x in rng.normal(0, 10, n)]],
        "w": ["int32", [int(x) for x in rng.integers(0, 4, n)]],
    }
    ot, pt = oracle_table(spec), product_table(spec)
    preds = [
        _contained_in_values("s", ["a", "b"]),
        _contained_in_values("s", ["it's", "z", ""]),  # quote escaped as '' (Check.scala:908-910)
        _contained_in_range("i", -10.0, 10.0),
        _contained_in_range("i", -10.5, 10.25, False, False),
        _contained_in_range("f", -3.5, 1e10, True, False),  # 1e10 prints as 1.0E10: a double literal
        _contained_in_range("f", -1.0, 1.0, False, True),
    ]
    for k, p in enumerate(preds):
        for where in (None, "w > 1"):
            a = d.Compliance("c%d" % k, p, where)
            _check_state(a, d.run_scan([a], pt)[a], ot)
    # all of them in one fused pass, as VerificationSuite would run them
    an = [d.Compliance("c%d" % k, p) for k, p in enumerate(preds)]
    st = d.run_scan(an, pt)
    for a in an:
        _check_state(a, st[a], ot)


def test_string_to_double_cast_in_predicates(gpu):
    """Spark 2.2 PromoteStrings: `strcol CMP number` compares Cast(strcol AS DOUBLE) in double;
    unparsable strings are NULL (not TRUE, not FALSE)."""
    texts = ["1", "2", " 3 ", "4.5", "-7", "1e3", "abc", "", "NaN", "-Infinity", "5d", "+6.25f", ".5",
             "0012", "1_0", "inf", None]
    rng = np.random.default_rng(3)
    n = 12000
    col = [texts[i] for i in rng.integers(0, len(texts), n)]
    spec = {"item": ["string", col], "v": ["int32", [int(x) for x in rng.integers(0, 10, n)]]}
    ot, pt = oracle_table(spec), product_table(spec)
    for p in ("item > 3", "item < 4", "item = 4.5", "item >= -7", "item != 2", "3 < item", "item <= 1000.5"):
        for where in (None, "v > 4"):
            a = d.Compliance(p, p, where)
            _check_state(a, d.run_scan([a], pt)[a], ot)
        for b in (d.Size(p), d.Completeness("v", p), d.Sum("v", p), d.ApproxCountDistinct("v", p)):
            _check_state(b, d.run_scan([b], pt)[b], ot)


def test_string_to_double_beyond_fast_path_is_exact(gpu):
    """Numbers off Clinger's fast path (> 19 significant digits, |exponent| > 22, hexadecimal,
    halfway points) cast exactly on the device (Eisel-Lemire + the big-integer comparison), so
    the op succeeds and matches the oracle's Java parseDouble (the fused pass's other analyzers
    are unaffected)."""
    vals = ["1", "2", "12345678901234567890123", "4", "3.0000000000000000000000001", "2.9999999999999999999999",
            "0x1.8p1", "3e-400", "1e400", "3.000000000000000444089209850062616169452667236328125"]
    spec = {"item": ["string", vals], "v": ["int32", list(range(1, len(vals) + 1))]}
    pt, ot = product_table(spec), oracle_table(spec)
    cast_op = d.Compliance("cast", "item > 3")
    others = [d.Size(), d.Sum("v"), d.Compliance("plain", "v > 2")]
    ctx = d.AnalysisRunner.onData(pt).addAnalyzers([cast_op] + others).run()
    assert ctx.metric(cast_op).value.get() == O.compliance_state(ot, "item > 3").metric_value()
    assert ctx.metric(d.Size()).value.get() == float(len(vals))
    assert ctx.metric(d.Sum("v")).value.get() == float(sum(range(1, len(vals) + 1)))
    assert ctx.metric(d.Compliance("plain", "v > 2")).value.get() == (len(vals) - 2) / len(vals)


def test_reference_string_cast_known_answers(gpu):
    """AnalyzerTests.scala:551-558 (ApproxCountDistinct with `unique < 4` = 2.0) and the
    CheckTest.scala:174-290 where-filtered checks on the string column `item`."""
    ka = known_answers()
    ids = {"acd_where_string_cast", "check_lt_where_item", "check_le_where_item", "check_gt_where_item",
           "check_ge_where_item", "check_satisfies_where", "check_satisfies_where_half"}
    cases = [c for c in ka["cases"] if c["id"] in ids]
    assert len(cases) == len(ids)
    for c in cases:
        table = product_table(ka["tables"][c["table"]])
        a = getattr(d, c["analyzer"])(*c["args"])
        assert a.calculate(table).value.get() == c["expected"], c


def test_float_column_vs_large_int_literal(gpu):
    """Spark 2.2 compares FloatType with an int literal in FloatType: 16777217 rounds to 2^24."""
    vals = [16777216.0, 16777218.0, 16777220.0, 3.0, None, 2.0 ** 31, 2.0 ** 31 + 256.0]
    spec = {"x": ["float32", vals * 300]}
    ot, pt = oracle_table(spec), product_table(spec)
    for p in ("x = 16777217", "x > 16777217", "x <= 16777219", "x >= 2147483647", "x < 2147483777",
              "x != 16777217"):
        a = d.Compliance(p, p)
        _check_state(a, d.run_scan([a], pt)[a], ot)
    got = d.run_scan([d.Compliance("e", "x = 16777217")], pt)[d.Compliance("e", "x = 16777217")]
    assert got.numMatches == 300  # 16777216f only: Spark's FloatType equality


@pytest.mark.parametrize("order,reps", [([1e306, -1e306, 5.0], 50), ([5.0, 1e306, -1e306], 50),
                                        ([-1.7e306, 3.0, 1.7e306, -2.0], 40), ([1e308, -1e308, 5.0], 1),
                                        ([1e307, -1e307, 5.0], 700), ([-1.7e307, 3.0, 1.7e307, -2.0], 700),
                                        ([1.7e308, -1.7e308], 700), ([-1.7e308, 1.7e308, 1.0], 700)])
def test_fp64_sum_near_dbl_max(gpu, order, reps):
    """Opposite-sign values near DBL_MAX: the Sum is taken over the raw values, so the
    moments' shift (dropped when |shift| > 2^1000) can no longer overflow it to Inf / NaN, in both
    scan kernels (no where: the 8-byte fast kernel; with a where filter: the general kernel).
    Summation order differs from Spark's sequential order (itself partition-dependent), so the
    bar is the error bound of any-order float summation: within 1e-12 * sum |x| of the exact sum,
    and finite, whenever sum |x| < DBL_MAX.  Past that bound a parallel sum may overflow where a
    sequential one does not (a lane accumulating rows of one sign); those cases check the
    extrema only."""
    rows = order * reps
    spec = {"f": ["float64", rows], "g": ["int32", [1] * len(rows)]}
    pt = product_table(spec)
    k = 2.0 ** -1000  # compare scaled: sum |x| itself may overflow
    exact = math.fsum(x * k for x in rows)
    scale = math.fsum(abs(x) * k for x in rows)
    bounded = scale < 1.7e308 * k
    for where in (None, "g > 0"):
        st = d.run_scan([d.Sum("f", where), d.Mean("f", where), d.Maximum("f", where), d.Minimum("f", where)], pt)
        got = st[d.Sum("f", where)].sum_value
        if bounded:
            assert math.isfinite(got), (where, got)
            assert abs(got * k - exact) <= 1e-12 * scale, (where, got, exact / k)
        assert st[d.Maximum("f", where)].maxValue == max(rows)
        assert st[d.Minimum("f", where)].minValue == min(rows)


def test_run_on_aggregated_states_over_gpu_states(gpu):
    """AnalysisRunner.runOnAggregatedStates (AnalysisRunner.scala:385-460): states of partitions
    computed on the GPU and kept in InMemoryStateProviders merge to the whole table's metrics
    (StateAggregationIntegrationTest.scala:55-127 pattern)."""
    rng = np.random.default_rng(12)
    n = 30000
    spec = {"i": ["int64", [None if rng.random() < 0.05 else int(x) for x in rng.integers(-1000, 10 ** 6, n)]],
            "f": ["float64", [None if rng.random() < 0.05 else float(x) for x in rng.normal(5e2, 50, n)]],
            "s": ["string", ["k%d" % x for x in rng.integers(0, 500, n)]]}
    analyzers = [d.Size(), d.Completeness("i"), d.Compliance("pos", "i >= 0"), d.Sum("i"), d.Mean("f"),
                 d.StandardDeviation("f"), d.Minimum("i"), d.Maximum("f"), d.ApproxCountDistinct("s"),
                 d.ApproxCountDistinct("i"), d.Uniqueness(["s"]), d.Entropy("s"), d.CountDistinct(["s"])]
    cuts = [0, 7001, 18000, n]
    providers = []
    for a0, b0 in zip(cuts, cuts[1:]):
        part = product_table({k: [t, v[a0:b0]] for k, (t, v) in spec.items()})
        prov = d.InMemoryStateProvider()
        d.AnalysisRunner.onData(part).addAnalyzers(analyzers).saveStatesWith(prov).run()
        providers.append(prov)
    schema = {"i": "int64", "f": "float64", "s": "string"}
    agg = d.AnalysisRunner.runOnAggregatedStates(schema, d.Analysis(analyzers), providers)
    whole = d.AnalysisRunner.onData(product_table(spec)).addAnalyzers(analyzers).run()
    for a in analyzers:
        got, want = agg.metric(a).value.get(), whole.metric(a).value.get()
        assert abs(got - want) <= 1e-12 * max(1.0, abs(want)), (a, got, want)
    # a loader without a state for some analyzer: the others still merge (missing = None)
    partial = d.AnalysisRunner.runOnAggregatedStates(schema, d.Analysis([d.Sum("i")]),
                                                     [providers[0], d.InMemoryStateProvider()])
    first = d.AnalysisRunner.onData(product_table({k: [t, v[:7001]] for k, (t, v) in spec.items()})) \
        .addAnalyzer(d.Sum("i")).run()
    assert partial.metric(d.Sum("i")).value.get() == first.metric(d.Sum("i")).value.get()


def test_run_on_aggregated_states_vs_oracle(gpu):
    """runOnAggregatedStates over GPU-computed partition states against the ORACLE's states of
    the same partitions merged with `Analyzers.merge` (Analyzer.scala:367-386, State.sum of each
    state class; oracle.merge_options), in the same partition order.  Bit-exact for counts,
    integral sums, Min/Max, HLL counts and the frequency metrics; fp64 within 1e-12."""
    rng = np.random.default_rng(29)
    n = 24000
    spec = {"i": ["int64", [None if rng.random() < 0.05 else int(x) for x in rng.integers(-1000, 10 ** 6, n)]],
            "f": ["float64", [None if rng.random() < 0.05 else float(x) for x in rng.normal(5e2, 50, n)]],
            "s": ["string", [None if rng.random() < 0.02 else "k%d" % x for x in rng.integers(0, 4000, n)]]}
    analyzers = [d.Size(), d.Completeness("i"), d.Compliance("pos", "i >= 0"), d.Sum("i"), d.Mean("f"),
                 d.StandardDeviation("f"), d.Minimum("i"), d.Maximum("f"), d.ApproxCountDistinct("s"),
                 d.ApproxCountDistinct("i"), d.Uniqueness(["s"]), d.Distinctness(["s"]), d.Entropy("s"),
                 d.CountDistinct(["s"]), d.UniqueValueRatio(["s"])]
    cuts = [0, 5003, 5004, 16000, n]
    providers, parts = [], []
    for a0, b0 in zip(cuts, cuts[1:]):
        sub = {k: [t, v[a0:b0]] for k, (t, v) in spec.items()}
        prov = d.InMemoryStateProvider()
        d.AnalysisRunner.onData(product_table(sub)).addAnalyzers(analyzers).saveStatesWith(prov).run()
        providers.append(prov)
        parts.append(oracle_table(sub))
    schema = {"i": "int64", "f": "float64", "s": "string"}
    agg = d.AnalysisRunner.runOnAggregatedStates(schema, d.Analysis(analyzers), providers)

    def merged(fn, *args):
        return O.merge_options(*[fn(p, *args) for p in parts])

    want = {
        d.Size(): merged(O.size_state).metric_value(),
        d.Completeness("i"): merged(O.completeness_state, "i").metric_value(),
        d.Compliance("pos", "i >= 0"): merged(O.compliance_state, "i >= 0").metric_value(),
        d.Sum("i"): merged(O.sum_state, "i").metric_value(),
        d.Minimum("i"): merged(O.min_state, "i").metric_value(),
        d.Maximum("f"): merged(O.max_state, "f").metric_value(),
        d.ApproxCountDistinct("s"): merged(O.approx_count_distinct_state, "s").metric_value(),
        d.ApproxCountDistinct("i"): merged(O.approx_count_distinct_state, "i").metric_value(),
    }
    freq = merged(O.frequencies_state, ["s"])
    want[d.Uniqueness(["s"])] = O.uniqueness_metric(freq)
    want[d.Distinctness(["s"])] = O.distinctness_metric(freq)
    want[d.CountDistinct(["s"])] = O.count_distinct_metric(freq)
    want[d.UniqueValueRatio(["s"])] = O.unique_value_ratio_metric(freq)
    close = {d.Mean("f"): merged(O.mean_state, "f").metric_value(),
             d.StandardDeviation("f"): merged(O.stddev_state, "f").metric_value(),
             d.Entropy("s"): O.entropy_exact(freq)}
    for a, w in want.items():
        assert agg.metric(a).value.get() == w, (a, agg.metric(a).value.get(), w)
    for a, w in close.items():
        got = agg.metric(a).value.get()
        assert abs(got - w) <= 1e-12 * abs(w), (a, got, w)


class _ExtractionFailingMean(d.Mean):
    """AnalysisTest.scala:228-253: fromAggregationResult throws."""

    def fromAggregationResult(self, raw):
        raise ValueError("-test-mean-failing-")


class _AggregationFailingMean(d.Mean):
    """AnalysisTest.scala:255-280: aggregationFunctions throws."""

    def aggregationFunctions(self, schema):
        raise ValueError("-test-agg-failing-")


def test_failure_scoping(gpu):
    pt = product_table(known_answers()["tables"]["dfNumeric"])
    # extraction failure: only that analyzer fails
    failing = _ExtractionFailingMean("att1")
    ctx = d.AnalysisRunner.onData(pt).addAnalyzers([failing, d.Minimum("att1"), d.Maximum("att1")]).run()
    assert isinstance(ctx.metric(failing).value, Failure)
    assert "-test-mean-failing-" in str(ctx.metric(failing).value.exception)
    assert ctx.metric(d.Minimum("att1")).value.get() == 1.0
    assert ctx.metric(d.Maximum("att1")).value.get() == 6.0
    # aggregation failure: every scan-shareable analyzer of the run fails with that error
    agg = _AggregationFailingMean("att1")
    ctx = d.AnalysisRunner.onData(pt).addAnalyzers([agg, d.Minimum("att1"), d.Maximum("att1")]).run()
    for a in (agg, d.Minimum("att1"), d.Maximum("att1")):
        assert isinstance(ctx.metric(a).value, Failure), a
        assert "-test-agg-failing-" in str(ctx.metric(a).value.exception), a
