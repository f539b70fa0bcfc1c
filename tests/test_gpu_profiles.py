"""DataType, the Spark string casts and the ColumnProfiler on the GPU.

* DataType (DataType.scala:152-183): the reference's known answers (AnalyzerTests.scala:294-420,
  NullHandlingTests.scala:72) and bit-exact parity with the oracle's regex restatement on
  randomized strings and numeric columns (including the Double.toString plain/scientific cut).
* dq_cast_utf8: Spark 2.2.2 Cast(StringType -> LongType | DoubleType) against the restatements
  below (UTF8String.toLong; java.lang.Double.parseDouble for the forms the exact path covers).
* ColumnProfiler (ColumnProfiler.scala:91-208): every known answer of ColumnProfilerTest.scala.
"""
import math
import struct

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd.profiles import ColumnProfiler, ColumnProfilerRunner, NumericColumnProfile, cast_string_column
from helpers import known_answers, oracle_table, product_table

pytestmark = pytest.mark.gpu
KA = known_answers()


@pytest.mark.parametrize("case", KA["datatype_cases"], ids=[c["id"] for c in KA["datatype_cases"]])
def test_datatype_known_answers(gpu, case):
    table = product_table(KA["tables"][case["table"]])
    a = d.DataType(case["column"])
    state = a.computeStateFrom(table)
    assert list(state.counts()) == case["expected"], case["source"]
    m = a.calculate(table)
    total = sum(case["expected"])
    for name, c in zip(d.DataTypeInstances.NAMES, case["expected"]):
        assert m.value.get()[name] == d.DistributionValue(c, c / total), (case["source"], name)


def test_datatype_fused_with_other_analyzers(gpu):
    spec = KA["tables"]["dfBoolNull"]
    table = product_table(spec)
    analyzers = [d.DataType("att1"), d.Completeness("att1"), d.ApproxCountDistinct("att1"), d.Size(),
                 d.DataType("item"), d.DataType("att1", "item != '4'")]
    ctx = d.AnalysisRunner.onData(table).addAnalyzers(analyzers).run()
    assert ctx.metric(analyzers[0]).value.get()["Boolean"].absolute == 2
    assert ctx.metric(analyzers[4]).value.get()["Integral"].absolute == 4
    # where-filtered rows are NULL inputs: "2.0" (item 4) becomes Unknown
    dist = ctx.metric(analyzers[5]).value.get()
    assert (dist["Unknown"].absolute, dist["Fractional"].absolute) == (2, 0)


_ALPHABET = ["0", "1", "7", "9", ".", "-", "+", " ", "a", "e", "E", "true", "false", "\n", "é", "x"]


def _random_strings(rng, n):
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.08:
            out.append(None)
        elif r < 0.14:
            out.append(["true", "false", "True", "", ".", "-", "+", " ", "-.", "+ .5", "- 12"][rng.integers(0, 11)])
        else:
            k = int(rng.integers(0, 9))
            out.append("".join(_ALPHABET[int(rng.integers(0, len(_ALPHABET)))] if rng.random() < 0.25
                               else str(int(rng.integers(0, 10))) for _ in range(k)))
    return out


@pytest.mark.parametrize("n", [1, 63, 2049, 20000])
def test_datatype_random_strings_match_oracle(gpu, n):
    rng = np.random.default_rng(n)
    spec = {"s": ["string", _random_strings(rng, n)], "w": ["int32", [int(x) for x in rng.integers(0, 3, n)]]}
    table, ot = product_table(spec), oracle_table(spec)
    for where in (None, "w > 0"):
        got = d.DataType("s", where).computeStateFrom(table)
        assert got.counts() == O.datatype_state(ot, "s", where), where


def test_datatype_numeric_looking_strings_match_oracle(gpu):
    """Digit-heavy strings of 0..30 bytes: the word-at-a-time classifier (<= 24 bytes) and the
    byte DFA (longer) against the oracle's regexes, prefixes and '.' counts included."""
    rng = np.random.default_rng(29)
    toks = ["0", "5", "9", "12", "345", ".", "-", "+", " ", "e", "true", "false"]
    vals = []
    for _ in range(30000):
        s = "".join(toks[int(rng.integers(0, len(toks) if rng.random() < 0.2 else 6))]
                    for _ in range(int(rng.integers(0, 16))))
        vals.append(None if rng.random() < 0.05 else s[:int(rng.integers(0, 31))])
    spec = {"s": ["string", vals]}
    table, ot = product_table(spec), oracle_table(spec)
    assert d.DataType("s").computeStateFrom(table).counts() == O.datatype_state(ot, "s")


def test_datatype_numeric_columns_match_oracle(gpu):
    rng = np.random.default_rng(3)
    n = 5000
    f64 = [float(x) for x in rng.choice([0.0, -0.0, 1e-3, 9.999999999999998e-4, 1e7, 9999999.999999998,
                                         float("nan"), float("inf"), -float("inf"), 2.5, -123.25, 1e-5, 3e9],
                                        n)]
    f32 = [float(np.float32(x)) for x in rng.choice([0.0, 1e-3, 9.99e-4, 1e7, 9999999.0, 1.5, float("nan"),
                                                     -2.25, 1e-8], n)]
    spec = {"f64": ["float64", [None if i % 9 == 0 else v for i, v in enumerate(f64)]],
            "f32": ["float32", f32],
            "i8": ["int8", [int(x) for x in rng.integers(-128, 127, n)]],
            "i64": ["int64", [int(x) for x in rng.integers(-2 ** 62, 2 ** 62, n)]],
            "b": ["bool", [bool(x) for x in rng.integers(0, 2, n)]]}
    table, ot = product_table(spec), oracle_table(spec)
    for c in spec:
        assert d.DataType(c).computeStateFrom(table).counts() == O.datatype_state(ot, c), c


# ---- string casts: restatements of Spark 2.2.2's two parsers (test-local)
def _spark_to_long(s):
    """UTF8String.toLong (Spark 2.2): sign, digits, optional '.' + digits (truncated)."""
    b = s.encode()
    if not b:
        return None
    neg = b[0:1] == b"-"
    i = 1 if (neg or b[0:1] == b"+") else 0
    if i and len(b) == 1:
        return None
    r = 0
    while i < len(b):
        c = b[i]
        i += 1
        if c == ord("."):
            break
        if not 48 <= c <= 57:
            return None
        r = r * 10 + (c - 48)
    if any(not 48 <= c <= 57 for c in b[i:]):
        return None
    r = -r if neg else r
    return r if -2 ** 63 <= r < 2 ** 63 else None


def _java_parse_double(s):
    """java.lang.Double.parseDouble for decimal forms (trim, sign, digits, '.', exponent,
    f/d suffix, NaN, Infinity); Python float() rounds correctly as Java does."""
    i, j = 0, len(s)
    while i < j and ord(s[i]) <= 32:  # String.trim()
        i += 1
    while j > i and ord(s[j - 1]) <= 32:
        j -= 1
    t = s[i:j]
    if not t:
        return None
    import re
    body = t[1:] if t[0] in "+-" else t
    if body in ("NaN", "Infinity"):
        return float(t.replace("Infinity", "inf").replace("NaN", "nan"))
    if not re.fullmatch(r"[+-]?([0-9]+\.?[0-9]*|\.[0-9]+)([eE][+-]?[0-9]+)?[fFdD]?", t):
        return None
    return float(t.rstrip("fFdD"))


def test_cast_to_long_matches_spark(gpu):
    vals = ["1", "-1", "+7", "", "-", "+", "12.5", "12.", "1.2.3", " 5", "5 ", "- 5", "007",
            "9223372036854775807", "9223372036854775808", "-9223372036854775808", "-9223372036854775809",
            "1e3", "abc", None, "0", "-0", "123456789012", "3.x"]
    col = d.Column.from_pylist(vals, "string")
    out = cast_string_column(col, "int64")
    got = out.to_pylist()
    assert got == [None if v is None else _spark_to_long(v) for v in vals]


def test_cast_to_long_random_digit_strings(gpu):
    """The word-at-a-time path (sign + 1..16 digits) and its fall-backs (longer, '.', junk)."""
    rng = np.random.default_rng(41)
    alpha = "0123456789" * 8 + "-+. a"
    vals = []
    for _ in range(20000):
        s = "".join(alpha[int(rng.integers(0, len(alpha)))] for _ in range(int(rng.integers(0, 21))))
        if s and rng.random() < 0.3:
            s = "-+"[int(rng.integers(0, 2))] + s[1:]
        vals.append(s)
    col = d.Column.from_pylist(vals, "string")
    got = cast_string_column(col, "int64").to_pylist()
    assert got == [_spark_to_long(v) for v in vals]


def test_cast_batch_equals_single_casts(gpu):
    """dq_cast_utf8_batch (pass 2's casts in one call, alternating over two streams) writes exactly
    what one dq_cast_utf8 per column writes: long and double targets mixed, NULLs, junk, the
    heap's last bytes, an odd column count."""
    from deequ_amd.profiles import cast_string_columns
    rng = np.random.default_rng(77)
    alpha = "0123456789" * 6 + "-+.eE a"
    cols, targets = [], []
    for k in range(5):
        vals = []
        for _ in range(3001):
            s = "".join(alpha[int(rng.integers(0, len(alpha)))] for _ in range(int(rng.integers(0, 19))))
            vals.append(None if rng.random() < 0.05 else s)
        vals[-1] = "12345"  # a string ending exactly at the heap end
        cols.append(d.Column.from_pylist(vals, "string"))
        targets.append("int64" if k % 2 == 0 else "float64")
    got = cast_string_columns(cols, targets)
    for c, t, g in zip(cols, targets, got):
        want = cast_string_column(c, t)
        assert g.dtype == t
        a, b = g.to_pylist(), want.to_pylist()
        if t == "int64":
            assert a == b
        else:
            assert [None if x is None else struct.pack("<d", x) for x in a] == \
                   [None if x is None else struct.pack("<d", x) for x in b]


def test_cast_to_double_matches_java(gpu):
    rng = np.random.default_rng(9)
    vals = ["1.5", "-0.25", ".5", "5.", ".", "-.", "", "  2.0  ", "- 1.5", "+3", "1e3", "1E-3", "2.5f", "7d",
            "NaN", "-Infinity", "Infinity", "1234567890123456", "0.1", "0", "-0.0", None, "1.0e22",
            "4.35", "123.456e-5", "abc", "1,5"]
    vals += ["%d.%0*d" % (int(rng.integers(0, 10 ** 6)), int(k), int(rng.integers(0, 10 ** int(k))))
             for k in rng.integers(1, 9, 400)]
    col = d.Column.from_pylist(vals, "string")
    got = cast_string_column(col, "float64").to_pylist()
    for v, g in zip(vals, got):
        want = None if v is None else _java_parse_double(v)
        if want is None:
            assert g is None, (v, g)
        elif math.isnan(want):
            assert g is not None and math.isnan(g), v
        else:
            assert g is not None and struct.pack("<d", g) == struct.pack("<d", want), (v, g, want)


def test_cast_to_double_full_range_on_device(gpu):
    """dq_cast_utf8 on the device, bit for bit against the oracle's Java parseDouble, for the
    inputs off Clinger's fast path (the CPU test of the host build, tests/test_numparse.py, uses
    the same generators): > 19 significant digits, exponents across the whole range, exact
    halfway points and one digit either side, 700-1200-digit strings, subnormals, overflow,
    hexadecimal literals, malformed strings.  Strings of <= 24 bytes take the word-loaded path,
    longer ones the pointer path."""
    import random
    from test_numparse import halfway_strings, random_decimal
    rng = random.Random(2024)
    vals = [random_decimal(rng) for _ in range(20000)] + halfway_strings(rng, 1500)
    vals += ["3.14159265358979323846264", "1.7976931348623158e308", "2.4703282292062328e-324", "0x1.8p1",
             "0x1.fffffffffffff8p1023", "1" + "0" * 400 + "e-400", "-0.0", "1e-400", "1e400", "x", "", None]
    for _ in range(50):
        n = rng.randint(700, 1200)
        dg = "".join(rng.choice("0123456789") for _ in range(n))
        vals.append(dg[0] + "." + dg[1:] + "e" + str(rng.randint(-330, 300)))
    col = d.Column.from_pylist(vals, "string")
    got = cast_string_column(col, "float64").to_pylist()
    bad = []
    for v, g in zip(vals, got):
        want = None if v is None else O.java_parse_double(v)
        if want is None or g is None:
            ok = want is None and g is None
        elif math.isnan(want):
            ok = math.isnan(g)
        else:
            ok = struct.pack("<d", g) == struct.pack("<d", want)
        if not ok:
            bad.append((v, g, want))
    assert not bad, bad[:5]


# ---- ColumnProfiler known answers
@pytest.mark.parametrize("case", KA["profile_cases"], ids=[c["id"] for c in KA["profile_cases"]])
def test_profiler_known_answers(gpu, case):
    table = product_table(KA["tables"][case["table"]])
    profiles = ColumnProfiler.profile(table, case["restrict"], False, case["threshold"],
                                      predefinedTypes=case["predefined"])
    p = profiles.profiles[case["column"]]
    e = case["expect"]
    if "histogram_values" in e:
        assert p.histogram is not None
        for k, (c, r) in e["histogram_values"].items():
            assert p.histogram[k] == d.DistributionValue(c, r), (case["source"], k)
        return
    assert isinstance(p, NumericColumnProfile) == (e["kind"] == "numeric"), case["source"]
    assert p.completeness == e["completeness"]
    assert p.approximateNumDistinctValues == e["approx"]
    assert p.dataType == e["dataType"]
    assert p.isDataTypeInferred == e["inferred"]
    assert p.typeCounts == e["typeCounts"]
    if e["histogram"] is None:
        assert p.histogram is None
    else:
        assert p.histogram.numberOfBins == e["histogram"]["bins"]
        assert {k: [v.absolute, v.ratio] for k, v in p.histogram.values.items()} == e["histogram"]["values"]
    if e["kind"] == "numeric":
        for f in ("mean", "maximum", "minimum", "sum", "stdDev"):
            assert getattr(p, f) == e[f], (case["source"], f)


def test_profiler_runner_and_json(gpu):
    table = product_table(KA["tables"]["dfCompleteIncomplete"])
    profiles = ColumnProfilerRunner().onData(table).withLowCardinalityHistogramThreshold(10).run()
    assert profiles.numRecords == 6
    assert set(profiles.profiles) == {"item", "att1", "att2"}
    assert profiles.profiles["att1"].histogram["a"] == d.DistributionValue(4, 4 / 6.0)
    import json
    from deequ_amd.profiles import ColumnProfiles
    j = json.loads(ColumnProfiles.toJson(list(profiles.profiles.values())))
    assert [c["column"] for c in j["columns"]] == ["item", "att1", "att2"]
    assert j["columns"][0]["dataType"] == "Integral" and j["columns"][0]["mean"] == 3.5


def test_bool_histograms_fused_scan(gpu):
    """Boolean profiler histograms come from one fused scan; they must equal the exact
    (value.toString, count) group-by of computeHistograms (ColumnProfiler.scala:564-606)."""
    from deequ_amd.profiles import compute_histograms
    rng = np.random.default_rng(3)
    n = 7000
    cols = {"b0": [None if rng.random() < 0.1 else bool(rng.integers(0, 2)) for _ in range(n)],
            "b1": [True] * n,                                   # one group
            "b2": [None if i % 3 == 0 else False for i in range(n)]}
    table = product_table({c: ["bool", v] for c, v in cols.items()})
    hist = compute_histograms(table, list(cols))
    for c, vals in cols.items():
        want = {}
        for v in vals:
            k = "NullValue" if v is None else ("true" if v else "false")
            want[k] = want.get(k, 0) + 1
        got = hist[c]
        assert got.numberOfBins == len(want), c
        assert {k: v.absolute for k, v in got.values.items()} == want, c
        assert all(v.ratio == v.absolute / n for v in got.values.values())


@pytest.mark.parametrize("n", [63, 2049, 20000])
def test_string_pass_datatype_and_hll_match_oracle(gpu, monkeypatch, n):
    """DataType + ApproxCountDistinct of the same string column in one run take the fused string
    pass (dq_string_pass_kernel: one read, word-form classifier and XXH64): DataType counts and
    HLL register words bit-exact against the oracle and against the separate kernels
    (DQ_NO_STRING_PASS=1), for strings of 0..40 bytes (word form <= 24, byte paths above, the
    >= 32-byte XXH64 path), NULLs and a `where` filter."""
    rng = np.random.default_rng(41 + n)
    vals = []
    for i in range(n):
        if rng.random() < 0.07:
            vals.append(None)
            continue
        k = int(rng.integers(0, 41))
        pool = "0123456789.-+ truefalsxyz" if rng.random() < 0.7 else "0123456789"
        vals.append("".join(pool[int(j)] for j in rng.integers(0, len(pool), k)))
    spec = {"s": ["string", vals], "w": ["int32", [int(x) for x in rng.integers(0, 3, n)]]}
    table, ot = product_table(spec), oracle_table(spec)
    states = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("DQ_NO_STRING_PASS", "0" if fused == "1" else "1")
        for where in (None, "w > 0"):
            prov = d.InMemoryStateProvider()
            an = [d.DataType("s", where), d.ApproxCountDistinct("s", where), d.Completeness("s", where)]
            d.AnalysisRunner.onData(table).addAnalyzers(an).saveStatesWith(prov).run()
            dt, hll = prov.load(an[0]), prov.load(an[1])
            assert dt.counts() == O.datatype_state(ot, "s", where), (fused, where)
            assert hll.words == O.approx_count_distinct_state(ot, "s", where).words, (fused, where)
            states[(fused, where)] = (dt.counts(), hll.words)
    assert states[("1", None)] == states[("0", None)] and states[("1", "w > 0")] == states[("0", "w > 0")]


def test_string_hll_only_matches_oracle(gpu):
    """ApproxCountDistinct of string columns alone (the HLL kernel) gives the oracle's register
    words bit for bit."""
    rng = np.random.default_rng(77)
    n = 30000
    vals = [None if rng.random() < 0.05 else
            "".join("0123456789abcdef"[int(j)] for j in rng.integers(0, 16, int(rng.integers(0, 40))))
            for _ in range(n)]
    spec = {"s": ["string", vals], "t": ["string", [v[:6] if v else v for v in vals]],
            "w": ["int32", [int(x) for x in rng.integers(0, 3, n)]]}
    table, ot = product_table(spec), oracle_table(spec)
    prov = d.InMemoryStateProvider()
    an = [d.ApproxCountDistinct("s"), d.ApproxCountDistinct("t"), d.ApproxCountDistinct("s", "w > 0")]
    d.AnalysisRunner.onData(table).addAnalyzers(an).saveStatesWith(prov).run()
    for a in an:
        assert prov.load(a).words == O.approx_count_distinct_state(ot, a.column, a.where).words, str(a)
