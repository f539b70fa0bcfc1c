"""CPU tests of the C-ABI library: it loads, exports every symbol include/deequ_amd.h
declares, and its host-side State algebra / HLL estimate / XXH64 agree with the oracle.
Also checks the SQL -> IR predicate compiler against the oracle's independent evaluator
(through a test-only IR interpreter).  No GPU compute is invoked here."""
import ctypes
import math
import os
import random
import re

import numpy as np
import pytest
import xxhash

import pyoracle as O
from helpers import known_answers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    from deequ_amd import _lib
    header = open(os.path.join(ROOT, "include", "deequ_amd.h")).read()
    declared = set(re.findall(r"^(?:const\s+)?[a-z_0-9]+\s*\*?\s*(dq_[a-z0-9_]+)\s*\(", header, re.M))
    assert len(declared) >= 19
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    # the ctypes signature table covers the whole header too
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    assert _lib.lib().dq_abi_version() == 4


def test_library_reports_no_device_without_gpu_cleanly():
    from deequ_amd import _lib
    assert _lib.device_count() >= 0


def test_xxh64_host_matches_reference():
    from deequ_amd import _lib
    rnd = random.Random(1)
    for n in list(range(0, 70)) + [255, 1024]:
        b = bytes(rnd.getrandbits(8) for _ in range(n))
        assert _lib.lib().dq_xxh64(b, n, 42) == xxhash.xxh64_intdigest(b, 42)


def _rand_regs(rnd, hi):
    return [rnd.randint(0, hi) if rnd.random() < 0.7 else 0 for _ in range(512)]


def test_hll_count_and_merge_match_oracle():
    import deequ_amd as d
    rnd = random.Random(5)
    for hi in (0, 1, 3, 8, 20, 40, 63):
        for _ in range(20):
            words = O.hll_pack(_rand_regs(rnd, hi))
            assert d.ApproxCountDistinctState(words).metricValue() == O.hll_count(words)
    for n in (1, 10, 100, 1000, 5000, 20000, 300000):
        vals = [rnd.getrandbits(64) - 2 ** 63 for _ in range(min(n, 20000))]
        words = O.hll_pack(O.hll_registers(vals, "int64"))
        assert d.ApproxCountDistinctState(words).metricValue() == O.hll_count(words)
    a, b = O.hll_pack(_rand_regs(rnd, 30)), O.hll_pack(_rand_regs(rnd, 30))
    merged = d.ApproxCountDistinctState(a).sum(d.ApproxCountDistinctState(b))
    assert list(merged.words) == O.hll_merge(a, b)
    st = d.ApproxCountDistinctState(a)
    assert st.to_bytes() == O.hll_words_to_bytes(a)
    assert d.ApproxCountDistinctState.from_bytes(st.to_bytes()) == st


def test_state_algebra_matches_oracle():
    import deequ_amd as d
    rnd = random.Random(9)
    for _ in range(200):
        a, b = rnd.randint(0, 10 ** 12), rnd.randint(0, 10 ** 12)
        c, e = rnd.randint(a, 2 * 10 ** 12), rnd.randint(b, 2 * 10 ** 12)
        assert d.NumMatches(a).sum(d.NumMatches(b)).numMatches == O.NumMatches(a).sum(O.NumMatches(b)).num_matches
        m = d.NumMatchesAndCount(a, c).sum(d.NumMatchesAndCount(b, e))
        om = O.NumMatchesAndCount(a, c).sum(O.NumMatchesAndCount(b, e))
        assert (m.numMatches, m.count) == (om.num_matches, om.count)
        assert m.metricValue() == om.metric_value()
        x, y = rnd.uniform(-1e9, 1e9), rnd.uniform(-1e9, 1e9)
        assert d.SumState(x).sum(d.SumState(y)).metricValue() == O.SumState(x).sum(O.SumState(y)).metric_value()
        assert d.MeanState(x, a + 1).sum(d.MeanState(y, b)).metricValue() == \
            O.MeanState(x, a + 1).sum(O.MeanState(y, b)).metric_value()
        n1, n2 = float(rnd.randint(1, 10 ** 6)), float(rnd.randint(1, 10 ** 6))
        s1 = (n1, rnd.uniform(-1e3, 1e3), rnd.uniform(0, 1e9))
        s2 = (n2, rnd.uniform(-1e3, 1e3), rnd.uniform(0, 1e9))
        ds = d.StandardDeviationState(*s1).sum(d.StandardDeviationState(*s2))
        os_ = O.StandardDeviationState(*s1).sum(O.StandardDeviationState(*s2))
        assert (ds.n, ds.avg, ds.m2) == (os_.n, os_.avg, os_.m2)  # bit-exact State.sum
        assert ds.metricValue() == os_.metric_value()
        assert d.MinState(x).sum(d.MinState(y)).minValue == min(x, y)
        assert d.MaxState(x).sum(d.MaxState(y)).maxValue == max(x, y)
    # Java Math.min/max: NaN propagates
    assert math.isnan(d.MinState(1.0).sum(d.MinState(float("nan"))).minValue)
    assert math.isnan(d.MaxState(float("nan")).sum(d.MaxState(1.0)).maxValue)
    assert d.NumMatchesAndCount(0, 0).metricValue() != d.NumMatchesAndCount(0, 0).metricValue()  # NaN
    with pytest.raises(ValueError):
        d.StandardDeviationState(0.0, 0.0, 0.0)


def test_correlation_state_algebra_matches_oracle():
    """CorrelationState.sum / metricValue through dq_state_merge / dq_state_metric, bit-exact
    with the oracle's restatement of Correlation.scala:37-56."""
    import deequ_amd as d
    rnd = random.Random(10)
    for _ in range(200):
        a = (float(rnd.randint(1, 10 ** 6)),) + tuple(rnd.uniform(-1e3, 1e3) for _ in range(3)) + \
            (rnd.uniform(0, 1e9), rnd.uniform(0, 1e9))
        b = (float(rnd.randint(1, 10 ** 6)),) + tuple(rnd.uniform(-1e3, 1e3) for _ in range(3)) + \
            (rnd.uniform(0, 1e9), rnd.uniform(0, 1e9))
        got = d.CorrelationState(*a).sum(d.CorrelationState(*b))
        want = O.CorrelationState(*a).sum(O.CorrelationState(*b))
        assert got.fields() == (want.n, want.xAvg, want.yAvg, want.ck, want.xMk, want.yMk)
        assert got.metricValue() == want.metric_value()
    assert math.isnan(d.CorrelationState(3.0, 2.0, 0.0, 0.0, 2.0, 0.0).metricValue())  # 0 / 0
    with pytest.raises(ValueError):
        d.CorrelationState(0.0, 0.0, 0.0, 0.0, 0.0, 0.0)


def test_new_ops_are_supported_and_typed():
    """MinLength/MaxLength need a utf8 column, Correlation two numeric ones; an empty string
    literal in a `where` filter (AnalyzerTests.scala:515) is a valid predicate."""
    import ctypes
    from deequ_amd import _lib as L
    from deequ_amd.engine import op_spec_for, op_supported
    from deequ_amd.metrics import MetricCalculationException  # noqa: F401
    import deequ_amd as d
    schema = {"s": "string", "i": "int64", "f": "float64"}
    for a in (d.MinLength("s"), d.MaxLength("s", "s != ''"), d.Correlation("i", "f", "s != 'x'")):
        op_supported(op_spec_for(a, schema), schema)
    for a in (d.MinLength("i"), d.Correlation("s", "f")):
        with pytest.raises(L.DeequAmdError):
            op_supported(op_spec_for(a, schema), schema)
    assert ctypes.sizeof(L.DqOp) == 4 * 4 + 2 * ctypes.sizeof(L.DqPredicate)


def test_merge_option_semantics():
    import deequ_amd as d
    from deequ_amd.states import merge
    assert merge(None, None) is None
    assert merge(d.NumMatches(3), None) == d.NumMatches(3)
    assert merge(None, d.NumMatches(4)) == d.NumMatches(4)
    assert merge(d.NumMatches(3), d.NumMatches(4), None, d.NumMatches(1)) == d.NumMatches(8)


# ----------------------------------------------------------------------------- predicates
def _interp(code, pool, table, names, nrows):
    """Test-only interpreter of the product IR (mirrors dq_pred.hip's semantics)."""
    from deequ_amd import _lib as L
    out = []
    for r in range(nrows):
        st = []
        for op, arg, i64, f64 in code:
            if op == L.DQ_P_COLUMN:
                col = table[names[arg]]
                v = col.values[r]
                kind = "s" if col.dtype == "string" else ("f" if col.dtype.startswith("float") else "i")
                if col.dtype == "bool" and v is not None:
                    v = int(v)
                st.append((kind, v))
            elif op == L.DQ_P_LIT_INT:
                st.append(("i", i64))
            elif op == L.DQ_P_LIT_FLOAT:
                st.append(("f", f64))
            elif op == L.DQ_P_LIT_NULL:
                st.append(("i", None))
            elif op == L.DQ_P_LIT_STRING:
                st.append(("s", pool[i64:i64 + arg].decode("utf-8")))
            elif op in (L.DQ_P_TRUE, L.DQ_P_FALSE):
                st.append(("b", op == L.DQ_P_TRUE))
            elif op == L.DQ_P_CAST_DOUBLE:  # Cast(-> DoubleType): Java parseDouble of a string
                a = st.pop()
                v = a[1] if a[1] is None else (O.java_parse_double(a[1]) if a[0] == "s" else float(a[1]))
                st.append(("f", v))
            elif op == L.DQ_P_COALESCE:
                b, a = st.pop(), st.pop()
                r_ = a if a[1] is not None else b
                if "f" in (a[0], b[0]) and r_[1] is not None:
                    r_ = ("f", float(r_[1]))
                st.append(r_)
            elif L.DQ_P_EQ <= op <= L.DQ_P_EQ_NULLSAFE:
                b, a = st.pop(), st.pop()
                if a[1] is None or b[1] is None:
                    st.append(("b", (a[1] is None and b[1] is None)) if op == L.DQ_P_EQ_NULLSAFE else ("b", None))
                    continue
                x, y = a[1], b[1]
                if a[0] == "s":
                    x, y = x.encode(), y.encode()
                elif arg == L.DQ_CMP_AS_FLOAT64:
                    x, y = float(x), float(y)
                if isinstance(x, float) and (x != x or y != y):
                    ordv = (x != x) - (y != y)
                else:
                    ordv = (x > y) - (x < y)
                res = {L.DQ_P_EQ: ordv == 0, L.DQ_P_NE: ordv != 0, L.DQ_P_LT: ordv < 0,
                       L.DQ_P_LE: ordv <= 0, L.DQ_P_GT: ordv > 0, L.DQ_P_GE: ordv >= 0,
                       L.DQ_P_EQ_NULLSAFE: ordv == 0}[op]
                st.append(("b", res))
            elif op in (L.DQ_P_IS_NULL, L.DQ_P_IS_NOT_NULL):
                a = st.pop()
                st.append(("b", (a[1] is None) == (op == L.DQ_P_IS_NULL)))
            elif op == L.DQ_P_NOT:
                a = st.pop()
                st.append(("b", None if a[1] is None else not a[1]))
            elif op in (L.DQ_P_AND, L.DQ_P_OR):
                b, a = st.pop()[1], st.pop()[1]
                if op == L.DQ_P_AND:
                    v = False if (a is False or b is False) else (None if (a is None or b is None) else True)
                else:
                    v = True if (a is True or b is True) else (None if (a is None or b is None) else False)
                st.append(("b", v))
        top = st[-1][1]
        out.append(None if top is None else bool(top))
    return out


PREDICATES = [
    "i >= 0", "i > 3.5", "i >= 3.5", "i < 3.5", "i <= 3.5", "i = 3.5", "i != 3.5", "i <=> 3.5",
    "i > 3", "f > 5e2", "f >= 0", "f < i", "i = f", "COALESCE(i, 0.0) >= 0", "COALESCE(f, 0) < 1",
    "i IN (1, 2, 3)", "i NOT IN (1, 2)", "i BETWEEN -2 AND 4", "NOT (i < 3) OR f IS NULL",
    "i IS NOT NULL AND f IS NULL", "s = 'k1'", "s IN ('k1', 'k2')", "s != 'k0'", "s > 'k1'",
    "s IS NULL", "b = true", "b", "NOT b", "i > -3", "i < 2 AND (s = 'k1' OR f > 1000.5)",
    "f > 1000.5", "i <=> NULL", "i = NULL", "TRUE", "FALSE", "i >= 3 OR i < 3",
    # Spark 2.2 PromoteStrings: string vs number compares Cast(string AS DOUBLE) in double
    "sn > 3", "sn <= 2.5", "3 < sn", "sn = f", "sn != -1", "i > '2'",
    # FloatType vs an int literal compares in FloatType (rounded once on the host)
    "g = 16777217", "g > 16777217",
]


@pytest.mark.parametrize("text", PREDICATES)
def test_predicate_compiler_matches_oracle_semantics(text):
    from deequ_amd.predicates import compile_predicate
    rng = np.random.default_rng(abs(hash(text)) % 2 ** 32)
    n = 60
    iv = [None if rng.random() < 0.2 else int(x) for x in rng.integers(-5, 8, n)]
    fv = [None if rng.random() < 0.2 else float(x) for x in rng.normal(1000, 3, n)]
    fv[0] = float("nan")
    sv = [None if rng.random() < 0.2 else "k%d" % x for x in rng.integers(0, 4, n)]
    bv = [None if rng.random() < 0.2 else bool(x) for x in rng.integers(0, 2, n)]
    texts = ["1", " 2 ", "2.5", "-1", "3e0", "x", "", "NaN", "4d", "1000.0"]
    snv = [None if rng.random() < 0.1 else texts[k] for k in rng.integers(0, len(texts), n)]
    gv = [float(x) for x in rng.choice([16777216.0, 16777218.0, 3.0, 16777220.0], n)]
    table = {"i": O.OColumn("int64", iv), "f": O.OColumn("float64", fv),
             "s": O.OColumn("string", sv), "b": O.OColumn("bool", bv),
             "sn": O.OColumn("string", snv), "g": O.OColumn("float32", gv)}
    names = ["i", "f", "s", "b", "sn", "g"]
    schema = {nm: (k, table[nm].dtype) for k, nm in enumerate(names)}
    prog = compile_predicate(text, schema)
    assert _interp(prog.code, prog.pool, table, names, n) == O.eval_predicate(text, table)


@pytest.mark.parametrize("text", ["i + 1 > 2", "upper(s) = 'A'", "s IN (1, 2)", "i IN ('1', 2)",
                                  "b > '1'", "cast(s as int) > 1"])
def test_unsupported_predicates_are_rejected(text):
    from deequ_amd.predicates import UnsupportedPredicate, compile_predicate
    schema = {"i": (0, "int64"), "s": (1, "string"), "b": (2, "bool"), "g": (3, "float32")}
    with pytest.raises((UnsupportedPredicate, ValueError)):
        compile_predicate(text, schema)


def test_known_answer_predicates_compile():
    from deequ_amd.predicates import compile_predicate
    ka = known_answers()
    for case in ka["cases"] + ka["merge_cases"]:
        table = ka["tables"][case.get("table") or case["table_a"]]
        schema = {nm: (k, spec[0]) for k, (nm, spec) in enumerate(table.items())}
        args = case["args"]
        texts = []
        if case["analyzer"] in ("Histogram", "MutualInformation"):
            texts = []
        elif case["analyzer"] == "Compliance":
            texts = args[1:]
        elif case["analyzer"] == "Correlation":
            texts = args[2:]
        elif len(args) > 1 or (case["analyzer"] == "Size" and args):
            texts = args[-1:]
        for t in texts:
            compile_predicate(t, schema)


def test_library_exports_every_diag_symbol():
    from deequ_amd import _lib
    header = open(os.path.join(ROOT, "include", "deequ_amd_diag.h")).read()
    declared = set(re.findall(r"^(?:const\s+)?[a-z_0-9]+\s*\*?\s*(dq_[a-z0-9_]+)\s*\(", header, re.M))
    assert declared == set(_lib.DIAG_SIGNATURES), declared ^ set(_lib.DIAG_SIGNATURES)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    assert all(hasattr(lib, s) for s in declared)
