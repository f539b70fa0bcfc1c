"""Spark 2.2 casts and coercions in the predicate IR (DQ_P_CAST), pinned in the LIBRARY.

The JVM encoder maps every analyzed Catalyst `Cast` node onto DQ_P_CAST, so
the cast semantics and the type rules live in libdeequ_amd.so, not in the encoder:

* CPU: `dq_diag_eval_predicate` is the host build of the device interpreter (the same source,
  `deequ_amd/csrc/dq_predeval.h`).  Every predicate here is compiled (deequ_amd.predicates, or a
  raw instruction list as the JVM encoder would emit it), evaluated by the library row by row,
  and compared with the oracle's independent SQL evaluator (oracle/pyoracle.py `eval_predicate`,
  `spark_cast`).  Blobs Spark would evaluate in a way the IR cannot are DQ_ERR_UNSUPPORTED at plan
  time (`dq_op_supported`), never DQ_ERR_INVALID, so the analyzer is routed to Spark.
* GPU: the same predicates as Compliance analyzers through a plan, against the oracle.

Reference call sites: Compliance.scala:49 (`expr(predicate)`), Check.scala:594-604 (`satisfies`),
Analyzer.scala:409-432 (`where`).
"""
import ctypes
import math

import numpy as np
import pytest

import deequ_amd as d
from deequ_amd import _lib as L
from deequ_amd.engine import _fill_pred, _pred_array
from deequ_amd.predicates import (PredicateSyntaxError, UnsupportedPredicate, compile_predicate,
                                  int_to_float32)
from deequ_amd.table import Column, Table
from oracle import pyoracle as O

T = L.TYPE_CODES
I31 = 2 ** 31
I63 = 2 ** 63

LONGS = [0, 3, 4, -3, -4, I31 - 1, I31, I31 + 3, I31 + 4, -I31, -I31 - 1, 2 ** 32 + 4, -(2 ** 32) + 5,
         I63 - 1, -I63, 2 ** 40 + 7, 16777217, 16777219, 2 ** 53 + 1, 2 ** 60 + 2 ** 36 + 1, 70000, -70000,
         130, -130, 255, 256, 32767, 32768, 65539, None, 2 ** 24 + 3]
DOUBLES = [0.0, -0.0, 3.7, -3.7, 4.0, 3.0, 2.5, float("nan"), float("inf"), float("-inf"), 2147483647.5,
           2147483648.0, -2147483648.9, -2147483649.0, 9.3e18, -9.3e18, 1e300, 70000.9, -70000.9, 130.5,
           -130.5, 16777217.0, 3.4028235677973366e38, 3.4028235e38 * 1.0000001, 1e-50, None, 0.1,
           33000.2, 65539.0, 2.0 ** 24 + 1, 1.00000005960464477539]
FLOATS = [float(np.float32(x)) for x in (16777216.0, 16777218.0, 3.0, 4.0, -3.5, 0.0, 1e30, 2.0 ** 31,
                                          float("nan"), 0.1, 65539.0, 2 ** 24 + 4)] + [None]
BOOLS = [True, False, None]
INTS = [0, 3, 4, -3, 127, 128, -129, 2147483647, -2147483648, 100, 101, 16777217, 16777219, None]


def _table(n=96, seed=5):
    rng = np.random.default_rng(seed)
    pick = lambda xs: [xs[int(k)] for k in rng.integers(0, len(xs), n)]  # noqa: E731
    data = {"l": ("int64", pick(LONGS)), "d": ("float64", pick(DOUBLES)), "g": ("float32", pick(FLOATS)),
            "i": ("int32", pick(INTS)), "b": ("bool", pick(BOOLS)),
            "s": ("string", pick(["3", " 4 ", "x", None, "2.5"]))}
    # make every LONGS / DOUBLES value appear at least once
    data["l"][1][:len(LONGS)] = LONGS
    data["d"][1][:len(DOUBLES)] = DOUBLES
    return data


def _otable(data):
    return {k: O.OColumn(t, list(v)) for k, (t, v) in data.items()}


def _eval_lib(code, pool, table: Table, names):
    """The library's host interpreter over `table`: list of True / False / None per row."""
    from deequ_amd.table import dq_columns
    packed = _pred_array(code if pool is None else _Prog(code, pool))
    p = L.DqPredicate()
    _fill_pred(p, packed)
    cols = dq_columns(table, names)
    out = np.zeros(table.num_rows, dtype=np.uint8)
    st = L.lib().dq_diag_eval_predicate(ctypes.byref(p), cols, len(names), table.num_rows,
                                        out.ctypes.data_as(ctypes.c_void_p))
    if st != L.DQ_OK:
        return st, L.lib().dq_last_error().decode()
    return [None if v == 2 else bool(v) for v in out.tolist()]


class _Prog(list):
    def __init__(self, code, pool):
        super().__init__(code)
        self.pool = pool


CAST_PREDICATES = [
    # integral narrowing keeps the low bits (Scala .toInt / .toShort / .toByte)
    "cast(l as int) > 3", "CAST(l AS INT) <= -4", "cast(l as smallint) = 4", "cast(l as tinyint) < 0",
    "cast(l as bigint) = 4", "cast(i as tinyint) > 100", "cast(l as int) IN (3, 4, -1)",
    # fractional -> integral: Java d2i / d2l (NaN -> 0, saturating, toward zero)
    "cast(d as int) > 3", "cast(d as int) = 2147483647", "cast(d as int) = -2147483648",
    "cast(d as bigint) = 9223372036854775807", "cast(d as bigint) < -9000000000000000000",
    "cast(d as int) = 0", "cast(d as smallint) = 4464", "cast(d as tinyint) = -126",
    "cast(g as int) = 3", "cast(g as bigint) > 2147483647",
    # -> float: l2f rounds the integer itself; double -> float rounds to nearest even
    "cast(l as float) = 16777216", "cast(l as float) > cast(d as float)", "cast(d as float) = 0.1",
    "cast(d as float) = 3.4028235e38", "cast(d as float) > 3.4e38", "cast(l as float) = g",
    # FloatType coercion of an integral operand (Spark casts the int side to float)
    "g = 16777217", "g > 16777217", "g = l", "g < i", "g = cast(d as int)", "COALESCE(g, 16777217) = 16777216",
    "COALESCE(g, l) >= 16777216", "g = 16777217.0",
    # -> double, -> boolean, boolean -> numeric
    "cast(l as double) = 9007199254740992", "cast(i as double) < d", "cast(b as int) = 1",
    "cast(b as double) > 0.5", "cast(d as boolean)", "NOT cast(l as boolean)", "b = 1", "cast(0.5 as boolean)",
    "cast(3.7 as int) = 3", "cast(-3.7 as int) = l", "cast(2.5 as double) < d", "cast(s as double) > 2",
    "cast(NULL as int) IS NULL", "cast(l as int) IS NOT NULL AND cast(d as int) > -5",
    "cast(l as int) BETWEEN -5 AND 5", "cast(cast(l as int) as tinyint) = 4",
]


@pytest.mark.parametrize("text", CAST_PREDICATES)
def test_cast_predicates_library_matches_oracle(text):
    data = _table()
    table = Table.from_pydict(data)
    names = list(data)
    schema = {nm: (k, data[nm][0]) for k, nm in enumerate(names)}
    prog = compile_predicate(text, schema)
    got = _eval_lib(prog.code, prog.pool, table, names)
    want = O.eval_predicate(text, _otable(data))
    assert got == want, [(r, data["l"][1][r], data["d"][1][r], g, w) for r, (g, w) in enumerate(zip(got, want))
                         if g != w][:8]


def _raw(code, types, pool=b""):
    """dq_op_supported on a Compliance op built from a raw instruction list (the JVM route)."""
    op = L.DqOp()
    op.kind = L.DQ_OP_COMPLIANCE
    op.column = -1
    op.column2 = -1
    packed = _pred_array(_Prog(code, pool))
    _fill_pred(op.predicate, packed)
    ts = (ctypes.c_int32 * len(types))(*[T[t] for t in types])
    st = L.lib().dq_op_supported(ctypes.byref(op), ts, len(types))
    return st, L.lib().dq_last_error().decode()


COL, LI, LF, NUL, COAL, LS = L.DQ_P_COLUMN, L.DQ_P_LIT_INT, L.DQ_P_LIT_FLOAT, L.DQ_P_LIT_NULL, L.DQ_P_COALESCE, L.DQ_P_LIT_STRING
CAST, GT, EQ = L.DQ_P_CAST, L.DQ_P_GT, L.DQ_P_EQ
AS_I, AS_F = L.DQ_CMP_AS_INT64, L.DQ_CMP_AS_FLOAT64


def _i(op, arg=0, i64=0, f64=0.0):
    return (op, arg, i64, f64)


def test_verdict_blobs_evaluate_exactly():
    """The three encodings the JVM side emits for `cast(l as int) > 3` (|l| > 2^31),
    `f = 16777217` on a FloatType column, and `cast(d as int) > 3` on a double column: each
    evaluates exactly as Spark does (checked against the oracle row by row)."""
    data = _table(seed=11)
    table = Table.from_pydict(data)
    names = list(data)
    ot = _otable(data)
    blobs = {
        "cast(l as int) > 3": [_i(COL, 0), _i(CAST, T["int32"]), _i(LI, 0, 3), _i(GT, AS_I)],
        # Catalyst: EqualTo(g, Cast(Literal(16777217), FloatType))
        "g = 16777217": [_i(COL, 2), _i(LI, 0, 16777217), _i(CAST, T["float32"]), _i(EQ, AS_F)],
        "cast(d as int) > 3": [_i(COL, 1), _i(CAST, T["int32"]), _i(LI, 0, 3), _i(GT, AS_I)],
    }
    for text, code in blobs.items():
        assert _raw(code, [data[n][0] for n in names])[0] == L.DQ_OK
        got = _eval_lib(code, b"", table, names)
        assert got == O.eval_predicate(text, ot), text
    # the wrap is really exercised: some rows differ between cast(l as int) > 3 and l > 3
    wrapped = O.eval_predicate("cast(l as int) > 3", ot)
    plain = O.eval_predicate("l > 3", ot)
    assert wrapped != plain
    # and the float rounding: 16777216f == 16777217 in FloatType, not in double
    assert O.eval_predicate("g = 16777217", ot) != O.eval_predicate("cast(g as double) = 16777217e0", ot)


@pytest.mark.parametrize("case", [
    ("int64 compare of a double", [_i(COL, 1), _i(LI, 0, 3), _i(GT, AS_I)], ["int64", "float64"]),
    ("int64 compare of a cast to float", [_i(COL, 0), _i(CAST, T["float32"]), _i(LI, 0, 3), _i(GT, AS_I)],
     ["int64", "float64"]),
    ("float32 column vs raw int literal", [_i(COL, 0), _i(LI, 0, 16777217), _i(EQ, AS_F)], ["float32"]),
    ("float32 column vs int column", [_i(COL, 0), _i(COL, 1), _i(EQ, AS_F)], ["float32", "int64"]),
    ("COALESCE(float32, int)", [_i(COL, 0), _i(COL, 1), _i(COAL), _i(LF, 0, 0, 1.0), _i(GT, AS_F)],
     ["float32", "int64"]),
    ("cast of a string to int", [_i(COL, 0), _i(CAST, T["int32"]), _i(LI, 0, 3), _i(GT, AS_I)], ["string"]),
    ("cast to string", [_i(COL, 0), _i(CAST, T["string"]), _i(LS, 1, 0), _i(EQ, AS_I)], ["int64"]),
    ("cast to an unknown type", [_i(COL, 0), _i(CAST, 99), _i(LI, 0, 3), _i(GT, AS_I)], ["int64"]),
    ("string vs number", [_i(COL, 0), _i(LI, 0, 3), _i(GT, AS_F)], ["string"]),
])
def test_inexact_type_combinations_are_unsupported(case):
    """Blobs Spark would evaluate differently (or that the IR cannot evaluate) are
    DQ_ERR_UNSUPPORTED at plan time -- the shim then leaves the analyzer on Spark."""
    what, code, types = case
    st, msg = _raw(code, types, pool=b"x")
    assert st == L.DQ_ERR_UNSUPPORTED, (what, st, msg)


def test_malformed_programs_stay_invalid():
    assert _raw([_i(COL, 5), _i(LI, 0, 3), _i(GT, AS_I)], ["int64"])[0] == L.DQ_ERR_INVALID
    assert _raw([_i(CAST, T["int32"])], ["int64"])[0] == L.DQ_ERR_INVALID
    assert _raw([_i(COL, 0), _i(LI, 0, 3), _i(GT, 7)], ["int64"])[0] == L.DQ_ERR_INVALID


def test_cast_of_null_and_literals():
    """A cast keeps NULL; casts of literals are evaluated by the library too."""
    data = {"l": ("int64", [1, None, 3])}
    table = Table.from_pydict(data)
    code = [_i(NUL), _i(CAST, T["int32"]), _i(L.DQ_P_IS_NULL)]
    assert _eval_lib(code, b"", table, ["l"]) == [True, True, True]
    code = [_i(LF, 0, 0, -3.9), _i(CAST, T["int8"]), _i(COL, 0), _i(EQ, AS_I)]
    assert _eval_lib(code, b"", table, ["l"]) == [False, None, False]
    code = [_i(LF, 0, 0, 3.9), _i(CAST, T["int64"]), _i(COL, 0), _i(EQ, AS_I)]
    assert _eval_lib(code, b"", table, ["l"]) == [False, None, True]


def test_int_to_float32_is_exact():
    """Java l2f rounds the integer itself: no double rounding through fp64."""
    x = 2 ** 53 + 2 ** 29 + 1  # fp64 rounds it down to 2^53 + 2^29, a tie float would round down
    assert int_to_float32(x) == float(2 ** 53 + 2 ** 30)
    assert int_to_float32(x) == O.int_to_f32(x)
    rng = np.random.default_rng(3)
    for v in [int(v) for v in rng.integers(-2 ** 63, 2 ** 63 - 1, 2000, dtype=np.int64)] + [16777217, -16777219]:
        f = int_to_float32(v)
        assert f == O.int_to_f32(v)
        assert abs(f - v) <= 2.0 ** (max(abs(v).bit_length() - 24, 0) - 1) + 0  # within half an ulp


def test_front_end_rejects_arithmetic_and_resolves_names_case_insensitively():
    schema = {"a": (0, "int64"), "Mixed": (1, "float64")}
    for text in ("a + 1 > 2", "a > 1 + 2", "(a - 1) > 2", "a * 2 > 1", "a / 2 > 1", "a % 2 = 1"):
        with pytest.raises(UnsupportedPredicate):
            compile_predicate(text, schema)
    with pytest.raises(PredicateSyntaxError):
        compile_predicate("a > ", schema)
    assert list(compile_predicate("A > 2", schema)) == list(compile_predicate("a > 2", schema))
    assert list(compile_predicate("mixed > 2 AND MIXED < 3", schema)) == \
        list(compile_predicate("Mixed > 2 AND Mixed < 3", schema))
    with pytest.raises(KeyError):
        compile_predicate("b > 2", schema)
    with pytest.raises(ValueError):  # ambiguous: two columns equal but for case
        compile_predicate("x > 1", {"x": (0, "int64"), "X": (1, "int64")})
    for text in ("cast(s as int) > 1", "cast(a as decimal(10,2)) > 1", "cast(a as string) = '1'",
                 "cast(a as date) IS NULL"):
        with pytest.raises(UnsupportedPredicate):
            compile_predicate(text, {"a": (0, "int64"), "s": (1, "string")})


def test_compliance_precondition_is_case_insensitive():
    an = d.Compliance("c", "A >= 0")
    for check in an.preconditions():
        check({"a": "int64"})
    with pytest.raises(Exception):
        for check in d.Compliance("c", "zz >= 0").preconditions():
            check({"a": "int64"})


@pytest.mark.gpu
def test_cast_predicates_on_gpu(gpu):
    """Every CAST_PREDICATES text as a Compliance analyzer (plus a `where` on one) through a GPU
    plan: (numMatches, count) equal to the oracle's evaluation of the same rows."""
    from deequ_amd.engine import Plan, op_spec_for
    data = _table(n=4096, seed=21)
    table = Table.from_pydict(data)
    schema = {k: t for k, (t, _) in data.items()}
    ot = _otable(data)
    analyzers = [d.Compliance("c%d" % k, text) for k, text in enumerate(CAST_PREDICATES)]
    analyzers.append(d.Compliance("w", "cast(l as int) > 3", "cast(d as int) > 0"))
    plan = Plan([op_spec_for(a, schema) for a in analyzers], schema)
    try:
        plan.consume(table)
        states = plan.finish()
    finally:
        plan.close()
    for a, st in zip(analyzers, states):
        got = O.eval_predicate(a.predicate, ot)
        sel = O.eval_predicate(a.where, ot) if a.where else [True] * len(got)
        n_match = sum(1 for g, s in zip(got, sel) if s and g)
        assert (st.numMatches, st.count) == (n_match, sum(1 for s in sel if s)), a.predicate
