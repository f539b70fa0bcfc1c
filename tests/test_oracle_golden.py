"""The oracle (oracle/pyoracle.py) against the reference's own known answers and the
third-party XXH64 implementation it restates.  CPU only."""
import math
import random
import struct

import pytest
import xxhash

import pyoracle as O
from helpers import histogram_matches, known_answers, oracle_metric, oracle_state, oracle_table

KA = known_answers()


@pytest.mark.parametrize("case", KA["cases"], ids=[c["id"] for c in KA["cases"]])
def test_oracle_reproduces_reference_known_answer(case):
    table = oracle_table(KA["tables"][case["table"]])
    got = oracle_metric(oracle_state(case["analyzer"], case["args"], table), case["analyzer"], case["args"])
    if case["analyzer"] == "Histogram":
        assert histogram_matches(got, case["expected"]), (case["source"], got)
    else:
        assert got == case["expected"], (case["source"], got)


@pytest.mark.parametrize("case", KA["merge_cases"], ids=[c["id"] for c in KA["merge_cases"]])
def test_oracle_merge_equals_reference(case):
    ta = oracle_table(KA["tables"][case["table_a"]])
    tb = oracle_table(KA["tables"][case["table_b"]])
    sa = oracle_state(case["analyzer"], case["args"], ta)
    sb = oracle_state(case["analyzer"], case["args"], tb)
    name, args = case["analyzer"], case["args"]
    merged = sa.sum(sb) if isinstance(sa, O.FrequenciesAndNumRows) else O.merge_options(sa, sb)
    assert oracle_metric(merged, name, args) == case["expected"], case["source"]
    union = {k: O.OColumn(ta[k].dtype, ta[k].values + tb[k].values) for k in ta}
    assert oracle_metric(oracle_state(name, args, union), name, args) == case["expected"]


def test_oracle_xxh64_matches_reference_implementation():
    rnd = random.Random(7)
    for n in list(range(0, 80)) + [127, 128, 129, 1000]:
        data = bytes(rnd.getrandbits(8) for _ in range(n))
        for seed in (0, 42, 2 ** 63 + 5):
            assert O.xxh64(data, seed) == xxhash.xxh64_intdigest(data, seed % 2 ** 64)


def test_spark_hash_dispatch():
    # hashInt/hashLong are XXH64 over the 4/8 little-endian bytes (Spark 2.2.2 XXH64)
    assert O.spark_hash(5, "int32") == xxhash.xxh64_intdigest(struct.pack("<i", 5), 42)
    assert O.spark_hash(-5, "int64") == xxhash.xxh64_intdigest(struct.pack("<q", -5), 42)
    assert O.spark_hash(True, "bool") == O.spark_hash(1, "int32")
    assert O.spark_hash(float("nan"), "float64") == O.spark_hash(struct.unpack("<d", struct.pack("<Q", 0x7FF8000000000000))[0], "float64")
    assert O.spark_hash("é", "string") == xxhash.xxh64_intdigest("é".encode("utf-8"), 42)


def test_hll_pack_roundtrip_and_merge():
    rnd = random.Random(3)
    regs_a = [rnd.randint(0, 40) for _ in range(512)]
    regs_b = [rnd.randint(0, 40) for _ in range(512)]
    wa, wb = O.hll_pack(regs_a), O.hll_pack(regs_b)
    assert O.hll_unpack(wa) == regs_a
    assert O.hll_unpack(O.hll_merge(wa, wb)) == [max(x, y) for x, y in zip(regs_a, regs_b)]
    assert O.hll_words_from_bytes(O.hll_words_to_bytes(wa)) == wa


def test_hll_count_java_int_shift_quirk():
    # a register >= 32 wraps Java's `1 << m` (int shift masks the count to 5 bits)
    regs = [0] * 512
    regs[0] = 32  # 1 << 32 == 1 in Java
    regs[1] = 31  # 1 << 31 == Int.MinValue
    words = O.hll_pack(regs)
    z = 510.0 + 1.0 / 1 + 1.0 / -2147483648
    assert math.isclose(O.hll_count(words), float(math.floor(512 * math.log(512 / 510.0) + 0.5)))
    assert z != 0


def test_hll_relative_error_large():
    rnd = random.Random(11)
    vals = [rnd.getrandbits(63) for _ in range(100000)]
    est = O.hll_count(O.hll_pack(O.hll_registers(vals, "int64")))
    assert abs(est - 100000) / 100000 < 0.1  # RELATIVE_SD = 0.05


def test_welford_state_algebra():
    # StandardDeviationState.sum of two halves equals the single-pass state (within fp64)
    vals = [float(x) for x in range(1, 7)]
    t = {"x": O.OColumn("float64", vals)}
    a = O.stddev_state({"x": O.OColumn("float64", vals[:3])}, "x")
    b = O.stddev_state({"x": O.OColumn("float64", vals[3:])}, "x")
    assert a.sum(b).metric_value() == pytest.approx(O.stddev_state(t, "x").metric_value(), rel=1e-15)


def test_predicate_three_valued_logic():
    t = {"a": O.OColumn("int64", [1, None, 3]), "s": O.OColumn("string", ["x", "y", None])}
    assert O.eval_predicate("a > 2", t) == [False, None, True]
    assert O.eval_predicate("a > 2 OR s = 'y'", t) == [False, True, True]
    assert O.eval_predicate("a > 2 AND s = 'y'", t) == [False, None, None]
    assert O.eval_predicate("NOT (a > 2)", t) == [True, None, False]
    assert O.eval_predicate("COALESCE(a, 0.0) >= 0", t) == [True, True, True]
    assert O.eval_predicate("a IN (1, 3)", t) == [True, None, True]
    assert O.eval_predicate("a > 1.5", t) == [False, None, True]
    assert O.eval_predicate("a IS NULL", t) == [False, True, False]


@pytest.mark.parametrize("case", KA["datatype_cases"], ids=[c["id"] for c in KA["datatype_cases"]])
def test_oracle_datatype_known_answers(case):
    table = oracle_table(KA["tables"][case["table"]])
    assert list(O.datatype_state(table, case["column"])) == case["expected"], case["source"]


def test_datatype_host_logic():
    """DataTypeHistogram.toDistribution / determineType (DataType.scala:98-143) on the host."""
    import deequ_amd as d
    from deequ_amd.analyzers import data_type_distribution, determine_type
    h = d.DataTypeHistogram(1, 0, 5, 0, 0)
    dist = data_type_distribution(h)
    assert dist.numberOfBins == 5
    assert dist["Unknown"] == d.DistributionValue(1, 1.0 / 6.0)
    assert dist["Integral"] == d.DistributionValue(5, 5.0 / 6.0)
    I = d.DataTypeInstances
    assert determine_type(dist) == I.Integral
    assert determine_type(data_type_distribution(d.DataTypeHistogram(3, 0, 0, 0, 0))) == I.Unknown
    assert determine_type(data_type_distribution(d.DataTypeHistogram(0, 1, 1, 0, 0))) == I.Fractional
    assert determine_type(data_type_distribution(d.DataTypeHistogram(0, 0, 1, 1, 0))) == I.String
    assert determine_type(data_type_distribution(d.DataTypeHistogram(1, 0, 0, 2, 0))) == I.Boolean
    assert determine_type(data_type_distribution(d.DataTypeHistogram(0, 1, 0, 0, 1))) == I.String
    assert h.sum(d.DataTypeHistogram(1, 2, 3, 4, 5)) == d.DataTypeHistogram(2, 2, 8, 4, 5)
    assert d.DataTypeHistogram.fromBytes(h.toBytes()) == h and len(h.toBytes()) == 40


def _rare_fixture():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "hll_rare_values.json")) as f:
        return json.load(f)


def test_hll_rare_rank_fixture_is_rare():
    """The values in hll_rare_values.json really reach the device's rare HLL branches."""
    fx = _rare_fixture()
    for dtype, key in (("int64", "int64"), ("int32", "int32")):
        for e in fx[key]:
            x = O.spark_hash(e["value"], dtype)
            if e["kind"] == "rare2":
                assert (x >> 23) & 0xFFFFFFFF == 0
                assert O.hll_index_and_rank(x)[1] > 32
            else:
                assert (x >> 32) & 0x7FFFFF == 0 and (x >> 23) & 0xFFFFFFFF != 0
    assert any(e["kind"] == "rare2" for e in fx["int64"])


@pytest.mark.parametrize("case", KA["profile_cases"], ids=[c["id"] for c in KA["profile_cases"]])
def test_oracle_profiles_known_answers(case):
    """O.column_profiles pinned by every ColumnProfilerTest.scala known answer."""
    spec = KA["tables"][case["table"]]
    cols = case["restrict"] or list(spec)
    ot = oracle_table({c: spec[c] for c in cols})
    p = O.column_profiles(ot, case["threshold"], {k: int(v) for k, v in case["predefined"].items()})[case["column"]]
    e = case["expect"]
    if "histogram_values" in e:
        assert p["histogram"] == {k: tuple(v) for k, v in e["histogram_values"].items()}, case["source"]
        return
    assert ("mean" in p) == (e["kind"] == "numeric"), case["source"]
    assert (p["completeness"], p["approx"], p["dataType"], p["inferred"], p["typeCounts"]) == \
        (e["completeness"], e["approx"], e["dataType"], e["inferred"], e["typeCounts"]), case["source"]
    if e["histogram"] is None:
        assert p["histogram"] is None
    else:
        assert p["histogram"] == {k: tuple(v) for k, v in e["histogram"]["values"].items()}
    if e["kind"] == "numeric":
        for f in ("mean", "maximum", "minimum", "sum", "stdDev"):
            assert p[f] == e[f], (case["source"], f)


@pytest.mark.parametrize("dtype", ["int64", "float64", "string"])
def test_c_oracle_hll_registers_equal_python_oracle(dtype):
    """The C restatement's HLL registers (oracle/dq_oracle.c, used by the large GPU parity
    tests) == the Python oracle's, NULLs skipped, NaN / -0.0 / empty strings included."""
    import numpy as np
    import cdq_oracle as C
    rnd = random.Random(7)
    n = 4000
    if dtype == "int64":
        vals = [rnd.getrandbits(64) - (1 << 63) for _ in range(n)]
    elif dtype == "float64":
        vals = [rnd.uniform(-1e6, 1e6) for _ in range(n)] + [float("nan"), -0.0, 0.0, math.inf]
    else:
        vals = ["%016x" % rnd.getrandbits(64) for _ in range(n)] + ["", "é", "a" * 70]
    valid = [rnd.random() >= 0.1 for _ in vals]
    bitmap = np.packbits(np.array(valid, dtype=bool), bitorder="little")
    bitmap = np.concatenate([bitmap, np.zeros(8, np.uint8)])
    if dtype == "string":
        data = [v.encode() for v in vals]
        offs = np.zeros(len(data) + 1, dtype=np.int32)
        np.cumsum([len(b) for b in data], out=offs[1:])
        buf = np.frombuffer(b"".join(data) + b"\0" * 8, dtype=np.uint8)
        regs = C.hll_registers("string", buf, bitmap, offs)
    else:
        regs = C.hll_registers(dtype, np.array(vals, dtype=np.int64 if dtype == "int64" else np.float64), bitmap)
    want = O.hll_registers([v for v, ok in zip(vals, valid) if ok], dtype)
    assert regs.tolist() == list(want)
