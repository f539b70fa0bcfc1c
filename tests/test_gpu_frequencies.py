"""The GPU group-by (dq_freq) and the frequency-based analyzers against the oracle.

Bit-exact: the frequency table itself (every key and count), #groups, #unique, Histogram bins
and top-N.  Entropy / MutualInformation within 1e-12 relative (north_star tolerance; the
reference's own summation order over the frequency DataFrame is unspecified)."""
import math
import struct

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd.frequencies import FrequenciesAndNumRows, FrequencyTable, decode_key, encode_key
from deequ_amd.metrics import EmptyStateException, Failure, Success
from helpers import oracle_table, product_table, random_table, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-12


def _oracle_key(values, dtypes):
    out = []
    for v, t in zip(values, dtypes):
        if t == "float64":
            out.append(("f64bits", struct.unpack("<Q", struct.pack("<d", v))[0]))
        elif t == "float32":
            out.append(("f32bits", struct.unpack("<I", struct.pack("<f", v))[0]))
        else:
            out.append(v)
    return tuple(out)


def _product_freqs(state):
    dtypes = state.table.dtypes
    return {_oracle_key(decode_key(k, dtypes), dtypes): c for k, c in state.frequencies(raw=True).items()}


def _check_state(spec, cols):
    table = product_table(spec)
    otable = oracle_table(spec)
    state = d.Uniqueness(cols).computeStateFrom(table)
    ostate = O.frequencies_state(otable, cols)
    assert state.numRows == ostate.num_rows
    assert _product_freqs(state) == ostate.frequencies
    s = state.summary()
    assert s.num_groups == len(ostate.frequencies)
    assert s.num_unique == sum(1 for c in ostate.frequencies.values() if c == 1)
    assert s.grouped_rows == sum(ostate.frequencies.values())
    if ostate.frequencies:
        assert rel_err(s.entropy, O.entropy_exact(ostate)) <= TOL
    return table, otable, state, ostate


@pytest.mark.parametrize("dtype", ["bool", "int8", "int16", "int32", "int64", "float32", "float64", "string"])
@pytest.mark.parametrize("null_frac", [0.0, 0.3])
def test_single_column_frequencies_match_oracle(gpu, dtype, null_frac):
    rng = np.random.default_rng(11)
    spec = random_table(rng, 5000, null_frac, [dtype])
    if dtype in ("float32", "float64", "int64"):  # low cardinality so counts > 1 occur
        vals = spec["c_" + dtype][1]
        spec["c_" + dtype][1] = [None if v is None else (float(round(v / 10)) if "float" in dtype
                                                        else int(v) % 97) for v in vals]
    _check_state(spec, ["c_" + dtype])


def test_multi_column_keys_match_oracle(gpu):
    rng = np.random.default_rng(3)
    n = 4000
    spec = {
        "a": ["string", [None if rng.random() < 0.1 else "s%d" % rng.integers(0, 9) for _ in range(n)]],
        "b": ["int32", [int(v) for v in rng.integers(0, 5, n)]],
        "c": ["float64", [float(v) for v in rng.integers(0, 3, n)]],
        "e": ["bool", [bool(v) for v in rng.integers(0, 2, n)]],
        "f": ["string", ["long-string-value-%04d-xxxxxxxx" % rng.integers(0, 7) for _ in range(n)]],
    }
    for cols in (["a", "b"], ["b", "c", "e"], ["a", "f"], ["f", "b", "a", "c"]):
        _check_state(spec, cols)


def test_long_and_unicode_string_keys(gpu):
    rng = np.random.default_rng(5)
    words = ["", "a", "é", "短い", "x" * 15, "y" * 16, "z" * 17, "ü" * 40, "key-%s" % ("q" * 200),
             "NullValue"]
    vals = [words[i] if rng.random() > 0.05 else None for i in rng.integers(0, len(words), 3000)]
    _check_state({"s": ["string", vals]}, ["s"])


def test_special_float_keys_group_by_bits(gpu):
    """Spark 2.2 groups by the UnsafeRow bytes: -0.0 and 0.0 are different groups; NaNs with
    different payloads would be too (only the canonical NaN is used here)."""
    vals = [0.0, -0.0, float("nan"), float("inf"), -float("inf"), 1.0, 0.0, float("nan"), None] * 50
    for t in ("float64", "float32"):
        _, _, state, _ = _check_state({"x": [t, vals]}, ["x"])
        assert state.summary().num_groups == 6


def test_high_cardinality_grows_the_table(gpu, monkeypatch):
    """> 2^16 distinct keys, fed in sub-batches: the device table is rehashed while full."""
    monkeypatch.setenv("DQ_FREQ_SUBBATCH_ROWS", "50000")
    rng = np.random.default_rng(9)
    n = 400_000
    ints = rng.integers(0, 300_000, n)
    col = d.Column.from_numpy(ints.astype(np.int64))
    table = d.Table({"k": col})
    state = d.CountDistinct("k").computeStateFrom(table)
    uniq, counts = np.unique(ints, return_counts=True)
    s = state.summary()
    assert s.num_groups == len(uniq)
    assert s.num_unique == int((counts == 1).sum())
    assert s.grouped_rows == n
    got = state.frequencies()
    assert len(got) == len(uniq)
    assert all(got[(int(k),)] == int(c) for k, c in zip(uniq[:1000], counts[:1000]))


def test_counts_beyond_the_device_histogram(gpu):
    """A group with count >= 2^16 goes through the 'big counts' list."""
    vals = np.concatenate([np.zeros(70_000, np.int32), np.arange(1, 3001, dtype=np.int32),
                           np.full(66_000, 7, np.int32)])
    table = d.Table({"k": d.Column.from_numpy(vals)})
    state = d.Uniqueness("k").computeStateFrom(table)
    s = state.summary()
    n = len(vals)
    assert s.num_groups == 3001  # 0 and 1..3000
    assert s.num_unique == 2999  # value 7 occurs 66001 times
    exp_h = math.fsum(-(c / n) * math.log(c / n) for c in [70_000, 66_001] + [1] * 2999)
    assert rel_err(s.entropy, exp_h) <= TOL
    counts, keys = state.table.top(2)
    assert counts.tolist() == [70_000, 66_001]


def test_sub_batches_and_partitions(gpu, monkeypatch):
    """Rows processed in several insert launches (sub-batch knob) and several batches."""
    monkeypatch.setenv("DQ_FREQ_SUBBATCH_ROWS", "1000")
    rng = np.random.default_rng(17)
    spec = random_table(rng, 9001, 0.2, ["string"])
    _check_state(spec, ["c_string"])
    half = {k: [t, v[:4500]] for k, (t, v) in spec.items()}
    rest = {k: [t, v[4500:]] for k, (t, v) in spec.items()}
    part = d.PartitionedTable([product_table(half), product_table(rest)])
    state = d.Uniqueness("c_string").computeStateFrom(part)
    assert _product_freqs(state) == O.frequencies_state(oracle_table(spec), ["c_string"]).frequencies


def test_sliced_and_device_resident_columns(gpu):
    import pyarrow as pa
    rng = np.random.default_rng(21)
    vals = ["v%d" % v if rng.random() > 0.1 else None for v in rng.integers(0, 50, 5000)]
    arr = pa.array(vals, type=pa.string()).slice(13, 4000)
    table = d.Table.from_arrow(pa.table({"s": arr}))
    state = d.Uniqueness("s").computeStateFrom(table)
    exp = O.frequencies_state({"s": O.OColumn("string", vals[13:4013])}, ["s"])
    assert _product_freqs(state) == exp.frequencies
    dev = d.Uniqueness("s").computeStateFrom(table.to_device(0))
    assert _product_freqs(dev) == exp.frequencies


def test_empty_and_all_null(gpu):
    empty = product_table({"s": ["string", []]})
    state = d.CountDistinct("s").computeStateFrom(empty)
    assert state.numRows == 0 and state.summary().num_groups == 0
    assert d.CountDistinct("s").calculate(empty).value == Success(0.0)
    m = d.Uniqueness("s").calculate(empty)
    assert isinstance(m.value.exception, EmptyStateException)
    nulls = product_table({"s": ["string", [None] * 8], "x": ["float64", [None] * 8]})
    assert d.CountDistinct("s").computeStateFrom(nulls).numRows == 8
    r = d.UniqueValueRatio("s").calculate(nulls)
    assert isinstance(r.value, Failure) and not isinstance(r.value.exception, EmptyStateException)
    h = d.Histogram("x").calculate(nulls)
    assert h.value.get().numberOfBins == 1
    assert h.value.get().values["NullValue"].absolute == 8


@pytest.mark.parametrize("name", ["Uniqueness", "Distinctness", "CountDistinct", "UniqueValueRatio", "Entropy"])
def test_metrics_match_oracle(gpu, name):
    rng = np.random.default_rng(31)
    spec = random_table(rng, 6000, 0.1, ["string", "int32"])
    spec["c_int32"][1] = [None if v is None else v % 1000 for v in spec["c_int32"][1]]
    table, otable = product_table(spec), oracle_table(spec)
    for col in ("c_string", "c_int32"):
        a = getattr(d, name)(col) if name == "Entropy" else getattr(d, name)([col])
        got = a.calculate(table).value.get()
        st = O.frequencies_state(otable, [col])
        exp = {"Uniqueness": O.uniqueness_metric, "Distinctness": O.distinctness_metric,
               "CountDistinct": O.count_distinct_metric, "UniqueValueRatio": O.unique_value_ratio_metric,
               "Entropy": O.entropy_exact}[name](st)
        if name == "Entropy":
            assert rel_err(got, exp) <= TOL
        else:
            assert got == exp


def test_mutual_information_matches_oracle(gpu):
    rng = np.random.default_rng(41)
    n = 3000
    a = [int(v) for v in rng.integers(0, 20, n)]
    b = [None if rng.random() < 0.05 else "b%d" % ((x * 7 + int(rng.integers(0, 3))) % 11) for x in a]
    spec = {"a": ["int64", a], "b": ["string", b]}
    got = d.MutualInformation("a", "b").calculate(product_table(spec)).value.get()
    st = O.frequencies_state(oracle_table(spec), ["a", "b"])
    exp = O.mutual_information_metric(st, ["a", "b"], ["a", "b"])
    assert rel_err(got, exp) <= 1e-10


def test_state_sum_equals_union(gpu):
    rng = np.random.default_rng(51)
    spec = random_table(rng, 5000, 0.2, ["string", "float64"])
    spec["c_float64"][1] = [None if v is None else float(round(v)) for v in spec["c_float64"][1]]
    half = {k: [t, v[:2000]] for k, (t, v) in spec.items()}
    rest = {k: [t, v[2000:]] for k, (t, v) in spec.items()}
    for cols in (["c_string"], ["c_float64"], ["c_string", "c_float64"]):
        a = d.Uniqueness(cols)
        merged = a.computeStateFrom(product_table(half)).sum(a.computeStateFrom(product_table(rest)))
        union = a.computeStateFrom(product_table(spec))
        assert merged == union
        assert merged.summary().entropy == union.summary().entropy  # order independent


def test_state_from_host_frequencies_roundtrip(gpu):
    freqs = {("a", 1): 3, ("b", 2): 1, ("long" * 10, -5): 7}
    st = FrequenciesAndNumRows.from_frequencies(["s", "i"], ["string", "int64"], freqs, numRows=12)
    assert st.frequencies() == freqs
    assert st.numRows == 12
    assert d.Uniqueness(["s", "i"]).computeMetricFrom(st).value == Success(1 / 12)
    for k in freqs:
        assert decode_key(encode_key(k, ["string", "int64"]), ["string", "int64"]) == k


def test_histogram_matches_oracle(gpu):
    rng = np.random.default_rng(61)
    for t in ("string", "int32", "float64", "float32", "bool"):
        spec = random_table(rng, 3000, 0.15, [t])
        if t in ("int32", "float64", "float32"):
            spec["c_" + t][1] = [None if v is None else (v % 40 if t == "int32" else float(np.float32(round(v / 7) / 4)))
                                 for v in spec["c_" + t][1]]
        for bins in (1000, 5, 1):
            h = d.Histogram("c_" + t, maxDetailBins=bins).calculate(product_table(spec)).value.get()
            exp = O.histogram_metric(O.histogram_state(oracle_table(spec), "c_" + t), bins)
            assert h.numberOfBins == exp["number_of_bins"]
            assert {k: (v.absolute, v.ratio) for k, v in h.values.items()} == exp["values"]


def test_histogram_special_floats(gpu):
    vals = [float("nan"), -0.0, 0.0, 1e7, 1e-4, 123.5, float("inf"), None, float("nan")]
    spec = {"x": ["float64", vals * 3]}
    h = d.Histogram("x").calculate(product_table(spec)).value.get()
    exp = O.histogram_metric(O.histogram_state(oracle_table(spec), "x"))
    assert h.numberOfBins == exp["number_of_bins"] == 8
    assert {k: (v.absolute, v.ratio) for k, v in h.values.items()} == exp["values"]
    assert set(h.values) == {"NaN", "-0.0", "0.0", "1.0E7", "1.0E-4", "123.5", "Infinity", "NullValue"}


def test_histogram_binning_udf(gpu):
    """AnalyzerTests.scala:229-247: a binning function applied before grouping."""
    spec = {"att1": ["string", ["a", "b", None, "a", "a", None, None, "b", "a", None, None, None]]}

    def binner(v):
        return "Value1" if v in ("a", "b") else "Value2"
    h = d.Histogram("att1", binner).calculate(product_table(spec)).value.get()
    assert h.numberOfBins == 2
    assert set(h.values) == {"Value1", "Value2"}
    assert h.values["Value1"].absolute == 6 and h.values["Value2"].absolute == 6


def test_histogram_parameter_check(gpu):
    spec = {"att1": ["string", ["a", "b"]]}
    m = d.Histogram("att1", None, 1001).calculate(product_table(spec))
    assert str(m.value.exception) == "Cannot return histogram values for more than 1000 values"


def test_missing_column_failure_metric(gpu):
    spec = {"unique": ["string", ["1", "2"]]}
    m = d.Uniqueness(["nonExistingColumn", "unique"]).calculate(product_table(spec))
    assert m.entity == d.Entity.Mutlicolumn and m.instance == "nonExistingColumn,unique"
    assert type(m.value.exception).__name__ == "NoSuchColumnException"


def test_grouping_runner_shares_one_table_and_persists(gpu):
    spec = {"att1": ["string", ["a", "a", "a", "b"]], "att2": ["string", ["c", "c", "c", "d"]]}
    table = product_table(spec)
    provider = d.InMemoryStateProvider()
    analyzers = [d.Uniqueness(["att1", "att2"]), d.Distinctness(["att2", "att1"]),
                 d.MutualInformation("att1", "att2"), d.Entropy("att1"), d.Size()]
    ctx = d.AnalysisRunner.onData(table).addAnalyzers(analyzers).saveStatesWith(provider).run()
    assert ctx.metric(analyzers[0]).value == Success(0.25)
    assert ctx.metric(analyzers[1]).value == Success(0.5)
    h = -(0.75 * math.log(0.75) + 0.25 * math.log(0.25))
    assert ctx.metric(analyzers[2]).value == Success(h)
    assert ctx.metric(analyzers[3]).value == Success(h)
    # one state per grouping, stored under the first analyzer of that grouping
    assert provider.load(analyzers[0]) is not None and provider.load(analyzers[1]) is None
    # aggregate with the saved state: every count doubles -> no unique group, 2 of 8 distinct
    ctx2 = d.AnalysisRunner.onData(table).addAnalyzers(analyzers[:2]).aggregateWith(provider).run()
    assert ctx2.metric(analyzers[0]).value == Success(0.0)
    assert ctx2.metric(analyzers[1]).value == Success(0.25)


@pytest.mark.parametrize("t", ["string", "int64", "bool"])
def test_histogram_shares_the_frequency_table(gpu, t):
    """Histogram run beside a frequency analyzer of its column takes its metric from that
    table (one group-by); the result equals the oracle and Histogram run alone, including a
    literal "NullValue" string merging with the NULL bin (Histogram.scala:63-64)."""
    rng = np.random.default_rng(62)
    spec = random_table(rng, 4000, 0.1, [t])
    col = "c_" + t
    if t == "int64":
        spec[col][1] = [None if v is None else v % 50 for v in spec[col][1]]
    if t == "string":
        spec[col][1] = [("NullValue" if i % 97 == 0 else v) for i, v in enumerate(spec[col][1])]
    data = product_table(spec)
    for bins in (1000, 7, 1):
        hist = d.Histogram(col, maxDetailBins=bins)
        ctx = d.AnalysisRunner.onData(data).addAnalyzers([d.Uniqueness([col]), hist]).run()
        shared = ctx.metric(hist).value.get()
        alone = hist.calculate(data).value.get()
        exp = O.histogram_metric(O.histogram_state(oracle_table(spec), col), bins)
        for h in (shared, alone):
            assert h.numberOfBins == exp["number_of_bins"]
            assert {k: (v.absolute, v.ratio) for k, v in h.values.items()} == exp["values"]
