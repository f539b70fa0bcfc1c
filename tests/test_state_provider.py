"""HdfsStateProvider (analyzers/StateProvider.scala:72-311): the reference's on-disk state layout.

CPU: the MurmurHash3 arithmetic behind the file identifiers (pinned against the standard
MurmurHash3_x86_32 of scikit-learn), every scalar state's byte layout and round trip, the
overwrite rule (StateProviderTest.scala:105-147).  GPU: frequency states through parquet
(StateProviderTest.scala:57-60, 97-100) and incremental runs aggregating persisted states."""
import os
import random
import struct

import pytest

import deequ_amd as d
from deequ_amd.state_provider import COUNT_COL, _mix, _mix_last, scala_string_hash
from helpers import product_table

# StateProviderTest.someData (:226-238)
SOME_DATA = {
    "item": ["string", ["1", "2", "3", "4", "5", "6", "7"]],
    "att1": ["string", ["a", None, "b", "b", None, "a", None]],
    "count": ["int32", [17, 12, 15, 12, 1, 21, 12]],
    "price": ["float64", [1.3, 76.0, 89.0, 12.7, 1.0, 78.0, 0.0]],
}


def _murmur3_x86_32(data: bytes, seed: int) -> int:
    """Standard MurmurHash3_x86_32 written with the provider's mix helpers."""
    h = seed & 0xFFFFFFFF
    n = len(data) // 4
    for i in range(n):
        h = _mix(h, int.from_bytes(data[4 * i:4 * i + 4], "little"))
    tail = data[4 * n:]
    if tail:
        h = _mix_last(h, int.from_bytes(tail, "little"))
    h ^= len(data)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h - (1 << 32) if h & 0x80000000 else h


def test_murmur_mixing_matches_reference_implementation():
    from sklearn.utils import murmurhash3_32
    rnd = random.Random(3)
    for _ in range(300):
        b = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 40)))
        seed = rnd.randrange(0, 2 ** 31)
        assert _murmur3_x86_32(b, seed) == murmurhash3_32(b, seed=seed)


def test_string_hash_framing():
    """stringHash = the x86_32 rounds over blocks (c0 << 16) + c1 of UTF-16 units, an odd last
    unit mixed alone, the length counted in units.  For an ASCII string of even length that is
    the standard hash of the units laid out as little-endian blocks, finalised with len(s)
    instead of the byte count: rebuild it from the standard implementation's pieces."""
    for s in ["Size(None)", "Completeness(att1,None)", "Mean(price,None)", "Uniqueness(List(att1))"]:
        units = [ord(c) for c in s]
        h = 42
        for i in range(0, len(units) - 1, 2):
            h = _mix(h, (units[i] << 16) + units[i + 1])
        if len(units) % 2:
            h = _mix_last(h, units[-1])
        h ^= len(units)
        h ^= h >> 16
        h = (h * 0x85EBCA6B) & 0xFFFFFFFF
        h ^= h >> 13
        h = (h * 0xC2B2AE35) & 0xFFFFFFFF
        h ^= h >> 16
        assert scala_string_hash(s) == (h - (1 << 32) if h & 0x80000000 else h)
    assert -2 ** 31 <= scala_string_hash("Mean(price,None)") < 2 ** 31


def _scalar_cases():
    return [
        (d.Size(), d.NumMatches(7), struct.pack(">q", 7)),
        (d.Completeness("att1"), d.NumMatchesAndCount(4, 7), struct.pack(">qq", 4, 7)),
        (d.Compliance("att1", "att1 = 'b'"), d.NumMatchesAndCount(2, 7), struct.pack(">qq", 2, 7)),
        (d.Sum("price"), d.SumState(258.0), struct.pack(">d", 258.0)),
        (d.Mean("price"), d.MeanState(258.0, 7), struct.pack(">dq", 258.0, 7)),
        (d.Minimum("price"), d.MinState(0.0), struct.pack(">d", 0.0)),
        (d.Maximum("price"), d.MaxState(89.0), struct.pack(">d", 89.0)),
        (d.MinLength("att1"), d.MinState(1.0), struct.pack(">d", 1.0)),
        (d.MaxLength("att1"), d.MaxState(1.0), struct.pack(">d", 1.0)),
        (d.StandardDeviation("price"), d.StandardDeviationState(7.0, 36.857, 9000.5),
         struct.pack(">3d", 7.0, 36.857, 9000.5)),
        (d.Correlation("count", "price"), d.CorrelationState(7.0, 12.8, 36.9, 10.0, 20.0, 30.0),
         struct.pack(">6d", 7.0, 12.8, 36.9, 10.0, 20.0, 30.0)),
        (d.DataType("item"), d.DataTypeHistogram(0, 0, 7, 0, 0), struct.pack(">i5q", 40, 0, 0, 7, 0, 0)),
    ]


def test_scalar_states_layout_and_roundtrip(tmp_path):
    provider = d.HdfsStateProvider(str(tmp_path / "states"))
    for analyzer, state, raw in _scalar_cases():
        provider.persist(analyzer, state)
        path = "%s-%d.bin" % (tmp_path / "states", scala_string_hash(str(analyzer), 42))
        with open(path, "rb") as f:
            assert f.read() == raw, analyzer
        assert provider.load(analyzer) == state, analyzer
    hll = d.ApproxCountDistinctState([i * 7919 for i in range(52)])
    provider.persist(d.ApproxCountDistinct("att1"), hll)
    loaded = provider.load(d.ApproxCountDistinct("att1"))
    assert loaded.words == hll.words


def test_overwrite_rule(tmp_path):
    provider = d.HdfsStateProvider(str(tmp_path / "s"))
    provider.persist(d.Size(), d.NumMatches(1))
    with pytest.raises(FileExistsError, match="already exists"):
        provider.persist(d.Size(), d.NumMatches(2))
    over = d.HdfsStateProvider(str(tmp_path / "s"), allowOverwrite=True)
    over.persist(d.Size(), d.NumMatches(2))
    assert over.load(d.Size()) == d.NumMatches(2)


@pytest.mark.gpu
def test_frequency_states_roundtrip(gpu, tmp_path):
    """StateProviderTest.scala:57-60 / 97-100: Uniqueness(att1), Uniqueness(att1, count),
    Entropy(att1) states survive parquet; Histogram too."""
    import pyarrow.parquet as pq
    data = product_table(SOME_DATA)
    provider = d.HdfsStateProvider(str(tmp_path / "freq"))
    for a in (d.Uniqueness(["att1"]), d.Uniqueness(["att1", "count"]), d.Entropy("att1"), d.Histogram("count")):
        state = a.computeStateFrom(data)
        provider.persist(a, state)
        back = provider.load(a)
        assert back.numRows == state.numRows == 7
        assert back.frequencies() == state.frequencies() or isinstance(a, d.Histogram)
        assert a.computeMetricFrom(back).value == a.computeMetricFrom(state).value, a
        ident = scala_string_hash(str(a), 42)
        pdir = "%s-%d-frequencies.pqt" % (tmp_path / "freq", ident)
        t = pq.ParquetFile(os.path.join(pdir, os.listdir(pdir)[0])).read()  # (duplicate names: no dataset API)
        # Histogram's state is groupBy(column).count(): Spark names the count "count"
        assert t.column_names[-1] == ("count" if isinstance(a, d.Histogram) else COUNT_COL)
    with pytest.raises(FileExistsError):
        provider.persist(d.Uniqueness(["att1"]), d.Uniqueness(["att1"]).computeStateFrom(data))


@pytest.mark.gpu
def test_incremental_run_through_files(gpu, tmp_path):
    """Persist states of one run, aggregate a second run with them: equals the union."""
    first = {k: (v[0], v[1][:4]) for k, v in SOME_DATA.items()}
    second = {k: (v[0], v[1][4:]) for k, v in SOME_DATA.items()}
    analyzers = [d.Size(), d.Completeness("att1"), d.Mean("price"), d.StandardDeviation("price"),
                 d.Correlation("count", "price"), d.MaxLength("att1"), d.ApproxCountDistinct("att1"),
                 d.Uniqueness(["att1"]), d.Entropy("att1")]
    histograms = [d.Histogram("count"), d.Histogram("att1")]  # an int column: string-keyed on disk
    store = d.HdfsStateProvider(str(tmp_path / "inc"))
    d.AnalysisRunner.onData(d.Table.from_pydict(first)).addAnalyzers(analyzers + histograms).saveStatesWith(store).run()
    ctx = d.AnalysisRunner.onData(d.Table.from_pydict(second)).addAnalyzers(analyzers + histograms).aggregateWith(store).run()
    whole = d.AnalysisRunner.onData(product_table(SOME_DATA)).addAnalyzers(analyzers + histograms).run()
    for a in analyzers:
        got, want = ctx.metric(a).value.get(), whole.metric(a).value.get()
        assert abs(got - want) <= 1e-12 * max(1.0, abs(want)), (a, got, want)
    for a in histograms:
        got, want = ctx.metric(a).value.get(), whole.metric(a).value.get()
        assert got.numberOfBins == want.numberOfBins, a
        assert {k: v.absolute for k, v in got.values.items()} == {k: v.absolute for k, v in want.values.items()}, a
    assert os.path.exists("%s-%d.bin" % (tmp_path / "inc", scala_string_hash("Size(None)", 42)))


@pytest.mark.gpu
def test_loads_reference_layout_histogram_state(gpu, tmp_path):
    """A Histogram state as Spark deequ writes it (Histogram.scala:63-66 + StateProvider.scala:
    222-240): parquet (column, "count") with the values cast to string, plus num_rows."""
    import struct
    import pyarrow as pa
    import pyarrow.parquet as pq
    a = d.Histogram("count")
    base = str(tmp_path / "ref")
    ident = scala_string_hash(str(a), 42)
    pdir = "%s-%d-frequencies.pqt" % (base, ident)
    os.makedirs(pdir)
    pq.write_table(pa.table({"count": pa.array(["1", "2", "NullValue"]), "count_": pa.array([3, 2, 1], pa.int64())})
                   .rename_columns(["count", "count"]), os.path.join(pdir, "part-00000.snappy.parquet"))
    with open("%s-%d-num_rows.bin" % (base, ident), "wb") as f:
        f.write(struct.pack(">q", 6))
    state = d.HdfsStateProvider(base).load(a)
    assert state.numRows == 6
    assert state.frequencies() == {("1",): 3, ("2",): 2, ("NullValue",): 1}
    fresh = a.computeStateFrom(d.Table.from_pydict({"count": ("int32", [1, 2, 2, None])}))
    total = fresh.sum(state)
    assert total.numRows == 10
    assert total.frequencies() == {("1",): 4, ("2",): 4, ("NullValue",): 2}
