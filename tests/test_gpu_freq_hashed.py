"""Long (> 15 B) and multi-column grouping keys on the partition path (round 6): hashed records.

The reference groups any key type in one hash aggregate (GroupingAnalyzers.scala:67-71); its
most common callers on such keys are isUnique / isPrimaryKey / hasUniqueness (Check.scala:140-230)
on UUID-like ids and composite keys.  Here a batch holding a key that does not fit a 16-byte
record switches the table to hashed records: the stage copies every key's bytes into the key heap
and stages {table hash, heap reference}; the two-level split and an LDS aggregation by hash follow,
each record of a hash group compared byte for byte with the group's first.  Checked exactly
(every group and count) against Python counts / the oracle, for:

* 36-character UUID strings with duplicates and NULLs, Histogram's "NullValue" included;
* composite (int64, utf8) keys whose encoding is longer than 15 bytes (oracle);
* tables that already hold groups (early aggregations, short keys first, batches beyond the
  reserved rows) and tables of fewer than 2^20 slots: the global inserts (exact, slower);
* every operation after it (summary, top, export, lookup, merge, further batches).
"""
import struct

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd.frequencies import FrequencyTable, encode_key
from helpers import oracle_table, product_table

pytestmark = pytest.mark.gpu


@pytest.fixture
def part(monkeypatch):
    monkeypatch.setenv("DQ_FREQ_PART_MIN", "1")
    monkeypatch.setenv("DQ_FREQ_PATH", "sorted")


def _uuid(v: int) -> str:
    x = (v * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) % 2 ** 64
    y = ((v ^ 0x5DEECE66D) * 0xC2B2AE3D27D4EB4F) % 2 ** 64
    h = "%016x%016x" % (x, y)
    return "%s-%s-%s-%s-%s" % (h[:8], h[8:12], h[12:16], h[16:20], h[20:32])


def _count(keys, hist=False):
    want = {}
    for k in keys:
        if k is None and not hist:
            continue
        kb = b"NullValue" if k is None else k.encode()
        want[kb] = want.get(kb, 0) + 1
    return want


def _export(t):
    counts, keys = t.export()
    return dict(zip(keys, counts.tolist()))


def _consume(keys, hist, batches, **kw):
    t = FrequencyTable(["key"], {"key": "string"}, histogram=hist, **kw)
    t.reserve(len(keys))  # (as compute_frequencies does: one staging for every batch)
    step = (len(keys) + batches - 1) // batches
    for s in range(0, len(keys), step):
        t.consume(d.Table.from_pydict({"key": ("string", keys[s:s + step])}))
    return t


@pytest.mark.parametrize("hist", [False, True])
def test_uuid_keys_exact(gpu, part, hist):
    """~260k UUID groups of 1-8 rows (2^20 slots: one slice per level-1 region), NULLs, 3 batches."""
    rng = np.random.default_rng(41)
    n = 600_000
    ids = rng.integers(0, 300_000, n)
    keys = [None if i % 41 == 0 else _uuid(int(v)) for i, v in enumerate(ids)]
    t = _consume(keys, hist, 3)
    want = _count(keys, hist)
    s = t.summary()
    assert (s.num_groups, s.num_unique, s.grouped_rows) == (
        len(want), sum(1 for c in want.values() if c == 1), sum(want.values()))
    top_c, top_k = t.top(5)
    best = sorted(want.items(), key=lambda kv: (-kv[1], kv[0]))
    cut = best[4][1]
    assert sorted(zip(top_c.tolist(), top_k)) == sorted((c, k) for k, c in want.items() if c >= cut)
    paths = t.paths()
    assert paths["hashed_runs"] >= 1, paths
    # (Histogram: "NullValue" holds 1/41 of the rows, more than its region's room -- the rest
    # takes the overflow list, inserted globally)
    assert paths["hashed_inserts"] <= (keys.count(None) if hist else 0), paths
    assert _export(t) == want
    assert t.lookup(best[0][0]) == best[0][1]
    t.close()


def test_uuid_keys_unique_ids(gpu, part):
    """isPrimaryKey-shaped: every id distinct (no hash group of two records to compare); 2^21
    slots, so the level-2 split runs too."""
    n = 500_000
    keys = [_uuid(v) for v in range(n)]
    t = _consume(keys, False, 2)
    s = t.summary()
    assert (s.num_groups, s.num_unique, s.grouped_rows) == (n, n, n)
    assert t.paths()["hashed_runs"] >= 1
    t.close()


def test_composite_keys_against_oracle(gpu, part, monkeypatch):
    """(int64, utf8) grouping keys of 8 + 4 + 9..12 encoded bytes: hashed records; groups equal
    to the oracle's FrequenciesAndNumRows (GroupingAnalyzers.scala:53-80), NULL in either column
    dropping the row."""
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))  # (the LDS aggregation's slice layout)
    rng = np.random.default_rng(43)
    n = 120_000
    a = rng.integers(0, 3000, n)
    spec = {"id": ["int64", [None if i % 31 == 0 else int(a[i] % 700) for i in range(n)]],
            "name": ["string", [None if i % 37 == 0 else "name-%05d" % (a[i] % 900) for i in range(n)]]}
    table = product_table(spec)
    t = FrequencyTable(["id", "name"], dict(table.schema))
    t.reserve(n)
    t.consume(table)
    got = _export(t)
    st = O.frequencies_state(oracle_table(spec), ["id", "name"])
    want = {encode_key(list(k), ["int64", "string"]): c for k, c in st.frequencies.items()}
    assert got == want
    assert t.paths()["hashed_runs"] >= 1
    s = t.summary()
    assert s.num_groups == len(want) and s.num_rows == n
    t.close()


@pytest.mark.parametrize("mode", ["budget", "short_first"])
def test_hashed_into_table_with_groups(gpu, part, monkeypatch, mode):
    """budget: an early aggregation fills the table, the next hashed regions go in by global
    inserts; short_first: 12-digit keys first (packed records), then UUIDs.  Exact either way."""
    rng = np.random.default_rng(47)
    n = 300_000
    uu = [_uuid(int(v)) for v in rng.integers(0, 80_000, n)]
    if mode == "budget":
        monkeypatch.setenv("DQ_FREQ_STAGE_BUDGET", "200000")
        keys = uu
    else:
        keys = ["%012d" % v for v in rng.integers(0, 90_000, n)] + uu
    t = _consume(keys, False, 4)
    assert _export(t) == _count(keys)
    assert t.paths()["hashed_inserts"] > 0
    t.close()


def test_hashed_operations_after(gpu, part):
    """A hashed (compacted) table through every later operation: further batches, a merge from
    another hashed table, imports; exact against Python counts."""
    rng = np.random.default_rng(53)
    k1 = [_uuid(int(v)) for v in rng.integers(0, 600_000, 600_000)]  # ~380k groups: 2^20 slots
    k2 = [_uuid(int(v)) for v in rng.integers(300_000, 900_000, 200_000)]
    t = _consume(k1, False, 2)
    assert t.paths()["compacted"] == 1
    t.consume(d.Table.from_pydict({"key": ("string", k2)}))
    other = _consume(k2, False, 1)
    t.merge_from(other)
    other.close()
    want = _count(k1 + k2 + k2)
    assert _export(t) == want
    counts, offs, blob = t.export_flat()
    t2 = FrequencyTable(["key"], {"key": "string"})
    t2.import_flat(counts, offs, blob, num_rows=5)
    assert _export(t2) == want
    t.close()
    t2.close()


def test_composite_few_groups_many_rows(gpu):
    """A composite key of few groups over many rows (a (region, city)-shaped pair, 24 encoded
    bytes): every group's rows land in a few level-1 regions, whose overflow fills up, so the
    hashed staging rolls back (heap cursor included) and the batch takes the insert kernel's LDS
    pre-aggregation.  Exact."""
    rng = np.random.default_rng(59)
    n = 6_000_000
    a = rng.integers(0, 40, n)
    b = rng.integers(0, 25, n)
    valid = rng.random(n) > 0.02
    names = np.array(["city-%07d" % k for k in range(25)])
    table = d.Table({"a": d.Column.from_numpy(a, valid, "int64"),
                     "b": d.Column.from_pylist(names[b].tolist(), "string")})
    t = FrequencyTable(["a", "b"], dict(table.schema))
    t.reserve(n)
    t.consume(table)
    s = t.summary()
    pairs, counts = np.unique(a[valid] * 100 + b[valid], return_counts=True)
    assert (s.num_groups, s.grouped_rows, s.num_rows) == (len(pairs), int(valid.sum()), n)
    assert s.num_unique == int((counts == 1).sum())
    got = {(int.from_bytes(k[:8], "little", signed=True), k[12:].decode()): c for k, c in _export(t).items()}
    want = {(int(p // 100), "city-%07d" % (p % 100)): int(c) for p, c in zip(pairs, counts)}
    assert got == want
    paths = t.paths()
    assert paths["hashed_runs"] == 0 and paths["wait_timeouts"] == 0, paths
    t.close()


# ---- canonical UUID keys (dq_uuidpack.h): the table stages each UUID as its 128 bits (UuidRec)
# and compares keys in LDS; the text is written once per group.  Other key shapes keep the
# hashed records above.

def test_uuid_records_against_hashed(gpu, part, monkeypatch):
    """The same UUID batches grouped with UuidRec records and, DQ_FREQ_UUID=0, with hashed
    records: equal exports, summaries, top-N and lookups, both exact against Python counts."""
    rng = np.random.default_rng(61)
    keys = [None if i % 53 == 0 else _uuid(int(v)) for i, v in enumerate(rng.integers(0, 400_000, 900_000))]
    want = _count(keys)
    got = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("DQ_FREQ_UUID", mode)
        t = _consume(keys, False, 3)
        paths = t.paths()
        assert (paths["uuid_runs"] >= 1) == (mode == "1"), paths
        assert paths["hashed_inserts"] == 0, paths
        s = t.summary()
        got[mode] = (_export(t), (s.num_groups, s.num_unique, s.grouped_rows, s.num_rows),
                     sorted(zip(t.top(7)[0].tolist(), t.top(7)[1])))
        k = next(iter(want))
        assert t.lookup(k) == want[k]
        assert t.lookup(k.upper()) == 0
        t.close()
    assert got["1"][0] == want
    assert got["1"] == got["0"]


def test_uuid_batch_with_other_keys_rolls_back(gpu, part, monkeypatch):
    """Batch 1 holds canonical UUIDs only (UuidRec regions); batch 2 adds an uppercase UUID and a
    40-byte string: it is rolled back, the UUID regions are aggregated (2^20 slots: the slice
    aggregation), and the table stages hashed records from then on (inserted globally into the
    table that now holds groups).  Exact."""
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))
    rng = np.random.default_rng(67)
    b1 = [_uuid(int(v)) for v in rng.integers(0, 150_000, 300_000)]
    b2 = [_uuid(int(v)) for v in rng.integers(100_000, 250_000, 300_000)]
    b2[17] = b2[17].upper()
    b2[99] = "x" * 40
    t = FrequencyTable(["key"], {"key": "string"})
    t.reserve(len(b1) + len(b2))
    t.consume(d.Table.from_pydict({"key": ("string", b1)}))
    t.consume(d.Table.from_pydict({"key": ("string", b2)}))
    assert _export(t) == _count(b1 + b2)
    paths = t.paths()
    assert paths["uuid_runs"] >= 1 and paths["hashed_inserts"] >= len(b2) - 2, paths
    t.close()


def test_uuid_uppercase_keeps_hashed_records(gpu, part, monkeypatch):
    """Uppercase UUID text is not canonical: the probe keeps the hashed records (2^20 slots: the
    hashed slice aggregation).  Exact."""
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))
    rng = np.random.default_rng(71)
    keys = [_uuid(int(v)).upper() for v in rng.integers(0, 100_000, 250_000)]
    t = _consume(keys, False, 2)
    assert _export(t) == _count(keys)
    paths = t.paths()
    assert paths["uuid_runs"] == 0 and paths["hashed_runs"] >= 1, paths
    t.close()


def test_uuid_slices_handed_back(gpu, part, monkeypatch):
    """More groups than a 2^20-slot table's slices hold in LDS (2048 each): every slice hands its
    UUID records back; they are turned into hashed records (text into the heap) and inserted
    globally into a grown table.  Exact."""
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))
    n = 1_300_000
    keys = [_uuid(v) for v in range(n)] + [_uuid(v) for v in range(0, n, 7)]
    t = _consume(keys, False, 2)
    s = t.summary()
    assert (s.num_groups, s.grouped_rows) == (n, len(keys))
    assert s.num_unique == n - len(range(0, n, 7))
    paths = t.paths()
    assert paths["uuid_runs"] >= 1 and paths["hashed_inserts"] > 0, paths
    c, k = t.top(3)
    assert set(c.tolist()) == {2} and len(c) == len(range(0, n, 7))  # (top-N keeps the ties)
    assert sorted(k) == sorted(_uuid(v).encode() for v in range(0, n, 7))
    t.close()


# ---- 16-byte keys (Raw16Rec): a single string column of 16-byte keys, or two 8-byte key columns
# (make_key's encoding is then the two values' 16 bytes): the record is the key, compared in LDS
# and written inline into its slot.

def test_int64_pair_keys_against_oracle(gpu, part, monkeypatch):
    """(int64, int64) keys with NULLs in either column and negative values: 16-byte-key records,
    groups equal to the oracle's FrequenciesAndNumRows (GroupingAnalyzers.scala:53-80)."""
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))
    rng = np.random.default_rng(83)
    n = 150_000
    a = rng.integers(-2000, 2000, n)
    b = rng.integers(0, 300, n)
    spec = {"a": ["int64", [None if i % 29 == 0 else int(a[i]) for i in range(n)]],
            "b": ["int64", [None if i % 31 == 0 else int(b[i]) * 1_000_000_007 for i in range(n)]]}
    table = product_table(spec)
    t = FrequencyTable(["a", "b"], dict(table.schema))
    t.reserve(n)
    t.consume(table)
    st = O.frequencies_state(oracle_table(spec), ["a", "b"])
    want = {encode_key(list(k), ["int64", "int64"]): c for k, c in st.frequencies.items()}
    assert _export(t) == want
    paths = t.paths()
    assert paths["raw16_runs"] >= 1 and paths["hashed_inserts"] == 0, paths
    k = next(iter(want))
    assert t.lookup(k) == want[k]
    t.close()


def test_16_byte_string_keys_against_hashed(gpu, part, monkeypatch):
    """16-character keys (hex ids) with NULLs: 16-byte-key records against hashed records
    (DQ_FREQ_UUID=0): equal exports, summaries and top-N, exact against Python counts; then a
    batch with a 17-byte key is rolled back to hashed records."""
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))
    rng = np.random.default_rng(89)
    keys = [None if i % 43 == 0 else "%016x" % (int(v) * 0x9E3779B97F4A7C15 % 2 ** 64)
            for i, v in enumerate(rng.integers(0, 300_000, 700_000))]
    want = _count(keys)
    got = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("DQ_FREQ_UUID", mode)
        t = _consume(keys, False, 2)
        paths = t.paths()
        assert (paths["raw16_runs"] >= 1) == (mode == "1"), paths
        s = t.summary()
        top_c, top_k = t.top(5)
        got[mode] = (_export(t), (s.num_groups, s.num_unique, s.grouped_rows), sorted(zip(top_c.tolist(), top_k)))
        t.close()
    assert got["1"][0] == want and got["1"] == got["0"]
    monkeypatch.setenv("DQ_FREQ_UUID", "1")
    b2 = keys[:200_000] + ["x" * 17]
    t = FrequencyTable(["key"], {"key": "string"})
    t.reserve(len(keys) + len(b2))
    t.consume(d.Table.from_pydict({"key": ("string", keys)}))
    t.consume(d.Table.from_pydict({"key": ("string", b2)}))
    assert _export(t) == _count(keys + b2)
    assert t.paths()["raw16_runs"] >= 1
    t.close()


def _oracle_float_key(k, dtypes):
    # the oracle keys floats by their bits (-0.0 and 0.0 apart): back to the float of those bits
    return [struct.unpack("<d", struct.pack("<Q", v[1]))[0] if t == "float64" else v for v, t in zip(k, dtypes)]


@pytest.mark.parametrize("dtypes", [("int64", "float64"), ("float64", "float64")])
def test_float_pair_keys_group_by_bits(gpu, part, monkeypatch, dtypes):
    """Two 8-byte key columns with a float64 among them, holding 0.0 and -0.0, NaN, +-inf and
    NULLs: 16-byte-key records; groups equal to the oracle's, which keys floats by their bits
    (Spark 2.2 groups by the UnsafeRow bytes: -0.0 and 0.0 are different groups)."""
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))
    rng = np.random.default_rng(97)
    n = 160_000
    special = [0.0, -0.0, float("nan"), float("inf"), -float("inf")]

    def col(t, salt):
        out = []
        for i, v in enumerate(rng.integers(0, 3000, n)):
            if (i + salt) % 37 == 0:
                out.append(None)
            elif t == "int64":
                out.append(int(v) - 1500)
            elif v % 11 == 0:
                out.append(special[int(v) % len(special)])
            else:
                out.append(float(v % 700) * 0.25 - 40.0)
        return out
    spec = {"a": [dtypes[0], col(dtypes[0], 0)], "b": [dtypes[1], col(dtypes[1], 5)]}
    table = product_table(spec)
    t = FrequencyTable(["a", "b"], dict(table.schema))
    t.reserve(n)
    t.consume(table)
    st = O.frequencies_state(oracle_table(spec), ["a", "b"])
    want = {encode_key(_oracle_float_key(k, dtypes), list(dtypes)): c for k, c in st.frequencies.items()}
    assert _export(t) == want
    zero = {k[8:] for k in want} if dtypes[0] == "int64" else {k[:8] for k in want}
    assert struct.pack("<d", 0.0) in zero and struct.pack("<d", -0.0) in zero
    paths = t.paths()
    assert paths["raw16_runs"] >= 1 and paths["hashed_inserts"] == 0, paths
    s = t.summary()
    assert (s.num_groups, s.num_rows) == (len(want), n)
    t.close()
