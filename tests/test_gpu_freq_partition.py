"""The partition path of the sorted-bucket group-by (dq_freq_part_kernel P1/P2 +
dq_freq_agg_region_kernel), forced onto small stagings with DQ_FREQ_PART_MIN=1, against the
oracle, numpy and the radix-sort path (DQ_FREQ_PART=0).

Covers: several key encodings and batches; a table that is not empty when the partition runs
(a small staging budget aggregates early); high cardinality (many slice regions, P2 on); a hot
key that overflows its region into the overflow list (aggregated afterwards by the sort path);
a hot key large enough to fill the overflow list (the whole staging falls back to the sort);
few groups (one pass, no P2).  Bit-exact: every group and count."""
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


def _export(t):
    counts, keys = t.export()
    return dict(zip(keys, counts.tolist()))


def _int_groups(t):
    counts, keys = t.export()
    return {int.from_bytes(k, "little", signed=True): int(c) for k, c in zip(keys, counts.tolist())}


@pytest.mark.parametrize("budget", [None, "3000"])
def test_partition_matches_oracle(gpu, part, monkeypatch, budget):
    if budget:
        monkeypatch.setenv("DQ_FREQ_STAGE_BUDGET", budget)
    rng = np.random.default_rng(11)
    n = 20000
    a = rng.integers(0, n // 3 + 1, n)
    spec = {"key": ["string", [None if i % 19 == 0 else "k%d" % a[i] for i in range(n)]],
            "i": ["int64", [None if i % 23 == 0 else int(a[i] % 1000) for i in range(n)]]}
    table = product_table(spec)
    schema = dict(table.schema)
    for cols in (["key"], ["i"], ["key", "i"]):
        t = FrequencyTable(cols, schema)
        step = n // 4
        for s in range(0, n, step):
            t.consume(d.Table.from_pydict({c: (schema[c], table.columns[c].to_pylist()[s:s + step])
                                           for c in schema}))
        got = _export(t)
        st = O.frequencies_state(oracle_table(spec), cols)
        want = {encode_key(list(k), [spec[c][0] for c in cols]): c for k, c in st.frequencies.items()}
        assert got == want, cols
        s = t.summary()
        assert s.num_groups == len(want)
        assert s.num_unique == sum(1 for c in want.values() if c == 1)


@pytest.mark.parametrize("n,distinct", [(3_000_000, 1_500_000), (5_000_000, 200_000), (2_000_000, 40),
                                        (2_000_000, 10)])
def test_partition_counts_exact(gpu, part, n, distinct):
    rng = np.random.default_rng(12)
    vals = rng.integers(0, distinct, n)
    valid = rng.random(n) > 0.01
    table = d.Table({"v": d.Column.from_numpy(vals, valid, "int64")})
    t = FrequencyTable(["v"], {"v": "int64"})
    t.consume(table)
    s = t.summary()
    u, c = np.unique(vals[valid], return_counts=True)
    assert s.num_groups == len(u)
    assert s.num_unique == int((c == 1).sum())
    assert s.grouped_rows == int(valid.sum())
    ent = -np.sum((c / n) * np.log(c / n))
    assert abs(s.entropy - ent) <= 1e-9 * abs(ent)
    counts, _ = t.top(5)  # (the slice maxima let the export skip slices below the threshold)
    assert sorted(counts.tolist(), reverse=True)[:5] == sorted(c.tolist(), reverse=True)[:5]
    if len(u) <= 1_000_000:
        assert _int_groups(t) == dict(zip(u.tolist(), c.tolist()))


@pytest.mark.parametrize("hot_frac", [0.5, 0.03])
def test_partition_hot_key_overflow(gpu, part, hot_frac):
    """0.03: the hot key's rows overflow its level-1 region into the overflow list; 0.5: they
    overflow the list too and the staging is sorted instead.  Exact either way."""
    rng = np.random.default_rng(13)
    n = 4_000_000
    vals = rng.integers(0, 300_000, n)
    vals[rng.random(n) < hot_frac] = 987_654_321
    table = d.Table({"v": d.Column.from_numpy(vals, None, "int64")})
    t = FrequencyTable(["v"], {"v": "int64"})
    t.consume(table)
    u, c = np.unique(vals, return_counts=True)
    assert _int_groups(t) == dict(zip(u.tolist(), c.tolist()))


def test_partition_equals_sort_path_strings(gpu, monkeypatch):
    """12-digit keys (the C4 shape) on both paths: identical groups and counts."""
    rng = np.random.default_rng(14)
    n = 2_000_000
    keys = ["%012d" % v for v in rng.integers(0, 400_000, n)]
    spec = {"key": ["string", keys]}
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DQ_FREQ_PART", mode)
        monkeypatch.setenv("DQ_FREQ_PART_MIN", "1")
        table = product_table(spec)
        t = FrequencyTable(["key"], dict(table.schema))
        t.consume(table)
        res[mode] = _export(t)
        t.close()
    assert res["0"] == res["1"]
    vals, cnt = np.unique(np.array(keys), return_counts=True)
    assert len(res["1"]) == len(vals)
    assert sorted(res["1"].values()) == sorted(cnt.tolist())


@pytest.mark.parametrize("long_frac", [0.0, 0.2])
def test_region_staging_batches_and_rollback(gpu, part, long_frac):
    """Region staging across several batches; a batch holding a key longer than 15 bytes is
    rolled back (fills, overflow and staged counts restored) and grouped on the general path
    after the regions staged so far are aggregated."""
    rng = np.random.default_rng(15)
    n = 40000
    a = rng.integers(0, 9000, n)
    keys = [None if i % 29 == 0 else ("a-much-longer-grouping-key-%d" % a[i] if rng.random() < long_frac
                                      else "%012d" % a[i]) for i in range(n)]
    spec = {"key": ["string", keys]}
    table = product_table(spec)
    schema = dict(table.schema)
    for hist in (False, True):
        t = FrequencyTable(["key"], schema, histogram=hist)
        step = n // 5
        for s in range(0, n, step):
            t.consume(d.Table.from_pydict({"key": ("string", keys[s:s + step])}))
        got = _export(t)
        want = {}
        for k in keys:
            if k is None and not hist:
                continue
            kb = b"NullValue" if k is None else k.encode()
            want[kb] = want.get(kb, 0) + 1
        assert got == want, hist
        t.close()


# ---- packed digit-key records (dq_keypack.h) -------------------------------------------------

def _count(keys, hist):
    want = {}
    for k in keys:
        if k is None and not hist:
            continue
        kb = b"NullValue" if k is None else k.encode()
        want[kb] = want.get(kb, 0) + 1
    return want


def _consume_batches(keys, hist, batches, **kw):
    t = FrequencyTable(["key"], {"key": "string"}, histogram=hist, **kw)
    step = (len(keys) + batches - 1) // batches
    for s in range(0, len(keys), step):
        t.consume(d.Table.from_pydict({"key": ("string", keys[s:s + step])}))
    return t


@pytest.mark.parametrize("other_frac", [0.0, 0.02])
@pytest.mark.parametrize("hist", [False, True])
def test_packed_digit_keys(gpu, part, hist, other_frac):
    """Digit keys of every length 0..15 (leading zeros kept), NULLs ("NullValue" for Histogram,
    its own packed code), and a few keys that are not digit strings (16-B records on the
    overflow list, aggregated after the packed regions): exact groups and counts."""
    rng = np.random.default_rng(21)
    n = 600_000  # ~350k groups: a 2^20-slot table, one slice per level-1 region
    a = rng.integers(0, 500_000, n)
    ln = rng.integers(0, 16, n)
    keys = []
    for i in range(n):
        if i % 37 == 0:
            keys.append(None)
        elif rng.random() < other_frac:
            keys.append("id-%d" % (a[i] % 500))
        else:
            keys.append(("%015d" % a[i])[15 - ln[i]:] if ln[i] else "")
    t = _consume_batches(keys, hist, 3)
    assert _export(t) == _count(keys, hist)
    paths = t.paths()
    assert paths["packed_runs"] >= 1, paths
    s = t.summary()
    want = _count(keys, hist)
    assert s.num_groups == len(want)
    assert s.num_unique == sum(1 for c in want.values() if c == 1)
    t.close()


def test_packed_then_other_keys(gpu, part):
    """Digit batches staged packed, then a batch of hex keys overflows the overflow list: the
    packed regions are aggregated, the table switches to 16-B records, and the result is exact."""
    rng = np.random.default_rng(22)
    n = 400_000  # ~330k digit groups: the packed regions are aggregated on the partition path
    digits = ["%012d" % v for v in rng.integers(0, 1_000_000, n)]
    hexes = ["%012x" % v for v in rng.integers(0, 2**40, n)]  # 99.6 % not digit strings
    keys = digits + hexes + digits[: n // 2]
    t = _consume_batches(keys, False, 5)  # batches 1-2 digits, 3 hex (the switch), 4-5 mixed
    assert _export(t) == _count(keys, False)
    assert t.paths()["packed_runs"] >= 1
    t.close()


@pytest.mark.parametrize("frac", [0.0, 0.03, 0.2, 1.0])
def test_pack_probe_mixed_first_batch(gpu, part, frac):
    """The table's first batch holds a fraction `frac` of hex keys: the pack probe samples it and
    stages packed records (few keys that do not pack: the overflow list takes them) or 16-B
    records from the start (many: no packed staging to roll back).  Exact either way."""
    rng = np.random.default_rng(24)
    n = 300_000
    keys = [("%012x" % v) if rng.random() < frac else ("%012d" % (v % 10**12))
            for v in rng.integers(0, 2**40, n)]
    t = _consume_batches(keys, False, 2)
    assert _export(t) == _count(keys, False)
    assert t.paths()["wait_timeouts"] == 0
    t.close()


@pytest.mark.parametrize("mode", ["budget", "load", "few"])
def test_packed_paths_equal_unpacked(gpu, part, monkeypatch, mode):
    """The same digit keys with DQ_FREQ_PACK=0 (16-B records) and packed: identical tables.
    budget: early aggregations into a non-empty table (existing digit and non-digit groups
    loaded into the packed LDS image); load: a table of fewer slots than groups, whose slices
    overflow the LDS image (their records return to the retry list as 16-B records); few: fewer slices than
    level-1 regions (the packed regions are unpacked to a contiguous staging for the sort path)."""
    rng = np.random.default_rng(23)
    batches = 4
    if mode == "few":
        n, distinct = 100_000, 300
    else:  # ~700k groups: 2^21 slots, level-2 split on
        n, distinct = 1_600_000, 1_000_000
    vals = rng.integers(0, distinct, n)
    keys = ["%010d" % v if i % 11 else "k%d" % (v % 97) for i, v in enumerate(vals)]
    if mode == "budget":  # the second batch is aggregated into the first one's table
        monkeypatch.setenv("DQ_FREQ_STAGE_BUDGET", "700000")
        batches = 2
    if mode == "load":  # 2^20 slots for ~1.1M groups: most slices overflow their LDS image
        monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))
        n, distinct = 1_500_000, 2_000_000
        vals = rng.integers(0, distinct, n)
        keys = ["%010d" % v if i % 11 else "k%d" % (v % 97) for i, v in enumerate(vals)]
    res = {}
    for pack in ("0", "1"):
        monkeypatch.setenv("DQ_FREQ_PACK", pack)
        t = _consume_batches(keys, True, batches)
        res[pack] = _export(t)
        res[pack + "paths"] = t.paths()
        t.close()
    assert res["1"] == res["0"] == _count(keys, True)
    assert res["0paths"]["packed_runs"] == 0
    if mode != "few":
        assert res["1paths"]["packed_runs"] >= (2 if mode == "budget" else 1), res["1paths"]
    if mode == "load":
        assert res["1paths"]["sort_records"] > 0, res["1paths"]  # slices overflowed LDS


def test_compacted_table_equals_slot_image(gpu, part, monkeypatch):
    """Round 6: the packed aggregation into a fresh table writes only its occupied slots
    (compacted); summary() and top() read that form, every other operation rebuilds the slot
    image first (dq_freq_expand_kernel).  The same operations with DQ_FREQ_COMPACT=0: identical
    summaries, top groups, exports, lookups, and results of further batches, imports and merges."""
    rng = np.random.default_rng(31)
    n = 1_200_000  # ~650k groups: 2^21 slots, level-2 split on, packed records
    keys = ["%011d" % v if i % 53 else None for i, v in enumerate(rng.integers(0, 1_000_000, n))]
    more = ["%011d" % v for v in rng.integers(500_000, 1_500_000, 300_000)]
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DQ_FREQ_COMPACT", mode)
        out = {}
        t = _consume_batches(keys, True, 3)
        s = t.summary()
        out["summary"] = (s.num_groups, s.num_unique, s.grouped_rows, s.num_rows, s.entropy)
        out["top"] = t.top(9)[0].tolist(), sorted(t.top(9)[1])
        out["export"] = _export(t)
        out["lookup"] = [t.lookup(k.encode()) for k in keys[:50] if k is not None]
        t.consume(d.Table.from_pydict({"key": ("string", more)}))
        out["after_consume"] = _export(t)
        src = _consume_batches(more[:100_000], True, 1)
        t.merge_from(src)
        src.close()
        out["after_merge"] = _export(t)
        out["paths"] = t.paths()["packed_runs"]
        t.close()
        res[mode] = out
    for k in ("summary", "top", "export", "lookup", "after_consume", "after_merge"):
        assert res["0"][k] == res["1"][k], k
    assert res["1"]["export"] == _count(keys, True)
    assert res["1"]["paths"] >= 1
