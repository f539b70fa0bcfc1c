"""Both group-by paths of dq_freq against the oracle, and against each other.

* sorted-bucket path (default for keys of <= 15 bytes): rows staged as 16-B records, sorted by
  slice, aggregated per slice in LDS;
* atomic path (keys > 15 bytes, or DQ_FREQ_PATH=atomic): per-row inserts with device atomics;
* a tiny staging budget (DQ_FREQ_STAGE_BUDGET) forces aggregation in the middle of a batch
  sequence, and a table mixing short and long keys exercises both paths on one table.
Bit-exact: every group and count; #groups, #unique, top-N."""
import os

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd.frequencies import FrequencyTable, encode_key
from helpers import oracle_table, product_table

pytestmark = pytest.mark.gpu


def _spec(n, seed, long_frac=0.0):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, n // 3 + 1, n)
    keys = [None if i % 19 == 0 else ("a-much-longer-grouping-key-%d" % a[i] if rng.random() < long_frac
                                      else "k%d" % a[i]) for i in range(n)]
    ints = [None if i % 23 == 0 else int(a[i] % 1000) for i in range(n)]
    return {"key": ["string", keys], "i": ["int64", ints]}


def _freqs(table, cols, batches=1):
    schema = dict(table.schema)
    t = FrequencyTable(cols, schema)
    n = table.num_rows
    step = (n + batches - 1) // batches
    for s in range(0, n, step):
        part = d.Table.from_pydict({c: (schema[c], table.columns[c].to_pylist()[s:s + step]) for c in schema})
        t.consume(part)
    counts, keys = t.export()
    s = t.summary()
    return dict(zip(keys, counts.tolist())), s


def _want(spec, cols):
    st = O.frequencies_state(oracle_table(spec), cols)
    dtypes = [spec[c][0] for c in cols]
    return {encode_key(list(k), dtypes): c for k, c in st.frequencies.items()}


@pytest.mark.parametrize("path", ["sorted", "atomic"])
@pytest.mark.parametrize("budget", [None, "700"])
@pytest.mark.parametrize("long_frac", [0.0, 0.2])
def test_paths_match_oracle(gpu, monkeypatch, path, budget, long_frac):
    monkeypatch.setenv("DQ_FREQ_PATH", path)
    if budget:
        monkeypatch.setenv("DQ_FREQ_STAGE_BUDGET", budget)
    spec = _spec(20000, 1, long_frac)
    table = product_table(spec)
    for cols in (["key"], ["i"], ["key", "i"]):
        got, s = _freqs(table, cols, batches=4)
        want = _want(spec, cols)
        assert got == want, (cols, path)
        assert s.num_groups == len(want) and s.num_unique == sum(1 for c in want.values() if c == 1)
        assert s.num_rows == 20000


def test_high_cardinality_grows_table(gpu):
    """~1.5M distinct int64 keys: the table grows through many slice doublings; the sketch
    sizes it before aggregation."""
    rng = np.random.default_rng(2)
    n = 3_000_000
    vals = rng.integers(0, 1_500_000, n)
    table = d.Table({"v": d.Column.from_numpy(vals, None, "int64")})
    t = FrequencyTable(["v"], {"v": "int64"})
    t.consume(table)
    s = t.summary()
    u, c = np.unique(vals, return_counts=True)
    assert s.num_groups == len(u)
    assert s.num_unique == int((c == 1).sum())
    assert s.grouped_rows == n
    counts, keys = t.top(5)
    assert sorted(counts.tolist())[-1] == int(c.max())


@pytest.mark.parametrize("hot_frac", [0.5, 0.02])
def test_hot_key_buckets_split_across_workgroups(gpu, hot_frac):
    """A key holding a large share of the rows fills one slice's bucket far beyond one work
    item (kFreqAggPiece records): its pieces are pre-aggregated in LDS and merged atomically.
    Exact counts, also for the cold keys sharing that slice."""
    rng = np.random.default_rng(3)
    n = 4_000_000
    vals = rng.integers(0, 200_000, n)
    hot = rng.random(n) < hot_frac
    vals[hot] = 123_456_789
    valid = rng.random(n) > 0.01
    table = d.Table({"v": d.Column.from_numpy(vals, valid, "int64")})
    for hist in (False, True):
        t = FrequencyTable(["v"], {"v": "int64"}, histogram=hist)
        t.consume(table)
        s = t.summary()
        u, c = np.unique(vals[valid], return_counts=True)
        extra = 1 if hist and (~valid).any() else 0
        assert s.num_groups == len(u) + extra
        assert s.num_unique == int((c == 1).sum()) + (1 if extra and (~valid).sum() == 1 else 0)
        counts, keys = t.top(3)
        want = sorted(c.tolist() + ([int((~valid).sum())] if extra else []), reverse=True)[:3]
        assert sorted(counts.tolist(), reverse=True)[:3] == want  # top() keeps ties at the threshold


def test_low_cardinality_many_rows(gpu):
    """16 distinct keys over 3M rows: every bucket is split into pieces (the table is tiny)."""
    rng = np.random.default_rng(4)
    n = 3_000_000
    vals = rng.integers(0, 16, n).astype(np.int32)
    table = d.Table({"v": d.Column.from_numpy(vals, None, "int32")})
    t = FrequencyTable(["v"], {"v": "int32"})
    t.consume(table)
    counts, keys = t.export()
    got = {int.from_bytes(k, "little", signed=True): int(c) for k, c in zip(keys, counts.tolist())}
    u, c = np.unique(vals, return_counts=True)
    assert got == dict(zip(u.tolist(), c.tolist()))


@pytest.mark.parametrize("distinct,hint", [(90, 100), (3_000_000, 100)])
def test_few_group_hint_single_launch_and_fallback(gpu, distinct, hint):
    """dq_freq_expect_groups: a right hint takes one insert launch over the whole batch; a wrong
    one (3M groups behind a hint of 100) overflows the optimistic table, which is cleared and
    re-filled on the sized path.  Both must give the exact group-by."""
    rng = np.random.default_rng(5)
    n = 6_000_000  # more rows than one sized sub-launch (4M)
    vals = rng.integers(0, distinct, n).astype(np.int64)
    valid = rng.random(n) >= 0.02
    table = d.Table({"v": d.Column.from_numpy(vals, valid, "int64")})
    t = FrequencyTable(["v"], {"v": "int64"})
    t.expect_groups(hint)
    t.consume(table)
    counts, keys = t.export()
    s = t.summary()
    t.close()
    got = {int.from_bytes(k, "little", signed=True): int(c) for k, c in zip(keys, counts.tolist())}
    u, c = np.unique(vals[valid], return_counts=True)
    assert s.num_groups == len(u)
    assert got == dict(zip(u.tolist(), c.tolist()))


@pytest.mark.parametrize("hot_frac", [0.0, 0.3])
def test_bucket_split_two_levels(gpu, monkeypatch, hot_frac):
    """The sort path's hand-written bucket split at > 2^11 slices (two multi-split levels: the
    top 11 slice bits, then the rest inside each level-1 region), with and without a hot key
    (one atomic per tile, not per record): exact group counts against numpy."""
    monkeypatch.setenv("DQ_FREQ_PART", "0")  # every record through the sort path
    rng = np.random.default_rng(11)
    n = 9_000_000
    vals = rng.integers(0, 6_000_000, n)
    if hot_frac:
        vals[rng.random(n) < hot_frac] = 987_654_321
    table = d.Table({"v": d.Column.from_numpy(vals, None, "int64")})
    t = FrequencyTable(["v"], {"v": "int64"})
    t.consume(table)
    s = t.summary()
    p = t.paths()
    u, c = np.unique(vals, return_counts=True)
    assert p["slots"] >= (1 << 23) and p["sort_records"] >= n, p  # >= 2^12 slices: two levels
    assert s.num_groups == len(u)
    assert s.num_unique == int((c == 1).sum())
    assert s.grouped_rows == n
    hist = np.bincount(c)
    ent = -sum(float(k) * (cc / n) * np.log(cc / n) for cc, k in enumerate(hist) if k and cc)
    assert abs(s.entropy - ent) <= 1e-12 * abs(ent)
    counts, keys = t.top(3)
    assert sorted(counts.tolist(), reverse=True)[:3] == sorted(c.tolist(), reverse=True)[:3]
