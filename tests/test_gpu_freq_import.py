"""Frequency-state merges on the device (round 4): the key-hash exchange's receiver
(dq_freq_import_parts) and dq_freq_merge -- FrequenciesAndNumRows.sum, the outer join of two key
sets (GroupingAnalyzers.scala:128-148) -- merged slice by slice in LDS from parts that the
sender wrote in slice order (dq_freq_partition: 16-B packed records for digit keys, 32-B records
for the rest).  Checked bit-exact: against the oracle on mixed keys (digits, other short keys,
long keys, Histogram's NullValue), into empty and non-empty tables, with runs out of slice order,
with slices that overflow their LDS image, and at C4 scale (8e7 rows, 8 parts) against numpy."""
import time

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd.frequencies import FrequencyTable, encode_key
from helpers import oracle_table

pytestmark = pytest.mark.gpu


def _groups(t):
    counts, keys = t.export()
    return dict(zip(keys, counts.tolist()))


def _spec(n, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, n // 2 + 1, n)
    keys = []
    for i in range(n):
        if i % 29 == 0:
            keys.append(None)
        elif i % 7 == 0:
            keys.append("long-grouping-key-%015d" % a[i])  # > 16 B: key heap
        elif i % 3 == 0:
            keys.append("k%d" % a[i])                      # short, not digits: 32-B records
        else:
            keys.append("%d" % a[i])                       # digits: 16-B packed records
    return {"key": ["string", keys]}


def _table(spec, hist=False, batches=3):
    t = FrequencyTable(["key"], {"key": "string"}, histogram=hist)
    vals = spec["key"][1]
    step = (len(vals) + batches - 1) // batches
    for s in range(0, len(vals), step):
        t.consume(d.Table.from_pydict({"key": ("string", vals[s:s + step])}))
    return t


def _want(spec, hist=False):
    if hist:  # Histogram: NULL is the "NullValue" group (Histogram.scala:63-64)
        st = O.histogram_state(oracle_table(spec), "key")
        return {k[0].encode(): c for k, c in st.frequencies.items()}
    st = O.frequencies_state(oracle_table(spec), ["key"])
    return {encode_key(list(k), ["string"]): c for k, c in st.frequencies.items()}


def _parts(t, n_parts):
    import torch
    pp, pg, pk = t.partition_sizes(n_parts)
    nb = sum(t.part_bytes(p, g) for p, g in zip(pp, pg))
    buf = torch.empty(max(16, nb), dtype=torch.uint8, device="cuda")
    keys = torch.empty(max(8, sum(pk)), dtype=torch.uint8, device="cuda")
    assert t.partition_into(n_parts, buf, keys) == (pp, pg, pk)
    return buf, keys, pp, pg, pk


def _slices(buf, keys, pp, pg, pk, p):
    """Part p alone: (parts tensor, keys tensor) views."""
    off = sum(16 * a + 32 * b for a, b in zip(pp[:p], pg[:p]))
    koff = sum(pk[:p])
    return buf[off:off + 16 * pp[p] + 32 * pg[p]], keys[koff:koff + max(1, pk[p])]


@pytest.mark.parametrize("hist", [False, True])
@pytest.mark.parametrize("n_parts", [1, 3, 8])
def test_partition_import_matches_oracle(gpu, hist, n_parts):
    spec = _spec(40000, 3)
    t = _table(spec, hist)
    want = _want(spec, hist)
    buf, keys, pp, pg, pk = _parts(t, n_parts)
    assert sum(pp) > 0 and sum(pg) > 0 and sum(pk) > 0  # every record kind travels
    # every part into its own owner table: disjoint, and the union is the whole state
    union = {}
    for p in range(n_parts):
        o = FrequencyTable.like(t)
        g, k = _slices(buf, keys, pp, pg, pk, p)
        o.import_parts(g, [pp[p]], [pg[p]], k, [pk[p]])
        got = _groups(o)
        assert not (set(got) & set(union))
        union.update(got)
        o.close()
    assert union == want
    # all parts into one fresh table, then all of them again into the (now non-empty) table
    o = FrequencyTable.like(t)
    o.import_parts(buf, pp, pg, keys, pk)
    assert _groups(o) == want
    o.import_parts(buf, pp, pg, keys, pk)
    assert _groups(o) == {k: 2 * c for k, c in want.items()}
    s = o.summary()
    assert s.num_groups == len(want)
    o.close()
    t.close()


def test_import_runs_out_of_slice_order(gpu):
    """General records shuffled (dq_freq_import_wire accepts any order): the bounds pass finds the
    run out of slice order and it is inserted group by group -- same result."""
    import torch
    spec = _spec(30000, 5)
    t = _table(spec)
    want = _want(spec)
    counts, ks = t.export()
    short = [(k, c) for k, c in zip(ks, counts.tolist()) if len(k) <= 16]
    rng = np.random.default_rng(1)
    rng.shuffle(short)
    rec = np.zeros(len(short), dtype=[("ctrl", "<u8"), ("count", "<i8"), ("k0", "<u8"), ("k1", "<u8")])
    for i, (k, c) in enumerate(short):
        kk = k.ljust(16, b"\0")
        rec[i] = (len(k), c, int.from_bytes(kk[:8], "little"), int.from_bytes(kk[8:], "little"))
    g = torch.from_numpy(rec.view(np.uint8).copy()).cuda()
    o = FrequencyTable.like(t)
    o.import_wire(g, len(short), torch.zeros(8, dtype=torch.uint8, device="cuda"), 0)
    assert _groups(o) == {k: c for k, c in want.items() if len(k) <= 16}
    o.close()
    t.close()


@pytest.mark.parametrize("sizes", [(30000, 30000), (200000, 3000), (3000, 200000)])
def test_merge_tables(gpu, sizes):
    """dq_freq_merge: the source table's slot array as one run (its slices map onto the
    destination's whatever the two sizes), into an empty and a non-empty destination."""
    a_spec, b_spec = _spec(sizes[0], 7), _spec(sizes[1], 8)
    a, b = _table(a_spec), _table(b_spec)
    wa, wb = _want(a_spec), _want(b_spec)
    a.merge_from(b)
    want = dict(wa)
    for k, c in wb.items():
        want[k] = want.get(k, 0) + c
    assert _groups(a) == want
    e = FrequencyTable.like(b)
    e.merge_from(b)
    assert _groups(e) == wb
    for t in (a, b, e):
        t.close()


@pytest.mark.parametrize("n_parts", [2, 20])
def test_import_wide_weights(gpu, n_parts):
    """Packed runs (digit keys only) imported twice over in one call -- 2 parts take the flat
    merge (one index space over <= 16 runs), 20 parts the run-by-run merge -- with weights that do
    not fit the LDS image's 32-bit counts: one record of 2^33 + 3 and one of 2^32 - 16 whose double
    wraps 32 bits.  Their slices take the overflow path (64-bit, group by group): exact counts."""
    import torch
    keys_in = ["%d" % (v % 50000) for v in range(120000)]
    t = _table({"key": ["string", keys_in]}, batches=1)
    want = _want({"key": ["string", keys_in]})
    buf, keys, pp, pg, pk = _parts(t, n_parts)
    assert sum(pg) == 0 and sum(pk) == 0 and pp[0] >= 2
    recs = buf[:16 * sum(pp)].view(torch.int64).view(-1, 2)
    wide = {0: (1 << 33) + 3, 1: (1 << 32) - 16}
    for i, w in wide.items():
        recs[i, 1] = w
    o = FrequencyTable.like(t)
    o.import_parts(torch.cat([buf[:16 * sum(pp)]] * 2), pp * 2, pg * 2, keys, pk * 2)
    got = _groups(o)
    assert len(got) == len(want)
    changed = 0
    for k, c in want.items():
        if got[k] != 2 * c:
            changed += 1
            assert got[k] in (2 * wide[0], 2 * wide[1]), (k, got[k])
    assert changed == 2 and sorted(v for v in got.values() if v > 1 << 31) == sorted(2 * w for w in wide.values())
    o.close()
    t.close()


def test_import_slices_overflow_lds(gpu, monkeypatch):
    """A destination forced far too small (DQ_FREQ_PART_SLOTS: 2^20 slots for 2M keys, ~4000 per
    2048-slot slice): every slice overflows its LDS image, is listed, the table grows, and the
    listed slices' records are inserted group by group -- the same counts."""
    spec = {"key": ["string", ["%d" % v for v in range(2_000_000)]]}
    t = _table(spec, batches=1)
    buf, keys, pp, pg, pk = _parts(t, 4)
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(1 << 20))
    o = FrequencyTable.like(t)
    o.import_parts(buf, pp, pg, keys, pk)
    s = o.summary()
    assert s.num_groups == 2_000_000 and s.num_unique == 2_000_000 and s.grouped_rows == 2_000_000
    assert o.lookup(b"1234567") == 1 and o.lookup(b"1999999") == 1 and o.lookup(b"2000000") == 0
    o.close()
    t.close()


def test_c4_scale_partition_import(gpu):
    """The verdict's C4 case: an 8e7-row table of 12-digit keys (2e8-key domain, 1% NULL) is
    partitioned into 8 parts and all 8 are imported into one fresh table.  Exact against numpy:
    the count-of-counts histogram, #groups, #unique, grouped rows, top-20, and a sample of 2000
    keys looked up one by one.  Prints the import's wall time beside the grouping's."""
    import torch
    n, key_range = 80_000_000, 201_500_000
    g = torch.Generator(device="cuda").manual_seed(11)
    ids = torch.randint(0, key_range, (n,), device="cuda", generator=g, dtype=torch.int64)
    valid = torch.rand(n, device="cuda", generator=g) >= 0.01
    chars = torch.empty((n, 12), dtype=torch.uint8, device="cuda")
    rest = ids.clone()
    for k in range(11, -1, -1):
        chars[:, k] = (rest % 10 + 48).to(torch.uint8)
        rest //= 10
    del rest
    data = torch.cat([chars.view(-1), torch.zeros(8, dtype=torch.uint8, device="cuda")])
    del chars
    offsets = (torch.arange(n + 1, device="cuda", dtype=torch.int64) * 12).to(torch.int32)
    bits = torch.zeros(n // 8, dtype=torch.uint8, device="cuda")
    vb = valid.view(-1, 8).to(torch.uint8)
    for b in range(8):
        bits |= vb[:, b] << b
    del vb
    col = d.Column("string", n, data, bits, offsets=offsets, device=True)
    t = FrequencyTable(["key"], {"key": "string"})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t.consume(d.Table({"key": col}))
    s_local = t.summary()
    t1 = time.perf_counter()
    buf, keys, pp, pg, pk = _parts(t, 8)
    assert sum(pg) == 0 and sum(pk) == 0  # 12-digit keys: every group travels as a 16-B packed record
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    o = FrequencyTable.like(t)
    o.import_parts(buf, pp, pg, keys, pk)
    s = o.summary()
    t3 = time.perf_counter()
    print("\n[c4 import] group-by %.1f ms, partition %.1f ms, import of 8 parts (%d groups) %.1f ms"
          % (1e3 * (t1 - t0), 1e3 * (t2 - t1), sum(pp), 1e3 * (t3 - t2)))
    ids_h, valid_h = ids.cpu().numpy(), valid.cpu().numpy()
    u, c = np.unique(ids_h[valid_h], return_counts=True)
    assert s.num_groups == s_local.num_groups == len(u)
    assert s.num_unique == int((c == 1).sum())
    assert s.grouped_rows == int(valid_h.sum())
    hist, big = o.count_histogram(1 << 10)
    want_hist = np.bincount(c, minlength=1 << 10)[:1 << 10]
    want_hist[0] = 0
    assert np.array_equal(hist, want_hist) and len(big) == int((c >= 1 << 10).sum())
    order = np.argsort(-c, kind="stable")
    cut = c[order[19]]
    want = {("%012d" % k).encode(): int(v) for k, v in zip(u[c >= cut].tolist(), c[c >= cut].tolist())}
    top_counts, top_keys = o.top(20)
    assert dict(zip(top_keys, top_counts.tolist())) == want
    rng = np.random.default_rng(2)
    for i in rng.integers(0, len(u), 2000).tolist():
        assert o.lookup(("%012d" % u[i]).encode()) == int(c[i])
    assert o.lookup(b"not-a-key") == 0
    o.close()
    t.close()


@pytest.mark.parametrize("grow", [1, 2, 3, 5])
def test_import_into_finer_receiver(gpu, monkeypatch, grow):
    """a receiver table with more slice bits than the sender's (2^grow times the
    slots; e.g. owners of disjoint key sets sized independently).  The sender's runs are in order
    only by its own coarser slices: they are cut at those (each receiver slice reads the
    enclosing range and filters) when the difference is at most 3 bits -- no group-by-group
    fallback -- and inserted group by group beyond that.  Exact either way."""
    spec = _spec(60000, 12)
    t = _table(spec)
    want = _want(spec)
    buf, keys, pp, pg, pk = _parts(t, 2)
    send_slots = t.paths()["slots"]
    monkeypatch.setenv("DQ_FREQ_PART_SLOTS", str(send_slots << grow))
    o = FrequencyTable.like(t)
    o.import_parts(buf, pp, pg, keys, pk)
    assert _groups(o) == want
    paths = o.paths()
    assert paths["slots"] == send_slots << grow
    n_wire = sum(1 for v in pp + pg if v)
    if grow <= 3:
        assert paths["import_coarse_runs"] == n_wire and paths["import_skipped_runs"] == 0, paths
    else:
        assert paths["import_skipped_runs"] == n_wire, paths
    # a second import into the now non-empty table: the same cut, doubled counts
    o.import_parts(buf, pp, pg, keys, pk)
    assert _groups(o) == {k: 2 * c for k, c in want.items()}
    o.close()
    t.close()
