"""Frequency states as columns (dq_freq_export_flat / dq_freq_import_flat): exact against the
per-group export and the oracle on small tables, then a C4-scale state (>= 5e7 groups) persisted
and reloaded through HdfsStateProvider's layout (StateProvider.scala:222-240 persist, :280-311
load; AnalysisRunner.scala:543 persists every grouping state) -- with no per-group Python
object on the way, inside 15 s, and compared exactly against torch.unique over the same ids."""
import os
import time

import numpy as np
import pytest

import deequ_amd as d
from deequ_amd.frequencies import FrequenciesAndNumRows, FrequencyTable, encode_key
from deequ_amd.state_provider import HdfsStateProvider

pytestmark = pytest.mark.gpu


def _table(spec, key_columns, histogram=False):
    data = d.Table.from_pydict(spec).to_device(0)
    t = FrequencyTable(key_columns, {c: spec[c][0] for c in spec}, histogram)
    t.consume(data)
    return t


def _flat_dict(t):
    counts, offs, blob = t.export_flat()
    raw = blob.tobytes()
    return {raw[offs[i]:offs[i + 1]]: int(counts[i]) for i in range(len(counts))}


def _want(spec, key_columns, histogram=False):
    dtypes = [spec[c][0] for c in key_columns]
    out = {}
    for row in zip(*[spec[c][1] for c in key_columns]):
        if not histogram and any(v is None for v in row):
            continue
        k = encode_key(row, dtypes, histogram)
        out[k] = out.get(k, 0) + 1
    return out


SPECS = [
    ({"s": ["string", ["k%d" % (i % 777) if i % 5 else "a-long-key-over-sixteen-bytes-%d" % (i % 31)
                       for i in range(20000)] + ["", None, ""]]}, ["s"], False),
    ({"s": ["string", [None if i % 9 == 0 else str(i % 100) for i in range(5000)]]}, ["s"], True),
    ({"i": ["int64", [(i * 7919) % 3001 - 1500 for i in range(30000)]]}, ["i"], False),
    ({"f": ["float64", [float(i % 13) * 0.5 if i % 11 else None for i in range(3000)]]}, ["f"], True),
    ({"a": ["string", ["x" * (i % 20) for i in range(4000)]], "b": ["int32", [i % 7 for i in range(4000)]],
      "c": ["bool", [i % 3 == 0 for i in range(4000)]]}, ["a", "b", "c"], False),
]


@pytest.mark.parametrize("case", range(len(SPECS)))
def test_flat_export_matches_groups(gpu, case):
    spec, keys, hist = SPECS[case]
    t = _table(spec, keys, hist)
    got = _flat_dict(t)
    assert got == _want(spec, keys, hist)
    # slot order: the same table exports the same columns; device export equals host export
    c1, o1, b1 = t.export_flat()
    c2, o2, b2 = t.export_flat(device=True)
    assert np.array_equal(c1, c2.cpu().numpy()) and np.array_equal(o1, o2.cpu().numpy())
    assert np.array_equal(b1, b2.cpu().numpy())
    # import from host arrays and from device tensors: the same groups; twice -> doubled counts
    u = FrequencyTable.like(t)
    u.import_flat(c1, o1, b1, 10)
    u.import_flat(c2, o2, b2, 5)
    assert _flat_dict(u) == {k: 2 * c for k, c in got.items()}
    assert u.num_rows == 15
    # the arrow form (Histogram: cast to string) loads back as the same state
    st = FrequenciesAndNumRows(t)
    back = FrequenciesAndNumRows.from_arrow(st.to_arrow(strings=False), keys, [spec[c][0] for c in keys],
                                            st.numRows, histogram=hist)
    assert back.frequencies(raw=True) == st.frequencies(raw=True)
    for x in (t, u, back.table):
        x.close()


def test_flat_import_rejects_bad_offsets(gpu):
    t = FrequencyTable(["s"], {"s": "string"})
    from deequ_amd import _lib as L
    with pytest.raises(L.DeequAmdError):
        t.import_flat(np.array([1, 1]), np.array([0, 5, 3]), np.zeros(8, np.uint8))
    assert t.summary().num_groups == 0
    assert t.num_rows == 0  # (a failing import adds no numRows)
    t.close()


def test_flat_import_tensor_inputs(gpu):
    """Device tensors: a CPU tensor is refused (ValueError, nothing imported); int32 offsets and
    int32 counts -- Arrow's string offsets -- are converted, not misread as int64."""
    import torch
    t = FrequencyTable(["s"], {"s": "string"})
    dev = t.torch_device
    blob = torch.tensor(list(b"abxyz"), dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        t.import_flat(torch.tensor([2, 3]), torch.tensor([0, 2, 5], device=dev), blob, 5)
    assert t.summary().num_groups == 0 and t.num_rows == 0
    t.import_flat(torch.tensor([2, 3], dtype=torch.int32, device=dev),
                  torch.tensor([0, 2, 5], dtype=torch.int32, device=dev), blob, 5)
    assert _flat_dict(t) == {b"ab": 2, b"xyz": 3}
    assert t.num_rows == 5
    t.close()


def test_c4_scale_state_persist_and_load(gpu, tmp_path):
    import torch
    import bench
    rows, distinct = 80_000_000, 100_000_000
    shard = bench.make_c4_batches(rows, rows, distinct, 0, 0)
    table = FrequencyTable(["key"], {"key": "string"})
    table.reserve(rows)
    for b in shard.batches():
        table.consume(b)
    state = FrequenciesAndNumRows(table)
    groups = state.summary().num_groups
    assert groups >= 50_000_000
    del shard
    torch.cuda.empty_cache()
    prov = HdfsStateProvider(str(tmp_path / "state"))
    an = d.Uniqueness(["key"])
    t0 = time.perf_counter()
    prov.persist(an, state)
    t1 = time.perf_counter()
    loaded = prov.load(an)
    t2 = time.perf_counter()
    part = str(tmp_path / "state") + "-%s-frequencies.pqt" % prov._identifier(an)
    size = sum(os.path.getsize(os.path.join(part, f)) for f in os.listdir(part))
    print("\n[state scale] groups %d: persist %.2f s, load %.2f s, parquet %.1f MB"
          % (groups, t1 - t0, t2 - t1, size / 1e6))
    assert t2 - t0 < 15.0, (t1 - t0, t2 - t1)
    assert loaded.numRows == rows and loaded.summary().num_groups == groups

    def by_id(t):  # (id, count) sorted by id, from the flat export on the device
        c, o, b = t.export_flat(device=True)
        assert bool(((o[1:] - o[:-1]) == 12).all())
        digits = (b.view(-1, 12).to(torch.int64) - 48)
        ids = (digits * torch.tensor([10 ** (11 - i) for i in range(12)], device=b.device)).sum(1)
        ids, order = torch.sort(ids)
        return ids, c[order]
    a_ids, a_c = by_id(table)
    b_ids, b_c = by_id(loaded.table)
    assert torch.equal(a_ids, b_ids) and torch.equal(a_c, b_c)
    ref = bench.c4_valid_ids(rows, rows, distinct, 0, 0)
    u, c = torch.unique(ref, sorted=True, return_counts=True)
    assert torch.equal(u, b_ids) and torch.equal(c, b_c)
    table.close()
    loaded.table.close()
