"""Parity at the shapes of BASELINE.json's configs C3 and C4, beyond what
the small-table tests reach:

* C3: ApproxCountDistinct over 64 high-cardinality int64 columns in ONE plan (the
  `dq_scan_fast_kernel<long, PK_NONE, STATS=false, HLL=true>` group, 64 tasks), and the string
  variant (16-char lowercase hex, `dq_hll_kernel`).  Registers bit-exact against the oracle's C
  restatement (oracle/dq_oracle.c, pinned to the Python oracle by
  tests/test_oracle_golden.py::test_c_oracle_hll_registers_equal_python_oracle);
  StatefulHyperloglogPlus.scala:89-115.
* C4: a 12-digit zero-padded decimal key column of 8e7 rows over [0, 201.5M) -- ~6.6e7
  distinct keys, so the partition path sizes its table at 2^28 slots = 2^17 slices of 2048, the
  regime of the 1e9-row C4 run -- against numpy's unique over the integer ids: grouped rows,
  groups, unique groups, Entropy (GroupingAnalyzers.scala:53-80, Entropy.scala:31-41) and the
  top-20 with ties (Histogram.scala:78-79)."""
import math

import numpy as np
import pytest

import cdq_oracle as C
import deequ_amd as d
import pyoracle as O
from deequ_amd.frequencies import FrequencyTable

pytestmark = pytest.mark.gpu


def _bitmap(valid):
    return np.concatenate([np.packbits(valid, bitorder="little"), np.zeros(8, np.uint8)])


def test_c3_shape_64_int64_hll_columns(gpu):
    rng = np.random.default_rng(3)
    n, ncol = 250_000, 64
    cols, expect = {}, {}
    for c in range(ncol):
        v = rng.integers(0, 2 ** 64, n, dtype=np.uint64).view(np.int64)
        valid = (rng.random(n) >= 0.05) if c % 2 else np.ones(n, dtype=bool)
        if c == 5:
            v[: n // 3] = v[0]  # a column with a heavy duplicate
        name = "c%02d" % c
        cols[name] = d.Column.from_numpy(v, None if valid.all() else valid, "int64")
        expect[name] = O.hll_pack(C.hll_registers("int64", v, None if valid.all() else _bitmap(valid)).tolist())
    table = d.Table(cols).to_device(0)
    an = [d.ApproxCountDistinct(name) for name in cols]
    st = d.run_scan(an, table)
    for a in an:
        assert list(st[a].words) == expect[a.column], a


def test_c3_string_variant_hll(gpu):
    rng = np.random.default_rng(4)
    n, ncol = 120_000, 16
    cols, expect = {}, {}
    for c in range(ncol):
        keys = ["%016x" % x for x in rng.integers(0, 2 ** 64, n, dtype=np.uint64).tolist()]
        valid = rng.random(n) >= 0.05
        col = d.Column.from_pylist([k if ok else None for k, ok in zip(keys, valid)], "string")
        name = "s%02d" % c
        cols[name] = col
        expect[name] = O.hll_pack(C.hll_registers("string", col.values, _bitmap(valid), col.offsets).tolist())
    table = d.Table(cols).to_device(0)
    an = [d.ApproxCountDistinct(name) for name in cols]
    st = d.run_scan(an, table)
    for a in an:
        assert list(st[a].words) == expect[a.column], a


def test_c4_scale_partition_group_by(gpu):
    import torch
    n, key_range = 80_000_000, 201_500_000
    g = torch.Generator(device="cuda").manual_seed(7)
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
    t.consume(d.Table({"key": col}))
    paths = t.paths()
    s = t.summary()
    top_counts, top_keys = t.top(20)

    ids_h, valid_h = ids.cpu().numpy(), valid.cpu().numpy()
    u, c = np.unique(ids_h[valid_h], return_counts=True)
    assert paths["slots"] >= 1 << 28, paths            # >= 2^17 slices
    assert paths["partition_runs"] >= 1, paths
    assert paths["packed_runs"] >= 1, paths            # 12-digit keys: 8-byte records
    assert paths["sort_records"] <= n // 100, paths    # retries only
    assert s.num_rows == n
    assert s.grouped_rows == int(valid_h.sum())
    assert s.num_groups == len(u)
    assert s.num_unique == int((c == 1).sum())
    p = c.astype(np.float64) / n
    ent = float(np.sum(-p * np.log(p)))
    assert abs(s.entropy - ent) <= 1e-12 * ent, (s.entropy, ent)
    order = np.argsort(-c, kind="stable")
    cut = c[order[19]]
    want = {("%012d" % k).encode(): int(v) for k, v in zip(u[c >= cut].tolist(), c[c >= cut].tolist())}
    got = dict(zip(top_keys, top_counts.tolist()))
    assert got == want
    t.close()
