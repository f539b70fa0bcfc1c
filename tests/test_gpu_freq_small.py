"""The few-groups group-by (round 4, dq_freq_small_kernel): the profiler's low-cardinality
histograms (ColumnProfiler.scala:564-606, columns with at most 120 distinct values) and any table
hinted with dq_freq_expect_groups.  Per-workgroup LDS counts, staging lists, one merge.  Bit-exact
against the oracle for string keys (NULL as "NullValue" for Histogram) and fixed-width keys (NaN
canonical, NULL as the empty key), into empty and non-empty tables; a wrong hint (too many keys)
and keys longer than 15 bytes fall back to the general path with the same result.  Also: a slot
publish that never comes (a test-only broken publish, dq_diag_freq_test_flags) is a hard error,
never a miscount."""
import math

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd import _lib as L
from deequ_amd.frequencies import FrequencyTable, encode_key
from helpers import oracle_table

pytestmark = pytest.mark.gpu


def _groups(t):
    counts, keys = t.export()
    return dict(zip(keys, counts.tolist()))


def _want(spec, col, hist):
    if hist:
        st = O.histogram_state(oracle_table(spec), col)
        dtype = spec[col][0]
        out = {}
        for (k,), c in st.frequencies.items():
            out[k] = out.get(k, 0) + c
        return out, dtype
    st = O.frequencies_state(oracle_table(spec), [col])
    return {encode_key(list(k), [spec[col][0]]): c for k, c in st.frequencies.items()}, spec[col][0]


def _consume(t, spec, col, batches=2):
    vals = spec[col][1]
    step = (len(vals) + batches - 1) // batches
    for s in range(0, len(vals), step):
        t.consume(d.Table.from_pydict({col: (spec[col][0], vals[s:s + step])}))


@pytest.mark.parametrize("hist", [False, True])
def test_small_strings_match_oracle(gpu, hist):
    rng = np.random.default_rng(4)
    n = 300_000
    a = rng.integers(0, 100, n)
    spec = {"c": ["string", [None if i % 17 == 0 else "cat_%02d" % a[i] for i in range(n)]]}
    t = FrequencyTable(["c"], {"c": "string"}, histogram=hist)
    t.expect_groups(101)
    _consume(t, spec, "c")
    assert t.paths()["small_runs"] == 2
    got = _groups(t)
    if hist:
        want, _ = _want(spec, "c", True)
        assert {k.decode(): v for k, v in got.items()} == want
    else:
        want, _ = _want(spec, "c", False)
        assert got == want
    _consume(t, spec, "c")  # into the non-empty table
    assert sum(_groups(t).values()) == 2 * sum(got.values())
    t.close()


@pytest.mark.parametrize("dtype", ["int64", "int32", "float64", "bool"])
def test_small_fixed_width_histogram(gpu, dtype):
    rng = np.random.default_rng(5)
    n = 200_000
    a = rng.integers(0, 60, n)
    if dtype == "bool":
        vals = [None if i % 13 == 0 else bool(a[i] & 1) for i in range(n)]
    elif dtype == "float64":
        pool = [float(v) / 4 for v in range(57)] + [math.nan, -0.0, math.inf]
        vals = [None if i % 13 == 0 else pool[a[i]] for i in range(n)]
    else:
        vals = [None if i % 13 == 0 else int(a[i]) - 30 for i in range(n)]
    spec = {"x": [dtype, vals]}
    t = FrequencyTable(["x"], {"x": dtype}, histogram=True)
    t.expect_groups(61)
    _consume(t, spec, "x")
    assert t.paths()["small_runs"] == 2
    got = _groups(t)
    want = {}
    for v in vals:
        k = encode_key([v], [dtype], True)
        want[k] = want.get(k, 0) + 1
    assert got == want
    t.close()


def test_small_wrong_hint_falls_back(gpu):
    """5000 distinct keys with a hint of 100 groups: more keys than an LDS table holds -- nothing
    is merged from the few-groups kernel, the batch takes the general path, same result."""
    n = 100_000
    spec = {"c": ["string", ["key%d" % (i % 5000) for i in range(n)]]}
    t = FrequencyTable(["c"], {"c": "string"})
    t.expect_groups(100)
    _consume(t, spec, "c", batches=1)
    assert t.paths()["small_runs"] == 0
    assert _groups(t) == _want(spec, "c", False)[0]
    t.close()


def test_small_long_keys_fall_back(gpu):
    n = 50_000
    spec = {"c": ["string", ["a-key-longer-than-fifteen-%d" % (i % 7) if i % 3 else "short%d" % (i % 5)
                             for i in range(n)]]}
    t = FrequencyTable(["c"], {"c": "string"})
    t.expect_groups(12)
    _consume(t, spec, "c", batches=1)
    assert t.paths()["small_runs"] == 0
    assert _groups(t) == _want(spec, "c", False)[0]
    t.close()


def test_publish_wait_timeout_is_an_error(gpu, monkeypatch):
    """A claimed global slot that never turns READY (dq_diag_freq_test_flags, per-row inserts):
    the lanes waiting on it time out and the batch fails with that error -- it is not reported as
    a full slice and the rows are not regrouped."""
    monkeypatch.setenv("DQ_FREQ_PATH", "atomic")
    n = 60_000
    spec = {"c": ["string", ["k%d" % (i % 6000) for i in range(n)]]}  # > 1024 keys: LDS overflows
    t = FrequencyTable(["c"], {"c": "string"})
    L.check(L.lib().dq_diag_freq_test_flags(t.handle, 1))
    with pytest.raises(L.DeequAmdError, match="timed out"):
        _consume(t, spec, "c", batches=1)
    assert t.paths()["wait_timeouts"] == 1
    t.close()


def test_no_wait_timeouts_in_normal_runs(gpu):
    """Every path's tables report no publish wait timeout (hot keys included)."""
    rng = np.random.default_rng(9)
    n = 400_000
    hot = ["hot"] * (n // 2)
    spec = {"c": ["string", hot + ["k%d" % v for v in rng.integers(0, 50_000, n - len(hot))]]}
    for path in ("atomic", "sorted"):
        import os
        os.environ["DQ_FREQ_PATH"] = path
        try:
            t = FrequencyTable(["c"], {"c": "string"})
            _consume(t, spec, "c", batches=3)
            assert _groups(t) == _want(spec, "c", False)[0]
            assert t.paths()["wait_timeouts"] == 0
            t.close()
        finally:
            del os.environ["DQ_FREQ_PATH"]


def test_group_bys_on_two_threads(gpu):
    """Two group-bys on separate host threads against one device (the profiler runs pass 3 beside
    pass 2 this way): each equals the same group-by run alone."""
    from concurrent.futures import ThreadPoolExecutor
    rng = np.random.default_rng(12)
    n = 300_000
    specs = [{"c": ["string", ["%d" % v for v in rng.integers(0, 90_000, n)]]},
             {"c": ["string", ["cat_%02d" % v for v in rng.integers(0, 80, n)]]}]

    def run(spec, hint):
        t = FrequencyTable(["c"], {"c": "string"}, histogram=True)
        if hint:
            t.expect_groups(hint)
        try:
            _consume(t, spec, "c", batches=4)
            return _groups(t)
        finally:
            t.close()
    serial = [run(specs[0], 0), run(specs[1], 81)]
    for _ in range(3):
        with ThreadPoolExecutor(max_workers=2) as ex:
            futs = [ex.submit(run, specs[0], 0), ex.submit(run, specs[1], 81)]
            assert [f.result() for f in futs] == serial
