"""Pass 1 of the ColumnProfiler on few-valued string columns (round 5): the column is grouped by
the few-groups kernel alone (DQ_FREQ_FEW_ONLY) and its ApproxCountDistinct / DataType states
come from its distinct values weighted by their counts (dq_profile_string_groups).

* The states equal the per-row string pass's bit for bit (HLL registers are maxima; DataType
  counts are sums): StatefulHyperloglogPlus.update / StatefulDataType.update over every row
  (StatefulHyperloglogPlus.scala:89-115, catalyst/StatefulDataType.scala:26-83).
* A column with more distinct values than the kernel holds, or a value longer than 15 bytes,
  fails with DQ_ERR_SPACE (and keeps failing), so the profiler takes the per-row pass.
* Whole profiles are identical with the path on and off (DEEQU_AMD_PROFILE_FEW=0), including
  NULLs, the literal "NullValue", empty strings, and numeric strings cast in pass 2."""
import numpy as np
import pytest

import deequ_amd as d
from deequ_amd import _lib as L
from deequ_amd.frequencies import FrequencyTable
from deequ_amd.profiles import ColumnProfilerRunner
from deequ_amd.states import state_from_dq

pytestmark = pytest.mark.gpu

_VALUES = ["", "true", "false", "+ .5", "- 12", "12", "3.5", "-0", "é", "NullValue", "x" * 15, "0123456789abcde",
           "  ", ".", "1e5", "TRUE"]


def _column(rng, n, values, null_frac=0.07):
    pick = rng.integers(0, len(values), n)
    nulls = rng.random(n) < null_frac
    return [None if z else values[i] for i, z in zip(pick, nulls)]


def _table(cols):
    return d.Table({name: d.Column.from_pylist(v, "string") for name, v in cols.items()}).to_device(0)


def _few_states(table, c):
    t = FrequencyTable([c], dict(table.schema), few_only=True)
    for b in table.batches():
        t.consume(b)
    s = t.summary()
    counts, offs, blob = t.export_flat()
    t.close()
    hll, dt = L.DqState(), L.DqState()
    ctx = L.Context.get(0)
    L.check(L.lib().dq_profile_string_groups(ctx.handle, counts.ctypes.data, offs.ctypes.data,
                                             blob.ctypes.data if len(blob) else None, len(counts),
                                             s.num_rows - s.grouped_rows, 0, hll, dt))
    return state_from_dq(hll), state_from_dq(dt)


@pytest.mark.parametrize("n", [64, 1000, 300_000])
def test_group_states_equal_row_pass(gpu, n):
    rng = np.random.default_rng(n)
    table = _table({"s": _column(rng, n, _VALUES)})
    hll, dt = _few_states(table, "s")
    want_hll = d.ApproxCountDistinct("s").computeStateFrom(table)
    want_dt = d.DataType("s").computeStateFrom(table)
    assert hll.words == want_hll.words
    assert tuple(dt.counts()) == tuple(want_dt.counts())


def test_group_states_device_buffers(gpu):
    """The same call on device tensors (DQ_FLAT_DEVICE)."""
    rng = np.random.default_rng(7)
    table = _table({"s": _column(rng, 50_000, _VALUES)})
    t = FrequencyTable(["s"], dict(table.schema), few_only=True)
    for b in table.batches():
        t.consume(b)
    s = t.summary()
    counts, offs, blob = t.export_flat(device=True)
    t.close()
    hll, dt = L.DqState(), L.DqState()
    L.check(L.lib().dq_profile_string_groups(L.Context.get(0).handle, counts.data_ptr(), offs.data_ptr(),
                                             blob.data_ptr(), counts.numel(), s.num_rows - s.grouped_rows,
                                             L.DQ_FLAT_DEVICE, hll, dt))
    assert state_from_dq(hll).words == d.ApproxCountDistinct("s").computeStateFrom(table).words
    assert tuple(state_from_dq(dt).counts()) == tuple(d.DataType("s").computeStateFrom(table).counts())


@pytest.mark.parametrize("kind", ["many", "long", "tiny_heap"])
def test_few_only_refuses(gpu, kind):
    n = 100_000
    if kind == "many":
        vals = ["k%d" % i for i in range(n)]
    elif kind == "long":
        vals = ["a", "b", "c" * 16] * (n // 3)
    else:  # a string heap under 16 bytes: the kernel's 16-byte key loads need one
        vals = ["ab", None, "c"]
    table = _table({"s": vals})
    t = FrequencyTable(["s"], dict(table.schema), few_only=True)
    with pytest.raises(L.DeequAmdError) as e:
        for b in table.batches():
            t.consume(b)
    assert e.value.status == L.DQ_ERR_SPACE
    with pytest.raises(L.DeequAmdError) as e2:  # and every later batch
        t.consume(next(iter(table.batches())))
    assert e2.value.status == L.DQ_ERR_SPACE
    t.close()


def _batched_few(table, names):
    """dq_profile_few_strings over one batch: {column: (ok, groups, nulls, states)}."""
    batch = next(iter(table.batches()))
    n = len(names)
    res = (L.DqFewResult * n)()
    counts = np.zeros(n * L.DQ_FEW_MAX_GROUPS, dtype=np.int64)
    keys = np.zeros(n * L.DQ_FEW_MAX_GROUPS * 16, dtype=np.uint8)
    lens = np.zeros(n * L.DQ_FEW_MAX_GROUPS, dtype=np.int32)
    cols = (L.DqColumn * n)(*[batch.columns[c].to_dq() for c in names])
    L.check(L.lib().dq_profile_few_strings(L.Context.get(0).handle, n, cols, batch.num_rows, res, counts.ctypes.data,
                                           keys.ctypes.data, lens.ctypes.data))
    out = {}
    for i, c in enumerate(names):
        r = res[i]
        base = i * L.DQ_FEW_MAX_GROUPS
        groups = {keys[(base + j) * 16:(base + j) * 16 + lens[base + j]].tobytes(): int(counts[base + j])
                  for j in range(r.n_groups)}
        out[c] = (r.ok, groups, r.n_nulls, state_from_dq(r.completeness) if r.ok else None,
                  state_from_dq(r.hll) if r.ok else None, state_from_dq(r.dtype) if r.ok else None)
    return out


def test_batched_few_strings(gpu):
    """Several columns in one call: the ones that fit give the per-row pass's states and the
    exact groups; the others (too many values, too long, tiny heap) report ok = 0."""
    rng = np.random.default_rng(5)
    n = 200_000
    cols = {"a": _column(rng, n, _VALUES), "b": _column(rng, n, ["x", "yy", "zzz"], null_frac=0.5),
            "many": ["k%d" % i for i in range(n)], "long": _column(rng, n, ["a" * 16, "b"]),
            "c": _column(rng, n, ["NullValue", "", "1.5"])}
    table = _table(cols)
    got = _batched_few(table, list(cols))
    for c in ("a", "b", "c"):
        ok, groups, nulls, comp, hll, dt = got[c]
        assert ok == 1, c
        want = {}
        for v in cols[c]:
            if v is not None:
                k = v.encode("utf-8")
                want[k] = want.get(k, 0) + 1
        assert groups == want, c
        assert nulls == sum(v is None for v in cols[c])
        assert hll.words == d.ApproxCountDistinct(c).computeStateFrom(table).words
        assert tuple(dt.counts()) == tuple(d.DataType(c).computeStateFrom(table).counts())
        want_comp = d.Completeness(c).computeStateFrom(table)
        assert (comp.numMatches, comp.count) == (want_comp.numMatches, want_comp.count)
    assert got["many"][0] == 0 and got["long"][0] == 0


def _profile_json(table, monkeypatch, few: bool):
    monkeypatch.setenv("DEEQU_AMD_PROFILE_FEW", "1" if few else "0")
    return ColumnProfilerRunner().onData(table).run()


def test_profiles_equal_with_and_without(gpu, monkeypatch):
    rng = np.random.default_rng(11)
    n = 400_000
    cols = {
        "mixed": _column(rng, n, _VALUES),
        "ints": _column(rng, n, ["1", "-7", "12", "+3", "0"]),          # Integral: cast in pass 2
        "fracs": _column(rng, n, ["1.5", "-0.25", "3", ".5", "2."]),    # Fractional
        "bools": _column(rng, n, ["true", "false"], null_frac=0.0),
        "many": ["id%07d" % i for i in rng.permutation(n)],              # too many values: row pass
        "long": _column(rng, n, ["a" * 20, "b" * 17, "short"]),          # too long: row pass
        "nullish": _column(rng, n, ["NullValue", "x"], null_frac=0.3),
    }
    table = _table(cols)
    on = _profile_json(table, monkeypatch, True)
    off = _profile_json(table, monkeypatch, False)
    for c in cols:
        a, b = on.profiles[c], off.profiles[c]
        assert a == b, c


def test_wide_table_chunks(gpu):
    """More string columns than one library chunk (32): every column comes back, each chunk's
    columns with the per-row pass's states (bounded scratch per call)."""
    rng = np.random.default_rng(17)
    n = 20_000
    cols = {"c%02d" % k: _column(rng, n, _VALUES[:3 + k % 10]) for k in range(70)}
    cols["c05"] = ["k%d" % i for i in range(n)]  # one that does not fit, in the first chunk
    table = _table(cols)
    got = _batched_few(table, list(cols))
    for c, vals in cols.items():
        ok, groups, nulls, comp, hll, dt = got[c]
        if c == "c05":
            assert ok == 0
            continue
        assert ok == 1, c
        assert sum(groups.values()) + nulls == n
        assert hll.words == d.ApproxCountDistinct(c).computeStateFrom(table).words, c


def test_profiler_raises_when_few_groups_fail(gpu, monkeypatch):
    """An error in the few-groups step (after the other pass-1 plan was submitted, gated) is
    raised by the profiler, not turned into a hang."""
    import threading
    import deequ_amd.profiles as P

    def boom(data, columns, before_launch=None):
        if before_launch is not None:
            before_launch()
        raise RuntimeError("injected few-groups failure")
    monkeypatch.setattr(P, "_few_group_strings", boom)
    rng = np.random.default_rng(3)
    n = 10_000
    table = d.Table({"s": d.Column.from_pylist(_column(rng, n, _VALUES), "string"),
                     "i": d.Column.from_numpy(rng.integers(0, 9, n))}).to_device(0)
    done = threading.Event()
    result = {}

    def run():
        try:
            ColumnProfilerRunner().onData(table).run()
        except BaseException as e:  # noqa: BLE001
            result["e"] = e
        finally:
            done.set()
    th = threading.Thread(target=run, daemon=True)
    th.start()
    assert done.wait(60), "the profiler hung after a few-groups failure"
    assert isinstance(result.get("e"), RuntimeError) and "injected" in str(result["e"])
