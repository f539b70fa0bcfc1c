"""The Arrow C Data Interface path on the GPU: AnalysisRunner over an ArrowTable consumes every
record batch through dq_plan_consume_arrow / dq_freq_consume_arrow (the entry points a JNI shim
binds).  States must equal the oracle's on the same rows -- including batches
sliced at non-multiple-of-8 offsets (bitmap realignment) and several partitions -- and the
metrics must equal the dq_column (Table) path's."""
import numpy as np
import pyarrow as pa
import pytest

import deequ_amd as d
from helpers import oracle_table
from test_gpu_parity import _check_state

pytestmark = pytest.mark.gpu


def _spec(n, seed):
    rng = np.random.default_rng(seed)
    nul = lambda vals, f=0.1: [None if rng.random() < f else v for v in vals]  # noqa: E731
    return {
        "i64": ["int64", nul([int(x) for x in rng.integers(-10 ** 9, 10 ** 9, n)])],
        "i32": ["int32", nul([int(x) for x in rng.integers(-50, 50, n)])],
        "f64": ["float64", nul([float(x) for x in rng.normal(10, 3, n)])],
        "f32": ["float32", nul([float(np.float32(x)) for x in rng.normal(0, 1, n)])],
        "s": ["string", nul(["k%d" % x for x in rng.integers(0, 300, n)])],
        "b": ["bool", nul([bool(x) for x in rng.integers(0, 2, n)])],
    }


_PA = {"int64": pa.int64(), "int32": pa.int32(), "float64": pa.float64(), "float32": pa.float32(),
       "string": pa.string(), "bool": pa.bool_()}


def _arrow_table(spec, cuts):
    full = pa.record_batch({k: pa.array(v, _PA[t]) for k, (t, v) in spec.items()})
    return d.ArrowTable([full.slice(a, b - a) for a, b in zip(cuts, cuts[1:])])


def _analyzers():
    out = [d.Size(), d.Size("i32 > 0")]
    for c in ("i64", "i32", "f64", "f32"):
        out += [d.Completeness(c), d.Sum(c), d.Mean(c), d.StandardDeviation(c), d.Minimum(c), d.Maximum(c),
                d.ApproxCountDistinct(c), d.Sum(c, "b")]
    out += [d.Completeness("s"), d.ApproxCountDistinct("s"), d.MinLength("s"), d.MaxLength("s"),
            d.Compliance("pos", "i64 >= 0"), d.Compliance("in", "s IN ('k1', 'k2')"), d.Correlation("i64", "f64"),
            d.ApproxCountDistinct("b"), d.Completeness("b")]
    return out


@pytest.mark.parametrize("cuts", [[0, 9001], [0, 3, 1027, 4099, 9001], [5, 13, 8000]])
def test_arrow_batches_match_oracle(gpu, cuts):
    spec = _spec(9001, 21)
    lo, hi = cuts[0], cuts[-1]
    sub = {k: [t, v[lo:hi]] for k, (t, v) in spec.items()}
    ot = oracle_table(sub)
    at = _arrow_table(spec, cuts)
    an = _analyzers()
    st = d.run_scan(an, at)
    for a in an:
        _check_state(a, st[a], ot)


def test_arrow_runner_metrics_equal_table_path(gpu):
    spec = _spec(12000, 4)
    at = _arrow_table(spec, [0, 2500, 7001, 12000])
    table = d.Table.from_pydict({k: (t, v) for k, (t, v) in spec.items()})
    an = _analyzers() + [d.Uniqueness(["s"]), d.Distinctness(["s", "i32"]), d.Entropy("s"), d.CountDistinct(["i32"]),
                         d.Histogram("s"), d.Histogram("b"), d.DataType("s")]
    got = d.AnalysisRunner.onData(at).addAnalyzers(an).run()
    want = d.AnalysisRunner.onData(table).addAnalyzers(an).run()
    for a in an:
        g, w = got.metric(a).value, want.metric(a).value
        assert g.isSuccess and w.isSuccess, (a, g, w)
        gv, wv = g.get(), w.get()
        if isinstance(gv, float) and gv == gv:
            assert abs(gv - wv) <= 1e-12 * max(1.0, abs(wv)), (a, gv, wv)
        else:
            assert gv == wv or (gv != gv and wv != wv), (a, gv, wv)


def test_arrow_type_mismatch_is_invalid(gpu):
    from deequ_amd import _lib as L
    from deequ_amd.engine import Plan, op_spec_for
    schema = {"x": "int64"}
    plan = Plan([op_spec_for(d.Sum("x"), schema)], schema)
    try:
        bad = d.ArrowBatch(pa.record_batch({"x": pa.array([1.0, 2.0], pa.float64())}))
        with pytest.raises(L.DeequAmdError):
            plan.consume(bad)
        plan.consume(d.ArrowBatch(pa.record_batch({"x": pa.array([1, 2, None], pa.int64())})))
        assert plan.finish()[0].sum_value == 3.0
    finally:
        plan.close()
