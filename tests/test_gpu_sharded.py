"""The sharded path end to end on the GPU: AnalysisRunner and ColumnProfiler over a ShardedTable
(deequ_amd.distributed) with 2 ranks -- gloo for the collectives, both ranks on cuda:0 (the
one-GPU box cannot run RCCL between two ranks on one device) -- must give the metrics of the
whole table computed by one rank: counts, HLL, min/max, frequency metrics and histograms
exactly, fp64 sums and moments within 1e-12 (the rank-ordered State.sum merge reorders them).
A string -> double cast of a long-digit number held by one rank's shard agrees across ranks
(the per-op failure scope itself is tested on CPU, test_distributed.py).
Also: the C-ABI's RCCL group (dq_group_*) at world size 1 on the real device, and the nccl
backend with 2 ranks when the box has 2 GPUs."""
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 24000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spec(lo, hi, bad_rank_rows=None):
    rng = np.random.default_rng(8)
    nul = lambda vals, f=0.07: [None if rng.random() < f else v for v in vals]  # noqa: E731
    spec = {
        "i": ["int64", nul([int(x) for x in rng.integers(-10 ** 6, 10 ** 6, N)])],
        "f": ["float64", nul([float(x) for x in rng.normal(50, 7, N)])],
        "k": ["string", nul(["key%d" % x for x in rng.integers(0, 700, N)])],
        "n": ["string", nul([str(int(x)) for x in rng.integers(0, 90, N)])],
        "c": ["int32", nul([int(x) for x in rng.integers(0, 12, N)])],
        "b": ["bool", nul([bool(x) for x in rng.integers(0, 2, N)])],
    }
    if bad_rank_rows is not None:  # a number off Clinger's fast path, in one shard only
        spec["n"][1][bad_rank_rows] = "1234567890123456789012345"
    return {k: [t, v[lo:hi]] for k, (t, v) in spec.items()}


def _analyzers(d):
    out = [d.Size(), d.Size("c > 5"), d.Compliance("cast", "n > 40")]
    for c in ("i", "f"):
        out += [d.Completeness(c), d.Sum(c), d.Mean(c), d.StandardDeviation(c), d.Minimum(c), d.Maximum(c),
                d.ApproxCountDistinct(c), d.Sum(c, "b")]
    out += [d.ApproxCountDistinct("k"), d.DataType("n"), d.MaxLength("k"), d.Correlation("i", "f"),
            d.Uniqueness(["k"]), d.Distinctness(["k", "c"]), d.Entropy("k"), d.CountDistinct(["c"]),
            d.UniqueValueRatio(["k"]), d.Histogram("c"), d.Histogram("k", maxDetailBins=20), d.Histogram("b")]
    return out


def _metric_values(ctx, analyzers):
    out = {}
    for a in analyzers:
        v = ctx.metric(a).value
        if not v.isSuccess:
            out[str(a)] = ("failure", type(v.exception).__name__)
            continue
        g = v.get()
        if hasattr(g, "values"):  # Distribution
            g = (g.numberOfBins, sorted((k, x.absolute, x.ratio) for k, x in g.values.items()))
        out[str(a)] = g
    return out


def _profile_values(profiles):
    out = {}
    for name, p in profiles.profiles.items():
        out[name] = {k: (None if getattr(p, k, None) is None else
                         (p.histogram.numberOfBins, sorted((h, x.absolute, x.ratio) for h, x in p.histogram.values.items()))
                         if k == "histogram" else getattr(p, k))
                     for k in ("completeness", "approximateNumDistinctValues", "dataType", "isDataTypeInferred",
                               "typeCounts", "histogram", "mean", "maximum", "minimum", "sum", "stdDev")}
    return out, profiles.numRecords


def _worker(rank, world, port, q, bad_rank):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import deequ_amd as d
    from deequ_amd.distributed import ShardedTable
    from deequ_amd.profiles import ColumnProfilerRunner
    d.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    lo, hi = rank * N // world, (rank + 1) * N // world
    bad = (N // world + 5) if bad_rank else None  # row in rank 1's shard
    shard = d.Table.from_pydict({k: (t, v) for k, (t, v) in _spec(lo, hi, bad).items()})
    data = ShardedTable(shard)
    an = _analyzers(d)
    res = {"metrics": _metric_values(d.AnalysisRunner.onData(data).addAnalyzers(an).run(), an),
           "count": data.global_count()}
    if not bad_rank:
        res["profile"] = _profile_values(ColumnProfilerRunner().onData(data).run())
    if rank == 0:  # the reference result: the whole table on one rank, no collectives
        whole = d.Table.from_pydict({k: (t, v) for k, (t, v) in _spec(0, N, bad).items()})
        res["whole"] = _metric_values(d.AnalysisRunner.onData(whole).addAnalyzers(an).run(), an)
        if not bad_rank:
            res["whole_profile"] = _profile_values(ColumnProfilerRunner().onData(whole).run())
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def _close(got, want):
    if isinstance(want, float) and isinstance(got, float):
        if math.isnan(want):
            return math.isnan(got)
        return abs(got - want) <= 1e-12 * max(1.0, abs(want))
    return got == want


def _run(world, bad_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, bad_rank)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return results


def _oracle_metrics(d):
    """The oracle's metric of every analyzer with an oracle restatement, over the whole table."""
    from helpers import oracle_metric, oracle_state, oracle_table
    ot = oracle_table(_spec(0, N))
    out = {}
    for a in _analyzers(d):
        name = type(a).__name__
        if name in ("Size",):
            args = [a.where]
        elif name == "Compliance":
            args = [a.instance_name, a.predicate, a.where]
        elif name == "Correlation":
            args = [a.firstColumn, a.secondColumn, a.where]
        elif name == "Entropy":
            args = [a.column]
        elif name in ("Uniqueness", "Distinctness", "CountDistinct", "UniqueValueRatio"):
            args = [list(a.columns)]
        elif name in ("Histogram", "DataType"):
            continue
        else:
            args = [a.column, a.where]
        out[str(a)] = oracle_metric(oracle_state(name, args, ot), name, args)
    return out


def test_sharded_runner_and_profiler_equal_whole_table(gpu):
    import deequ_amd as d
    res = _run(2, False)
    whole = res[0]["whole"]
    # the sharded result against the ORACLE too, not only against the one-rank GPU run
    for name, want in _oracle_metrics(d).items():
        got = res[0]["metrics"][name]
        if want == "failure":
            assert got[0] == "failure", (name, got)
        else:
            assert _close(got, want), (name, got, want)
    for r in (0, 1):
        assert res[r]["count"] == N
        assert res[r]["metrics"] == res[0]["metrics"]  # every rank holds the same metrics
        for name, want in whole.items():
            got = res[r]["metrics"][name]
            assert _close(got, want), (name, got, want)
    (wp, wn), (gp, gn) = res[0]["whole_profile"], res[1]["profile"]
    assert gn == wn == N
    for col, fields in wp.items():
        for k, want in fields.items():
            assert _close(gp[col][k], want), (col, k, gp[col][k], want)


def test_sharded_long_digit_cast_agrees(gpu):
    """`n > 40` casts strings to double; rank 1's shard holds a 25-digit number (Eisel-Lemire on
    the device): every rank gets the whole table's metric, and so does one rank alone."""
    res = _run(2, True)
    for r in (0, 1):
        m = res[r]["metrics"]
        assert not isinstance(m["Compliance(cast,n > 40,None)"], tuple), m["Compliance(cast,n > 40,None)"]
        assert m["Compliance(cast,n > 40,None)"] == res[0]["whole"]["Compliance(cast,n > 40,None)"]
        assert m["Size(None)"] == float(N)


def test_c_abi_group_world_one(gpu):
    """dq_group over RCCL on the real device (world size 1: the box has one GPU): the fold leaves
    the states unchanged, the exchange hands the whole table to its only owner, and the summary
    equals the table's own."""
    import deequ_amd as d
    from deequ_amd.engine import Plan, op_spec_for
    from deequ_amd.frequencies import FrequencyTable
    from deequ_amd.group import DqGroup, unique_id
    spec = _spec(0, N)
    table = d.Table.from_pydict({k: (t, v) for k, (t, v) in spec.items()})
    g = DqGroup(1, 0, unique_id())
    try:
        an = [a for a in _analyzers(d) if hasattr(a, "DQ_KIND") and a.DQ_KIND]
        plan = Plan([op_spec_for(a, table.schema) for a in an], table.schema)
        try:
            plan.consume(table)
            raw = plan.finish_raw()
            before = bytes(raw)
            g.allgather_merge(raw, len(an))
            assert bytes(raw) == before
        finally:
            plan.close()
        local = FrequencyTable(["k"], dict(table.schema))
        local.consume(table)
        owned, rows = g.freq_exchange(local)
        assert rows == N
        s_own, s_loc = g.freq_summary(owned, rows), local.summary()
        for f in ("num_rows", "num_groups", "num_unique", "grouped_rows", "entropy"):
            assert getattr(s_own, f) == getattr(s_loc, f), f
        counts, keys = owned.export()
        c2, k2 = local.export()
        assert dict(zip(keys, counts.tolist())) == dict(zip(k2, c2.tolist()))
        tc, tk = g.freq_top(owned, 7)
        lc, lk = local.top(7)
        assert tc.tolist() == lc.tolist() and tk == lk
        local.close()
        owned.close()
    finally:
        g.close()


def _nccl_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist
    import deequ_amd as d
    from deequ_amd.distributed import ShardedTable
    torch.cuda.set_device(rank)
    d.set_device(rank)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world,
                            device_id=torch.device("cuda", rank))
    lo, hi = rank * N // world, (rank + 1) * N // world
    shard = d.Table.from_pydict({k: (t, v) for k, (t, v) in _spec(lo, hi).items()})
    an = _analyzers(d)
    q.put((rank, _metric_values(d.AnalysisRunner.onData(ShardedTable(shard)).addAnalyzers(an).run(), an)))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_runner_over_rccl(gpu):
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("the nccl (RCCL) backend needs one GPU per rank; this box has %d" % torch.cuda.device_count())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_nccl_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert results[0] == results[1]
    import deequ_amd as d
    whole = d.Table.from_pydict({k: (t, v) for k, (t, v) in _spec(0, N).items()})
    an = _analyzers(d)
    want = _metric_values(d.AnalysisRunner.onData(whole).addAnalyzers(an).run(), an)
    for name, w in want.items():
        assert _close(results[0][name], w), (name, results[0][name], w)
