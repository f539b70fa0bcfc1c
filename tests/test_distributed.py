"""Multi-rank state exchange (deequ_amd/distributed.py) on CPU with gloo, world_size 2.

Each rank holds the states of its own row shard (built here with the oracle, since these CPU
tests run no GPU compute), the ranks all-gather the POD states and fold them in rank order
with dq_state_merge.  The result must equal the states of the whole table: exactly for counts,
int sums, min/max and HLL registers, and as the State.sum formulas prescribe for fp64 moments.
"""
import ctypes
import os
import socket

import pytest
import torch.multiprocessing as mp

import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _to_dq(kind, st):
    import deequ_amd as d
    from deequ_amd import _lib as L
    if st is None:
        s = L.DqState()
        s.kind = kind
        return s
    mapping = {
        L.DQ_OP_SIZE: lambda: d.NumMatches(st.num_matches),
        L.DQ_OP_COMPLETENESS: lambda: d.NumMatchesAndCount(st.num_matches, st.count),
        L.DQ_OP_SUM: lambda: d.SumState(st.sum_),
        L.DQ_OP_MEAN: lambda: d.MeanState(st.sum_, st.count),
        L.DQ_OP_STDDEV: lambda: d.StandardDeviationState(st.n, st.avg, st.m2),
        L.DQ_OP_MINIMUM: lambda: d.MinState(st.min_value),
        L.DQ_OP_MAXIMUM: lambda: d.MaxState(st.max_value),
        L.DQ_OP_APPROX_COUNT_DISTINCT: lambda: d.ApproxCountDistinctState(st.words),
    }
    out = mapping[kind]().to_dq()
    out.kind = kind
    return out


def _states_for(table):
    from deequ_amd import _lib as L
    return [
        (L.DQ_OP_SIZE, O.size_state(table)),
        (L.DQ_OP_COMPLETENESS, O.completeness_state(table, "x")),
        (L.DQ_OP_SUM, O.sum_state(table, "x")),
        (L.DQ_OP_MEAN, O.mean_state(table, "f")),
        (L.DQ_OP_STDDEV, O.stddev_state(table, "f")),
        (L.DQ_OP_MINIMUM, O.min_state(table, "x")),
        (L.DQ_OP_MAXIMUM, O.max_state(table, "f")),
        (L.DQ_OP_APPROX_COUNT_DISTINCT, O.approx_count_distinct_state(table, "x")),
        (L.DQ_OP_SUM, O.sum_state(table, "empty")),  # None on every rank
    ]


def _table(lo, hi):
    xs = [None if i % 7 == 0 else (i * 37) % 1000 - 300 for i in range(lo, hi)]
    fs = [None if i % 11 == 0 else 0.5 * i for i in range(lo, hi)]
    return {"x": O.OColumn("int64", xs), "f": O.OColumn("float64", fs),
            "empty": O.OColumn("int64", [None] * (hi - lo))}


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    from deequ_amd import _lib as L
    from deequ_amd.distributed import allgather_merge
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    n = 3000
    lo, hi = rank * n // world, (rank + 1) * n // world
    local = _states_for(_table(lo, hi))
    arr = (L.DqState * len(local))()
    for i, (kind, st) in enumerate(local):
        arr[i] = _to_dq(kind, st)
    merged = allgather_merge(arr, len(local))
    q.put((rank, bytes(merged)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_merge_equals_whole_table(world):
    from deequ_amd import _lib as L
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = _states_for(_table(0, 3000))
    n_ops = len(whole)
    size = ctypes.sizeof(L.DqState)
    for r in range(world):
        blob = results[r]
        assert blob == results[0]  # every rank holds the same merged states
        for i, (kind, want) in enumerate(whole):
            got = L.DqState.from_buffer_copy(blob, i * size)
            if want is None:
                assert not got.has_value
                continue
            assert got.has_value
            if kind == L.DQ_OP_SIZE:
                assert got.num_matches == want.num_matches
            elif kind == L.DQ_OP_COMPLETENESS:
                assert (got.num_matches, got.count) == (want.num_matches, want.count)
            elif kind == L.DQ_OP_SUM:
                assert got.sum == want.sum_  # integral sum: exact
            elif kind == L.DQ_OP_MEAN:
                assert got.count == want.count and got.sum == pytest.approx(want.sum_, rel=1e-15)
            elif kind == L.DQ_OP_STDDEV:
                assert got.n == want.n
                assert got.avg == pytest.approx(want.avg, rel=1e-13)
                assert got.m2 == pytest.approx(want.m2, rel=1e-12)
            elif kind == L.DQ_OP_MINIMUM:
                assert got.value == want.min_value
            elif kind == L.DQ_OP_MAXIMUM:
                assert got.value == want.max_value
            elif kind == L.DQ_OP_APPROX_COUNT_DISTINCT:
                assert list(got.words) == list(want.words)


@pytest.mark.parametrize("world", [1, 2, 5])
def test_c_abi_rank_fold_equals_whole_table(world):
    """dq_states_merge_ranks -- the fold dq_group_allgather_merge applies after its RCCL
    all-gather -- on the shards' states equals the whole table's states, and the same bytes as
    the torch.distributed route's fold."""
    from deequ_amd import _lib as L
    from deequ_amd.distributed import merge_raw
    from deequ_amd.group import merge_ranks
    n = 3000
    shards = [_states_for(_table(r * n // world, (r + 1) * n // world)) for r in range(world)]
    n_ops = len(shards[0])
    gathered = (L.DqState * (world * n_ops))()
    for r, local in enumerate(shards):
        for i, (kind, st) in enumerate(local):
            gathered[r * n_ops + i] = _to_dq(kind, st)
    out = merge_ranks(gathered, world, n_ops)
    for i in range(n_ops):
        acc = L.DqState.from_buffer_copy(gathered[i])
        for r in range(1, world):
            acc = merge_raw(acc, gathered[r * n_ops + i])
        assert bytes(acc) == bytes(out[i])
    whole = _states_for(_table(0, n))
    for i, (kind, want) in enumerate(whole):
        got = out[i]
        if want is None:
            assert not got.has_value
        elif kind in (L.DQ_OP_SIZE, L.DQ_OP_COMPLETENESS):
            assert (got.num_matches, got.count if kind == L.DQ_OP_COMPLETENESS else 0) == \
                (want.num_matches, want.count if kind == L.DQ_OP_COMPLETENESS else 0)
        elif kind == L.DQ_OP_APPROX_COUNT_DISTINCT:
            assert list(got.words) == list(want.words)
        elif kind == L.DQ_OP_STDDEV:
            assert got.n == want.n and got.m2 == pytest.approx(want.m2, rel=1e-12)
        elif kind in (L.DQ_OP_MINIMUM, L.DQ_OP_MAXIMUM):
            assert got.value == (want.min_value if kind == L.DQ_OP_MINIMUM else want.max_value)


def test_c_abi_rank_fold_rejects_bad_arguments():
    from deequ_amd import _lib as L
    arr = (L.DqState * 2)()
    out = (L.DqState * 2)()
    assert L.lib().dq_states_merge_ranks(arr, 0, 2, out) == L.DQ_ERR_INVALID
    arr[0].kind, arr[1].kind = L.DQ_OP_SUM, L.DQ_OP_MEAN  # kinds differ across ranks
    assert L.lib().dq_states_merge_ranks(arr, 2, 1, out) != L.DQ_OK


def _scope_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    from deequ_amd import _lib as L
    from deequ_amd.distributed import merge_scan_results
    from deequ_amd.engine import OpUnsupported
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    local = _states_for(_table(rank * 100, (rank + 1) * 100))
    kinds = [k for k, _ in local]
    states = [_to_dq(k, st) for k, st in local]
    # rank 1 could not evaluate op 2 on its shard (dq_plan_op_status): that op fails on every
    # rank, the others merge as usual (AnalysisRunner.scala:340-353 over the whole dataset)
    if rank == 1:
        states[2] = OpUnsupported(L.UnsupportedOnGpu(L.DQ_ERR_UNSUPPORTED, "injected"))
    out = merge_scan_results(states, None, kinds)
    q.put((rank, [isinstance(o, OpUnsupported) for o in out]))
    # and an aggregation failure on rank 0 fails every rank (the all-fail scope, :320-323)
    err = None
    try:
        merge_scan_results(None if rank == 0 else states, RuntimeError("boom") if rank == 0 else None, kinds)
    except Exception as e:  # noqa: BLE001
        err = type(e).__name__
    q.put((rank + 100, err))
    dist.barrier()
    dist.destroy_process_group()


def test_failure_scopes_span_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_scope_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2 * world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r][2] and sum(res[r]) == 1, res[r]
    assert res[100] == "RuntimeError" and res[101] == "DeequAmdError"
