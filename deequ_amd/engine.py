"""Plan execution over the C-ABI: the replacement for the fused `data.agg(...)` job.

`AnalysisRunner.runScanningAnalyzers` (runners/AnalysisRunner.scala:306-313) concatenates
every scan-shareable analyzer's aggregation columns into ONE Spark job.  Here the same set
of analyzers becomes ONE `dq_plan`; every batch (partition) of the table is consumed by one
fused pass of the gfx950 kernels, and `dq_plan_finish` returns one POD state per analyzer.
"""
from __future__ import annotations

import collections
import contextvars
import ctypes
import os
import threading
from typing import Dict, List, Optional, Sequence

from . import _lib as L
from .predicates import compile_predicate
from .states import State, state_from_dq

_DEVICE: Optional[int] = None


def set_device(device: int) -> None:
    """Select the GPU used by subsequent plans in this process (one process per GPU)."""
    global _DEVICE
    _DEVICE = int(device)


def current_device() -> int:
    if _DEVICE is not None:
        return _DEVICE
    return int(os.environ.get("DEEQU_AMD_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def _pred_array(pred):
    if not pred:
        return None
    code = list(pred)
    arr = (L.DqPredInsn * len(code))()
    for i, (op, arg, i64, f64) in enumerate(code):
        arr[i].opcode, arr[i].arg, arr[i].i64, arr[i].f64 = op, arg, i64, f64
    pool = getattr(pred, "pool", b"")
    return arr, (ctypes.create_string_buffer(pool, max(1, len(pool))) if pool else None), len(pool)


def _fill_pred(dst: L.DqPredicate, packed) -> None:
    arr, pool, n_pool = packed
    dst.code = arr
    dst.n_insns = len(arr)
    if pool is not None:
        dst.strings = ctypes.cast(pool, ctypes.c_void_p)
        dst.strings_len = n_pool


class OpSpec:
    """One dq_op: kind, column index, compiled predicate / where programs."""

    def __init__(self, kind: int, column: int = -1, predicate=None, where=None, column2: int = -1):
        self.kind = kind
        self.column = column
        self.column2 = column2
        self.predicate = _pred_array(predicate)
        self.where = _pred_array(where)

    def fill(self, op: L.DqOp) -> None:
        op.kind = self.kind
        op.column = self.column
        op.column2 = self.column2
        if self.predicate is not None:
            _fill_pred(op.predicate, self.predicate)
        if self.where is not None:
            _fill_pred(op.where, self.where)


PACKED_MAGIC = 0x504F5144  # "DQOP", include/deequ_amd.h


def pack_ops(specs: Sequence[OpSpec]) -> bytes:
    """The analyzer list in the byte layout of dq_plan_create_packed -- what the JVM side's
    GpuPlanEncoder writes into a little-endian ByteBuffer."""
    import struct

    def pred(p):
        if p is None:
            return [], b""
        arr, pool, n_pool = p
        return [(arr[i].opcode, arr[i].arg, arr[i].i64, arr[i].f64) for i in range(len(arr))], \
            (pool.raw[:n_pool] if pool is not None else b"")
    out = [struct.pack("<III", PACKED_MAGIC, 1, len(specs))]
    for s in specs:
        pc, ps = pred(s.predicate)
        wc, ws = pred(s.where)
        out.append(struct.pack("<7i", s.kind, s.column, s.column2, len(pc), len(ps), len(wc), len(ws)))
        out += [struct.pack("<iiqd", *ins) for ins in pc] + [ps]
        out += [struct.pack("<iiqd", *ins) for ins in wc] + [ws]
    return b"".join(out)


_SCHEMA_CACHE: Dict[tuple, tuple] = {}
_SCHEMA_BY_ID: Dict[int, tuple] = {}


def _schema_info(schema: Dict[str, str]):
    """(name -> (index, dtype), dq type codes) of a schema, memoised on its contents: a profiler
    run builds hundreds of ops over the same 100-column schema.  A table's schema dict is fixed,
    so the same dict object is answered by identity (it is kept referenced, so its id stays its
    own) without rebuilding the content key."""
    e = _SCHEMA_BY_ID.get(id(schema))
    if e is not None and e[0] is schema and e[1] == len(schema):
        return e[2]
    key = tuple(schema.items())
    hit = _SCHEMA_CACHE.get(key)
    if hit is None:
        idx = {name: (i, dtype) for i, (name, dtype) in enumerate(schema.items())}
        codes = [L.TYPE_CODES[t] for t in schema.values()]
        hit = (idx, (ctypes.c_int32 * max(1, len(codes)))(*codes))
        if len(_SCHEMA_CACHE) > 256:
            _SCHEMA_CACHE.clear()
        _SCHEMA_CACHE[key] = hit
    if len(_SCHEMA_BY_ID) > 256:
        _SCHEMA_BY_ID.clear()
    _SCHEMA_BY_ID[id(schema)] = (schema, len(schema), hit)
    return hit


def schema_index(schema: Dict[str, str]) -> Dict[str, tuple]:
    return _schema_info(schema)[0]


def op_spec_for(analyzer, schema: Dict[str, str]) -> OpSpec:
    idx = schema_index(schema)
    where = compile_predicate(analyzer.where, idx) if getattr(analyzer, "where", None) else None
    kind = analyzer.DQ_KIND
    if kind == L.DQ_OP_SIZE:
        return OpSpec(kind, -1, None, where)
    if kind == L.DQ_OP_COMPLIANCE:
        return OpSpec(kind, -1, compile_predicate(analyzer.predicate, idx), where)
    if kind == L.DQ_OP_CORRELATION:
        return OpSpec(kind, idx[analyzer.firstColumn][0], None, where, idx[analyzer.secondColumn][0])
    return OpSpec(kind, idx[analyzer.column][0], None, where)


_SUPPORTED: Dict[tuple, bool] = {}


def op_supported(spec: OpSpec, schema: Dict[str, str]) -> None:
    """Raises UnsupportedOnGpu / DeequAmdError if the op is not GPU-eligible.  The answer for an
    op without predicate programs depends only on (kind, column types), so accepted ones are
    remembered: a profiler run checks hundreds of such ops, again on every run."""
    types = _schema_info(schema)[1]
    key = None
    if spec.predicate is None and spec.where is None:
        n = len(schema)
        t1 = types[spec.column] if 0 <= spec.column < n else None
        t2 = types[spec.column2] if 0 <= spec.column2 < n else None
        key = (spec.kind, spec.column, spec.column2, n, t1, t2)
        if key in _SUPPORTED:
            return
    op = L.DqOp()
    spec.fill(op)
    L.check(L.lib().dq_op_supported(ctypes.byref(op), types, len(schema)))
    if key is not None:
        if len(_SUPPORTED) > 65536:
            _SUPPORTED.clear()
        _SUPPORTED[key] = True


class Plan:
    """Owns a dq_plan for a fixed analyzer list and schema; reusable across datasets."""

    def __init__(self, specs: Sequence[OpSpec], schema: Dict[str, str], device: Optional[int] = None):
        self.device = current_device() if device is None else device
        self.ctx = L.Context.get(self.device)
        self.schema = dict(schema)
        self.names = list(schema.keys())
        self.specs = list(specs)  # keep predicate arrays alive
        self.n_ops = len(self.specs)
        ops = (L.DqOp * max(1, self.n_ops))()
        for i, s in enumerate(self.specs):
            s.fill(ops[i])
        types = (ctypes.c_int32 * max(1, len(self.names)))(*[L.TYPE_CODES[schema[n]] for n in self.names])
        h = ctypes.c_void_p()
        L.check(L.lib().dq_plan_create(self.ctx.handle, ops, self.n_ops, types, len(self.names),
                                       ctypes.byref(h)))
        self.handle = h
        self._out = (L.DqState * max(1, self.n_ops))()

    def consume(self, batch) -> None:
        from .arrow import ArrowBatch
        from .table import dq_columns
        if isinstance(batch, ArrowBatch):  # the Arrow C Data Interface entry point
            schema, array = batch.c_structs(self.names)
            L.check(L.lib().dq_plan_consume_arrow(self.handle, ctypes.byref(schema), ctypes.byref(array), 0))
            return
        cols = dq_columns(batch, self.names)
        L.check(L.lib().dq_plan_consume(self.handle, cols, len(self.names), batch.num_rows))

    def finish_raw(self):
        L.check(L.lib().dq_plan_finish(self.handle, self._out, self.n_ops))
        return self._out

    def finish(self) -> List[Optional[State]]:
        out = self.finish_raw()
        for i in range(self.n_ops):  # an op the GPU could not evaluate exactly fails loudly
            L.check(L.lib().dq_plan_op_status(self.handle, i))
        return [state_from_dq(out[i]) for i in range(self.n_ops)]

    def reset(self) -> None:
        L.check(L.lib().dq_plan_reset(self.handle))

    @property
    def stream(self) -> int:
        return L.lib().dq_plan_stream(self.handle) or 0

    def close(self) -> None:
        if getattr(self, "handle", None):
            L.lib().dq_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OpUnsupported:
    """In place of an op's POD state: the batch held input the GPU could not evaluate exactly
    for this op (dq_plan_op_status); the error is raised by fromAggregationResult, so only this
    analyzer fails -- the JNI layer would rerun it on Spark."""

    def __init__(self, error: Exception):
        self.error = error


# A threading.Event the scans of this context wait on before their first launch (LAUNCH_GATE),
# and one they set once their kernels are queued (LAUNCH_SIGNAL): the profiler orders pass 1's
# launches across its threads with them (profiles.py).
LAUNCH_GATE: "contextvars.ContextVar" = contextvars.ContextVar("deequ_amd_launch_gate", default=None)
LAUNCH_SIGNAL: "contextvars.ContextVar" = contextvars.ContextVar("deequ_amd_launch_signal", default=None)


# Idle plans by (device, schema, packed analyzer list): dq_plan_create allocates the plan's
# device state (task table, per-block partials, HLL registers) and a profiler run builds five or
# six plans -- the same ones on every run.  A finished plan goes back here and the next run of the
# same analyzers over the same schema takes it (dq_plan_reset) instead of creating one; each plan
# is used by one thread at a time.  DEEQU_AMD_PLAN_CACHE=0 turns it off.
_PLAN_POOL: "collections.OrderedDict[tuple, List[Plan]]" = collections.OrderedDict()
_PLAN_POOL_LOCK = threading.Lock()
_PLAN_POOL_IDLE = 32  # idle plans kept (least recently returned dropped first)


def _take_plan(specs: Sequence[OpSpec], schema: Dict[str, str]):
    if os.environ.get("DEEQU_AMD_PLAN_CACHE", "1") == "0":
        return Plan(specs, schema), None
    key = (current_device(), tuple(schema.items()), pack_ops(specs))
    plan = None
    with _PLAN_POOL_LOCK:
        idle = _PLAN_POOL.get(key)
        if idle:
            plan = idle.pop()
    if plan is not None:
        try:
            plan.reset()
        except Exception:  # noqa: BLE001 - a plan that cannot be reset is dropped, a fresh one made
            plan.close()
            plan = None
    return (plan if plan is not None else Plan(specs, schema)), key


def _return_plan(plan: "Plan", key) -> None:
    if key is None:
        plan.close()
        return
    drop = []
    with _PLAN_POOL_LOCK:
        _PLAN_POOL.setdefault(key, []).append(plan)
        _PLAN_POOL.move_to_end(key)
        n = sum(len(v) for v in _PLAN_POOL.values())
        while n > _PLAN_POOL_IDLE:
            k, v = next(iter(_PLAN_POOL.items()))
            drop.append(v.pop(0))
            n -= 1
            if not v:
                del _PLAN_POOL[k]
    for p in drop:
        p.close()


def clear_plan_cache() -> None:
    """Releases every idle plan (their device memory)."""
    with _PLAN_POOL_LOCK:
        plans = [p for v in _PLAN_POOL.values() for p in v]
        _PLAN_POOL.clear()
    for p in plans:
        p.close()


def _scan_local(specs: Sequence[OpSpec], data) -> List:
    plan, key = _take_plan(specs, data.schema)
    ok = False
    try:
        gate = LAUNCH_GATE.get()
        if gate is not None:
            gate.wait()
        for batch in data.batches():
            plan.consume(batch)
        signal = LAUNCH_SIGNAL.get()
        if signal is not None:
            signal.set()
        out = plan.finish_raw()
        res = []
        for i in range(plan.n_ops):
            try:
                L.check(L.lib().dq_plan_op_status(plan.handle, i))
                res.append(L.DqState.from_buffer_copy(out[i]))
            except L.DeequAmdError as e:
                res.append(OpUnsupported(e))
        ok = True
        return res
    finally:
        if ok:
            _return_plan(plan, key)  # (the next run of the same analyzers resets and reuses it)
        else:
            plan.close()  # (a failed run's plan may hold a half-consumed batch)


def run_scan_raw(specs: Sequence[OpSpec], data) -> List:
    """One fused GPU pass over every batch of `data` for the given ops; the POD dq_states
    (copies, in op order) for each analyzer's fromAggregationResult, or OpUnsupported.  With a
    ShardedTable every rank scans its shard and the results are those of the whole dataset
    (collective, distributed.merge_scan_results)."""
    from .distributed import is_sharded, merge_scan_results
    if not is_sharded(data):
        return _scan_local(specs, data)
    local, error = None, None
    try:
        local = _scan_local(specs, data.local)
    except Exception as e:  # noqa: BLE001 - reported to every rank before anyone raises
        error = e
    return merge_scan_results(local, error, [s.kind for s in specs], data.group)


def run_scan(analyzers: Sequence, data) -> Dict[object, Optional[State]]:
    """One fused GPU pass over every batch of `data` for all `analyzers` (collective over the
    ranks for a ShardedTable); an op the GPU could not evaluate exactly raises."""
    schema = data.schema
    raw = run_scan_raw([op_spec_for(a, schema) for a in analyzers], data)
    states = []
    for r in raw:
        if isinstance(r, OpUnsupported):
            raise r.error
        states.append(state_from_dq(r))
    return dict(zip(analyzers, states))
