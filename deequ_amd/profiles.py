"""ColumnProfilerRunner / ColumnProfiler -- the reference's three-pass profiler on the GPU path.

Follows `src/main/scala/com/amazon/deequ/profiles/ColumnProfiler.scala` (profile :91-208):

* pass 1 (:115-145, analyzers :220-238): Completeness + ApproxCountDistinct for every column,
  + DataType for string columns without a predefined type, + Size -- ONE AnalysisRunner run,
  i.e. one fused GPU plan (scan, HLL and DataType kernels over each column once).
* pass 2 (:147-173, :240-251): string columns typed Integral / Fractional are cast to
  LongType / DoubleType on the GPU (dq_cast_utf8, Spark 2.2.2 Cast semantics, :346-355,
  :427-445); then Minimum, Maximum, Mean, StandardDeviation and Sum of every numeric column in one
  fused plan.  The reference's KLLSketch (a randomized sketch, :249) is out of scope, so `kll`
  and `approxPercentiles` are None.
* pass 3 (:175-205, :535-606): exact histograms of the low-cardinality columns with the GPU
  group-by (NULL -> "NullValue", values as Java toString), ratio = count / rows (:598-601).

Profiles, `GenericColumnStatistics.typeOf` and the JSON writer follow ColumnProfile.scala and
ColumnProfiler.scala:18-57, 357-424, 658-710.
"""
from __future__ import annotations

import re
import ctypes
import os
import sys
import json
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from . import _lib as L
from .analyzers import (ApproxCountDistinct, Completeness, DataType, DataTypeInstances, Maximum, Mean,
                        Minimum, Size, StandardDeviation, Sum, determine_type)
from .metrics import Distribution, DistributionValue

DEFAULT_CARDINALITY_THRESHOLD = 120  # ColumnProfiler.DEFAULT_CARDINALITY_THRESHOLD (:71)
NULL_FIELD_REPLACEMENT = "NullValue"
_HISTOGRAM_TYPES = ("string", "bool", "float64", "float32", "int32", "int64", "int16")  # :541-543


@dataclass
class StandardColumnProfile:
    """StandardColumnProfile (ColumnProfile.scala:34-42)."""
    column: str
    completeness: float
    approximateNumDistinctValues: int
    dataType: int
    isDataTypeInferred: bool
    typeCounts: Dict[str, int]
    histogram: Optional[Distribution]


@dataclass
class NumericColumnProfile:
    """NumericColumnProfile (ColumnProfile.scala:44-59)."""
    column: str
    completeness: float
    approximateNumDistinctValues: int
    dataType: int
    isDataTypeInferred: bool
    typeCounts: Dict[str, int]
    histogram: Optional[Distribution]
    kll: Optional[object] = None
    mean: Optional[float] = None
    maximum: Optional[float] = None
    minimum: Optional[float] = None
    sum: Optional[float] = None
    stdDev: Optional[float] = None
    approxPercentiles: Optional[List[float]] = None


@dataclass
class ColumnProfiles:
    """ColumnProfiles(profiles, numRecords) (ColumnProfile.scala:61-63)."""
    profiles: Dict[str, object]
    numRecords: int

    @staticmethod
    def toJson(columnProfiles: Sequence[object]) -> str:
        """ColumnProfiles.toJson (ColumnProfile.scala:68-177), including its quirk that the
        built typeCounts object is never attached."""
        cols = []
        for p in columnProfiles:
            j = OrderedDict()
            j["column"] = p.column
            j["dataType"] = DataTypeInstances.name_of(p.dataType)
            j["isDataTypeInferred"] = "true" if p.isDataTypeInferred else "false"
            j["completeness"] = p.completeness
            j["approximateNumDistinctValues"] = p.approximateNumDistinctValues
            if p.histogram is not None:
                j["histogram"] = [OrderedDict([("value", k), ("count", v.absolute), ("ratio", v.ratio)])
                                  for k, v in p.histogram.values.items()]
            if isinstance(p, NumericColumnProfile):
                for name in ("mean", "maximum", "minimum", "sum", "stdDev"):
                    v = getattr(p, name)
                    if v is not None:
                        j[name] = v
                j["approxPercentiles"] = list(p.approxPercentiles or [])
            cols.append(j)
        return json.dumps({"columns": cols}, indent=2)


@dataclass
class GenericColumnStatistics:
    """GenericColumnStatistics (ColumnProfiler.scala:31-46)."""
    numRecords: int
    inferredTypes: Dict[str, int]
    knownTypes: Dict[str, int]
    typeDetectionHistograms: Dict[str, Dict[str, int]]
    approximateNumDistincts: Dict[str, int]
    completenesses: Dict[str, float]
    predefinedTypes: Dict[str, int] = field(default_factory=dict)

    def typeOf(self, column: str) -> int:
        merged = dict(self.inferredTypes)
        merged.update(self.knownTypes)
        merged.update(self.predefinedTypes)
        return merged[column]


def _known_type(dtype: str) -> int:
    """The schema-type mapping of extractGenericStatistics (:401-420); ByteType is not in the
    reference's match and maps to Unknown."""
    if dtype in ("int16", "int32", "int64"):
        return DataTypeInstances.Integral
    if dtype in ("float32", "float64"):
        return DataTypeInstances.Fractional
    if dtype == "bool":
        return DataTypeInstances.Boolean
    return DataTypeInstances.Unknown


def _java_long(x: float) -> int:
    return int(x)  # Double.toLong truncates toward zero


class ColumnProfiler:
    DEFAULT_CARDINALITY_THRESHOLD = DEFAULT_CARDINALITY_THRESHOLD

    @staticmethod
    def profile(data, restrictToColumns: Optional[Sequence[str]] = None, printStatusUpdates: bool = False,
                lowCardinalityHistogramThreshold: int = DEFAULT_CARDINALITY_THRESHOLD,
                kllParameters=None, predefinedTypes: Optional[Dict[str, int]] = None) -> ColumnProfiles:
        # The passes run on up to three host threads that mostly wait inside library calls (no
        # GIL held).  A call that returns while another thread runs Python waits for the GIL for
        # up to the interpreter's switch interval (5 ms by default) -- on the critical path of a
        # 40 ms profile -- so the interval is shortened for the run and restored afterwards
        # (DEEQU_AMD_PROFILE_SWITCH_US, 0 = leave it).
        us = float(os.environ.get("DEEQU_AMD_PROFILE_SWITCH_US", "200"))
        old = sys.getswitchinterval()
        if us > 0:
            sys.setswitchinterval(min(old, us * 1e-6))
        try:
            return ColumnProfiler._profile(data, restrictToColumns, printStatusUpdates,
                                           lowCardinalityHistogramThreshold, kllParameters, predefinedTypes)
        finally:
            sys.setswitchinterval(old)

    @staticmethod
    def _profile(data, restrictToColumns, printStatusUpdates, lowCardinalityHistogramThreshold, kllParameters,
                 predefinedTypes) -> ColumnProfiles:
        from .runner import AnalysisRunner
        predefined = dict(predefinedTypes or {})
        schema = data.schema
        if restrictToColumns is not None:
            for c in restrictToColumns:
                if c not in schema:
                    raise ValueError("requirement failed: Unable to find column %s" % c)
        relevant = [c for c in schema if restrictToColumns is None or c in restrictToColumns]

        if printStatusUpdates:
            print("### PROFILING: Computing generic column statistics in pass (1/3)...")
        # Pass 2's statistics of a column whose type the schema already fixes as numeric (a native
        # int / float column, not predefined otherwise) are known before pass 1 runs and read the
        # same uncast column, so they ride along in pass 1's scan: the column is read once and its
        # statistics and HLL come out of one fused kernel (the states are the same aggregations
        # over the same rows; only string columns typed numeric by pass 1 wait for pass 2's cast).
        numeric_types = (DataTypeInstances.Integral, DataTypeInstances.Fractional)

        def _fixed_numeric(c):
            if schema[c] == "string":
                return False
            t = predefined[c] if c in predefined else _known_type(schema[c])
            return t in numeric_types

        def _stats(c):
            return [Minimum(c), Maximum(c), Mean(c), StandardDeviation(c), Sum(c)]

        early = [c for c in relevant if _fixed_numeric(c)]
        strings = [c for c in relevant if schema[c] == "string" and c not in predefined]

        def _first(cols):
            out = []
            for c in cols:
                out += [Completeness(c), ApproxCountDistinct(c)]
                if c in strings:
                    out.append(DataType(c))
            return out + [a for c in early if c in cols for a in _stats(c)]

        from concurrent.futures import ThreadPoolExecutor
        from .distributed import is_sharded
        from .runner import AnalyzerContext
        overlap = os.environ.get("DEEQU_AMD_PROFILE_SERIAL", "0") != "1"  # (A/B and debugging knob)
        sharded = is_sharded(data)
        casted, few, ctx2_s, bool_hist, few_hist = None, {}, None, {}, {}
        if sharded or not overlap or not strings:
            # one fused pass over every column (over a ShardedTable every pass is collective)
            ctx1 = AnalysisRunner.onData(data).addAnalyzers(_first(relevant)).addAnalyzer(Size()).run()
        else:
            # Pass 1 in three steps.  First every string column is tried as a few-valued column
            # (_few_group_strings): one that fits gets Completeness, ApproxCountDistinct and
            # DataType from its distinct values weighted by their counts -- the same states as
            # the per-row pass -- and, should it become a histogram target, its groups are pass
            # 3's histogram.  Then two plans run side by side: the columns that need no string
            # pass (every non-string column, predefined string columns) on a thread of their own,
            # the other string columns' per-row string pass here.  As soon as the string
            # columns' types are known, pass 2's casts start: they need nothing else from pass 1.
            # (The metrics are those of the one fused pass; only the failure scope of an error
            # inside a plan is the plan's columns.)
            others = [c for c in relevant if c not in strings]
            import threading
            from .engine import LAUNCH_GATE
            gate = threading.Event()
            if os.environ.get("DEEQU_AMD_PROFILE_GATE", "1") == "0":  # (A/B knob)
                gate.set()

            def gated(fn, *args):
                token = LAUNCH_GATE.set(gate)
                try:
                    return fn(*args)
                finally:
                    LAUNCH_GATE.reset(token)
            pool = ThreadPoolExecutor(max_workers=3)
            bools = [c for c in relevant if schema[c] == "bool" and _IDENT.match(c)]
            started = {}

            def start_others():
                # the other plan is planned while the few-groups launch runs (the library call
                # holds no GIL) and launches once the string pass is queued: the few-groups launch
                # is latency-bound and would starve beside its VALU-bound scans
                started["fut"] = pool.submit(gated, lambda: AnalysisRunner.onData(data).addAnalyzers(_first(others))
                                             .addAnalyzer(Size()).run())
                # a boolean column has at most three values, so it is a histogram target unless
                # the threshold is below that: its histogram scan runs beside pass 1, used if so
                started["bool"] = pool.submit(gated, _bool_histograms, data, bools) if bools else None
            try:
                few = _few_group_strings(data, strings, before_launch=start_others)
                if "fut" not in started:
                    start_others()
                fut, fut_bool = started["fut"], started["bool"]
                rest = [c for c in strings if c not in few]
                # the string pass is the head of the critical path (its types -> the casts -> their
                # statistics): it is queued first, the other plan's scans after it
                from .engine import LAUNCH_SIGNAL
                token = LAUNCH_SIGNAL.set(gate)
                try:
                    ctx_s = AnalysisRunner.onData(data).addAnalyzers(_first(rest)).run() if rest else AnalyzerContext()
                finally:
                    LAUNCH_SIGNAL.reset(token)
                    gate.set()
                # the few-valued columns' histograms, built while the casts run
                fut_hist = pool.submit(lambda: {c: g.histogram() for c, g in few.items()}) if few else None
                ctx_s = ctx_s + _few_group_metrics(few)
                gen_s = _extract_generic_statistics(strings, schema, ctx_s, predefined)
                casted = _cast_numeric_string_columns(relevant, data, gen_s)
                # pass 2's statistics of the string columns typed numeric: they need only the casts
                early_s = [a for c in strings if gen_s.typeOf(c) in numeric_types for a in _stats(c)]
                if early_s:
                    ctx2_s = AnalysisRunner.onData(casted).addAnalyzers(early_s).run()
                ctx1 = fut.result() + ctx_s
                if fut_bool is not None:
                    bool_hist = fut_bool.result()
                if fut_hist is not None:
                    few_hist = fut_hist.result()
            finally:
                # every exit path opens the gate: a pass-1 plan already submitted (start_others
                # runs before the few-groups launch) waits on it, and an error raised before the
                # string pass must surface instead of leaving that thread -- and this shutdown --
                # blocked forever
                gate.set()
                pool.shutdown(wait=True, cancel_futures=True)
        generic = _extract_generic_statistics(relevant, schema, ctx1, predefined)

        if printStatusUpdates:
            print("### PROFILING: Computing numeric column statistics in pass (2/3)...")
        # Pass 3 needs only pass 1's results (the inferred types and distinct estimates), so on
        # one device its group-bys run beside pass 2's casts and scan (each on its own streams;
        # the library releases the GIL).  Over a ShardedTable both passes are collective, so
        # they stay in order there.  A pass-2 failure is raised as the sequential run would.
        targets = _find_target_columns_for_histograms(schema, generic, lowCardinalityHistogramThreshold)
        known = {c: few_hist[c] if c in few_hist else few[c].histogram() for c in targets if c in few}
        known.update({c: bool_hist[c] for c in targets if c in bool_hist})
        todo = [c for c in targets if c not in known]
        side = ThreadPoolExecutor(max_workers=1) if overlap and todo and not sharded else None
        if side and printStatusUpdates:
            print("### PROFILING: Computing histograms of low-cardinality columns in pass (3/3), beside pass 2...")
        pending = (side.submit(compute_histograms, data, targets, generic.approximateNumDistincts, known)
                   if side else None)
        try:
            if casted is None:
                casted = _cast_numeric_string_columns(relevant, data, generic)
            second = []
            done = set(ctx2_s.metricMap) if ctx2_s is not None else set()
            for c in relevant:
                if c not in early and generic.typeOf(c) in numeric_types:
                    second += [a for a in _stats(c) if a not in done]
            numeric = _extract_numeric_statistics(ctx1)
            if ctx2_s is not None:
                for k, v in _extract_numeric_statistics(ctx2_s).items():
                    numeric[k].update(v)
            if second:
                ctx2 = AnalysisRunner.onData(casted).addAnalyzers(second).run()
                for k, v in _extract_numeric_statistics(ctx2).items():
                    numeric[k].update(v)
        except BaseException:
            if side:  # raised as the sequential run would, once the histogram pass has stopped:
                # a running pass still launches GPU work, so it is awaited (its own error, if
                # any, is dropped in favour of pass 2's, which the sequential run raises first)
                pending.cancel()
                side.shutdown(wait=True, cancel_futures=True)
            raise

        if printStatusUpdates and not side:
            print("### PROFILING: Computing histograms of low-cardinality columns in pass (3/3)...")
        if side:
            try:
                histograms = pending.result()
            finally:
                side.shutdown(wait=True)
        else:
            histograms = compute_histograms(data, targets, generic.approximateNumDistincts, known)
        return _create_profiles(relevant, generic, numeric, histograms)


class _FewGroups:
    """A string column pass 1 found few-valued (dq_profile_few_strings): its distinct non-NULL
    strings with their counts, its NULL count, and its pass-1 states (Completeness,
    ApproxCountDistinct, DataType) computed from them."""

    def __init__(self, groups: Dict[bytes, int], nulls: int, comp, hll, dtype):
        self.groups, self.nulls = groups, int(nulls)
        self.comp, self.hll, self.dtype = comp, hll, dtype

    def merge(self, other: "_FewGroups") -> "_FewGroups":
        """The union of two batches' results (State.sum of each state; group counts added)."""
        for k, c in other.groups.items():
            self.groups[k] = self.groups.get(k, 0) + c
        self.nulls += other.nulls
        for name in ("comp", "hll", "dtype"):
            out = L.DqState()
            L.check(L.lib().dq_state_merge(getattr(self, name), getattr(other, name), out))
            setattr(self, name, out)
        return self

    def histogram(self) -> Distribution:
        """computeHistograms' distribution (NULL -> "NullValue", merged with that literal)."""
        keys, counts = list(self.groups.keys()), list(self.groups.values())
        if self.nulls:
            keys.append(NULL_FIELD_REPLACEMENT.encode("utf-8"))
            counts.append(self.nulls)
        return _histogram_distribution(counts, keys, "string")


def _few_group_metrics(few: Dict[str, "_FewGroups"]):
    """Pass 1's metrics of the few-valued string columns from their states."""
    from .runner import AnalyzerContext
    out = OrderedDict()
    for c, g in few.items():
        for a, st in ((Completeness(c), g.comp), (ApproxCountDistinct(c), g.hll), (DataType(c), g.dtype)):
            try:
                out[a] = a.metricFromAggregationResult(st, None, None)
            except Exception as e:  # noqa: BLE001
                out[a] = a.toFailureMetric(e)
    return AnalyzerContext(out)


def _few_group_strings(data, columns: Sequence[str], before_launch=None) -> Dict[str, _FewGroups]:
    """Pass 1's string columns tried as few-valued columns, all in one library call per batch
    (dq_profile_few_strings: the few-groups kernel and a merge per column, launches overlapped,
    one wait); a column must fit in every batch.  Not over a ShardedTable (its passes are
    collective) and off with DEEQU_AMD_PROFILE_FEW=0."""
    from .distributed import is_sharded
    if not columns or is_sharded(data) or os.environ.get("DEEQU_AMD_PROFILE_FEW", "1") == "0":
        if before_launch is not None:
            before_launch()
        return {}
    from .arrow import ArrowBatch
    from .engine import current_device
    from .table import Table
    ctx = L.Context.get(current_device())
    import numpy as np
    out: Dict[str, _FewGroups] = {}
    live = list(columns)
    first = True
    for batch in data.batches():
        if not live:
            break
        if isinstance(batch, ArrowBatch):  # zero-copy host view of the record batch
            batch = Table.from_arrow(batch.batch)
        n, rows = len(live), batch.num_rows
        res = (L.DqFewResult * n)()
        counts = np.zeros(n * L.DQ_FEW_MAX_GROUPS, dtype=np.int64)
        keys = np.zeros(n * L.DQ_FEW_MAX_GROUPS * 16, dtype=np.uint8)
        lens = np.zeros(n * L.DQ_FEW_MAX_GROUPS, dtype=np.int32)
        cols = (L.DqColumn * n)(*[batch.columns[c].to_dq() for c in live])
        if before_launch is not None:  # (once: the caller's other threads start here, while the
            before_launch()            # library call below holds no GIL)
            before_launch = None
        L.check(L.lib().dq_profile_few_strings(ctx.handle, n, cols, rows, res, counts.ctypes.data, keys.ctypes.data,
                                               lens.ctypes.data))
        kept = []
        for i, c in enumerate(live):
            r = res[i]
            if not r.ok or (not first and c not in out):
                out.pop(c, None)
                continue
            base = i * L.DQ_FEW_MAX_GROUPS
            raw = keys[base * 16:(base + r.n_groups) * 16].tobytes()
            g = {raw[16 * j:16 * j + int(lens[base + j])]: int(counts[base + j]) for j in range(r.n_groups)}
            got = _FewGroups(g, r.n_nulls, r.completeness, r.hll, r.dtype)
            out[c] = out[c].merge(got) if c in out else got
            kept.append(c)
        live, first = kept, False
    return out


def _extract_generic_statistics(columns, schema, ctx, predefined) -> GenericColumnStatistics:
    """extractGenericStatistics (:357-424)."""
    num_records = None
    inferred, type_counts, approx, completeness = {}, {}, {}, {}
    for a, m in ctx.metricMap.items():
        if isinstance(a, Size):
            num_records = _java_long(m.value.get())
        elif isinstance(a, DataType):
            if a.column in predefined:
                continue
            dist = m.value.get()
            inferred[a.column] = determine_type(dist)
            type_counts[a.column] = {k: v.absolute for k, v in dist.values.items()}
        elif isinstance(a, ApproxCountDistinct):
            approx[a.column] = _java_long(m.value.get())
        elif isinstance(a, Completeness):
            completeness[a.column] = m.value.get()
    known = {c: _known_type(schema[c]) for c in columns if c not in predefined and schema[c] != "string"}
    return GenericColumnStatistics(num_records, inferred, known, type_counts, approx, completeness, predefined)


def cast_string_column(col, to_dtype: str, device: Optional[int] = None):
    """Spark 2.2.2 Cast(StringType -> LongType | DoubleType) of one utf8 column on the GPU
    (dq_cast_utf8); the result is a device-resident column.  Doubles are Java's parseDouble,
    correctly rounded for every input (dq_numparse.h)."""
    import torch
    from .engine import current_device
    from .table import Column
    dev_idx = current_device() if device is None else device
    dev = torch.device("cuda", dev_idx)
    n = col.length
    vals = torch.empty(max(1, n), dtype=torch.int64 if to_dtype == "int64" else torch.float64, device=dev)
    valid = torch.empty((n + 7) // 8 + 8, dtype=torch.uint8, device=dev)
    unsupported = ctypes.c_int64()
    src = col.to_dq()
    L.check(L.lib().dq_cast_utf8(L.Context.get(dev_idx).handle, ctypes.byref(src), n, L.TYPE_CODES[to_dtype],
                                 vals.data_ptr(), valid.data_ptr(), ctypes.byref(unsupported)))
    return Column(to_dtype, n, vals, valid, device=True)


def cast_string_columns(cols, to_dtypes, device: Optional[int] = None):
    """cast_string_column over several columns of one batch in ONE library call
    (dq_cast_utf8_batch: the casts overlap on the device, one wait for all)."""
    import torch
    from .engine import current_device
    from .table import Column
    dev_idx = current_device() if device is None else device
    dev = torch.device("cuda", dev_idx)
    n = len(cols)
    if n == 0:
        return []
    rows = cols[0].length
    if any(c.length != rows for c in cols):
        raise ValueError("cast_string_columns: columns of one batch have one length")
    outs = []
    for t in to_dtypes:
        vals = torch.empty(max(1, rows), dtype=torch.int64 if t == "int64" else torch.float64, device=dev)
        valid = torch.empty((rows + 7) // 8 + 8, dtype=torch.uint8, device=dev)
        outs.append((vals, valid))
    srcs = (L.DqColumn * n)(*[c.to_dq() for c in cols])
    types = (ctypes.c_int32 * n)(*[L.TYPE_CODES[t] for t in to_dtypes])
    vptr = (ctypes.c_void_p * n)(*[v.data_ptr() for v, _ in outs])
    bptr = (ctypes.c_void_p * n)(*[b.data_ptr() for _, b in outs])
    L.check(L.lib().dq_cast_utf8_batch(L.Context.get(dev_idx).handle, n, srcs, rows, types, vptr, bptr))
    return [Column(t, rows, v, b, device=True) for t, (v, b) in zip(to_dtypes, outs)]


def _cast_numeric_string_columns(columns, data, generic):
    """castNumericStringColumns (:427-445): string columns typed Integral -> LongType, Fractional
    -> DoubleType.  (Numeric columns keep their type: the reference's cast of them is value
    preserving and the GPU aggregates every numeric width with Spark's semantics.)"""
    from .table import PartitionedTable, Table
    targets = {}
    for c in columns:
        if data.schema[c] != "string":
            continue
        t = generic.typeOf(c)
        if t == DataTypeInstances.Integral:
            targets[c] = "int64"
        elif t == DataTypeInstances.Fractional:
            targets[c] = "float64"
    if not targets:
        return data
    from .distributed import agree, is_sharded
    if is_sharded(data):  # every rank casts its shard; a failure on any rank fails them all
        local, error = None, None
        try:
            local = _cast_batches(data.local, targets)
        except L.DeequAmdError as e:
            error = e
        agree(error, "the string cast of pass 2", data.group)
        return data.with_local(local)
    return _cast_batches(data, targets)


def _cast_batches(data, targets):
    from .arrow import ArrowBatch
    from .table import PartitionedTable, Table
    parts = []
    for batch in data.batches():
        if isinstance(batch, ArrowBatch):  # zero-copy host view of the record batch
            batch = Table.from_arrow(batch.batch)
        names = [name for name in batch.columns if name in targets]
        casted = dict(zip(names, cast_string_columns([batch.columns[n] for n in names], [targets[n] for n in names])))
        cols = OrderedDict()
        for name, col in batch.columns.items():
            cols[name] = casted.get(name, col)
        parts.append(Table(cols))
    return parts[0] if len(parts) == 1 else PartitionedTable(parts)


def _extract_numeric_statistics(ctx):
    """extractNumericStatistics (:448-528): successful metrics only."""
    out = {"mean": {}, "stdDev": {}, "maximum": {}, "minimum": {}, "sum": {}}
    key = {Mean: "mean", StandardDeviation: "stdDev", Maximum: "maximum", Minimum: "minimum", Sum: "sum"}
    for a, m in ctx.metricMap.items():
        k = key.get(type(a))
        if k is not None and m.value.isSuccess:
            out[k][a.column] = m.value.get()
    return out


def _find_target_columns_for_histograms(schema, generic, threshold) -> List[str]:
    """findTargetColumnsForHistograms (:535-557)."""
    ok_types = (DataTypeInstances.String, DataTypeInstances.Boolean, DataTypeInstances.Integral,
                DataTypeInstances.Fractional)
    return [c for c, count in generic.approximateNumDistincts.items()
            if schema[c] in _HISTOGRAM_TYPES and generic.typeOf(c) in ok_types and count <= threshold]


_IDENT = re.compile(r"^[A-Za-z_][A-Za-z0-9_]*$")


def _bool_histograms(data, columns: Sequence[str]) -> Dict[str, Distribution]:
    """A boolean column has at most three groups ("true", "false", "NullValue"), so its exact
    histogram is three counts: all boolean target columns go through ONE fused scan (Size +
    Completeness + Compliance(c) per column) instead of one group-by per column.  Same
    (value.toString, count) pairs as computeHistograms (:564-606); empty groups do not exist
    in a group-by, so zero counts are dropped."""
    from .analyzers import Completeness, Compliance, Size
    from .engine import run_scan
    size = Size()
    per_col = {c: (Completeness(c), Compliance("histogram %s" % c, c)) for c in columns}
    st = run_scan([size] + [a for pair in per_col.values() for a in pair], data)
    n = st[size].numMatches
    out = {}
    for c, (comp, true_) in per_col.items():
        non_null = st[comp].numMatches if st[comp] is not None else 0
        t = st[true_].numMatches if st[true_] is not None else 0
        counts = {"true": t, "false": non_null - t, NULL_FIELD_REPLACEMENT: n - non_null}
        counts = {k: v for k, v in counts.items() if v > 0}
        total = sum(counts.values())
        out[c] = Distribution({k: DistributionValue(v, v / total) for k, v in sorted(counts.items())},
                              len(counts))
    return out


def compute_histograms(data, target_columns: Sequence[str],
                       expected_groups: Optional[Dict[str, int]] = None,
                       known: Optional[Dict[str, Distribution]] = None) -> Dict[str, Distribution]:
    """computeHistograms (:564-606): exact (column, value.toString) counts, NULL -> "NullValue",
    one GPU group-by per target column; ratio = count / (sum of the column's counts).  `known`:
    histograms already computed (pass 1's few-groups string columns)."""
    from .frequencies import FrequencyTable
    schema = data.schema
    out = dict(known or {})
    target_columns = [c for c in target_columns if c not in out]
    order = [c for c in out]
    bool_cols = [c for c in target_columns if schema[c] == "bool" and _IDENT.match(c)]
    order += bool_cols  # (the boolean columns' histograms first, as computed sequentially)
    from .distributed import is_sharded
    from .engine import current_device
    rest = [c for c in target_columns if c not in bool_cols]
    if bool_cols and (is_sharded(data) or len(rest) <= 1):
        out.update(_bool_histograms(data, bool_cols))
        bool_cols = []
    if is_sharded(data):  # the key-hash exchanged table of the whole dataset (collective, in order)
        from .frequencies import compute_frequencies
        for c in rest:
            counts, keys = compute_frequencies(data, [c], histogram=True).table.export()
            out[c] = _histogram_distribution(counts, keys, schema[c])
        return out
    device = current_device()

    def one(c):
        table = FrequencyTable([c], dict(schema), histogram=True, device=device)
        if expected_groups and c in expected_groups:  # the pass-1 estimate (<= the threshold)
            table.expect_groups(int(expected_groups[c]) + 1)
        try:
            for batch in data.batches():
                table.consume(batch)
            counts, keys = table.export()
        finally:
            table.close()
        return _histogram_distribution(counts, keys, schema[c])

    if len(rest) <= 1:
        for c in rest:
            out[c] = one(c)
        return out
    # Each table has its own HIP stream and the library releases the GIL in every call, so the
    # group-bys of several columns run concurrently on the device (each alone is latency-bound:
    # few groups, LDS pre-aggregation), and beside them the boolean columns' fused scan (its own
    # plan and stream).  Results are per column, so the order does not matter.
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(rest) + (1 if bool_cols else 0), 8)) as ex:
        bools = ex.submit(_bool_histograms, data, bool_cols) if bool_cols else None
        for c, dist in zip(rest, ex.map(one, rest)):
            out[c] = dist
        if bools is not None:
            out.update(bools.result())
    return {c: out[c] for c in order + rest}


def _histogram_distribution(counts, keys, dtype) -> Distribution:
    """(value.toString, count) pairs of one column, ratio = count / sum (:590-602)."""
    from .frequencies import decode_key
    from .javafmt import spark_cast_to_string
    per_value: Dict[str, int] = {}
    for k, n in zip(keys, list(counts)):
        v = decode_key(k, [dtype], histogram=True)[0]
        s = NULL_FIELD_REPLACEMENT if v is None else spark_cast_to_string(v, dtype)
        per_value[s] = per_value.get(s, 0) + int(n)
    total = sum(per_value.values())
    values = {s: DistributionValue(n, n / total) for s, n in sorted(per_value.items())}
    return Distribution(values, len(values))


def _create_profiles(columns, generic, numeric, histograms) -> ColumnProfiles:
    """createProfiles (:658-710)."""
    profiles = OrderedDict()
    for name in columns:
        t = generic.typeOf(name)
        common = dict(column=name, completeness=generic.completenesses[name],
                      approximateNumDistinctValues=generic.approximateNumDistincts[name], dataType=t,
                      isDataTypeInferred=name in generic.inferredTypes,
                      typeCounts=generic.typeDetectionHistograms.get(name, {}),
                      histogram=histograms.get(name))
        if t in (DataTypeInstances.Integral, DataTypeInstances.Fractional):
            profiles[name] = NumericColumnProfile(
                **common, kll=None, mean=numeric["mean"].get(name), maximum=numeric["maximum"].get(name),
                minimum=numeric["minimum"].get(name), sum=numeric["sum"].get(name),
                stdDev=numeric["stdDev"].get(name), approxPercentiles=None)
        else:
            profiles[name] = StandardColumnProfile(**common)
    return ColumnProfiles(profiles, generic.numRecords)


class ColumnProfilerRunner:
    """ColumnProfilerRunner (ColumnProfilerRunner.scala:38-84)."""

    def onData(self, data) -> "ColumnProfilerRunBuilder":
        return ColumnProfilerRunBuilder(data)


class ColumnProfilerRunBuilder:
    """ColumnProfilerRunBuilder (ColumnProfilerRunBuilder.scala:24-157)."""

    def __init__(self, data):
        self.data = data
        self._print = False
        self._threshold = DEFAULT_CARDINALITY_THRESHOLD
        self._restrict = None
        self._kll = None
        self._predefined = {}

    def printStatusUpdates(self, flag: bool) -> "ColumnProfilerRunBuilder":
        self._print = flag
        return self

    def cacheInputs(self, flag: bool) -> "ColumnProfilerRunBuilder":
        return self  # inputs already live in HBM or host memory; nothing to cache

    def withLowCardinalityHistogramThreshold(self, threshold: int) -> "ColumnProfilerRunBuilder":
        self._threshold = threshold
        return self

    def restrictToColumns(self, columns: Sequence[str]) -> "ColumnProfilerRunBuilder":
        self._restrict = list(columns)
        return self

    def setKLLParameters(self, params) -> "ColumnProfilerRunBuilder":
        self._kll = params
        return self

    def setPredefinedTypes(self, types: Dict[str, int]) -> "ColumnProfilerRunBuilder":
        self._predefined = dict(types)
        return self

    def run(self) -> ColumnProfiles:
        return ColumnProfiler.profile(self.data, self._restrict, self._print, self._threshold, self._kll,
                                      self._predefined)
