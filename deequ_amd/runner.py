"""AnalysisRunner / AnalyzerContext / state providers -- the reference's runner on the GPU path.

Follows `runners/AnalysisRunner.scala`:
* doAnalysisRun (:97-203): de-duplicate, schema-only precondition failures (:137-145,
  :242-257), scan-shareable analyzers in ONE fused pass (:289-336) with the same failure
  scoping (an aggregation error fails every shareable analyzer :320-323, an extraction error
  fails one :340-353), then the non-shareable ones.
* runOnAggregatedStates (:385-460): metrics from persisted states only, no data scan.
Plus `AnalyzerContext` (AnalyzerContext.scala:29-105) and `InMemoryStateProvider`
(StateProvider.scala:47-70).
"""
from __future__ import annotations

import json
import math
import threading
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence

from . import _lib as L
from .analyzers import Analyzer, Preconditions, ScanShareableAnalyzer
from .metrics import DoubleMetric, Entity


class AnalyzerContext:
    def __init__(self, metricMap: Optional[Dict[Analyzer, object]] = None):
        self.metricMap = OrderedDict(metricMap or {})

    @staticmethod
    def empty() -> "AnalyzerContext":
        return AnalyzerContext()

    def allMetrics(self) -> List:
        return list(self.metricMap.values())

    def metric(self, analyzer) -> Optional[object]:
        return self.metricMap.get(analyzer)

    def __add__(self, other: "AnalyzerContext") -> "AnalyzerContext":
        m = OrderedDict(self.metricMap)
        m.update(other.metricMap)
        return AnalyzerContext(m)

    def successMetricsAsJson(self, forAnalyzers: Sequence[Analyzer] = ()) -> str:
        """AnalyzerContext.successMetricsAsJson (AnalyzerContext.scala:61-76)."""
        rows = []
        for analyzer, metric in self.metricMap.items():
            if forAnalyzers and analyzer not in forAnalyzers:
                continue
            for m in metric.flatten():
                if m.value.isSuccess:
                    rows.append(OrderedDict([("entity", m.entity.value), ("instance", m.instance),
                                             ("name", m.name), ("value", m.value.get())]))
        return json.dumps(rows)


class InMemoryStateProvider:
    """StateLoader + StatePersister backed by a dict (StateProvider.scala:47-70)."""

    def __init__(self):
        self._states = {}
        self._lock = threading.Lock()

    def load(self, analyzer):
        with self._lock:
            return self._states.get(analyzer)

    def persist(self, analyzer, state) -> None:
        with self._lock:
            self._states[analyzer] = state

    def __str__(self):
        return "InMemoryStateProvider(%s)" % ", ".join("%s -> %r" % kv for kv in self._states.items())


def _distinct(analyzers: Iterable[Analyzer]) -> List[Analyzer]:
    seen, out = set(), []
    for a in analyzers:
        if a not in seen:
            seen.add(a)
            out.append(a)
    return out


class AnalysisRunner:
    @staticmethod
    def onData(data) -> "AnalysisRunBuilder":
        return AnalysisRunBuilder(data)

    @staticmethod
    def run(data, analysis: "Analysis", aggregateWith=None, saveStatesWith=None) -> AnalyzerContext:
        return AnalysisRunner.doAnalysisRun(data, analysis.analyzers, aggregateWith, saveStatesWith)

    @staticmethod
    def doAnalysisRun(data, analyzers: Sequence[Analyzer], aggregateWith=None,
                      saveStatesWith=None) -> AnalyzerContext:
        analyzers = _distinct(analyzers)
        if not analyzers:
            return AnalyzerContext.empty()
        schema = data.schema
        passed, failed = [], OrderedDict()
        for a in analyzers:
            err = Preconditions.findFirstFailing(schema, a.preconditions())
            if err is None:
                passed.append(a)
            else:
                failed[a] = a.toFailureMetric(err)
        ctx = AnalyzerContext(failed)
        ctx = ctx + AnalysisRunner._runScanningAnalyzers(data, passed, aggregateWith, saveStatesWith)
        # keep the caller's order
        return AnalyzerContext(OrderedDict((a, ctx.metricMap[a]) for a in analyzers if a in ctx.metricMap))

    @staticmethod
    def _runGroupingAnalyzers(data, analyzers, aggregateWith, saveStatesWith, states_out=None) -> AnalyzerContext:
        """One GPU group-by per sorted grouping-column set (AnalysisRunner.scala:172-186,
        259-287), metrics of all analyzers of that grouping from the one table (:480-548)."""
        from .frequencies import compute_frequencies
        from .states import merge
        groups = OrderedDict()
        for a in analyzers:
            groups.setdefault(tuple(sorted(a.groupingColumns())), []).append(a)
        results = OrderedDict()
        for cols, group in groups.items():
            try:
                state = compute_frequencies(data, list(cols))
                if aggregateWith is not None:
                    state = merge(state, aggregateWith.load(group[0]))
            except Exception as e:  # noqa: BLE001 - the group-by itself failed
                for a in group:
                    results[a] = a.toFailureMetric(e)
                continue
            for a in group:
                try:
                    results[a] = a.computeMetricFrom(state)
                except Exception as e:  # noqa: BLE001 (:517-520, :528-531)
                    results[a] = a.toFailureMetric(e)
            if saveStatesWith is not None:
                saveStatesWith.persist(group[0], state)
            if states_out is not None:
                states_out[cols] = state
        return AnalyzerContext(results)

    @staticmethod
    def _runScanningAnalyzers(data, analyzers, aggregateWith, saveStatesWith) -> AnalyzerContext:
        from .analyzers import GroupingAnalyzer
        from .engine import op_spec_for, op_supported, run_scan_raw
        shareable = [a for a in analyzers if isinstance(a, ScanShareableAnalyzer)]
        grouping = [a for a in analyzers if isinstance(a, GroupingAnalyzer)]
        others = [a for a in analyzers if not isinstance(a, (ScanShareableAnalyzer, GroupingAnalyzer))]
        results = OrderedDict()
        # GPU eligibility is decided per analyzer at plan time (the reference's JNI shim
        # would leave an ineligible analyzer on Spark; here it becomes a failure metric)
        eligible = []
        for a in shareable:
            try:
                op_supported(op_spec_for(a, data.schema), data.schema)
                eligible.append(a)
            except Exception as e:  # noqa: BLE001
                results[a] = a.toFailureMetric(e)
        if eligible:
            try:  # AnalysisRunner.scala:305-323: one fused pass; any error fails them all
                raw = run_scan_raw([a.aggregationFunctions(data.schema) for a in eligible], data)
                for i, a in enumerate(eligible):
                    try:  # successOrFailureMetricFrom (:340-353): an error fails this one
                        results[a] = a.metricFromAggregationResult(raw[i], aggregateWith, saveStatesWith)
                    except Exception as e:  # noqa: BLE001
                        results[a] = a.toFailureMetric(e)
            except Exception as e:  # noqa: BLE001
                for a in eligible:
                    results[a] = a.toFailureMetric(e)
        tables = OrderedDict()
        if grouping:
            results.update(AnalysisRunner._runGroupingAnalyzers(
                data, grouping, aggregateWith, saveStatesWith, tables).metricMap)
        for a in others:
            shared = AnalysisRunner._sharedFrequencies(a, data.schema, tables, aggregateWith, saveStatesWith)
            if shared is not None:
                results[a] = a.metricFromFrequencies(shared)
            else:
                results[a] = a.calculate(data, aggregateWith, saveStatesWith)
        return AnalyzerContext(results)

    @staticmethod
    def _sharedFrequencies(analyzer, schema, tables, aggregateWith, saveStatesWith):
        """A Histogram (no binning UDF, no state loading/saving: its persisted state has its own
        form) whose column was just grouped by a frequency analyzer reuses that table instead of
        running a second group-by over the data (the reference runs a separate Spark job)."""
        from .analyzers import Histogram
        if not isinstance(analyzer, Histogram) or analyzer.binningUdf is not None:
            return None
        if aggregateWith is not None or saveStatesWith is not None:
            return None
        if schema.get(analyzer.column) not in Histogram.SHARES_FREQUENCIES:
            return None
        return tables.get((analyzer.column,))

    @staticmethod
    def runOnAggregatedStates(schema: Dict[str, str], analysis: "Analysis", stateLoaders,
                              saveStatesWith=None) -> AnalyzerContext:
        """Metrics from the merge of persisted states, no data scan (AnalysisRunner.scala:385-460):
        every analyzer's states are summed over the loaders (aggregateStateTo, Analyzer.scala:
        130-147); scanning analyzers compute their metric from that; grouping analyzers of one
        grouping-column set share the one frequency state any of them has (only the first of a
        set is persisted, :543; findStateForParticularGrouping, :462-476)."""
        from .analyzers import GroupingAnalyzer
        from .states import merge
        analyzers = _distinct(analysis.analyzers)
        if not analyzers or not stateLoaders:
            return AnalyzerContext.empty()
        results = OrderedDict()
        passed = []
        for a in analyzers:
            err = Preconditions.findFirstFailing(schema, a.preconditions())
            if err is not None:
                results[a] = a.toFailureMetric(err)
            else:
                passed.append(a)
        aggregated = {}
        for a in passed:
            try:
                state = None
                for loader in stateLoaders:
                    state = merge(loader.load(a), state)
                aggregated[a] = state
            except Exception as e:  # noqa: BLE001
                results[a] = a.toFailureMetric(e)
        grouping = OrderedDict()
        for a in passed:
            if a in results:
                continue
            if isinstance(a, GroupingAnalyzer):
                grouping.setdefault(tuple(sorted(a.groupingColumns())), []).append(a)
                continue
            try:
                state = aggregated.get(a)
                if state is not None and saveStatesWith is not None:
                    saveStatesWith.persist(a, state)
                results[a] = a.computeMetricFrom(state)
            except Exception as e:  # noqa: BLE001
                results[a] = a.toFailureMetric(e)
        for _, group in grouping.items():
            states = [aggregated.get(a) for a in group if aggregated.get(a) is not None]
            for a in group:
                try:
                    if not states:  # require(states.nonEmpty) (:474)
                        raise ValueError("no persisted frequency state for grouping %s" % a.groupingColumns())
                    results[a] = a.computeMetricFrom(states[0])
                except Exception as e:  # noqa: BLE001
                    results[a] = a.toFailureMetric(e)
            if states and saveStatesWith is not None:
                saveStatesWith.persist(group[0], states[0])
        return AnalyzerContext(OrderedDict((a, results[a]) for a in analyzers if a in results))


class AnalysisRunBuilder:
    """AnalysisRunBuilder (runners/AnalysisRunBuilder.scala:25-116)."""

    def __init__(self, data):
        self.data = data
        self.analyzers: List[Analyzer] = []
        self._aggregate_with = None
        self._save_states_with = None

    def addAnalyzer(self, analyzer: Analyzer) -> "AnalysisRunBuilder":
        self.analyzers.append(analyzer)
        return self

    def addAnalyzers(self, analyzers: Sequence[Analyzer]) -> "AnalysisRunBuilder":
        self.analyzers.extend(analyzers)
        return self

    def aggregateWith(self, loader) -> "AnalysisRunBuilder":
        self._aggregate_with = loader
        return self

    def saveStatesWith(self, persister) -> "AnalysisRunBuilder":
        self._save_states_with = persister
        return self

    def run(self) -> AnalyzerContext:
        return AnalysisRunner.doAnalysisRun(self.data, self.analyzers, self._aggregate_with,
                                            self._save_states_with)


class Analysis:
    """Analysis (analyzers/Analysis.scala): a list of analyzers run together."""

    def __init__(self, analyzers: Sequence[Analyzer] = ()):
        self.analyzers = list(analyzers)

    def addAnalyzer(self, analyzer: Analyzer) -> "Analysis":
        return Analysis(self.analyzers + [analyzer])

    def addAnalyzers(self, analyzers: Sequence[Analyzer]) -> "Analysis":
        return Analysis(self.analyzers + list(analyzers))

    def run(self, data, aggregateWith=None, saveStatesWith=None) -> AnalyzerContext:
        return AnalysisRunner.doAnalysisRun(data, self.analyzers, aggregateWith, saveStatesWith)
