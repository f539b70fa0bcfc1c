"""Analyzers -- the reference's Analyzer / ScanShareableAnalyzer API on the GPU path.

Names, constructor arguments, preconditions, NULL -> None rules and failure metrics follow
`src/main/scala/com/amazon/deequ/analyzers/`:

* Analyzer.calculate / calculateMetric      Analyzer.scala:88-128
* StandardScanShareableAnalyzer             Analyzer.scala:200-226
* Preconditions.hasColumn / isNumeric        Analyzer.scala:324-344
* Size, Completeness, Compliance, Sum, Mean, StandardDeviation, Minimum, Maximum,
  ApproxCountDistinct                        Size.scala, Completeness.scala, ... (one file each)

`computeStateFrom` runs the fused GPU scan (deequ_amd.engine.run_scan); there is no CPU path.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

from . import _lib as L
from .metrics import (DoubleMetric, Entity, NoSuchColumnException, WrongColumnTypeException,
                      empty_state_exception, metric_from_failure, metric_from_value)
from .states import State, merge

NUMERIC_TYPES = ("int8", "int16", "int32", "int64", "float32", "float64")


def _opt(x: Optional[str]) -> str:
    return "None" if x is None else "Some(%s)" % x


class Preconditions:
    @staticmethod
    def hasColumn(column: str) -> Callable[[Dict[str, str]], None]:
        def check(schema):
            if column not in schema:
                raise NoSuchColumnException("Input data does not include column %s!" % column)
        return check

    @staticmethod
    def isNumeric(column: str) -> Callable[[Dict[str, str]], None]:
        def check(schema):
            t = schema[column]
            if t not in NUMERIC_TYPES:
                raise WrongColumnTypeException(
                    "Expected type of column %s to be one of (ByteType,ShortType,IntegerType,"
                    "LongType,FloatType,DoubleType,DecimalType), but found %s instead!" % (column, t))
        return check

    @staticmethod
    def findFirstFailing(schema, conditions) -> Optional[Exception]:
        for c in conditions:
            try:
                c(schema)
            except Exception as e:  # noqa: BLE001 - mirrors the reference's catch-all
                return e
        return None


class Analyzer:
    """Analyzer[S, M] (Analyzer.scala:56-165)."""

    name = "Analyzer"
    entity = Entity.Column

    def instance(self) -> str:
        raise NotImplementedError

    def preconditions(self) -> List[Callable]:
        return []

    def computeStateFrom(self, data) -> Optional[State]:
        raise NotImplementedError

    def computeMetricFrom(self, state: Optional[State]):
        raise NotImplementedError

    def toFailureMetric(self, error: BaseException):
        return metric_from_failure(error, self.name, self.instance(), self.entity)

    def calculate(self, data, aggregateWith=None, saveStatesWith=None):
        try:
            for cond in self.preconditions():
                cond(data.schema)
            state = self.computeStateFrom(data)
            return self.calculateMetric(state, aggregateWith, saveStatesWith)
        except Exception as e:  # noqa: BLE001
            return self.toFailureMetric(e)

    def calculateMetric(self, state, aggregateWith=None, saveStatesWith=None):
        loaded = aggregateWith.load(self) if aggregateWith is not None else None
        merged = merge(state, loaded)
        if merged is not None and saveStatesWith is not None:
            saveStatesWith.persist(self, merged)
        return self.computeMetricFrom(merged)


class ScanShareableAnalyzer(Analyzer):
    """Runs in the single fused pass; one dq_op per analyzer."""

    DQ_KIND = 0
    where: Optional[str] = None

    def computeStateFrom(self, data) -> Optional[State]:
        from .engine import run_scan
        return run_scan([self], data)[self]


class StandardScanShareableAnalyzer(ScanShareableAnalyzer):
    def computeMetricFrom(self, state: Optional[State]) -> DoubleMetric:
        if state is None:
            return metric_from_failure(empty_state_exception(self), self.name, self.instance(), self.entity)
        return metric_from_value(state.metricValue(), self.name, self.instance(), self.entity)

    def additionalPreconditions(self) -> List[Callable]:
        return []

    def preconditions(self):
        return self.additionalPreconditions()


@dataclass(frozen=True)
class Size(StandardScanShareableAnalyzer):
    where: Optional[str] = None
    name = "Size"
    entity = Entity.Dataset
    DQ_KIND = L.DQ_OP_SIZE

    def instance(self):
        return "*"

    def __str__(self):
        return "Size(%s)" % _opt(self.where)


@dataclass(frozen=True)
class Completeness(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    name = "Completeness"
    DQ_KIND = L.DQ_OP_COMPLETENESS

    def instance(self):
        return self.column

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column)]

    def __str__(self):
        return "Completeness(%s,%s)" % (self.column, _opt(self.where))


@dataclass(frozen=True)
class Compliance(StandardScanShareableAnalyzer):
    instance_name: str
    predicate: str
    where: Optional[str] = None
    name = "Compliance"
    DQ_KIND = L.DQ_OP_COMPLIANCE

    def instance(self):
        return self.instance_name

    def preconditions(self):
        # Spark fails the aggregation (AnalysisException) on an unknown column; deequ turns
        # it into a failure metric.  Checked on the schema here, before any data is touched.
        from .predicates import referenced_columns

        def check(schema):
            for c in referenced_columns(self.predicate) + (
                    referenced_columns(self.where) if self.where else []):
                if c not in schema:
                    raise NoSuchColumnException("Input data does not include column %s!" % c)
        return [check]

    def __str__(self):
        return "Compliance(%s,%s,%s)" % (self.instance_name, self.predicate, _opt(self.where))


class _NumericColumnAnalyzer(StandardScanShareableAnalyzer):
    def instance(self):
        return self.column

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column), Preconditions.isNumeric(self.column)]

    def __str__(self):
        return "%s(%s,%s)" % (self.name, self.column, _opt(self.where))


@dataclass(frozen=True)
class Sum(_NumericColumnAnalyzer):
    column: str
    where: Optional[str] = None
    name = "Sum"
    DQ_KIND = L.DQ_OP_SUM

    __str__ = _NumericColumnAnalyzer.__str__


@dataclass(frozen=True)
class Mean(_NumericColumnAnalyzer):
    column: str
    where: Optional[str] = None
    name = "Mean"
    DQ_KIND = L.DQ_OP_MEAN

    __str__ = _NumericColumnAnalyzer.__str__


@dataclass(frozen=True)
class StandardDeviation(_NumericColumnAnalyzer):
    column: str
    where: Optional[str] = None
    name = "StandardDeviation"
    DQ_KIND = L.DQ_OP_STDDEV

    __str__ = _NumericColumnAnalyzer.__str__


@dataclass(frozen=True)
class Minimum(_NumericColumnAnalyzer):
    column: str
    where: Optional[str] = None
    name = "Minimum"
    DQ_KIND = L.DQ_OP_MINIMUM

    __str__ = _NumericColumnAnalyzer.__str__


@dataclass(frozen=True)
class Maximum(_NumericColumnAnalyzer):
    column: str
    where: Optional[str] = None
    name = "Maximum"
    DQ_KIND = L.DQ_OP_MAXIMUM

    __str__ = _NumericColumnAnalyzer.__str__


@dataclass(frozen=True)
class ApproxCountDistinct(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    name = "ApproxCountDistinct"
    DQ_KIND = L.DQ_OP_APPROX_COUNT_DISTINCT

    def instance(self):
        return self.column

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column)]

    def __str__(self):
        return "ApproxCountDistinct(%s,%s)" % (self.column, _opt(self.where))
