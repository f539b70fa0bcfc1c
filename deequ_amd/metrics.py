"""Metric values and the failure taxonomy, mirroring the reference's result types.

* `Entity`, `DoubleMetric` -- metrics/Metric.scala:21-49
* `Success` / `Failure` -- scala.util.Try, as carried by every metric
* exceptions -- analyzers/runners/MetricCalculationException.scala:19-78
"""
from __future__ import annotations

import enum
import math
from dataclasses import dataclass
from typing import Any


class Entity(enum.Enum):
    Dataset = "Dataset"
    Column = "Column"
    Mutlicolumn = "Mutlicolumn"  # sic: the reference's spelling (Metric.scala:22)


class MetricCalculationException(Exception):
    pass


class MetricCalculationRuntimeException(MetricCalculationException):
    pass


class MetricCalculationPreconditionException(MetricCalculationException):
    pass


class NoSuchColumnException(MetricCalculationPreconditionException):
    pass


class WrongColumnTypeException(MetricCalculationPreconditionException):
    pass


class NoColumnsSpecifiedException(MetricCalculationPreconditionException):
    pass


class NumberOfSpecifiedColumnsException(MetricCalculationPreconditionException):
    pass


class IllegalAnalyzerParameterException(MetricCalculationPreconditionException):
    pass


class EmptyStateException(MetricCalculationRuntimeException):
    pass


def wrap_if_necessary(error: BaseException) -> MetricCalculationException:
    """MetricCalculationException.wrapIfNecessary (:69-76)."""
    if isinstance(error, MetricCalculationException):
        return error
    wrapped = MetricCalculationRuntimeException(str(error))
    wrapped.__cause__ = error
    return wrapped


class Try:
    def is_success(self) -> bool:
        raise NotImplementedError

    isSuccess = property(lambda self: self.is_success())
    isFailure = property(lambda self: not self.is_success())


@dataclass(frozen=True)
class Success(Try):
    value: Any

    def is_success(self):
        return True

    def get(self):
        return self.value

    def __eq__(self, other):
        if not isinstance(other, Success):
            return False
        a, b = self.value, other.value
        if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
            return True
        return a == b

    def __hash__(self):
        return hash(("Success", self.value))


@dataclass(frozen=True, eq=False)
class Failure(Try):
    exception: BaseException

    def is_success(self):
        return False

    def get(self):
        raise self.exception

    def __eq__(self, other):
        return isinstance(other, Failure) and type(self.exception) is type(other.exception) and \
            str(self.exception) == str(other.exception)

    def __hash__(self):
        return hash(("Failure", type(self.exception).__name__, str(self.exception)))


@dataclass(frozen=True)
class DoubleMetric:
    entity: Entity
    name: str
    instance: str
    value: Try

    def flatten(self):
        return [self]


def metric_from_value(value: float, name: str, instance: str, entity: Entity = Entity.Column):
    return DoubleMetric(entity, name, instance, Success(float(value)))


def metric_from_failure(error: BaseException, name: str, instance: str,
                        entity: Entity = Entity.Column):
    return DoubleMetric(entity, name, instance, Failure(wrap_if_necessary(error)))


def empty_state_exception(analyzer) -> EmptyStateException:
    """Analyzers.emptyStateException (Analyzer.scala:444-446)."""
    return EmptyStateException("Empty state for analyzer %s, all input values were NULL." % analyzer)


@dataclass(frozen=True)
class DistributionValue:
    """DistributionValue(absolute, ratio) (metrics/HistogramMetric.scala:21)."""
    absolute: int
    ratio: float


@dataclass(frozen=True)
class Distribution:
    """Distribution(values, numberOfBins) (metrics/HistogramMetric.scala:23-36)."""
    values: Any  # Dict[str, DistributionValue]
    numberOfBins: int

    def __getitem__(self, key: str) -> DistributionValue:
        return self.values[key]

    def argmax(self) -> str:
        return max(self.values.items(), key=lambda kv: kv[1].absolute)[0]

    def __hash__(self):
        return hash((tuple(sorted(self.values.items())), self.numberOfBins))


@dataclass(frozen=True)
class HistogramMetric:
    """HistogramMetric(column, value: Try[Distribution]) (metrics/HistogramMetric.scala:38-64)."""
    column: str
    value: Try

    entity = Entity.Column
    name = "Histogram"

    @property
    def instance(self) -> str:
        return self.column

    def flatten(self):
        if not self.value.isSuccess:
            return [DoubleMetric(self.entity, "%s.bins" % self.name, self.instance, self.value)]
        dist = self.value.get()
        out = [DoubleMetric(self.entity, "%s.bins" % self.name, self.instance,
                            Success(float(dist.numberOfBins)))]
        for key, dv in dist.values.items():
            out.append(DoubleMetric(self.entity, "%s.abs.%s" % (self.name, key), self.instance,
                                    Success(float(dv.absolute))))
            out.append(DoubleMetric(self.entity, "%s.ratio.%s" % (self.name, key), self.instance,
                                    Success(dv.ratio)))
        return out
