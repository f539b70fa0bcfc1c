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

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from . import _lib as L
from .metrics import (DoubleMetric, Entity, Failure, IllegalAnalyzerParameterException,
                      MetricCalculationRuntimeException, NoColumnsSpecifiedException,
                      NoSuchColumnException, NumberOfSpecifiedColumnsException,
                      WrongColumnTypeException, empty_state_exception, metric_from_failure,
                      metric_from_value, wrap_if_necessary)
from . import engine as _engine
from .states import State, merge, state_from_dq

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
    def isString(column: str) -> Callable[[Dict[str, str]], None]:
        def check(schema):
            t = schema[column]
            if t != "string":
                raise WrongColumnTypeException(
                    "Expected type of column %s to be StringType, but found %s instead!" % (column, t))
        return check

    @staticmethod
    def atLeastOne(columns) -> Callable[[Dict[str, str]], None]:
        def check(_schema):
            if len(columns) == 0:
                raise NoColumnsSpecifiedException("At least one column needs to be specified!")
        return check

    @staticmethod
    def exactlyNColumns(columns, n: int) -> Callable[[Dict[str, str]], None]:
        def check(_schema):
            if len(columns) != n:
                raise NumberOfSpecifiedColumnsException(
                    "%d columns have to be specified! Currently, columns contains only %d column(s): %s!"
                    % (n, len(columns), ",".join(columns)))
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

    def __getstate__(self):
        # the memoised hash (_memoise_hashes) is per process: str hashes are salted per
        # interpreter, so a pickled copy must recompute it where it is unpickled
        state = dict(self.__dict__)
        state.pop("_dq_hash", None)
        return state

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
    """Runs in the single fused pass; one dq_op per analyzer (ScanShareableAnalyzer,
    Analyzer.scala:169-197).  The two hooks mirror the reference's seam so a subclass can
    override them exactly as AnalysisTest.scala:206-280 does:

    * aggregationFunctions(schema) -> the dq_op this analyzer contributes to the plan (the
      reference's Seq[Column]); an exception here fails every shareable analyzer of the run
      (AnalysisRunner.scala:305-323);
    * fromAggregationResult(raw) -> the State from this analyzer's POD dq_state (the reference
      reads its Row slice at `offset`); an exception here fails this analyzer only (:340-353).
    """

    DQ_KIND = 0
    where: Optional[str] = None

    def aggregationFunctions(self, schema):
        return _engine.op_spec_for(self, schema)

    def fromAggregationResult(self, raw) -> Optional[State]:
        if isinstance(raw, _engine.OpUnsupported):
            raise raw.error
        return state_from_dq(raw)

    def metricFromAggregationResult(self, raw, aggregateWith=None, saveStatesWith=None):
        """Analyzer.metricFromAggregationResult (Analyzer.scala:185-195)."""
        return self.calculateMetric(self.fromAggregationResult(raw), aggregateWith, saveStatesWith)

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
        from .predicates import referenced_columns, resolve_column

        def check(schema):
            for c in referenced_columns(self.predicate) + (
                    referenced_columns(self.where) if self.where else []):
                try:  # case-insensitive, as Spark 2.2 resolves names
                    resolve_column(c, schema)
                except KeyError:
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


@dataclass(frozen=True)
class MinLength(StandardScanShareableAnalyzer):
    """min(length(sel)).cast(double) over a string column (MinLength.scala:25-41)."""
    column: str
    where: Optional[str] = None
    name = "MinLength"
    DQ_KIND = L.DQ_OP_MIN_LENGTH

    def instance(self):
        return self.column

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column), Preconditions.isString(self.column)]

    def __str__(self):
        return "MinLength(%s,%s)" % (self.column, _opt(self.where))


@dataclass(frozen=True)
class MaxLength(StandardScanShareableAnalyzer):
    """max(length(sel)).cast(double) over a string column (MaxLength.scala:25-41)."""
    column: str
    where: Optional[str] = None
    name = "MaxLength"
    DQ_KIND = L.DQ_OP_MAX_LENGTH

    def instance(self):
        return self.column

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column), Preconditions.isString(self.column)]

    def __str__(self):
        return "MaxLength(%s,%s)" % (self.column, _opt(self.where))


@dataclass(frozen=True)
class Correlation(StandardScanShareableAnalyzer):
    """Pearson correlation of two numeric columns (Correlation.scala:65-105); state
    CorrelationState, metric ck / sqrt(xMk * yMk)."""
    firstColumn: str
    secondColumn: str
    where: Optional[str] = None
    name = "Correlation"
    entity = Entity.Mutlicolumn
    DQ_KIND = L.DQ_OP_CORRELATION

    def instance(self):
        return "%s,%s" % (self.firstColumn, self.secondColumn)

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.firstColumn), Preconditions.isNumeric(self.firstColumn),
                Preconditions.hasColumn(self.secondColumn), Preconditions.isNumeric(self.secondColumn)]

    def __str__(self):
        return "Correlation(%s,%s,%s)" % (self.firstColumn, self.secondColumn, _opt(self.where))


class DataTypeInstances:
    """DataTypeInstances enumeration (DataType.scala:32-38): value ids and names."""
    Unknown, Fractional, Integral, Boolean, String = 0, 1, 2, 3, 4
    NAMES = ("Unknown", "Fractional", "Integral", "Boolean", "String")

    @classmethod
    def name_of(cls, v: int) -> str:
        return cls.NAMES[v]


def data_type_distribution(h):
    """DataTypeHistogram.toDistribution (DataType.scala:98-114)."""
    from .metrics import Distribution, DistributionValue
    total = h.numNull + h.numString + h.numBoolean + h.numIntegral + h.numFractional
    vals = {"Unknown": h.numNull, "Fractional": h.numFractional, "Integral": h.numIntegral,
            "Boolean": h.numBoolean, "String": h.numString}
    return Distribution({k: DistributionValue(c, (c / total) if total else float("nan"))
                         for k, c in vals.items()}, 5)


def determine_type(dist) -> int:
    """DataTypeHistogram.determineType (DataType.scala:116-143)."""
    def ratio(name):
        v = dist.values.get(name)
        return 0.0 if v is None else v.ratio
    if ratio("Unknown") == 1.0:
        return DataTypeInstances.Unknown
    if ratio("String") > 0.0 or (ratio("Boolean") > 0.0 and (ratio("Integral") > 0.0 or ratio("Fractional") > 0.0)):
        return DataTypeInstances.String
    if ratio("Boolean") > 0.0:
        return DataTypeInstances.Boolean
    if ratio("Fractional") > 0.0:
        return DataTypeInstances.Fractional
    return DataTypeInstances.Integral


@dataclass(frozen=True)
class DataType(ScanShareableAnalyzer):
    """DataType(column, where) (DataType.scala:152-183): the StatefulDataType UDAF's regex type
    classification of the column cast to string, as the GPU op DQ_OP_DATATYPE (dq_profile.hip).
    The metric is a HistogramMetric over the five type names."""
    column: str
    where: Optional[str] = None
    name = "DataType"
    DQ_KIND = L.DQ_OP_DATATYPE

    def instance(self):
        return self.column

    def preconditions(self):
        return [Preconditions.hasColumn(self.column)]

    def computeMetricFrom(self, state):
        from .metrics import HistogramMetric, Success as _S
        if state is None:
            return HistogramMetric(self.column, Failure(wrap_if_necessary(empty_state_exception(self))))
        return HistogramMetric(self.column, _S(data_type_distribution(state)))

    def toFailureMetric(self, error):
        from .metrics import HistogramMetric
        return HistogramMetric(self.column, Failure(wrap_if_necessary(error)))

    def __str__(self):
        return "DataType(%s,%s)" % (self.column, _opt(self.where))


# ---------------------------------------------------------------- frequency-based analyzers
def _columns_tuple(columns) -> tuple:
    return (columns,) if isinstance(columns, str) else tuple(columns)


def _scala_seq(columns) -> str:
    return "List(%s)" % ", ".join(columns)


class GroupingAnalyzer(Analyzer):
    """GroupingAnalyzer (Analyzer.scala:273-282)."""

    def groupingColumns(self) -> List[str]:
        raise NotImplementedError

    def preconditions(self):
        return [Preconditions.hasColumn(c) for c in self.groupingColumns()]


class FrequencyBasedAnalyzer(GroupingAnalyzer):
    """FrequencyBasedAnalyzer (GroupingAnalyzers.scala:29-42): the state is the GPU group-by
    of the grouping columns (deequ_amd.frequencies)."""

    columns: tuple = ()

    def __post_init__(self):
        object.__setattr__(self, "columns", _columns_tuple(self.columns))

    def groupingColumns(self) -> List[str]:
        return list(self.columns)

    @property
    def entity(self):
        return Entity.Column if len(self.columns) == 1 else Entity.Mutlicolumn

    def instance(self) -> str:
        return ",".join(self.columns)

    def computeStateFrom(self, data):
        from .frequencies import compute_frequencies
        return compute_frequencies(data, self.groupingColumns())

    def preconditions(self):
        return [Preconditions.atLeastOne(self.columns)] + \
            [Preconditions.hasColumn(c) for c in self.columns]

    def __str__(self):
        return "%s(%s)" % (self.name, _scala_seq(self.columns))


class ScanShareableFrequencyBasedAnalyzer(FrequencyBasedAnalyzer):
    """ScanShareableFrequencyBasedAnalyzer (GroupingAnalyzers.scala:84-121).  The Spark job
    `frequencies.agg(...)` becomes the device summary (#groups, #count==1, entropy) of the
    frequency table; `metric_from_summary` restates each analyzer's aggregation."""

    def metric_from_summary(self, s) -> Optional[float]:
        raise NotImplementedError

    def computeMetricFrom(self, state):
        if state is None:
            return metric_from_failure(empty_state_exception(self), self.name, self.instance(), self.entity)
        value = self.metric_from_summary(state.summary())
        if value is None:  # the aggregation over the frequency table is NULL (:113-119)
            return metric_from_failure(empty_state_exception(self), self.name, self.instance(), self.entity)
        return metric_from_value(value, self.name, self.instance(), self.entity)


@dataclass(frozen=True)
class Uniqueness(ScanShareableFrequencyBasedAnalyzer):
    """Σ[count == 1] / numRows (Uniqueness.scala:29-31)."""
    columns: tuple
    name = "Uniqueness"

    def metric_from_summary(self, s):
        return None if s.num_groups == 0 else float(s.num_unique) / s.num_rows

    __str__ = FrequencyBasedAnalyzer.__str__


@dataclass(frozen=True)
class Distinctness(ScanShareableFrequencyBasedAnalyzer):
    """Σ[count >= 1] / numRows (Distinctness.scala:32-34)."""
    columns: tuple
    name = "Distinctness"

    def metric_from_summary(self, s):
        return None if s.num_groups == 0 else float(s.num_groups) / s.num_rows

    __str__ = FrequencyBasedAnalyzer.__str__


@dataclass(frozen=True)
class CountDistinct(ScanShareableFrequencyBasedAnalyzer):
    """count(*) over the frequency table (CountDistinct.scala:27-33): never NULL."""
    columns: tuple
    name = "CountDistinct"

    def metric_from_summary(self, s):
        return float(s.num_groups)

    __str__ = FrequencyBasedAnalyzer.__str__


@dataclass(frozen=True)
class UniqueValueRatio(ScanShareableFrequencyBasedAnalyzer):
    """Σ[count == 1] / count(*) (UniqueValueRatio.scala:28-37).  With no groups the sum is
    NULL and the reference's `Row.getDouble` throws, which surfaces as a failure metric."""
    columns: tuple
    name = "UniqueValueRatio"

    def metric_from_summary(self, s):
        if s.num_groups == 0:
            raise MetricCalculationRuntimeException("Value at index 0 is null")
        return float(s.num_unique) / float(s.num_groups)

    __str__ = FrequencyBasedAnalyzer.__str__


@dataclass(frozen=True)
class Entropy(ScanShareableFrequencyBasedAnalyzer):
    """Σ −(c/N)·ln(c/N) over the groups (Entropy.scala:31-41)."""
    column: str
    name = "Entropy"

    def __post_init__(self):
        object.__setattr__(self, "columns", (self.column,))

    def metric_from_summary(self, s):
        return None if s.num_groups == 0 else s.entropy

    def __str__(self):
        return "Entropy(%s)" % self.column


@dataclass(frozen=True)
class MutualInformation(FrequencyBasedAnalyzer):
    """Mutual information of two columns from their joint frequencies (MutualInformation.scala:
    34-84).  The joint table is the GPU group-by; the marginals and the sum are taken over the
    exported groups in a fixed (encoded-key) order."""
    columns: tuple
    columnB: Optional[str] = field(default=None, compare=False, repr=False)  # MutualInformation(a, b)
    name = "MutualInformation"

    def __post_init__(self):
        cols = _columns_tuple(self.columns)
        if self.columnB is not None:
            cols = cols + (self.columnB,)
            object.__setattr__(self, "columnB", None)
        object.__setattr__(self, "columns", cols)

    @property
    def entity(self):
        return Entity.Mutlicolumn

    def preconditions(self):
        return [Preconditions.exactlyNColumns(self.columns, 2)] + super().preconditions()

    def computeMetricFrom(self, state):
        if state is None:
            return metric_from_failure(empty_state_exception(self), self.name, self.instance(), self.entity)
        import math
        from .frequencies import decode_key
        total = state.numRows
        counts, keys = state.table.export()
        if len(keys) == 0:
            return metric_from_failure(empty_state_exception(self), self.name, self.instance(), self.entity)
        cols = state.columns
        i1, i2 = cols.index(self.columns[0]), cols.index(self.columns[1])
        order = sorted(range(len(keys)), key=lambda i: keys[i])
        joint = [(decode_key(keys[i], state.table.dtypes), int(counts[i])) for i in order]
        m1, m2 = {}, {}
        for k, c in joint:
            m1[k[i1]] = m1.get(k[i1], 0) + c
            m2[k[i2]] = m2.get(k[i2], 0) + c
        value = 0.0
        for k, c in joint:
            px, py, pxy = float(m1[k[i1]]), float(m2[k[i2]]), float(c)
            value += (pxy / total) * math.log((pxy / total) / ((px / total) * (py / total)))
        return metric_from_value(value, self.name, self.instance(), self.entity)

    def __str__(self):
        return "MutualInformation(%s)" % _scala_seq(self.columns)


MAXIMUM_ALLOWED_DETAIL_BINS = 1000  # Histogram.MaximumAllowedDetailBins (Histogram.scala:109)


@dataclass(frozen=True)
class Histogram(Analyzer):
    """Histogram (Histogram.scala:41-116): value counts of `column` cast to string (NULL ->
    "NullValue"), the top `maxDetailBins` by count and the number of bins.

    The group-by runs on the GPU over the raw values (DQ_FREQ_NULL_AS_KEY: NULL is a group,
    NaNs are one group); values become Java strings only for the few reported bins.  A
    `binningUdf` (a Python callable on the column's values, None for NULL) is applied per
    distinct value after the group-by -- the same result as binning every row first, since
    the UDF is a function of the value."""
    column: str
    binningUdf: Optional[Callable] = None
    maxDetailBins: int = MAXIMUM_ALLOWED_DETAIL_BINS
    name = "Histogram"

    def instance(self):
        return self.column

    def preconditions(self):
        def param_check(_schema):
            if self.maxDetailBins > MAXIMUM_ALLOWED_DETAIL_BINS:
                raise IllegalAnalyzerParameterException(
                    "Cannot return histogram values for more than %d values" % MAXIMUM_ALLOWED_DETAIL_BINS)
        return [param_check, Preconditions.hasColumn(self.column)]

    def computeStateFrom(self, data):
        from .frequencies import FrequenciesAndNumRows, compute_frequencies, decode_key
        if self.binningUdf is None:
            return compute_frequencies(data, [self.column], histogram=True)
        state = compute_frequencies(data, [self.column])
        dtype = state.table.dtypes[0]
        s = state.summary()
        counts, keys = state.table.export()
        binned: Dict[tuple, int] = {}

        def add(value, c):
            b = self.binningUdf(value)
            key = NULL_FIELD_REPLACEMENT if b is None else _udf_result_to_string(b)
            binned[(key,)] = binned.get((key,), 0) + c
        for k, c in zip(keys, counts.tolist()):
            add(decode_key(k, [dtype])[0], c)
        if s.num_rows > s.grouped_rows:
            add(None, s.num_rows - s.grouped_rows)
        return FrequenciesAndNumRows.from_frequencies([self.column], ["string"], binned, s.num_rows,
                                                      histogram=True)

    def computeMetricFrom(self, state):
        from .metrics import Distribution, DistributionValue, HistogramMetric, Success as _S
        if state is None:
            return HistogramMetric(self.column, Failure(wrap_if_necessary(empty_state_exception(self))))
        try:
            from .frequencies import decode_key
            from .javafmt import spark_cast_to_string
            dtype = state.table.dtypes[0]
            n_rows = state.numRows
            counts, keys = state.table.top(self.maxDetailBins)
            if dtype == "string":
                # a string key's encoding is its UTF-8 bytes, and top() is already ordered by
                # (count desc, encoded key asc) -- the order below: decode only what is kept
                items = [(k.decode("utf-8"), c) for k, c in zip(keys[:self.maxDetailBins],
                                                               counts[:self.maxDetailBins].tolist())]
            else:
                items = []
                for k, c in zip(keys, counts.tolist()):
                    v = decode_key(k, [dtype], histogram=True)[0]
                    items.append((NULL_FIELD_REPLACEMENT if v is None else spark_cast_to_string(v, dtype), c))
                items.sort(key=lambda kv: (-kv[1], kv[0].encode("utf-8")))
            values = {k: DistributionValue(c, c / n_rows) for k, c in items[:self.maxDetailBins]}
            return HistogramMetric(self.column, _S(Distribution(values, state.summary().num_groups)))
        except Exception as e:  # noqa: BLE001
            return self.toFailureMetric(e)

    # column types whose frequency table groups exactly as Histogram's string cast does
    # (distinct values <-> distinct strings); floats are excluded: Histogram merges NaN payloads
    SHARES_FREQUENCIES = ("string", "bool", "int8", "int16", "int32", "int64")

    def metricFromFrequencies(self, state):
        """The metric from the frequency table of `column` that a FrequencyBasedAnalyzer of the
        same run already built (no second group-by).  Histogram.scala:54-69 groups
        `col.cast(string)` with NULL replaced by "NullValue"; the shared table holds the
        non-NULL groups, so the NULL bin is numRows - (grouped rows), plus the count of a
        literal "NullValue" string when the column holds one (the replacement merges them)."""
        from .metrics import Distribution, DistributionValue, HistogramMetric, Success as _S
        if state is None:
            return HistogramMetric(self.column, Failure(wrap_if_necessary(empty_state_exception(self))))
        try:
            from .frequencies import decode_key
            from .javafmt import spark_cast_to_string
            dtype = state.table.dtypes[0]
            s = state.summary()
            n_rows = s.num_rows
            null_key = NULL_FIELD_REPLACEMENT.encode("utf-8")
            literal = state.table.lookup(null_key) if dtype == "string" else 0
            null_bin = (n_rows - s.grouped_rows) + literal
            counts, keys = state.table.top(self.maxDetailBins)
            if dtype == "string":
                # top() is ordered by (count desc, UTF-8 key asc), the order below: decode only the
                # keys that can be kept (one more for the literal "NullValue" key, skipped here),
                # and put the NULL bin in its place
                m = self.maxDetailBins + 1
                items = [(k.decode("utf-8"), c) for k, c in zip(keys[:m], counts[:m].tolist()) if k != null_key]
                if null_bin:
                    import bisect
                    pos = bisect.bisect_left([(-c, k.encode("utf-8")) for k, c in items],
                                             (-null_bin, null_key))
                    items.insert(pos, (NULL_FIELD_REPLACEMENT, null_bin))
            else:
                items = []
                for k, c in zip(keys, counts.tolist()):
                    items.append((spark_cast_to_string(decode_key(k, [dtype])[0], dtype), c))
                if null_bin:
                    items.append((NULL_FIELD_REPLACEMENT, null_bin))
                items.sort(key=lambda kv: (-kv[1], kv[0].encode("utf-8")))
            bins = s.num_groups + (1 if null_bin and not literal else 0)
            values = {k: DistributionValue(c, c / n_rows) for k, c in items[:self.maxDetailBins]}
            return HistogramMetric(self.column, _S(Distribution(values, bins)))
        except Exception as e:  # noqa: BLE001
            return self.toFailureMetric(e)

    def toFailureMetric(self, error):
        from .metrics import HistogramMetric
        return HistogramMetric(self.column, Failure(wrap_if_necessary(error)))

    def __str__(self):
        return "Histogram(%s,%s,%d)" % (self.column, "None" if self.binningUdf is None else
                                        "Some(%r)" % self.binningUdf, self.maxDetailBins)


NULL_FIELD_REPLACEMENT = "NullValue"


def _udf_result_to_string(b) -> str:
    from .javafmt import spark_cast_to_string
    if isinstance(b, str):
        return b
    if isinstance(b, bool):
        return spark_cast_to_string(b, "bool")
    if isinstance(b, int):
        return str(b)
    if isinstance(b, float):
        return spark_cast_to_string(b, "float64")
    return str(b)


def _memoise_hashes() -> None:
    """Analyzers are frozen dataclasses: their hash never changes, but the generated __hash__
    rebuilds and hashes the field tuple on every call, and a profiler run keys several dicts by
    hundreds of analyzers.  Each class's hash is computed once per instance and kept, with the
    class mixed in: Completeness(c), Mean(c), Sum(c) ... have equal field tuples, so without it
    they collide in every dict and each insert pays two __eq__ calls."""
    def caching(h):
        def __hash__(self):
            try:
                return self.__dict__["_dq_hash"]
            except KeyError:
                v = hash((type(self).__qualname__, h(self)))
                object.__setattr__(self, "_dq_hash", v)
                return v
        __hash__._dq_cached = True
        return __hash__
    stack, seen = [Analyzer], set()
    while stack:
        for sub in stack.pop().__subclasses__():
            if sub in seen:
                continue
            seen.add(sub)
            stack.append(sub)
            h = sub.__dict__.get("__hash__")
            if h is not None and not getattr(h, "_dq_cached", False):
                sub.__hash__ = caching(h)


_memoise_hashes()
