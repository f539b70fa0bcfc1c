"""deequ_amd -- MI355X-native backend for deequ's metric-computation hot path.

The public names mirror the reference's Scala API (`com.amazon.deequ.analyzers`,
`...analyzers.runners`): analyzers, states, `AnalysisRunner`, `AnalyzerContext`.  All compute
goes through the C-ABI library `libdeequ_amd.so` (hand-written gfx950 HIP kernels); there is
no CPU fallback.
"""
from .analyzers import (Analyzer, ApproxCountDistinct, Completeness, Compliance, CountDistinct, DataType,
                        DataTypeInstances,
                        Distinctness, Entropy, FrequencyBasedAnalyzer, GroupingAnalyzer, Histogram,
                        Correlation, MaxLength, Maximum, Mean, MinLength, Minimum, MutualInformation,
                        Preconditions,
                        ScanShareableAnalyzer, ScanShareableFrequencyBasedAnalyzer, Size,
                        StandardDeviation, StandardScanShareableAnalyzer, Sum, Uniqueness,
                        UniqueValueRatio)
from .frequencies import FrequenciesAndNumRows, FrequencyTable
from .engine import Plan, current_device, run_scan, set_device
from .metrics import (Distribution, DistributionValue, DoubleMetric, EmptyStateException, Entity,
                      Failure, HistogramMetric,
                      IllegalAnalyzerParameterException, MetricCalculationException,
                      MetricCalculationRuntimeException, NoSuchColumnException, Success,
                      WrongColumnTypeException)
from .runner import (Analysis, AnalysisRunBuilder, AnalysisRunner, AnalyzerContext,
                     InMemoryStateProvider)
from .states import (ApproxCountDistinctState, CorrelationState, DataTypeHistogram, MaxState, MeanState, MinState,
                     NumMatches,
                     NumMatchesAndCount, StandardDeviationState, State, SumState)
from .state_provider import HdfsStateProvider
from .arrow import ArrowBatch, ArrowTable
from .table import Column, PartitionedTable, Table

__all__ = [n for n in dir() if not n.startswith("_")]
