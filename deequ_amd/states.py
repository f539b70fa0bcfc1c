"""The reference's `State` case classes, backed by the C-ABI's state algebra.

Every `sum` and `metricValue` goes through `dq_state_merge` / `dq_state_metric`
(deequ_amd/csrc/dq_api.cpp), which restate each Scala `State.sum` exactly, so states produced
on different GPUs, batches or runs (or loaded from a StateProvider) combine the way Spark
partial states do.

* NumMatches -- Size.scala:23-31
* NumMatchesAndCount -- Analyzer.scala:230-244
* SumState -- Sum.scala:25-33;  MeanState -- Mean.scala:25-34
* StandardDeviationState -- StandardDeviation.scala:25-45
* MinState / MaxState -- Minimum.scala:25-33 / Maximum.scala:25-33
* ApproxCountDistinctState -- ApproxCountDistinct.scala:26-40
* DataTypeHistogram -- DataType.scala:40-52
* CorrelationState -- Correlation.scala:26-57
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

from . import _lib as L


class State:
    KIND = 0

    def to_dq(self) -> L.DqState:
        raise NotImplementedError

    @classmethod
    def from_dq(cls, s: L.DqState) -> "State":
        raise NotImplementedError

    def sum(self, other: "State") -> "State":
        if type(other) is not type(self):
            raise TypeError("cannot sum %s with %s" % (type(self).__name__, type(other).__name__))
        a, b, out = self.to_dq(), other.to_dq(), L.DqState()
        L.check(L.lib().dq_state_merge(ctypes.byref(a), ctypes.byref(b), ctypes.byref(out)))
        return type(self).from_dq(out)

    __add__ = sum

    def metricValue(self) -> float:
        s, out = self.to_dq(), ctypes.c_double()
        L.check(L.lib().dq_state_metric(ctypes.byref(s), ctypes.byref(out)))
        return out.value

    def _dq(self, **fields) -> L.DqState:
        s = L.DqState()
        s.kind = self.KIND
        s.has_value = 1
        for k, v in fields.items():
            setattr(s, k, v)
        return s


class NumMatches(State):
    KIND = L.DQ_OP_SIZE

    def __init__(self, numMatches: int):
        self.numMatches = int(numMatches)

    def to_dq(self):
        return self._dq(num_matches=self.numMatches)

    @classmethod
    def from_dq(cls, s):
        return cls(s.num_matches)

    def __eq__(self, o):
        return isinstance(o, NumMatches) and o.numMatches == self.numMatches

    def __hash__(self):
        return hash(("NumMatches", self.numMatches))

    def __repr__(self):
        return "NumMatches(%d)" % self.numMatches


class NumMatchesAndCount(State):
    KIND = L.DQ_OP_COMPLETENESS

    def __init__(self, numMatches: int, count: int):
        self.numMatches = int(numMatches)
        self.count = int(count)

    def to_dq(self):
        return self._dq(num_matches=self.numMatches, count=self.count)

    @classmethod
    def from_dq(cls, s):
        return cls(s.num_matches, s.count)

    def __eq__(self, o):
        return isinstance(o, NumMatchesAndCount) and (o.numMatches, o.count) == (self.numMatches, self.count)

    def __hash__(self):
        return hash(("NumMatchesAndCount", self.numMatches, self.count))

    def __repr__(self):
        return "NumMatchesAndCount(%d,%d)" % (self.numMatches, self.count)


class SumState(State):
    KIND = L.DQ_OP_SUM

    def __init__(self, sum: float):  # noqa: A002 - mirrors the Scala field name
        self.sum_value = float(sum)

    def to_dq(self):
        return self._dq(sum=self.sum_value)

    @classmethod
    def from_dq(cls, s):
        return cls(s.sum)

    def __eq__(self, o):
        return isinstance(o, SumState) and o.sum_value == self.sum_value

    def __hash__(self):
        return hash(("SumState", self.sum_value))

    def __repr__(self):
        return "SumState(%r)" % self.sum_value


class MeanState(State):
    KIND = L.DQ_OP_MEAN

    def __init__(self, sum: float, count: int):  # noqa: A002
        self.sum_value = float(sum)
        self.count = int(count)

    def to_dq(self):
        return self._dq(sum=self.sum_value, count=self.count)

    @classmethod
    def from_dq(cls, s):
        return cls(s.sum, s.count)

    def __eq__(self, o):
        return isinstance(o, MeanState) and (o.sum_value, o.count) == (self.sum_value, self.count)

    def __hash__(self):
        return hash(("MeanState", self.sum_value, self.count))

    def __repr__(self):
        return "MeanState(%r,%d)" % (self.sum_value, self.count)


class StandardDeviationState(State):
    KIND = L.DQ_OP_STDDEV

    def __init__(self, n: float, avg: float, m2: float):
        if not n > 0.0:  # StandardDeviation.scala:31
            raise ValueError("requirement failed: Standard deviation is undefined for n = 0.")
        self.n, self.avg, self.m2 = float(n), float(avg), float(m2)

    def to_dq(self):
        return self._dq(n=self.n, avg=self.avg, m2=self.m2)

    @classmethod
    def from_dq(cls, s):
        return cls(s.n, s.avg, s.m2)

    def __eq__(self, o):
        return isinstance(o, StandardDeviationState) and (o.n, o.avg, o.m2) == (self.n, self.avg, self.m2)

    def __hash__(self):
        return hash(("StandardDeviationState", self.n, self.avg, self.m2))

    def __repr__(self):
        return "StandardDeviationState(%r,%r,%r)" % (self.n, self.avg, self.m2)


class MinState(State):
    KIND = L.DQ_OP_MINIMUM

    def __init__(self, minValue: float):
        self.minValue = float(minValue)

    def to_dq(self):
        return self._dq(value=self.minValue)

    @classmethod
    def from_dq(cls, s):
        return cls(s.value)

    def __eq__(self, o):
        return isinstance(o, MinState) and o.minValue == self.minValue

    def __hash__(self):
        return hash(("MinState", self.minValue))

    def __repr__(self):
        return "MinState(%r)" % self.minValue


class MaxState(State):
    KIND = L.DQ_OP_MAXIMUM

    def __init__(self, maxValue: float):
        self.maxValue = float(maxValue)

    def to_dq(self):
        return self._dq(value=self.maxValue)

    @classmethod
    def from_dq(cls, s):
        return cls(s.value)

    def __eq__(self, o):
        return isinstance(o, MaxState) and o.maxValue == self.maxValue

    def __hash__(self):
        return hash(("MaxState", self.maxValue))

    def __repr__(self):
        return "MaxState(%r)" % self.maxValue


class ApproxCountDistinctState(State):
    KIND = L.DQ_OP_APPROX_COUNT_DISTINCT

    def __init__(self, words: Sequence[int]):
        words = tuple(map(int, words))
        if len(words) != L.DQ_HLL_NUM_WORDS:
            raise ValueError("requirement failed: expected %d words" % L.DQ_HLL_NUM_WORDS)
        self.words: Tuple[int, ...] = words

    def to_dq(self):
        s = self._dq()
        s.words[:] = self.words
        return s

    @classmethod
    def from_dq(cls, s):
        return cls(s.words[:])

    def to_bytes(self) -> bytes:
        """DeequHyperLogLogPlusPlusUtils.wordsToBytes (StatefulHyperloglogPlus.scala:170-178)."""
        w = (ctypes.c_int64 * L.DQ_HLL_NUM_WORDS)(*self.words)
        out = (ctypes.c_uint8 * 416)()
        L.lib().dq_hll_words_to_bytes(w, out)
        return bytes(out)

    @classmethod
    def from_bytes(cls, b: bytes) -> "ApproxCountDistinctState":
        if len(b) != 416:
            raise ValueError("requirement failed: expected 416 bytes")
        buf = (ctypes.c_uint8 * 416)(*b)
        w = (ctypes.c_int64 * L.DQ_HLL_NUM_WORDS)()
        L.lib().dq_hll_words_from_bytes(buf, w)
        return cls(list(w))

    def __eq__(self, o):
        return isinstance(o, ApproxCountDistinctState) and o.words == self.words

    def __hash__(self):
        return hash(("ApproxCountDistinctState", self.words))

    def __repr__(self):
        return "ApproxCountDistinctState(%s)" % ",".join(str(w) for w in self.words)


class DataTypeHistogram(State):
    """DataTypeHistogram(numNull, numFractional, numIntegral, numBoolean, numString)
    (DataType.scala:40-52); sum adds the counts.  Not a DoubleValuedState."""
    KIND = L.DQ_OP_DATATYPE
    SIZE_IN_BYTES = 40

    def __init__(self, numNull: int, numFractional: int, numIntegral: int, numBoolean: int, numString: int):
        self.numNull, self.numFractional, self.numIntegral = int(numNull), int(numFractional), int(numIntegral)
        self.numBoolean, self.numString = int(numBoolean), int(numString)

    def counts(self) -> Tuple[int, int, int, int, int]:
        return (self.numNull, self.numFractional, self.numIntegral, self.numBoolean, self.numString)

    def to_dq(self):
        s = self._dq()
        for i, c in enumerate(self.counts()):
            s.words[i] = c
        return s

    @classmethod
    def from_dq(cls, s):
        return cls(*[s.words[i] for i in range(5)])

    def metricValue(self):
        raise TypeError("DataTypeHistogram is not a DoubleValuedState")

    def toBytes(self) -> bytes:
        """DataTypeHistogram.toBytes (DataType.scala:75-96): five big-endian longs."""
        import struct
        return struct.pack(">5q", *self.counts())

    @classmethod
    def fromBytes(cls, b: bytes) -> "DataTypeHistogram":
        import struct
        if len(b) != cls.SIZE_IN_BYTES:
            raise ValueError("requirement failed")
        return cls(*struct.unpack(">5q", b))

    def __eq__(self, o):
        return isinstance(o, DataTypeHistogram) and o.counts() == self.counts()

    def __hash__(self):
        return hash(("DataTypeHistogram",) + self.counts())

    def __repr__(self):
        return "DataTypeHistogram(%d,%d,%d,%d,%d)" % self.counts()


class CorrelationState(State):
    """CorrelationState(n, xAvg, yAvg, ck, xMk, yMk) (Correlation.scala:26-57)."""
    KIND = L.DQ_OP_CORRELATION

    def __init__(self, n: float, xAvg: float, yAvg: float, ck: float, xMk: float, yMk: float):
        if not n > 0.0:  # Correlation.scala:35
            raise ValueError("requirement failed: Correlation undefined for n = 0.")
        self.n, self.xAvg, self.yAvg = float(n), float(xAvg), float(yAvg)
        self.ck, self.xMk, self.yMk = float(ck), float(xMk), float(yMk)

    def fields(self) -> Tuple[float, ...]:
        return (self.n, self.xAvg, self.yAvg, self.ck, self.xMk, self.yMk)

    def to_dq(self):
        return self._dq(n=self.n, avg=self.xAvg, y_avg=self.yAvg, ck=self.ck, x_mk=self.xMk, y_mk=self.yMk)

    @classmethod
    def from_dq(cls, s):
        return cls(s.n, s.avg, s.y_avg, s.ck, s.x_mk, s.y_mk)

    def __eq__(self, o):
        return isinstance(o, CorrelationState) and o.fields() == self.fields()

    def __hash__(self):
        return hash(("CorrelationState",) + self.fields())

    def __repr__(self):
        return "CorrelationState(%r,%r,%r,%r,%r,%r)" % self.fields()


_BY_KIND = {
    L.DQ_OP_SIZE: NumMatches,
    L.DQ_OP_COMPLETENESS: NumMatchesAndCount,
    L.DQ_OP_COMPLIANCE: NumMatchesAndCount,
    L.DQ_OP_SUM: SumState,
    L.DQ_OP_MEAN: MeanState,
    L.DQ_OP_STDDEV: StandardDeviationState,
    L.DQ_OP_MINIMUM: MinState,
    L.DQ_OP_MAXIMUM: MaxState,
    L.DQ_OP_APPROX_COUNT_DISTINCT: ApproxCountDistinctState,
    L.DQ_OP_DATATYPE: DataTypeHistogram,
    L.DQ_OP_MIN_LENGTH: MinState,  # MinLength's state is a MinState (MinLength.scala:26)
    L.DQ_OP_MAX_LENGTH: MaxState,
    L.DQ_OP_CORRELATION: CorrelationState,
}


def state_from_dq(s: L.DqState) -> Optional[State]:
    """POD state from dq_plan_finish -> Option[State] (has_value = 0 is None)."""
    if not s.has_value:
        return None
    return _BY_KIND[s.kind].from_dq(s)


def merge(*states: Optional[State]) -> Optional[State]:
    """Analyzers.merge (Analyzer.scala:367-386)."""
    acc = None
    for s in states:
        if acc is None:
            acc = s
        elif s is not None:
            acc = acc.sum(s)
    return acc
