"""TEST INFRASTRUCTURE ONLY -- CPU restatement ("oracle") of deequ's metric hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import this module, and only as the checker.  The product (`deequ_amd`) never
imports it and has no CPU fallback.

What is restated (reference = /root/reference, deequ 1.0.3-SNAPSHOT on Spark 2.2.2):

* States and their algebra (`State.sum`, `metricValue`):
  NumMatches `Size.scala:23-31`, NumMatchesAndCount `Analyzer.scala:230-244`,
  SumState `Sum.scala:25-33`, MeanState `Mean.scala:25-34`,
  StandardDeviationState `StandardDeviation.scala:25-45`, MinState `Minimum.scala:25-33`,
  MaxState `Maximum.scala:25-33`, ApproxCountDistinctState `ApproxCountDistinct.scala:26-40`,
  FrequenciesAndNumRows `GroupingAnalyzers.scala:124-157`, Option merge `Analyzer.scala:367-386`.
* Aggregations with Spark 2.2.2 NULL semantics:
  Size `Size.scala:35-47`, Completeness `Completeness.scala:26-46`,
  Compliance `Compliance.scala:37-53`, Sum/Mean/Min/Max (`sum/count/min/max ... cast`),
  StandardDeviation = Spark `CentralMomentAgg` update/merge (row a-7 of SURVEY §8),
  conditionalSelection / conditionalCount `Analyzer.scala:409-432`.
* HLL++: `StatefulHyperloglogPlus.scala:89-115` (update), `:121-139`/`:188-208` (merge),
  `:210-297` (count / estimateBias), `:170-186` (words <-> bytes), constants
  `HLLConstants.scala:27-37` + the p=9 bias tables (`hll_p9_tables.py`).
  Hash: Spark 2.2.2 `XxHash64Function` = XXH64 with seed 42 over the 4-byte (int
  family, float bits), 8-byte (long, double bits) little-endian value or UTF-8 bytes.
  XXH64 itself is the third-party algorithm (Spark `XXH64` port of Yann Collet's
  xxHash64, not vendored); it is restated here from the published spec and pinned
  against the `xxhash` 3.8.1 Python binding.
* MinLength / MaxLength `MinLength.scala:25-41`, `MaxLength.scala:25-41`:
  min/max(length(sel)).cast(double), `length` = Spark 2.2.2 `UTF8String.numChars` (a walk
  over first bytes: 0xC0-0xDF skip 2, 0xE0-0xEF 3, 0xF0-0xF7 4, 0xF8-0xFB 5, 0xFC-0xFD 6,
  anything else 1).
* Correlation `Correlation.scala:26-105` + `catalyst/StatefulCorrelation.scala:24-49`
  (Spark 2.2.2 `Corr`: per-row update when both inputs are non-NULL, state
  (n, xAvg, yAvg, ck, xMk, yMk), merge `Correlation.scala:37-52`, metric ck/sqrt(xMk*yMk)).
* DataType: `StatefulDataType.scala:36-38,58-69` (regex classification of the value cast
  to string), `DataType.scala:98-143` (distribution, determineType).
* Frequency family: `GroupingAnalyzers.scala:53-80` (group-by, NULL rows dropped,
  numRows = all rows), Uniqueness `Uniqueness.scala:29-31`, Distinctness
  `Distinctness.scala:32-34`, Entropy `Entropy.scala:31-41`, CountDistinct
  `CountDistinct.scala:27-33`, UniqueValueRatio `UniqueValueRatio.scala:28-37`,
  Histogram `Histogram.scala:54-96` (cast to string, NULL -> "NullValue").

Parity pins: every known answer of the reference tests listed in SURVEY §8(c) is
encoded in `tests/golden/reference_known_answers.json` and checked against this
module by `tests/test_oracle_golden.py`.
"""
from __future__ import annotations

import math
import re
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

try:  # the oracle directory may be imported as a package or via sys.path
    from .hll_p9_tables import BIAS_P9, RAW_ESTIMATE_P9, THRESHOLD_P9
except ImportError:  # pragma: no cover
    from hll_p9_tables import BIAS_P9, RAW_ESTIMATE_P9, THRESHOLD_P9

MASK64 = (1 << 64) - 1

# ----------------------------------------------------------------------------
# XXH64 (published spec) + Spark 2.2.2 type dispatch
# ----------------------------------------------------------------------------
P1 = 0x9E3779B185EBCA87
P2 = 0xC2B2AE3D27D4EB4F
P3 = 0x165667B19E3779F9
P4 = 0x85EBCA77C2B2AE63
P5 = 0x27D4EB2F165667C5


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (64 - r))) & MASK64


def _round(acc: int, lane: int) -> int:
    acc = (acc + lane * P2) & MASK64
    acc = _rotl(acc, 31)
    return (acc * P1) & MASK64


def _merge_round(acc: int, val: int) -> int:
    acc ^= _round(0, val)
    return (acc * P1 + P4) & MASK64


def xxh64(data: bytes, seed: int = 42) -> int:
    """XXH64 over `data` (unsigned 64-bit result)."""
    n = len(data)
    seed &= MASK64
    i = 0
    if n >= 32:
        v1 = (seed + P1 + P2) & MASK64
        v2 = (seed + P2) & MASK64
        v3 = seed
        v4 = (seed - P1) & MASK64
        while i + 32 <= n:
            a, b, c, d = struct.unpack_from("<4Q", data, i)
            v1 = _round(v1, a)
            v2 = _round(v2, b)
            v3 = _round(v3, c)
            v4 = _round(v4, d)
            i += 32
        h = (_rotl(v1, 1) + _rotl(v2, 7) + _rotl(v3, 12) + _rotl(v4, 18)) & MASK64
        h = _merge_round(h, v1)
        h = _merge_round(h, v2)
        h = _merge_round(h, v3)
        h = _merge_round(h, v4)
    else:
        h = (seed + P5) & MASK64
    h = (h + n) & MASK64
    while i + 8 <= n:
        (k,) = struct.unpack_from("<Q", data, i)
        h ^= _round(0, k)
        h = (_rotl(h, 27) * P1 + P4) & MASK64
        i += 8
    if i + 4 <= n:
        (k,) = struct.unpack_from("<I", data, i)
        h ^= (k * P1) & MASK64
        h = (_rotl(h, 23) * P2 + P3) & MASK64
        i += 4
    while i < n:
        h ^= (data[i] * P5) & MASK64
        h = (_rotl(h, 11) * P1) & MASK64
        i += 1
    h ^= h >> 33
    h = (h * P2) & MASK64
    h ^= h >> 29
    h = (h * P3) & MASK64
    h ^= h >> 32
    return h


try:  # the reference C implementation, used for speed once xxh64() is pinned against it
    import xxhash as _xxhash

    def _xxh(data: bytes, seed: int) -> int:
        return _xxhash.xxh64_intdigest(data, seed)
except ImportError:  # pragma: no cover
    _xxh = None


def spark_hash(value, dtype: str, seed: int = 42) -> int:
    """Spark 2.2.2 `XxHash64Function.hash(value, dataType, seed)` for the types deequ
    feeds into HLL (unsigned 64-bit result; the caller reinterprets as signed)."""
    xxh64 = _xxh if _xxh is not None else globals()["xxh64"]
    if dtype in ("int8", "int16", "int32", "date32"):
        return xxh64(struct.pack("<i", int(value)), seed)
    if dtype == "bool":
        return xxh64(struct.pack("<i", 1 if value else 0), seed)
    if dtype in ("int64", "timestamp"):
        return xxh64(struct.pack("<q", int(value)), seed)
    if dtype == "float32":
        f = float(value)
        bits = 0x7FC00000 if math.isnan(f) else struct.unpack("<I", struct.pack("<f", f))[0]
        return xxh64(struct.pack("<I", bits), seed)
    if dtype == "float64":
        d = float(value)
        bits = 0x7FF8000000000000 if math.isnan(d) else struct.unpack("<Q", struct.pack("<d", d))[0]
        return xxh64(struct.pack("<Q", bits), seed)
    if dtype == "string":
        return xxh64(value.encode("utf-8") if isinstance(value, str) else bytes(value), seed)
    raise ValueError("unsupported hash type " + dtype)


# ----------------------------------------------------------------------------
# HLL++ (p = 9) exactly as StatefulHyperloglogPlus / DeequHyperLogLogPlusPlusUtils
# ----------------------------------------------------------------------------
HLL_P = 9
HLL_M = 1 << HLL_P
HLL_IDX_SHIFT = 64 - HLL_P
HLL_W_PADDING = 1 << (HLL_P - 1)
HLL_NUM_WORDS = 52
HLL_REGISTER_SIZE = 6
HLL_REGISTERS_PER_WORD = 10
HLL_REGISTER_WORD_MASK = (1 << HLL_REGISTER_SIZE) - 1
HLL_ALPHA_M2 = (0.7213 / (1.0 + 1.079 / HLL_M)) * HLL_M * HLL_M
HLL_K = 6


def _nlz64(x: int) -> int:
    return 64 - x.bit_length() if x else 64


def hll_index_and_rank(x: int) -> Tuple[int, int]:
    """`StatefulHyperloglogPlus.scala:96,99`: idx = x >>> 55; pw = nlz((x << 9) | 256) + 1."""
    idx = x >> HLL_IDX_SHIFT
    pw = _nlz64(((x << HLL_P) & MASK64) | HLL_W_PADDING) + 1
    return idx, pw


def hll_registers(values: Sequence, dtype: str) -> List[int]:
    """512 registers after updating with every non-null value (`:89-115`)."""
    regs = [0] * HLL_M
    for v in values:
        if v is None:
            continue
        idx, pw = hll_index_and_rank(spark_hash(v, dtype))
        if pw > regs[idx]:
            regs[idx] = pw
    return regs


def _to_signed64(u: int) -> int:
    return u - (1 << 64) if u >= (1 << 63) else u


def hll_pack(regs: Sequence[int]) -> List[int]:
    """Registers -> 52 signed Long words, 10 six-bit registers per word (`:102-113`)."""
    words = []
    for w in range(HLL_NUM_WORDS):
        word = 0
        for i in range(HLL_REGISTERS_PER_WORD):
            idx = w * HLL_REGISTERS_PER_WORD + i
            if idx < HLL_M:
                word |= (regs[idx] & HLL_REGISTER_WORD_MASK) << (HLL_REGISTER_SIZE * i)
        words.append(_to_signed64(word))
    return words


def hll_unpack(words: Sequence[int]) -> List[int]:
    regs = []
    for idx in range(HLL_M):
        w = words[idx // HLL_REGISTERS_PER_WORD] & MASK64
        regs.append((w >> (HLL_REGISTER_SIZE * (idx % HLL_REGISTERS_PER_WORD))) & HLL_REGISTER_WORD_MASK)
    return regs


def hll_merge(words1: Sequence[int], words2: Sequence[int]) -> List[int]:
    """`DeequHyperLogLogPlusPlusUtils.merge` (`:188-208`): per-register max."""
    return hll_pack([max(a, b) for a, b in zip(hll_unpack(words1), hll_unpack(words2))])


def _java_int_shift_one(m: int) -> int:
    """Java `1 << m` for Int with a Long shift count: the count is masked to 5 bits and
    the result is a signed 32-bit int (so 1 << 31 is negative, 1 << 32 == 1)."""
    r = (1 << (m & 31)) & 0xFFFFFFFF
    return r - (1 << 32) if r >= (1 << 31) else r


def _estimate_bias(e: float) -> float:
    """`DeequHyperLogLogPlusPlusUtils.estimateBias` (`:259-297`)."""
    estimates = RAW_ESTIMATE_P9
    n = len(estimates)
    # java.util.Arrays.binarySearch: index if found, else -(insertion point) - 1
    lo, hi, found = 0, n - 1, None
    while lo <= hi:
        mid = (lo + hi) >> 1
        if estimates[mid] < e:
            lo = mid + 1
        elif estimates[mid] > e:
            hi = mid - 1
        else:
            found = mid
            break
    nearest = found if found is not None else lo

    def distance(i):
        d = e - estimates[i]
        return d * d

    low = max(nearest - HLL_K + 1, 0)
    high = min(low + HLL_K, n)
    while high < n and distance(high) < distance(low):
        low += 1
        high += 1
    bias_sum = 0.0
    for i in range(low, high):
        bias_sum += BIAS_P9[i]
    return bias_sum / (high - low)


def _java_round(x: float) -> float:
    """Java `Math.round(double)` (floor(x + 0.5), saturating), returned as a double."""
    if math.isnan(x):
        return 0.0
    r = math.floor(x + 0.5)
    return float(max(min(r, 2 ** 63 - 1), -(2 ** 63)))


def hll_count(words: Sequence[int]) -> float:
    """`DeequHyperLogLogPlusPlusUtils.count` (`:210-257`), sequential order kept."""
    z_inverse = 0.0
    v = 0.0
    for idx in range(HLL_M):
        w = words[idx // HLL_REGISTERS_PER_WORD] & MASK64
        m = (w >> (HLL_REGISTER_SIZE * (idx % HLL_REGISTERS_PER_WORD))) & HLL_REGISTER_WORD_MASK
        z_inverse += 1.0 / _java_int_shift_one(m)
        if m == 0:
            v += 1.0

    def e_bias_corrected():
        e = HLL_ALPHA_M2 / z_inverse
        if HLL_P < 19 and e < 5.0 * HLL_M:
            return e - _estimate_bias(e)
        return e

    if v > 0:
        h = HLL_M * math.log(HLL_M / v)
        estimate = h if h <= THRESHOLD_P9 else e_bias_corrected()
    else:
        estimate = e_bias_corrected()
    return _java_round(estimate)


def hll_words_to_bytes(words: Sequence[int]) -> bytes:
    """`wordsToBytes` (`:170-178`): big-endian longs."""
    return struct.pack(">52q", *words)


def hll_words_from_bytes(b: bytes) -> List[int]:
    return list(struct.unpack(">52q", b))


# ----------------------------------------------------------------------------
# States (Scala case classes) and their algebra
# ----------------------------------------------------------------------------
@dataclass(frozen=True)
class NumMatches:
    num_matches: int

    def sum(self, o):
        return NumMatches(_wrap64(self.num_matches + o.num_matches))

    def metric_value(self):
        return float(self.num_matches)


@dataclass(frozen=True)
class NumMatchesAndCount:
    num_matches: int
    count: int

    def sum(self, o):
        return NumMatchesAndCount(_wrap64(self.num_matches + o.num_matches), _wrap64(self.count + o.count))

    def metric_value(self):
        return float("nan") if self.count == 0 else float(self.num_matches) / self.count


@dataclass(frozen=True)
class SumState:
    sum_: float

    def sum(self, o):
        return SumState(self.sum_ + o.sum_)

    def metric_value(self):
        return self.sum_


@dataclass(frozen=True)
class MeanState:
    sum_: float
    count: int

    def sum(self, o):
        return MeanState(self.sum_ + o.sum_, _wrap64(self.count + o.count))

    def metric_value(self):
        return float("nan") if self.count == 0 else self.sum_ / self.count


@dataclass(frozen=True)
class StandardDeviationState:
    n: float
    avg: float
    m2: float

    def __post_init__(self):
        if not self.n > 0.0:
            raise ValueError("Standard deviation is undefined for n = 0.")

    def sum(self, o):  # StandardDeviation.scala:37-44
        new_n = self.n + o.n
        delta = o.avg - self.avg
        delta_n = 0.0 if new_n == 0.0 else delta / new_n
        return StandardDeviationState(new_n, self.avg + delta_n * o.n,
                                      self.m2 + o.m2 + delta * delta_n * self.n * o.n)

    def metric_value(self):
        return math.sqrt(self.m2 / self.n)


def java_div(a: float, b: float) -> float:
    """Java double division (a / 0.0 is +-Infinity or NaN instead of an exception)."""
    if b != 0.0 or a != a or b != b:
        return a / b if b == b else float("nan")
    if a == 0.0:
        return float("nan")
    return math.copysign(math.inf, a) * math.copysign(1.0, b)


@dataclass
class CorrelationState:
    n: float
    xAvg: float
    yAvg: float
    ck: float
    xMk: float
    yMk: float

    def __post_init__(self):
        if not self.n > 0.0:
            raise ValueError("Correlation undefined for n = 0.")

    def sum(self, o):  # Correlation.scala:37-52
        n1, n2 = self.n, o.n
        new_n = n1 + n2
        dx = o.xAvg - self.xAvg
        dx_n = 0.0 if new_n == 0.0 else dx / new_n
        dy = o.yAvg - self.yAvg
        dy_n = 0.0 if new_n == 0.0 else dy / new_n
        return CorrelationState(new_n, self.xAvg + dx_n * n2, self.yAvg + dy_n * n2,
                                self.ck + o.ck + dx * dy_n * n1 * n2,
                                self.xMk + o.xMk + dx * dx_n * n1 * n2,
                                self.yMk + o.yMk + dy * dy_n * n1 * n2)

    def metric_value(self):  # ck / math.sqrt(xMk * yMk), Java arithmetic
        d = self.xMk * self.yMk
        return java_div(self.ck, math.sqrt(d) if d >= 0.0 else float("nan"))


def _java_min(a: float, b: float) -> float:
    """java.lang.Math.min(double, double): NaN-propagating, -0.0 < 0.0."""
    if a != a:
        return a
    if b != b:
        return b
    if a == 0.0 and b == 0.0:
        return a if math.copysign(1.0, a) < 0 else b
    return a if a <= b else b


def _java_max(a: float, b: float) -> float:
    if a != a:
        return a
    if b != b:
        return b
    if a == 0.0 and b == 0.0:
        return a if math.copysign(1.0, a) > 0 else b
    return a if a >= b else b


@dataclass(frozen=True)
class MinState:
    min_value: float

    def sum(self, o):
        return MinState(_java_min(self.min_value, o.min_value))

    def metric_value(self):
        return self.min_value


@dataclass(frozen=True)
class MaxState:
    max_value: float

    def sum(self, o):
        return MaxState(_java_max(self.max_value, o.max_value))

    def metric_value(self):
        return self.max_value


@dataclass(frozen=True)
class ApproxCountDistinctState:
    words: Tuple[int, ...]

    def sum(self, o):
        return ApproxCountDistinctState(tuple(hll_merge(self.words, o.words)))

    def metric_value(self):
        return hll_count(self.words)


@dataclass
class FrequenciesAndNumRows:
    frequencies: Dict[tuple, int]
    num_rows: int

    def sum(self, o):  # null-safe outer join, counts added (GroupingAnalyzers.scala:128-148)
        out = dict(self.frequencies)
        for k, c in o.frequencies.items():
            out[k] = out.get(k, 0) + c
        return FrequenciesAndNumRows(out, self.num_rows + o.num_rows)


def merge_options(*states):
    """`Analyzers.merge` (`Analyzer.scala:367-386`)."""
    acc = None
    for s in states:
        if acc is None:
            acc = s
        elif s is not None:
            acc = acc.sum(s)
    return acc


def _wrap64(x: int) -> int:
    x &= MASK64
    return x - (1 << 64) if x >= (1 << 63) else x


# ----------------------------------------------------------------------------
# Columns and the SQL predicate subset (independent evaluator, 3-valued logic)
# ----------------------------------------------------------------------------
@dataclass
class OColumn:
    """A column as Spark would see it: python values, None = SQL NULL."""
    dtype: str            # int8/int16/int32/int64/float32/float64/bool/string
    values: list

    @staticmethod
    def from_numpy(dtype: str, values: np.ndarray, valid: Optional[np.ndarray]):
        vals = values.tolist()
        if valid is not None:
            vals = [v if ok else None for v, ok in zip(vals, valid.tolist())]
        return OColumn(dtype, vals)


OTable = Dict[str, OColumn]

_INTEGRAL = ("int8", "int16", "int32", "int64")
_FRACTIONAL = ("float32", "float64")


class _Tok:
    def __init__(self, text: str):
        self.toks = self._lex(text)
        self.i = 0

    @staticmethod
    def _lex(s: str):
        out, i = [], 0
        while i < len(s):
            c = s[i]
            if c.isspace():
                i += 1
            elif c == "'":
                j = s.index("'", i + 1)
                out.append(("str", s[i + 1:j]))
                i = j + 1
            elif c.isdigit() or (c == "." and i + 1 < len(s) and s[i + 1].isdigit()):
                j = i
                while j < len(s) and (s[j].isdigit() or s[j] == "."):
                    j += 1
                if j < len(s) and s[j] in "eE":
                    j += 1
                    if s[j] in "+-":
                        j += 1
                    while j < len(s) and s[j].isdigit():
                        j += 1
                out.append(("num", s[i:j]))
                i = j
            elif c.isalpha() or c == "_" or c == "`":
                if c == "`":
                    j = s.index("`", i + 1)
                    out.append(("id", s[i + 1:j]))
                    i = j + 1
                    continue
                j = i
                while j < len(s) and (s[j].isalnum() or s[j] == "_"):
                    j += 1
                out.append(("id", s[i:j]))
                i = j
            else:
                for op in ("<=>", "<=", ">=", "!=", "<>", "==", "<", ">", "=", "(", ")", ",", "-"):
                    if s.startswith(op, i):
                        out.append(("op", op))
                        i += len(op)
                        break
                else:
                    raise ValueError("cannot lex %r" % s[i:])
        return out

    def peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else (None, None)

    def next(self):
        t = self.peek()
        self.i += 1
        return t

    def kw(self, word):
        t = self.peek()
        if t[0] == "id" and t[1].upper() == word:
            self.i += 1
            return True
        return False


def _java_to_string(v) -> str:
    """Cast(-> StringType) of an int / double literal or value (Java toString)."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    return java_double_to_string(float(v))


def java_parse_double(s: str) -> Optional[float]:
    """java.lang.Double.parseDouble of String.trim() (chars <= U+0020 trimmed), None when it
    throws NumberFormatException: Spark 2.2's Cast(StringType -> DoubleType)."""
    import re
    t = s
    while t and ord(t[0]) <= 0x20:
        t = t[1:]
    while t and ord(t[-1]) <= 0x20:
        t = t[:-1]
    m = re.fullmatch(r"([+-]?)(NaN|Infinity|((\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)[fFdD]?)", t, re.ASCII)
    if m:
        sign, body = m.group(1), m.group(2)
        if body == "NaN":
            return float("nan")
        if body == "Infinity":
            return float("-inf") if sign == "-" else float("inf")
        num = body.rstrip("fFdD")
        return float(sign + num)
    hm = re.fullmatch(r"([+-]?)0[xX]([0-9a-fA-F]*\.?[0-9a-fA-F]*)[pP]([+-]?\d+)[fFdD]?", t, re.ASCII)
    if hm and hm.group(2).strip("."):
        try:
            return float.fromhex(hm.group(1) + "0x" + hm.group(2) + "p" + hm.group(3))
        except OverflowError:  # rounds past Double.MAX_VALUE: Java gives Infinity
            return float("-inf") if hm.group(1) == "-" else float("inf")
    return None


_SQL_TYPES = {"TINYINT": "int8", "BYTE": "int8", "SMALLINT": "int16", "SHORT": "int16", "INT": "int32",
              "INTEGER": "int32", "BIGINT": "int64", "LONG": "int64", "FLOAT": "float32", "REAL": "float32",
              "DOUBLE": "float64", "BOOLEAN": "bool"}
_INT_BITS = {"int8": 8, "int16": 16, "int32": 32, "int64": 64}


def _wrap_bits(v: int, bits: int) -> int:
    """Scala .toByte / .toShort / .toInt / .toLong of an integral value: the low bits, signed."""
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >= (1 << (bits - 1)) else v


def _java_f2int(x: float, bits: int) -> int:
    """Java d2i (bits 32) / d2l (bits 64): NaN -> 0, saturating, truncation toward zero."""
    if x != x:
        return 0
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    if x >= hi:
        return hi
    if x <= lo:
        return lo
    return int(x)


def int_to_f32(v: int) -> float:
    """Java i2f / l2f: the exact integer rounded to the nearest float, ties to even."""
    if v == 0:
        return 0.0
    a = abs(v)
    sh = a.bit_length() - 24
    if sh > 0:
        q, rem = divmod(a, 1 << sh)
        if rem > (1 << (sh - 1)) or (rem == (1 << (sh - 1)) and q & 1):
            q += 1
        a = q << sh
    return float(a if v > 0 else -a)


def spark_cast(v, src: str, to: str):
    """Spark 2.2.2 Cast (non-ANSI) of one value of kind `src` (int / float / double / decimal /
    bool / string) to `to` (a dq type name): Cast.castToByte/Short/Int/Long (integral values keep
    their low bits; fractional ones go through Java d2i -- then the low bits for byte/short -- or
    d2l), castToFloat (l2f rounds the integer itself; a double rounds to nearest), castToDouble,
    castToBoolean (value != 0).  NULL stays NULL."""
    if v is None:
        return None
    if src == "bool":
        v = 1 if v else 0
        src = "int"
    if to in _INT_BITS:
        if src in ("float", "double"):
            x = _java_f2int(float(v), 64 if to == "int64" else 32)
            return _wrap_bits(x, _INT_BITS[to])
        if src == "decimal":  # Decimal.toLong (truncation), then the low bits
            from fractions import Fraction
            return _wrap_bits(math.trunc(Fraction(v)), _INT_BITS[to])
        if src == "int":
            return _wrap_bits(int(v), _INT_BITS[to])
        raise ValueError("cast of %s to %s is outside the restated subset" % (src, to))
    if to == "float32":
        if src == "int":
            return int_to_f32(int(v))
        if src in ("float", "double"):
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                return float(np.float32(float(v)))
        raise ValueError("cast of %s to float is outside the restated subset" % src)
    if to == "float64":
        if src == "string":
            return java_parse_double(v)
        return float(v)
    if to == "bool":
        if src == "string":
            raise ValueError("cast of a string to boolean is outside the restated subset")
        return float(v) != 0.0 if src in ("float", "double") else v != 0
    raise ValueError(to)


def eval_predicate(text: str, table: OTable) -> List[Optional[bool]]:
    """Evaluate a deequ SQL predicate string (the numeric subset deequ's checks emit:
    comparisons, IN, BETWEEN, IS [NOT] NULL, COALESCE, AND/OR/NOT, string equality)
    row by row with SQL three-valued logic.  Returns True/False/None per row."""
    nrows = len(next(iter(table.values())).values)
    tk = _Tok(text)

    def operand():
        t = tk.next()
        if t[0] == "op" and t[1] == "-":
            v = operand()
            return ("neg", v)
        if t[0] == "op" and t[1] == "(":
            e = or_expr()
            assert tk.next() == ("op", ")")
            return ("paren", e)
        if t[0] == "num":
            return ("lit", ("int" if all(ch.isdigit() for ch in t[1]) else
                            ("double" if "e" in t[1].lower() else "decimal")), t[1])
        if t[0] == "str":  # adjacent literals concatenate (Spark 2.2 grammar: STRING+)
            v = t[1]
            while tk.peek()[0] == "str":
                v += tk.next()[1]
            return ("lit", "string", v)
        if t[0] == "id":
            if t[1].upper() == "CAST" and tk.peek() == ("op", "("):
                tk.next()
                inner = operand()
                assert tk.kw("AS"), "CAST without AS in %r" % text
                tname = tk.next()[1].upper()
                assert tk.next() == ("op", ")")
                return ("cast", inner, _SQL_TYPES[tname])
            if t[1].upper() == "COALESCE":
                assert tk.next() == ("op", "(")
                args = [operand()]
                while tk.peek() == ("op", ","):
                    tk.next()
                    args.append(operand())
                assert tk.next() == ("op", ")")
                return ("coalesce", args)
            if t[1].upper() in ("TRUE", "FALSE"):
                return ("lit", "bool", t[1].upper() == "TRUE")
            if t[1].upper() == "NULL":
                return ("lit", "null", None)
            return ("col", t[1])
        raise ValueError("bad operand %r" % (t,))

    def comparison():
        left = operand()
        t = tk.peek()
        if t[0] == "op" and t[1] in ("<", "<=", ">", ">=", "=", "==", "!=", "<>", "<=>"):
            tk.next()
            return ("cmp", t[1], left, operand())
        negate = False
        if tk.kw("NOT"):
            negate = True
        if tk.kw("IN"):
            assert tk.next() == ("op", "(")
            items = [operand()]
            while tk.peek() == ("op", ","):
                tk.next()
                items.append(operand())
            assert tk.next() == ("op", ")")
            e = ("in", left, items)
            return ("not", e) if negate else e
        if tk.kw("BETWEEN"):
            lo = operand()
            assert tk.kw("AND")
            hi = operand()
            e = ("and", ("cmp", ">=", left, lo), ("cmp", "<=", left, hi))
            return ("not", e) if negate else e
        if tk.kw("IS"):
            neg = tk.kw("NOT")
            assert tk.kw("NULL")
            return ("isnotnull" if neg else "isnull", left)
        assert not negate
        return ("bool", left)

    def not_expr():
        if tk.kw("NOT"):
            return ("not", not_expr())
        return comparison()

    def and_expr():
        e = not_expr()
        while tk.kw("AND"):
            e = ("and", e, not_expr())
        return e

    def or_expr():
        e = and_expr()
        while tk.kw("OR"):
            e = ("or", e, and_expr())
        return e

    tree = or_expr()
    assert tk.peek() == (None, None), "trailing tokens in %r" % text

    def typed(node):
        """Returns (kind, getter) where kind in int/decimal/double/string/bool."""
        if node[0] == "lit":
            kind, v = node[1], node[2]
            if kind == "int":
                return "int", lambda r, x=int(v): x
            if kind == "decimal":
                from fractions import Fraction
                return "decimal", lambda r, x=Fraction(v): x
            if kind == "double":
                return "double", lambda r, x=float(v): x
            if kind == "string":
                return "string", lambda r, x=v: x
            if kind == "bool":
                return "bool", lambda r, x=v: x
            return "null", lambda r: None
        if node[0] == "col":
            col = table[node[1]]
            # FloatType keeps its own kind: Spark 2.2 compares float vs int/long as FloatType
            kind = ("int" if col.dtype in _INTEGRAL else "float" if col.dtype == "float32"
                    else "double" if col.dtype in _FRACTIONAL else col.dtype)
            return kind, lambda r, c=col: c.values[r]
        if node[0] == "paren":
            return typed(node[1])
        if node[0] == "cast":
            k, g = typed(node[1])
            to = node[2]
            kind = {"float32": "float", "float64": "double", "bool": "bool"}.get(to, "int")
            return kind, lambda r: spark_cast(g(r), k, to)
        if node[0] == "neg":
            k, g = typed(node[1])
            return k, lambda r: None if g(r) is None else -g(r)
        if node[0] == "coalesce":
            parts = [typed(a) for a in node[1]]
            kinds = [k for k, _ in parts if k != "null"]
            kind = _common(kinds)

            def get(r):
                for _, g in parts:
                    v = g(r)
                    if v is not None:
                        return v
                return None
            return kind, get
        return "bool", lambda r, n=node: ev(n, r)

    def _common(kinds):
        # Spark 2.2 TypeCoercion: float vs int/long -> FloatType; decimal vs float/double -> double
        if "double" in kinds:
            return "double"
        if "float" in kinds:
            return "double" if "decimal" in kinds else "float"
        if "decimal" in kinds:
            return "decimal"
        if "int" in kinds:
            return "int"
        return kinds[0] if kinds else "null"

    def conv(v, src, dst):
        if v is None:
            return None
        if dst == "double":
            return float(v)
        if dst == "float":  # Java i2f / l2f round the integer itself (no double rounding)
            if isinstance(v, int) and not isinstance(v, bool):
                return int_to_f32(v)
            return float(np.float32(v))
        if dst == "decimal":
            from fractions import Fraction
            return Fraction(v) if not isinstance(v, float) else Fraction(v)
        if dst == "int":
            return int(v)
        if dst == "string" and src in ("int", "double", "decimal"):
            return str(v)
        return v

    def coerced_pair(a, b):
        ka, ga = typed(a)
        kb, gb = typed(b)
        if ka == kb:
            return ka, ga, kb, gb, ka
        if "string" in (ka, kb) and ka in ("int", "float", "double", "decimal", "string") and kb in (
                "int", "float", "double", "decimal", "string"):
            # Spark 2.2 PromoteStrings: numeric vs string compares as double
            return ka, ga, kb, gb, "double_from_string"
        target = _common([ka, kb])
        return ka, ga, kb, gb, target

    def cmp_values(op, x, y):
        if op in ("=", "==", "<=>"):
            return x == y
        if op in ("!=", "<>"):
            return x != y
        if op == "<":
            return x < y
        if op == "<=":
            return x <= y
        if op == ">":
            return x > y
        if op == ">=":
            return x >= y
        raise ValueError(op)

    def ev(node, r):
        t = node[0]
        if t == "cmp":
            op = node[1]
            ka, ga, kb, gb, target = coerced_pair(node[2], node[3])
            x, y = ga(r), gb(r)
            if op == "<=>":
                if x is None or y is None:
                    return x is None and y is None
            if x is None or y is None:
                return None
            if target == "double_from_string":  # Cast(-> DoubleType): Java parseDouble
                x = java_parse_double(x) if isinstance(x, str) else float(x)
                y = java_parse_double(y) if isinstance(y, str) else float(y)
                if x is None or y is None:
                    return None
            else:
                x, y = conv(x, ka, target), conv(y, kb, target)
            if isinstance(x, float) and isinstance(y, float) and (x != x or y != y):
                # Spark double comparison: NaN = NaN is true and NaN is the largest value
                xn, yn = x != x, y != y
                if op in ("=", "==", "<=>"):
                    return xn and yn
                if op in ("!=", "<>"):
                    return not (xn and yn)
                order = (1 if xn else 0) - (1 if yn else 0)
                return {"<": order < 0, "<=": order <= 0, ">": order > 0, ">=": order >= 0}[op]
            return cmp_values(op, x, y)
        if t == "in":
            kx, gx = typed(node[1])
            x = gx(r)
            if x is None:
                return None
            kinds = {kx} | {typed(item)[0] for item in node[2]}
            if "string" in kinds and kinds - {"string", "null"}:
                # Spark 2.2 InConversion: a string/number IN list compares as strings
                xs = x if kx == "string" else _java_to_string(x)
                saw_null = False
                for item in node[2]:
                    v = typed(item)[1](r)
                    if v is None:
                        saw_null = True
                    elif xs == (v if isinstance(v, str) else _java_to_string(v)):
                        return True
                return None if saw_null else False
            saw_null = False
            for item in node[2]:
                res = ev(("cmp", "=", node[1], item), r)
                if res is True:
                    return True
                if res is None:
                    saw_null = True
            return None if saw_null else False
        if t == "and":
            a, b = ev(node[1], r), ev(node[2], r)
            if a is False or b is False:
                return False
            if a is None or b is None:
                return None
            return True
        if t == "or":
            a, b = ev(node[1], r), ev(node[2], r)
            if a is True or b is True:
                return True
            if a is None or b is None:
                return None
            return False
        if t == "not":
            a = ev(node[1], r)
            return None if a is None else (not a)
        if t == "isnull":
            return typed(node[1])[1](r) is None
        if t == "isnotnull":
            return typed(node[1])[1](r) is not None
        if t == "bool":
            return typed(node[1])[1](r)
        if t == "paren":
            return ev(node[1], r)
        raise ValueError(t)

    return [ev(tree, r) for r in range(nrows)]


# ----------------------------------------------------------------------------
# Analyzer aggregations (Spark 2.2.2 semantics) -> Optional[State]
# ----------------------------------------------------------------------------
def _where_mask(table: OTable, where: Optional[str]):
    n = len(next(iter(table.values())).values)
    if where is None:
        return [True] * n
    return eval_predicate(where, table)


def _selected_values(table: OTable, column: str, where: Optional[str]):
    """`conditionalSelection` (`Analyzer.scala:413-426`): when(cond, col) is NULL when the
    condition is false or NULL."""
    w = _where_mask(table, where)
    return [v if w[i] is True else None for i, v in enumerate(table[column].values)]


def _conditional_count(table: OTable, where: Optional[str]) -> Optional[int]:
    """`conditionalCount` (`Analyzer.scala:428-432`): count(*) or sum(cast(where as long))."""
    n = len(next(iter(table.values())).values)
    if where is None:
        return n
    w = _where_mask(table, where)
    nonnull = [x for x in w if x is not None]
    if not nonnull:
        return None
    return sum(1 for x in nonnull if x)


def size_state(table: OTable, where: Optional[str] = None):
    c = _conditional_count(table, where)
    return None if c is None else NumMatches(c)


def completeness_state(table: OTable, column: str, where: Optional[str] = None):
    n = len(table[column].values)
    if n == 0:
        return None  # sum over zero rows is NULL
    sel = _selected_values(table, column, where)
    matches = sum(1 for v in sel if v is not None)
    count = _conditional_count(table, where)
    return None if count is None else NumMatchesAndCount(matches, count)


def compliance_state(table: OTable, predicate: str, where: Optional[str] = None):
    pred = eval_predicate(predicate, table)
    w = _where_mask(table, where)
    sel = [p if w[i] is True else None for i, p in enumerate(pred)]
    nonnull = [p for p in sel if p is not None]
    if not nonnull:
        return None
    count = _conditional_count(table, where)
    if count is None:
        return None
    return NumMatchesAndCount(sum(1 for p in nonnull if p), count)


def _numeric_selected(table, column, where):
    col = table[column]
    vals = [v for v in _selected_values(table, column, where) if v is not None]
    return col.dtype, vals


def _spark_sum(dtype, vals):
    if dtype in _INTEGRAL:
        return float(_wrap64(sum(int(v) for v in vals)))
    acc = 0.0
    for v in vals:  # sequential fp64 as Spark's Sum within one partition
        acc += float(v)
    return acc


def sum_state(table: OTable, column: str, where: Optional[str] = None):
    dtype, vals = _numeric_selected(table, column, where)
    return None if not vals else SumState(_spark_sum(dtype, vals))


def mean_state(table: OTable, column: str, where: Optional[str] = None):
    dtype, vals = _numeric_selected(table, column, where)
    return None if not vals else MeanState(_spark_sum(dtype, vals), len(vals))


def stddev_state(table: OTable, column: str, where: Optional[str] = None):
    """Spark `CentralMomentAgg` (momentOrder 2) per-row update, one partition."""
    _, vals = _numeric_selected(table, column, where)
    n = avg = m2 = 0.0
    for v in vals:
        x = float(v)
        n += 1.0
        delta = x - avg
        delta_n = delta / n
        avg += delta_n
        m2 += delta * (delta - delta_n)
    return None if n == 0.0 else StandardDeviationState(n, avg, m2)


def _spark_double_lt(a: float, b: float) -> bool:
    """Spark NaN-safe ordering for doubles: NaN is the largest value, -0.0 == 0.0."""
    an, bn = a != a, b != b
    if an or bn:
        return (not an) and bn
    return a < b


def min_state(table: OTable, column: str, where: Optional[str] = None):
    dtype, vals = _numeric_selected(table, column, where)
    if not vals:
        return None
    if dtype in _INTEGRAL:
        return MinState(float(min(int(v) for v in vals)))
    best = float(vals[0])
    for v in vals[1:]:
        if _spark_double_lt(float(v), best):
            best = float(v)
    return MinState(best)


def max_state(table: OTable, column: str, where: Optional[str] = None):
    dtype, vals = _numeric_selected(table, column, where)
    if not vals:
        return None
    if dtype in _INTEGRAL:
        return MaxState(float(max(int(v) for v in vals)))
    best = float(vals[0])
    for v in vals[1:]:
        if _spark_double_lt(best, float(v)):
            best = float(v)
    return MaxState(best)


def utf8_num_chars(b: bytes) -> int:
    """Spark 2.2.2 `UTF8String.numChars`: count the first bytes visited by the walk
    `i += numBytesForFirstByte(b[i])` (0xFE/0xFF, an index error in 2.2.2, step 1 here)."""
    n = i = 0
    while i < len(b):
        c = b[i]
        i += 2 if 0xC0 <= c <= 0xDF else 3 if 0xE0 <= c <= 0xEF else 4 if 0xF0 <= c <= 0xF7 else \
            5 if 0xF8 <= c <= 0xFB else 6 if 0xFC <= c <= 0xFD else 1
        n += 1
    return n


def _lengths_selected(table, column, where):
    return [utf8_num_chars(v.encode("utf-8")) for v in _selected_values(table, column, where) if v is not None]


def min_length_state(table: OTable, column: str, where: Optional[str] = None):
    lens = _lengths_selected(table, column, where)
    return MinState(float(min(lens))) if lens else None


def max_length_state(table: OTable, column: str, where: Optional[str] = None):
    lens = _lengths_selected(table, column, where)
    return MaxState(float(max(lens))) if lens else None


def correlation_state(table: OTable, first: str, second: str, where: Optional[str] = None):
    """Spark 2.2.2 `Corr` update per row with both inputs non-NULL (cast to double), one
    partition; None when no row qualifies (Correlation.scala:77-96)."""
    xs = _selected_values(table, first, where)
    ys = _selected_values(table, second, where)
    n = xa = ya = ck = xmk = ymk = 0.0
    for xv, yv in zip(xs, ys):
        if xv is None or yv is None:
            continue
        x, y = float(xv), float(yv)
        new_n = n + 1.0
        dx = x - xa
        dx_n = dx / new_n
        dy = y - ya
        dy_n = dy / new_n
        new_xa = xa + dx_n
        new_ya = ya + dy_n
        ck += dx * (y - new_ya)
        xmk += dx * (x - new_xa)
        ymk += dy * (y - new_ya)
        n, xa, ya = new_n, new_xa, new_ya
    return CorrelationState(n, xa, ya, ck, xmk, ymk) if n > 0.0 else None


def approx_count_distinct_state(table: OTable, column: str, where: Optional[str] = None):
    """Never None: the HLL aggregate is non-nullable (`StatefulHyperloglogPlus.scala:59`)."""
    col = table[column]
    vals = _selected_values(table, column, where)
    return ApproxCountDistinctState(tuple(hll_pack(hll_registers(vals, col.dtype))))


# ---------------------------------------------------------------------------- DataType
# `StatefulDataType.update` (catalyst/StatefulDataType.scala:36-38, 58-69): the value cast to
# string (Spark 2.2 Cast: Java toString for numbers/booleans) is matched, in this order, against
# FRACTIONAL / INTEGRAL / BOOLEAN with whole-string matching; Java `\d` is [0-9].
_DT_FRACTIONAL = re.compile(r"(-|\+)? ?[0-9]*\.[0-9]*")
_DT_INTEGRAL = re.compile(r"(-|\+)? ?[0-9]*")
_DT_BOOLEAN = re.compile(r"(true|false)")


def _datatype_class(v, dtype: str) -> int:
    """0 null, 1 fractional, 2 integral, 3 boolean, 4 string (DataTypeHistogram positions)."""
    if v is None:
        return 0
    s = v if dtype == "string" else _spark_cast_string(v, dtype)
    if _DT_FRACTIONAL.fullmatch(s):
        return 1
    if _DT_INTEGRAL.fullmatch(s):
        return 2
    if _DT_BOOLEAN.fullmatch(s):
        return 3
    return 4


def datatype_state(table: OTable, column: str, where: Optional[str] = None):
    """`DataType.computeStateFrom` (`DataType.scala:157-165`): never None (the UDAF always
    returns its buffer); where-filtered rows are NULL inputs (conditionalSelection)."""
    col = table[column]
    counts = [0, 0, 0, 0, 0]
    for v in _selected_values(table, column, where):
        counts[_datatype_class(v, col.dtype)] += 1
    return tuple(counts)


def frequencies_state(table: OTable, columns: Sequence[str]) -> FrequenciesAndNumRows:
    """`computeFrequencies` (`GroupingAnalyzers.scala:53-80`)."""
    n = len(table[columns[0]].values)
    freq: Dict[tuple, int] = {}
    for r in range(n):
        key = tuple(table[c].values[r] for c in columns)
        if any(k is None for k in key):
            continue
        key = tuple(_group_key(k, table[c].dtype) for k, c in zip(key, columns))
        freq[key] = freq.get(key, 0) + 1
    return FrequenciesAndNumRows(freq, n)


def _group_key(v, dtype):
    """Spark 2.2.2 groups by the UnsafeRow bytes of the key: floating keys group by their raw
    bits (-0.0 and 0.0 are different groups; float normalisation only arrived in Spark 3.0,
    SPARK-26021).  Python floats carry the bits, so the bit pattern is the group key."""
    if dtype == "float64":
        return ("f64bits", struct.unpack("<Q", struct.pack("<d", float(v)))[0])
    if dtype == "float32":
        return ("f32bits", struct.unpack("<I", struct.pack("<f", float(v)))[0])
    return v


def uniqueness_metric(state: FrequenciesAndNumRows) -> Optional[float]:
    if not state.frequencies:
        return None  # sum over an empty frequency table is NULL -> empty-state failure
    return sum(1.0 for c in state.frequencies.values() if c == 1) / state.num_rows


def distinctness_metric(state: FrequenciesAndNumRows) -> Optional[float]:
    if not state.frequencies:
        return None
    return sum(1.0 for c in state.frequencies.values() if c >= 1) / state.num_rows


def count_distinct_metric(state: FrequenciesAndNumRows) -> float:
    return float(len(state.frequencies))


def unique_value_ratio_metric(state: FrequenciesAndNumRows) -> float:
    """`UniqueValueRatio.scala:28-37`: with no groups the numerator sum is NULL and
    `Row.getDouble` throws -- a failure metric, signalled here by ValueError."""
    if not state.frequencies:
        raise ValueError("Value at index 0 is null")
    uniq = sum(1.0 for c in state.frequencies.values() if c == 1)
    return uniq / float(len(state.frequencies))


def mutual_information_metric(state: FrequenciesAndNumRows, columns: Sequence[str],
                              grouping: Sequence[str]) -> Optional[float]:
    """`MutualInformation.scala:34-84`: joint counts joined with both marginals, summing
    (pxy/N)·ln((pxy/N)/((px/N)(py/N))).  None (empty state) when there are no groups.
    `grouping` is the state's key column order."""
    if not state.frequencies:
        return None
    i1, i2 = grouping.index(columns[0]), grouping.index(columns[1])
    m1: Dict = {}
    m2: Dict = {}
    for k, c in state.frequencies.items():
        m1[k[i1]] = m1.get(k[i1], 0) + c
        m2[k[i2]] = m2.get(k[i2], 0) + c
    total = state.num_rows
    out = 0.0
    for k, c in state.frequencies.items():
        px, py, pxy = float(m1[k[i1]]), float(m2[k[i2]]), float(c)
        out += (pxy / total) * math.log((pxy / total) / ((px / total) * (py / total)))
    return out


def entropy_metric(state: FrequenciesAndNumRows, ordered_counts: Optional[Sequence[int]] = None):
    """Σ −(c/N)·ln(c/N); `ordered_counts` fixes the fp64 summation order."""
    counts = list(ordered_counts) if ordered_counts is not None else list(state.frequencies.values())
    if not counts:
        return None
    n = state.num_rows
    total = 0.0
    for c in counts:
        c = float(c)
        total += 0.0 if c == 0.0 else -(c / n) * math.log(c / n)
    return total


def entropy_exact(state: FrequenciesAndNumRows) -> Optional[float]:
    if not state.frequencies:
        return None
    n = state.num_rows
    return math.fsum(-(c / n) * math.log(c / n) for c in state.frequencies.values())


def java_double_to_string(d: float, single: bool = False) -> str:
    """Java `Double.toString` / `Float.toString` (`single`): the shortest decimal that
    rounds back to the value (when that has one digit, the closest decimal of at most two
    digits, e.g. 4.9E-324), plain for 1e-3 <= |d| < 1e7, else `d.dddE±n`.  The JDK 19+
    rule; older JDKs agree on the values the reference tests use."""
    import numpy as np
    if d != d:
        return "NaN"
    if d == math.inf:
        return "Infinity"
    if d == -math.inf:
        return "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    a = abs(d)
    to_bin = (lambda x: float(np.float32(x))) if single else float
    # shortest round-trip digit string, searched by precision (independent of repr())
    for prec in range(1, 18):
        cand = "%.*e" % (prec - 1, a) if not single else \
            np.format_float_scientific(np.float32(a), precision=prec - 1, unique=False)
        if to_bin(float(cand)) == a:
            break
    mant, exp = cand.lower().split("e")
    digits = mant.replace(".", "").rstrip("0") or "0"
    e10 = int(exp)
    if len(digits) == 1:
        two = "%.1e" % a if not single else np.format_float_scientific(np.float32(a), precision=1, unique=False)
        m2, x2 = two.lower().split("e")
        digits, e10 = m2.replace(".", "").rstrip("0") or "0", int(x2)  # closest 2-digit decimal
    point = e10 + 1
    sign = "-" if d < 0 else ""
    if 1e-3 <= a < 1e7:
        if point <= 0:
            body = "0." + "0" * (-point) + digits
        elif point >= len(digits):
            body = digits + "0" * (point - len(digits)) + ".0"
        else:
            body = digits[:point] + "." + digits[point:]
        return sign + body
    return sign + digits[0] + "." + (digits[1:] or "0") + "E" + str(e10)


def histogram_state(table: OTable, column: str) -> FrequenciesAndNumRows:
    """`Histogram.computeStateFrom` (`Histogram.scala:54-69`): cast to string, NULL ->
    "NullValue", group-by count, numRows = data.count()."""
    col = table[column]
    freq: Dict[tuple, int] = {}
    for v in col.values:
        key = "NullValue" if v is None else _spark_cast_string(v, col.dtype)
        freq[(key,)] = freq.get((key,), 0) + 1
    return FrequenciesAndNumRows(freq, len(col.values))


def _spark_cast_string(v, dtype):
    if dtype in _INTEGRAL:
        return str(int(v))
    if dtype in _FRACTIONAL:
        return java_double_to_string(float(v), single=(dtype == "float32"))
    if dtype == "bool":
        return "true" if v else "false"
    return str(v)


def histogram_metric(state: FrequenciesAndNumRows, max_detail_bins: int = 1000):
    """Distribution(values: top-N by count, numberOfBins).  Ties at the cut are broken by
    key (ascending) here; Spark's `rdd.top` breaks them arbitrarily."""
    items = sorted(state.frequencies.items(), key=lambda kv: (-kv[1], kv[0]))
    top = items[:max_detail_bins]
    return {
        "number_of_bins": len(state.frequencies),
        "values": {k[0]: (c, c / state.num_rows) for k, c in top},
    }


# ---------------------------------------------------------------------------- ColumnProfiler
# `ColumnProfiler.profile` (profiles/ColumnProfiler.scala:91-208) restated over the functions
# above: pass 1 (:220-238) Completeness + ApproxCountDistinct (+ DataType for string columns) +
# Size; type decision `DataType.determineType` (DataType.scala:116-143) or the schema type
# (:401-420); pass 2 (:240-251, casts :427-445) Min/Max/Mean/StdDev/Sum of the numeric columns,
# string columns typed Integral / Fractional cast to LongType / DoubleType first; pass 3
# (:535-606) exact histograms of the columns with approxNumDistinct <= threshold:
# (value.toString, count), NULL -> "NullValue", ratio = count / sum of the column's counts.
DT_UNKNOWN, DT_FRACTIONAL, DT_INTEGRAL, DT_BOOLEAN, DT_STRING = 0, 1, 2, 3, 4  # DataTypeInstances


def spark_string_to_long(s: str) -> Optional[int]:
    """Spark 2.2.2 Cast(StringType -> LongType) = `UTF8String.toLong`: optional sign, digits,
    optionally '.' and digits (truncated); no trimming; NULL on anything else or overflow."""
    b = s.encode("utf-8")
    if not b:
        return None
    neg = b[:1] == b"-"
    i = 1 if (neg or b[:1] == b"+") else 0
    if i and len(b) == 1:
        return None
    r = 0
    while i < len(b):
        c = b[i]
        i += 1
        if c == 0x2E:  # '.'
            break
        if not 0x30 <= c <= 0x39:
            return None
        r = r * 10 + (c - 0x30)
    if any(not 0x30 <= c <= 0x39 for c in b[i:]):
        return None
    r = -r if neg else r
    return r if -(1 << 63) <= r < (1 << 63) else None


def determine_type(counts: Sequence[int]) -> int:
    """`DataType.determineType` (DataType.scala:116-143) on the DataTypeHistogram counts
    (null, fractional, integral, boolean, string)."""
    n_null, n_frac, n_int, n_bool, n_str = counts
    total = sum(counts)
    if total == 0 or n_null == total:
        return DT_UNKNOWN
    if n_str > 0 or (n_bool > 0 and (n_int > 0 or n_frac > 0)):
        return DT_STRING
    if n_bool > 0:
        return DT_BOOLEAN
    if n_frac > 0:
        return DT_FRACTIONAL
    return DT_INTEGRAL


def _schema_type(dtype: str) -> int:
    """extractGenericStatistics' schema mapping (ColumnProfiler.scala:401-420)."""
    if dtype in ("int16", "int32", "int64"):
        return DT_INTEGRAL
    if dtype in _FRACTIONAL:
        return DT_FRACTIONAL
    if dtype == "bool":
        return DT_BOOLEAN
    return DT_UNKNOWN


def column_profiles(table: OTable, threshold: int = 120,
                    predefined: Optional[Dict[str, int]] = None) -> Dict[str, dict]:
    """{column: profile fields} as ColumnProfiler.profile builds them (no KLL, the reference's
    default).  Numeric fields are the Spark one-partition values (sequential sum, Welford).
    `predefined` types replace both inference and the schema type (typeOf, :31-46)."""
    predefined = predefined or {}
    n_rows = len(next(iter(table.values())).values) if table else 0
    out: Dict[str, dict] = {}
    for name, col in table.items():
        comp = completeness_state(table, name)
        words = approx_count_distinct_state(table, name).words
        approx = int(hll_count(words))  # Double.toLong of a rounded count
        p = {"completeness": comp.metric_value(), "approx": approx, "words": tuple(words),
             "typeCounts": {}, "inferred": False}
        if name in predefined:
            p["dataType"] = predefined[name]
        elif col.dtype == "string":
            counts = datatype_state(table, name)
            p["dataType"] = determine_type(counts)
            p["inferred"] = True
            p["typeCounts"] = dict(zip(("Unknown", "Fractional", "Integral", "Boolean", "String"), counts))
        else:
            p["dataType"] = _schema_type(col.dtype)
        # pass 2 on the (cast) column
        if p["dataType"] in (DT_INTEGRAL, DT_FRACTIONAL):
            if col.dtype == "string":
                if p["dataType"] == DT_INTEGRAL:
                    cast = OColumn("int64", [None if v is None else spark_string_to_long(v) for v in col.values])
                else:
                    cast = OColumn("float64", [None if v is None else java_parse_double(v) for v in col.values])
            else:
                cast = col
            t1 = {name: cast}
            for key, fn in (("minimum", min_state), ("maximum", max_state), ("mean", mean_state),
                            ("stdDev", stddev_state), ("sum", sum_state)):
                st = fn(t1, name)
                p[key] = None if st is None else st.metric_value()
            p["numeric_values"] = [v for v in cast.values if v is not None]
        # pass 3
        p["histogram"] = None
        if approx <= threshold and p["dataType"] in (DT_STRING, DT_BOOLEAN, DT_INTEGRAL, DT_FRACTIONAL) \
                and col.dtype in ("string", "bool", "float64", "float32", "int32", "int64", "int16"):
            counts: Dict[str, int] = {}
            for v in col.values:
                k = "NullValue" if v is None else _spark_cast_string(v, col.dtype)
                counts[k] = counts.get(k, 0) + 1
            total = sum(counts.values())
            p["histogram"] = {k: (c, c / total) for k, c in counts.items()}
        out[name] = p
    out["__numRecords__"] = n_rows  # type: ignore[assignment]
    return out
