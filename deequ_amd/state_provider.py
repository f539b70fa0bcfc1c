"""HdfsStateProvider: states on a filesystem in the reference's binary layout
(analyzers/StateProvider.scala:72-311), so states written here load in Spark deequ and the
other way round.  Local paths (the reference goes through Hadoop's FileSystem, which also
covers HDFS/S3; only the local filesystem is reachable from this backend).

Layout per analyzer, `id` = MurmurHash3.stringHash(analyzer.toString, 42) as a decimal Int
(StateProvider.scala:82-84), every number big-endian as java.io.DataOutputStream writes it:

  Size                              {prefix}-{id}.bin   long numMatches
  Completeness, Compliance          {prefix}-{id}.bin   long numMatches, long count
  Sum, Minimum, Maximum,
  MinLength, MaxLength              {prefix}-{id}.bin   double
  Mean                              {prefix}-{id}.bin   double sum, long count
  StandardDeviation                 {prefix}-{id}.bin   double n, avg, m2
  Correlation                       {prefix}-{id}.bin   double n, xAvg, yAvg, ck, xMk, yMk
  DataType                          {prefix}-{id}.bin   int 40, DataTypeHistogram.toBytes
  ApproxCountDistinct               {prefix}-{id}.bin   int 416, wordsToBytes (52 big-endian longs)
  FrequencyBasedAnalyzer, Histogram {prefix}-{id}-frequencies.pqt (parquet: the grouping columns +
                                    com_amazon_deequ_dq_metrics_count) and
                                    {prefix}-{id}-num_rows.bin (long)

Without `allowOverwrite` an existing state is an error, as the reference's
writeToFileOnDfs / SaveMode.ErrorIfExists make it (StateProviderTest.scala:105-130).
"""
from __future__ import annotations

import os
import shutil
import struct
from typing import List

import numpy as np

from .analyzers import (ApproxCountDistinct, Completeness, Compliance, Correlation, DataType,
                        FrequencyBasedAnalyzer, Histogram, MaxLength, Maximum, Mean, MinLength, Minimum,
                        Size, StandardDeviation, Sum)
from .states import (ApproxCountDistinctState, CorrelationState, DataTypeHistogram, MaxState, MeanState,
                     MinState, NumMatches, NumMatchesAndCount, StandardDeviationState, SumState)

COUNT_COL = "com_amazon_deequ_dq_metrics_count"  # Analyzer.scala:363-364
# Histogram's state is `data.select(col.cast(string)).groupBy(column).count()`
# (Histogram.scala:63-66): Spark names that count column "count".
HISTOGRAM_COUNT_COL = "count"

_M32 = 0xFFFFFFFF


def _i32(x: int) -> int:
    x &= _M32
    return x - (1 << 32) if x & 0x80000000 else x


def _rotl32(x: int, r: int) -> int:
    x &= _M32
    return ((x << r) | (x >> (32 - r))) & _M32


def _mix_last(h: int, k: int) -> int:
    k = (k * 0xCC9E2D51) & _M32
    k = _rotl32(k, 15)
    k = (k * 0x1B873593) & _M32
    return (h ^ k) & _M32


def _mix(h: int, k: int) -> int:
    h = _mix_last(h, k)
    h = _rotl32(h, 13)
    return (h * 5 + 0xE6546B64) & _M32


def scala_string_hash(s: str, seed: int = 42) -> int:
    """scala.util.hashing.MurmurHash3.stringHash (Scala 2.11): MurmurHash3_x86_32 over pairs of
    UTF-16 code units (hi << 16 + lo), the odd last unit mixed alone, finalised with the length
    in code units.  A third-party (Scala library) function, restated; no reference test pins it."""
    units = s.encode("utf-16-be")
    cu = [int.from_bytes(units[i:i + 2], "big") for i in range(0, len(units), 2)]
    h = seed & _M32
    i = 0
    while i + 1 < len(cu):
        h = _mix(h, ((cu[i] << 16) + cu[i + 1]) & _M32)
        i += 2
    if i < len(cu):
        h = _mix_last(h, cu[i])
    h ^= len(cu)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    h ^= h >> 16
    return _i32(h)


_PA_TYPES = {"bool": "bool_", "int8": "int8", "int16": "int16", "int32": "int32", "int64": "int64",
             "float32": "float32", "float64": "float64", "string": "string"}


class HdfsStateProvider:
    """StateLoader + StatePersister over files (StateProvider.scala:72-311)."""

    def __init__(self, locationPrefix: str, numPartitionsForHistogram: int = 10, allowOverwrite: bool = False):
        self.locationPrefix = locationPrefix
        self.numPartitionsForHistogram = numPartitionsForHistogram
        self.allowOverwrite = allowOverwrite

    # ------------------------------------------------------------ files
    def _identifier(self, analyzer) -> str:
        return str(scala_string_hash(str(analyzer), 42))

    def _path(self, identifier: str, suffix: str = ".bin") -> str:
        return "%s-%s%s" % (self.locationPrefix, identifier, suffix)

    def _write(self, path: str, data: bytes) -> None:
        if os.path.exists(path) and not self.allowOverwrite:
            raise FileExistsError("path %s already exists." % path)
        parent = os.path.dirname(path)
        if parent:
            os.makedirs(parent, exist_ok=True)
        with open(path, "wb") as f:
            f.write(data)

    def _read(self, path: str) -> bytes:
        with open(path, "rb") as f:
            return f.read()

    # ------------------------------------------------------------ persist
    def persist(self, analyzer, state) -> None:
        ident = self._identifier(analyzer)
        path = self._path(ident)
        if isinstance(analyzer, Size):
            self._write(path, struct.pack(">q", state.numMatches))
        elif isinstance(analyzer, (Completeness, Compliance)):
            self._write(path, struct.pack(">qq", state.numMatches, state.count))
        elif isinstance(analyzer, Sum):
            self._write(path, struct.pack(">d", state.sum_value))
        elif isinstance(analyzer, Mean):
            self._write(path, struct.pack(">dq", state.sum_value, state.count))
        elif isinstance(analyzer, (Minimum, MinLength)):
            self._write(path, struct.pack(">d", state.minValue))
        elif isinstance(analyzer, (Maximum, MaxLength)):
            self._write(path, struct.pack(">d", state.maxValue))
        elif isinstance(analyzer, (FrequencyBasedAnalyzer, Histogram)):
            self._persist_frequencies(ident, state)
        elif isinstance(analyzer, DataType):
            b = state.toBytes()
            self._write(path, struct.pack(">i", len(b)) + b)
        elif isinstance(analyzer, ApproxCountDistinct):
            b = state.to_bytes()
            self._write(path, struct.pack(">i", len(b)) + b)
        elif isinstance(analyzer, Correlation):
            self._write(path, struct.pack(">6d", *state.fields()))
        elif isinstance(analyzer, StandardDeviation):
            self._write(path, struct.pack(">3d", state.n, state.avg, state.m2))
        else:
            raise ValueError("Unable to persist state for analyzer %s." % analyzer)

    def _persist_frequencies(self, ident: str, state) -> None:
        from .distributed import DistributedFrequencies
        directory = self._path(ident, "-frequencies.pqt")
        if isinstance(state, DistributedFrequencies):
            self._persist_frequencies_sharded(ident, directory, state)
            return
        if os.path.exists(directory):
            if not self.allowOverwrite:
                raise FileExistsError("path %s already exists." % directory)
            shutil.rmtree(directory)
        os.makedirs(directory)
        _write_frequency_part(os.path.join(directory, "part-00000.snappy.parquet"), state.table)
        self._write(self._path(ident, "-num_rows.bin"), struct.pack(">q", state.numRows))

    def _persist_frequencies_sharded(self, ident: str, directory: str, state) -> None:
        """A frequency state held by the ranks of a process group (each owns disjoint keys after
        the key-hash exchange) is written as the reference's Spark job writes its partitions:
        rank r writes part-%05d with the groups it owns, rank 0 the numRows file -- no rank
        gathers the table (StateProvider.scala:222-240 writes the state DataFrame partition by
        partition).  Collective; the ranks share the filesystem (one node)."""
        import torch.distributed as dist
        from .distributed import agree, allreduce_flag
        group = state.group
        rank = dist.get_rank(group)
        exists = rank == 0 and os.path.exists(directory)
        if allreduce_flag(exists and not self.allowOverwrite, group):
            raise FileExistsError("path %s already exists." % directory)
        err = None
        if rank == 0:
            try:
                if exists:
                    shutil.rmtree(directory)
                os.makedirs(directory)
            except Exception as e:  # noqa: BLE001 -- agreed on, then re-raised
                err = e
        agree(err, "creating %s" % directory, group)
        try:
            _write_frequency_part(os.path.join(directory, "part-%05d.snappy.parquet" % rank), state.owned)
            if rank == 0:
                self._write(self._path(ident, "-num_rows.bin"), struct.pack(">q", state.numRows))
        except Exception as e:  # noqa: BLE001
            err = e
        agree(err, "writing the frequency state's parts", group)

    # ------------------------------------------------------------ load
    def load(self, analyzer):
        ident = self._identifier(analyzer)
        path = self._path(ident)
        if isinstance(analyzer, Size):
            return NumMatches(struct.unpack(">q", self._read(path))[0])
        if isinstance(analyzer, (Completeness, Compliance)):
            return NumMatchesAndCount(*struct.unpack(">qq", self._read(path)))
        if isinstance(analyzer, Sum):
            return SumState(struct.unpack(">d", self._read(path))[0])
        if isinstance(analyzer, Mean):
            return MeanState(*struct.unpack(">dq", self._read(path)))
        if isinstance(analyzer, (Minimum, MinLength)):
            return MinState(struct.unpack(">d", self._read(path))[0])
        if isinstance(analyzer, (Maximum, MaxLength)):
            return MaxState(struct.unpack(">d", self._read(path))[0])
        if isinstance(analyzer, (FrequencyBasedAnalyzer, Histogram)):
            return self._load_frequencies(ident, analyzer)
        if isinstance(analyzer, DataType):
            return DataTypeHistogram.fromBytes(self._load_bytes(path))
        if isinstance(analyzer, ApproxCountDistinct):
            return ApproxCountDistinctState.from_bytes(self._load_bytes(path))
        if isinstance(analyzer, Correlation):
            return CorrelationState(*struct.unpack(">6d", self._read(path)))
        if isinstance(analyzer, StandardDeviation):
            return StandardDeviationState(*struct.unpack(">3d", self._read(path)))
        raise ValueError("Unable to load state for analyzer %s." % analyzer)

    def _load_bytes(self, path: str) -> bytes:
        raw = self._read(path)
        (n,) = struct.unpack(">i", raw[:4])
        return raw[4:4 + n]

    def _load_frequencies(self, ident: str, analyzer):
        """The parquet parts -> one device table, part by part through the flat import (array
        operations only; a key in several parts adds up, as the reference's union of partitions
        does), then numRows (StateProvider.scala:280-311)."""
        import pyarrow.parquet as pq
        from .frequencies import FrequenciesAndNumRows, FrequencyTable
        from .keycols import encode_columns
        # file by file: Histogram("count")'s state has two columns named "count", which
        # pyarrow's dataset reader (read_table of a directory) refuses to unify
        directory = self._path(ident, "-frequencies.pqt")
        parts = sorted(f for f in os.listdir(directory) if f.endswith(".parquet")) if os.path.isdir(directory) else []
        paths = [os.path.join(directory, f) for f in parts] or [directory]
        num_rows = struct.unpack(">q", self._read(self._path(ident, "-num_rows.bin")))[0]
        histogram = isinstance(analyzer, Histogram)
        table = None
        try:
            for path in paths:
                part = pq.ParquetFile(path).read()
                # the count column: deequ's name for grouping states, Spark's "count" for Histogram;
                # anything else (a state written by another tool) -- the last column
                # (by position: Histogram("count") gives two columns named "count")
                names_all = list(part.column_names)
                ci = names_all.index(COUNT_COL) if COUNT_COL in names_all else len(names_all) - 1
                keys = [i for i in range(len(names_all)) if i != ci]
                if table is None:
                    names = [names_all[i] for i in keys]
                    dtypes = [_dtype_of(part.schema.field(i).type) for i in keys]
                    table = FrequencyTable(names, dict(zip(names, dtypes)), histogram)
                offs, blob = encode_columns([part.column(i) for i in keys], table.dtypes, histogram)
                counts = part.column(ci).combine_chunks().to_numpy(zero_copy_only=False)
                table.import_flat(counts.astype(np.int64, copy=False), offs, blob, 0)
            table.import_flat(np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.uint8), num_rows)
        except BaseException:
            if table is not None:
                table.close()
            raise
        return FrequenciesAndNumRows(table)


def _write_frequency_part(path: str, table) -> None:
    """One parquet part of a frequency state: the grouping columns + the count column (Histogram:
    the column cast to string, Histogram.scala:63-66, NULL -> "NullValue"), built from the flat
    export with array operations (FrequencyTable.to_arrow)."""
    import pyarrow.parquet as pq
    count_col = HISTOGRAM_COUNT_COL if table.histogram else COUNT_COL
    pq.write_table(table.to_arrow(count_column=count_col), path)


def _concat(tables):
    import pyarrow as pa
    cols = [pa.chunked_array([c for t in tables for c in t.column(i).chunks], type=tables[0].schema.field(i).type)
            for i in range(tables[0].num_columns)]
    return pa.Table.from_arrays(cols, names=tables[0].column_names)


def _dtype_of(t) -> str:
    import pyarrow as pa
    for name, attr in _PA_TYPES.items():
        if t == getattr(pa, attr)():
            return name
    if pa.types.is_large_string(t):
        return "string"
    raise ValueError("unsupported frequency column type %s" % t)


__all__: List[str] = ["HdfsStateProvider", "scala_string_hash", "COUNT_COL", "HISTOGRAM_COUNT_COL"]
