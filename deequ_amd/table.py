"""Columnar batches in the Arrow layout, handed to the C-ABI as `dq_column`s.

The reference scans a Spark DataFrame; the drop-in boundary hands the GPU
Arrow-layout column batches.  A `Table` here is one such batch (or several, via
`PartitionedTable`, like a DataFrame's partitions): per column a validity bitmap (LSB-first,
1 = valid), fixed-width values or int32 offsets + UTF-8 bytes.  Buffers live either in host
memory (numpy; the library copies them to HBM) or in HBM already (torch tensors on the GPU;
used in place) -- the latter is how the benchmark keeps 65 GB resident.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from . import _lib as L

DTYPES = ("bool", "int8", "int16", "int32", "int64", "float32", "float64", "string")
_NP = {"int8": np.int8, "int16": np.int16, "int32": np.int32, "int64": np.int64,
       "float32": np.float32, "float64": np.float64}
NUMERIC = ("int8", "int16", "int32", "int64", "float32", "float64")


def pack_validity(valid: Optional[np.ndarray]) -> Optional[np.ndarray]:
    if valid is None:
        return None
    valid = np.asarray(valid, dtype=bool)
    if valid.all():
        return None
    return np.packbits(valid, bitorder="little")


class Column:
    """One column of a batch.  `device=True` means every buffer is a torch tensor in HBM."""

    def __init__(self, dtype: str, length: int, values, validity=None, offsets=None,
                 offset: int = 0, device: bool = False):
        if dtype not in DTYPES:
            raise ValueError("unsupported column type %r" % dtype)
        self.dtype = dtype
        self.length = int(length)
        self.values = values
        self.validity = validity
        self.offsets = offsets
        self.offset = int(offset)
        self.device = device

    # ---------------------------------------------------------------- constructors
    @staticmethod
    def from_numpy(values: np.ndarray, valid: Optional[np.ndarray] = None,
                   dtype: Optional[str] = None) -> "Column":
        values = np.ascontiguousarray(values)
        if dtype is None:
            dtype = "bool" if values.dtype == np.bool_ else str(values.dtype)
        if dtype == "bool":
            bits = np.packbits(values.astype(bool), bitorder="little")
            return Column("bool", len(values), bits, pack_validity(valid))
        return Column(dtype, len(values), values.astype(_NP[dtype], copy=False), pack_validity(valid))

    @staticmethod
    def from_pylist(values: Sequence, dtype: str) -> "Column":
        valid = np.array([v is not None for v in values], dtype=bool)
        if dtype == "string":
            data = [(v if v is not None else "").encode("utf-8") for v in values]
            offs = np.zeros(len(data) + 1, dtype=np.int32)
            np.cumsum([len(d) for d in data], out=offs[1:])
            buf = np.frombuffer(b"".join(data) + b"\0" * 8, dtype=np.uint8)
            return Column("string", len(values), buf, pack_validity(valid), offsets=offs)
        fill = False if dtype == "bool" else 0
        arr = np.array([v if v is not None else fill for v in values],
                       dtype=bool if dtype == "bool" else _NP[dtype])
        return Column.from_numpy(arr, valid, dtype)

    @staticmethod
    def from_arrow(arr) -> "Column":
        """pyarrow.Array (single chunk) -> Column, zero-copy on the host."""
        import pyarrow as pa
        t = arr.type
        if pa.types.is_large_string(t):
            arr = arr.cast(pa.string())
            t = arr.type
        kind = {pa.bool_(): "bool", pa.int8(): "int8", pa.int16(): "int16", pa.int32(): "int32",
                pa.int64(): "int64", pa.float32(): "float32", pa.float64(): "float64",
                pa.string(): "string"}.get(t)
        if kind is None:
            raise TypeError("unsupported arrow type %s" % t)
        bufs = arr.buffers()
        validity = None
        if bufs[0] is not None and arr.null_count > 0:
            validity = np.frombuffer(bufs[0], dtype=np.uint8)
        if kind == "string":
            offs = np.frombuffer(bufs[1], dtype=np.int32)
            data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(8, np.uint8)
            return Column(kind, len(arr), data, validity, offsets=offs, offset=arr.offset)
        if kind == "bool":
            return Column(kind, len(arr), np.frombuffer(bufs[1], dtype=np.uint8), validity, offset=arr.offset)
        return Column(kind, len(arr), np.frombuffer(bufs[1], dtype=_NP[kind]), validity, offset=arr.offset)

    # ---------------------------------------------------------------- device residency
    def to_device(self, device: int = 0) -> "Column":
        """Copy every buffer to HBM (torch tensors on cuda:`device`)."""
        import torch
        if self.device:
            return self
        dev = torch.device("cuda", device)

        def up(a):
            if a is None:
                return None
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        return Column(self.dtype, self.length, up(self.values), up(self.validity), up(self.offsets),
                      self.offset, device=True)

    # ---------------------------------------------------------------- C-ABI view
    def _ptr(self, a):
        if a is None:
            return None
        if self.device:
            return a.data_ptr()
        return a.ctypes.data

    def to_dq(self) -> L.DqColumn:
        c = L.DqColumn()
        c.type = L.TYPE_CODES[self.dtype]
        c.flags = L.DQ_COL_DEVICE if self.device else 0
        c.length = self.length
        c.offset = self.offset
        c.validity = self._ptr(self.validity)
        c.values = self._ptr(self.values)
        c.offsets = self._ptr(self.offsets)
        return c

    # ---------------------------------------------------------------- host views (tests)
    def valid_mask(self) -> np.ndarray:
        if self.validity is None:
            return np.ones(self.length, dtype=bool)
        v = self.validity.cpu().numpy() if self.device else self.validity
        bits = np.unpackbits(np.asarray(v, dtype=np.uint8), bitorder="little")
        return bits[self.offset:self.offset + self.length].astype(bool)

    def to_pylist(self) -> List:
        valid = self.valid_mask()
        vals = self.values.cpu().numpy() if self.device else self.values
        if self.dtype == "string":
            offs = self.offsets.cpu().numpy() if self.device else self.offsets
            raw = bytes(np.asarray(vals, dtype=np.uint8))
            o = offs[self.offset:self.offset + self.length + 1]
            return [raw[o[i]:o[i + 1]].decode("utf-8") if valid[i] else None for i in range(self.length)]
        if self.dtype == "bool":
            bits = np.unpackbits(np.asarray(vals, dtype=np.uint8), bitorder="little")
            bits = bits[self.offset:self.offset + self.length].astype(bool)
            return [bool(b) if ok else None for b, ok in zip(bits, valid)]
        arr = np.asarray(vals)[self.offset:self.offset + self.length]
        return [x if ok else None for x, ok in zip(arr.tolist(), valid)]


class Table:
    """An ordered set of equally long named columns (one batch / one partition)."""

    def __init__(self, columns: "OrderedDict[str, Column]"):
        self.columns = OrderedDict(columns)
        lengths = {c.length for c in self.columns.values()}
        if len(lengths) > 1:
            raise ValueError("columns have different lengths: %s" % sorted(lengths))
        self.num_rows = lengths.pop() if lengths else 0
        self._schema = OrderedDict((k, c.dtype) for k, c in self.columns.items())

    @property
    def schema(self) -> Dict[str, str]:
        """{name: dtype} in column order (computed once: the columns of a Table are fixed)."""
        return self._schema

    @staticmethod
    def from_pydict(data: Dict[str, tuple]) -> "Table":
        """{name: (dtype, [values with None for NULL])}"""
        return Table(OrderedDict((k, Column.from_pylist(v, t)) for k, (t, v) in data.items()))

    @staticmethod
    def from_rows(names: Sequence[str], dtypes: Sequence[str], rows: Iterable[Sequence]) -> "Table":
        rows = list(rows)
        return Table.from_pydict({n: (t, [r[i] for r in rows]) for i, (n, t) in enumerate(zip(names, dtypes))})

    @staticmethod
    def from_arrow(tbl) -> "Table":
        """pyarrow.Table / RecordBatch with single-chunk columns."""
        cols = OrderedDict()
        for name in tbl.column_names:
            col = tbl.column(name)
            if hasattr(col, "chunks"):
                if col.num_chunks != 1:
                    col = col.combine_chunks() if hasattr(col, "combine_chunks") else col.chunk(0)
                else:
                    col = col.chunk(0)
            cols[name] = Column.from_arrow(col)
        return Table(cols)

    def to_device(self, device: int = 0) -> "Table":
        return Table(OrderedDict((k, c.to_device(device)) for k, c in self.columns.items()))

    def batches(self) -> List["Table"]:
        return [self]

    def count(self) -> int:
        return self.num_rows


class PartitionedTable:
    """Several batches with one schema, processed like a DataFrame's partitions."""

    def __init__(self, parts: Sequence[Table]):
        self.parts = list(parts)
        if not self.parts:
            raise ValueError("a PartitionedTable needs at least one partition")
        schema = self.parts[0].schema
        for p in self.parts[1:]:
            if p.schema != schema:
                raise ValueError("partitions have different schemas")

    @property
    def schema(self):
        return self.parts[0].schema

    def batches(self) -> List[Table]:
        return self.parts

    def count(self) -> int:
        return sum(p.num_rows for p in self.parts)

    @property
    def num_rows(self) -> int:
        return self.count()


def dq_columns(batch: Table, names: Sequence[str]):
    """ctypes array of dq_column for `names` (in plan column order)."""
    arr = (L.DqColumn * max(1, len(names)))()
    for i, n in enumerate(names):
        arr[i] = batch.columns[n].to_dq()
    return arr
