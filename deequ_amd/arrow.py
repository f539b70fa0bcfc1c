"""Arrow record batches handed to the library through the Arrow C Data Interface.

The JVM side of the seam exports each Spark partition as an
Arrow record batch and passes the two C structs (ArrowSchema, ArrowArray) to
dq_plan_consume_arrow / dq_freq_consume_arrow -- the replacement of the row handoff at
`data.agg` (AnalysisRunner.scala:313) and computeFrequencies (GroupingAnalyzers.scala:53-80).
This module is the same route from Python: pyarrow exports a RecordBatch into ctypes-allocated
structs (`RecordBatch._export_to_c`), and the engine consumes those, so a
`AnalysisRunner.onData(ArrowTable(...))` run goes through exactly the entry points a JNI shim
binds.  The library only borrows the buffers; the exported structs are re-imported into pyarrow
(which calls their release callbacks) when the batch is dropped.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

from . import _lib as L

# Arrow type -> the engine's dtype names (the formats dq_arrow_columns accepts)
_ARROW_DTYPES = {"bool": "bool", "int8": "int8", "int16": "int16", "int32": "int32", "int64": "int64",
                 "float": "float32", "double": "float64", "string": "string"}


def dtype_of(arrow_type) -> str:
    name = str(arrow_type)
    if name not in _ARROW_DTYPES:
        raise L.UnsupportedOnGpu(L.DQ_ERR_UNSUPPORTED, "Arrow type %s is not on the GPU path" % name)
    return _ARROW_DTYPES[name]


class _Exported:
    """One batch exported through the C Data Interface (owns the two structs)."""

    def __init__(self, batch):
        self.schema = L.ArrowSchema()
        self.array = L.ArrowArray()
        batch._export_to_c(ctypes.addressof(self.array), ctypes.addressof(self.schema))

    def close(self) -> None:
        if self.array.release:  # hand ownership back to pyarrow, which releases on collection
            import pyarrow as pa
            pa.RecordBatch._import_from_c(ctypes.addressof(self.array), ctypes.addressof(self.schema))

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class ArrowBatch:
    """A pyarrow.RecordBatch as one partition (host buffers; the library stages them in HBM)."""

    def __init__(self, batch):
        self.batch = batch
        self.num_rows = batch.num_rows
        self._exports: Dict[tuple, _Exported] = {}
        self._schema = None

    @property
    def schema(self) -> Dict[str, str]:
        if self._schema is None:
            self._schema = OrderedDict((f.name, dtype_of(f.type)) for f in self.batch.schema)
        return self._schema

    def c_structs(self, names: Sequence[str]):
        """(ArrowSchema, ArrowArray) of the batch's columns `names`, in that order."""
        key = tuple(names)
        if key not in self._exports:
            b = self.batch if list(names) == self.batch.schema.names else self.batch.select(list(names))
            self._exports[key] = _Exported(b)
        e = self._exports[key]
        return e.schema, e.array

    def batches(self) -> List["ArrowBatch"]:
        return [self]

    def count(self) -> int:
        return self.num_rows

    def close(self) -> None:
        for e in self._exports.values():
            e.close()
        self._exports.clear()


class ArrowTable:
    """A pyarrow.Table (or a list of RecordBatches) as a partitioned dataset: every record batch
    is one partition consumed through dq_plan_consume_arrow."""

    def __init__(self, data, max_chunksize: Optional[int] = None):
        import pyarrow as pa
        if isinstance(data, pa.Table):
            batches = data.to_batches(max_chunksize=max_chunksize)
            schema = data.schema
        elif isinstance(data, pa.RecordBatch):
            batches, schema = [data], data.schema
        else:
            batches = list(data)
            if not batches:
                raise ValueError("an ArrowTable needs at least one record batch")
            schema = batches[0].schema
        for b in batches:
            if not b.schema.equals(schema):
                raise ValueError("record batches have different schemas")
        self.arrow_schema = schema
        self.parts = [ArrowBatch(b) for b in batches] or [ArrowBatch(pa.RecordBatch.from_pylist([], schema=schema))]

    @property
    def schema(self) -> Dict[str, str]:
        if getattr(self, "_schema", None) is None:
            self._schema = OrderedDict((f.name, dtype_of(f.type)) for f in self.arrow_schema)
        return self._schema

    def batches(self) -> List[ArrowBatch]:
        return self.parts

    def count(self) -> int:
        return sum(p.num_rows for p in self.parts)

    @property
    def num_rows(self) -> int:
        return self.count()


def arrow_columns(batch, names: Optional[Sequence[str]] = None):
    """dq_arrow_columns of a RecordBatch (host only, no GPU): ([dq types], [DqColumn], n_rows)."""
    ab = batch if isinstance(batch, ArrowBatch) else ArrowBatch(batch)
    schema, array = ab.c_structs(names or ab.batch.schema.names)
    cap = max(1, ab.batch.num_columns)
    types = (ctypes.c_int32 * cap)()
    cols = (L.DqColumn * cap)()
    n, rows = ctypes.c_int(), ctypes.c_int64()
    L.check(L.lib().dq_arrow_columns(ctypes.byref(schema), ctypes.byref(array), 0, types, cols, cap,
                                     ctypes.byref(n), ctypes.byref(rows)))
    return list(types[:n.value]), [cols[i] for i in range(n.value)], rows.value, ab


__all__ = ["ArrowBatch", "ArrowTable", "arrow_columns", "dtype_of"]
