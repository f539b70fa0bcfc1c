"""Columnar codec of frequency-table keys: flat encoded keys <-> Arrow columns, vectorised.

A frequency state crosses the C-ABI as flat columns (`dq_freq_export_flat` /
`dq_freq_import_flat`): counts int64[n], key offsets int64[n + 1] and one byte array holding
every encoded key (the encoding of include/deequ_amd.h: fixed-width values as little-endian
bytes, a lone string column as its UTF-8 bytes, several columns concatenated with string parts
prefixed by a u32 length).  The reference keeps the same state as a DataFrame of the grouping
columns plus a count column (GroupingAnalyzers.scala:124-157) and persists it as parquet
(StateProvider.scala:222-240).  This module converts between the two with numpy / pyarrow
array operations only -- no Python object per group -- so a 2e8-group state (C4) can be
persisted, loaded and exchanged at array speed.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

_NP = {"bool": np.uint8, "int8": np.int8, "int16": np.int16, "int32": np.int32, "int64": np.int64,
       "float32": np.float32, "float64": np.float64}
_WIDTH = {"bool": 1, "int8": 1, "int16": 2, "int32": 4, "int64": 8, "float32": 4, "float64": 8}
NULL_VALUE = b"NullValue"  # Histogram.NullFieldReplacement (Histogram.scala:108)
_CHUNK = 1 << 22  # groups per vectorised step of the multi-column codec (bounds index arrays)


def _pa_type(dtype: str):
    import pyarrow as pa
    return {"bool": pa.bool_(), "int8": pa.int8(), "int16": pa.int16(), "int32": pa.int32(), "int64": pa.int64(),
            "float32": pa.float32(), "float64": pa.float64(), "string": pa.string()}[dtype]


def string_array(offsets: np.ndarray, blob: np.ndarray):
    """An Arrow utf8 array over flat bytes (offsets from 0): int32 offsets when they fit, else
    large_string -- both are parquet BYTE_ARRAY / UTF8, what Spark writes for StringType."""
    import pyarrow as pa
    n = len(offsets) - 1
    total = int(offsets[-1]) if n >= 0 else 0
    data = pa.py_buffer(np.ascontiguousarray(blob[:total]))
    if total < (1 << 31) - 1:
        return pa.StringArray.from_buffers(n, pa.py_buffer(np.ascontiguousarray(offsets, dtype=np.int32)), data)
    return pa.LargeStringArray.from_buffers(n, pa.py_buffer(np.ascontiguousarray(offsets, dtype=np.int64)), data)


def _gather_ranges(blob: np.ndarray, starts: np.ndarray, lens: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate blob[starts[i] : starts[i] + lens[i]] -> (bytes, offsets from 0)."""
    offs = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    total = int(offs[-1])
    if total == 0:
        return np.zeros(0, dtype=np.uint8), offs
    idx = np.repeat(starts.astype(np.int64) - offs[:-1], lens) + np.arange(total, dtype=np.int64)
    return blob[idx], offs


def _fixed_at(blob: np.ndarray, pos: np.ndarray, dtype: str) -> np.ndarray:
    w = _WIDTH[dtype]
    raw = blob[pos[:, None] + np.arange(w, dtype=np.int64)]
    return np.ascontiguousarray(raw).view(_NP[dtype]).reshape(len(pos))


def _u32_at(blob: np.ndarray, pos: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(blob[pos[:, None] + np.arange(4, dtype=np.int64)]).view("<u4").reshape(len(pos))


def decode_columns(offsets: np.ndarray, blob: np.ndarray, dtypes: Sequence[str], histogram: bool = False,
                   strings: bool = False) -> List:
    """Flat encoded keys -> one Arrow array per key column.

    `histogram`: a Histogram table (one column; NULL is the empty key of a non-string column and
    the literal "NullValue" of a string column).  `strings`: the key column cast to string as the
    reference's Histogram state holds it (Histogram.scala:63-66; NULL -> "NullValue")."""
    import pyarrow as pa
    import pyarrow.compute as pc
    offsets = np.asarray(offsets, dtype=np.int64)
    blob = np.asarray(blob, dtype=np.uint8)
    n = len(offsets) - 1
    base = int(offsets[0]) if n >= 0 else 0
    if base:
        offsets = offsets - base
        blob = blob[base:]
    lens = np.diff(offsets)
    if len(dtypes) == 1:
        t = dtypes[0]
        if t == "string":
            return [string_array(offsets, blob)]
        w = _WIDTH[t]
        null = lens == 0 if histogram else None
        if null is not None and null.any():
            vals = np.zeros(n, dtype=_NP[t])
            keep = ~null
            vals[keep] = _fixed_at(blob, offsets[:-1][keep], t)
        else:
            if n and not np.all(lens == w):
                raise ValueError("keys of a %s column must be %d bytes" % (t, w))
            vals = blob[:n * w].view(_NP[t]) if n else np.zeros(0, dtype=_NP[t])
        arr = pa.array(vals != 0 if t == "bool" else vals, type=_pa_type(t),
                       mask=null if null is not None and null.any() else None)
        if not strings:
            return [arr]
        return [_spark_string(arr, t)]
    # several columns: one vectorised pass per column, in chunks of groups
    parts: List[List] = [[] for _ in dtypes]
    for c0 in range(0, max(n, 0), _CHUNK):
        c1 = min(n, c0 + _CHUNK)
        pos = offsets[c0:c1].copy()
        for j, t in enumerate(dtypes):
            if t == "string":
                ln = _u32_at(blob, pos).astype(np.int64)
                data, offs = _gather_ranges(blob, pos + 4, ln)
                parts[j].append(string_array(offs, data))
                pos += 4 + ln
            else:
                v = _fixed_at(blob, pos, t)
                parts[j].append(pa.array(v != 0 if t == "bool" else v, type=_pa_type(t)))
                pos += _WIDTH[t]
        if not np.array_equal(pos, offsets[c0 + 1:c1 + 1]):
            raise ValueError("encoded keys do not match the key column types")
    return [pa.concat_arrays(p) if p else pa.array([], type=_pa_type(t)) for p, t in zip(parts, dtypes)]


def _spark_string(arr, dtype: str):
    """Spark 2.2's Cast(_ -> StringType) of a column, NULL -> "NullValue" (Histogram.scala:63-66)."""
    import pyarrow as pa
    import pyarrow.compute as pc
    if dtype in ("float32", "float64"):
        # Java's Double.toString / Float.toString have no vectorised equivalent; a Histogram
        # column is low-cardinality (ColumnProfiler's threshold), so its groups are few
        from .javafmt import spark_cast_to_string
        vals = arr.to_pylist()
        return pa.array(["NullValue" if v is None else spark_cast_to_string(v, dtype) for v in vals], type=pa.string())
    s = pc.cast(arr, pa.string())  # integers: decimal; booleans: "true" / "false" -- Spark's forms
    return pc.fill_null(s, "NullValue")


def encode_columns(columns: Sequence, dtypes: Sequence[str], histogram: bool = False) -> Tuple[np.ndarray, np.ndarray]:
    """Arrow arrays (one per key column, equal lengths) -> (offsets int64[n + 1], key bytes)."""
    import pyarrow as pa
    cols = [c.combine_chunks() if isinstance(c, pa.ChunkedArray) else c for c in columns]
    n = len(cols[0]) if cols else 0
    if len(dtypes) == 1:
        t, c = dtypes[0], cols[0]
        if t == "string":
            if c.null_count:
                if not histogram:
                    raise ValueError("a grouping column of a frequency state holds no NULL")
                c = pa.compute.fill_null(c, NULL_VALUE.decode())
            return _string_buffers(c)
        return _fixed_encode(c, t, histogram)
    if any(c.null_count for c in cols):
        raise ValueError("a grouping column of a frequency state holds no NULL")
    lens = np.zeros(n, dtype=np.int64)
    strs = {}
    for j, (c, t) in enumerate(zip(cols, dtypes)):
        if t == "string":
            so, sb = _string_buffers(c)
            strs[j] = (so, sb)
            lens += 4 + np.diff(so)
        else:
            lens += _WIDTH[t]
    offsets = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    blob = np.zeros(int(offsets[-1]), dtype=np.uint8)
    for c0 in range(0, n, _CHUNK):
        c1 = min(n, c0 + _CHUNK)
        pos = offsets[c0:c1].copy()
        for j, (c, t) in enumerate(zip(cols, dtypes)):
            if t == "string":
                so, sb = strs[j]
                ln = np.diff(so[c0:c1 + 1])
                blob[pos[:, None] + np.arange(4, dtype=np.int64)] = ln.astype("<u4").view(np.uint8).reshape(-1, 4)
                tot = int(ln.sum())
                if tot:
                    src = np.repeat(so[c0:c1] - (np.cumsum(ln) - ln), ln) + np.arange(tot, dtype=np.int64)
                    dst = np.repeat(pos + 4 - (np.cumsum(ln) - ln), ln) + np.arange(tot, dtype=np.int64)
                    blob[dst] = sb[src]
                pos += 4 + ln
            else:
                w = _WIDTH[t]
                v = _values(c.slice(c0, c1 - c0), t)
                blob[pos[:, None] + np.arange(w, dtype=np.int64)] = v.view(np.uint8).reshape(-1, w)
                pos += w
    return offsets, blob


def _values(c, t: str) -> np.ndarray:
    v = c.to_numpy(zero_copy_only=False)
    return np.ascontiguousarray(v.astype(np.uint8) if t == "bool" else v.astype(_NP[t], copy=False))


def _fixed_encode(c, t: str, histogram: bool) -> Tuple[np.ndarray, np.ndarray]:
    w = _WIDTH[t]
    n = len(c)
    null = None
    if c.null_count:
        if not histogram:
            raise ValueError("a grouping column of a frequency state holds no NULL")
        null = np.asarray(c.is_null().to_numpy(zero_copy_only=False), dtype=bool)
        c = c.fill_null(False if t == "bool" else 0)
    v = _values(c, t)
    if histogram and t in ("float32", "float64"):  # NaN groups as one canonical NaN (encode_key)
        nan = np.isnan(v)
        if nan.any():
            v = v.copy()
            v.view(np.uint64 if t == "float64" else np.uint32)[nan] = 0x7FF8000000000000 if t == "float64" else 0x7FC00000
    lens = np.full(n, w, dtype=np.int64)
    if null is not None:
        lens[null] = 0  # Histogram's NULL of a non-string column: the empty key
    offsets = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    raw = v.view(np.uint8).reshape(n, w)
    blob = raw[~null].reshape(-1) if null is not None else raw.reshape(-1)
    return offsets, np.ascontiguousarray(blob)


def _string_buffers(c) -> Tuple[np.ndarray, np.ndarray]:
    """(offsets int64 from 0, data bytes) of an Arrow (large_)string array, without copying keys."""
    import pyarrow as pa
    if pa.types.is_large_string(c.type):
        odt = np.int64
    elif pa.types.is_string(c.type):
        odt = np.int32
    else:
        raise ValueError("expected a string column, got %s" % c.type)
    bufs = c.buffers()
    n = len(c)
    offs = np.frombuffer(bufs[1], dtype=odt, count=n + 1 + c.offset)[c.offset:].astype(np.int64)
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, dtype=np.uint8)
    lo, hi = int(offs[0]), int(offs[-1])
    return offs - lo, data[lo:hi]


def concat_flat(parts: Sequence[Tuple[np.ndarray, np.ndarray, np.ndarray]]):
    """Several (counts, offsets, bytes) -> one, offsets rebased."""
    if not parts:
        return np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.uint8)
    counts = np.concatenate([p[0] for p in parts])
    blobs, offs, base = [], [np.zeros(1, np.int64)], 0
    for _, o, b in parts:
        o = np.asarray(o, dtype=np.int64)
        blobs.append(np.asarray(b, dtype=np.uint8)[int(o[0]):int(o[-1])])
        offs.append(o[1:] - o[0] + base)
        base += int(o[-1] - o[0])
    return counts, np.concatenate(offs), np.concatenate(blobs) if blobs else np.zeros(0, np.uint8)
