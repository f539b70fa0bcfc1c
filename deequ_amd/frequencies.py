"""Frequency group-by on the GPU: the state `FrequenciesAndNumRows` and its table handle.

Replaces `FrequencyBasedAnalyzer.computeFrequencies` (analyzers/GroupingAnalyzers.scala:53-80):

    SELECT cols, COUNT(*) FROM data WHERE cols NOT NULL GROUP BY cols      (+ data.count())

and the group-by of `Histogram.computeStateFrom` (Histogram.scala:54-69).  The table lives in
HBM (an open-addressing hash table built by deequ_amd/csrc/dq_freq.hip); the metrics of the
frequency family are derived on the device from a count-of-counts histogram, so a 200M-group
table never leaves the GPU unless the caller exports it (state persistence, Spark interop).

Group keys cross the C-ABI in an encoded form (see include/deequ_amd.h): fixed-width values
as their little-endian bytes (floats as raw bits -- Spark 2.2 groups by the UnsafeRow bytes),
strings as UTF-8; several columns concatenated, string parts prefixed by a u32 length.
"""
from __future__ import annotations

import ctypes
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .states import State

_FIXED = {"bool": ("<B", 1), "int8": ("<b", 1), "int16": ("<h", 2), "int32": ("<i", 4),
          "int64": ("<q", 8), "float32": ("<f", 4), "float64": ("<d", 8)}
NULL_FIELD_REPLACEMENT = "NullValue"  # Histogram.NullFieldReplacement (Histogram.scala:108)


# ---------------------------------------------------------------- key codec
def encode_key(values: Sequence, dtypes: Sequence[str], histogram: bool = False) -> bytes:
    """Python values (None = NULL, histogram tables only) -> encoded key bytes."""
    if histogram:
        (v,), (t,) = values, dtypes
        if v is None:
            return NULL_FIELD_REPLACEMENT.encode() if t == "string" else b""
        if t == "float64" and v != v:
            return struct.pack("<Q", 0x7FF8000000000000)
        if t == "float32" and v != v:
            return struct.pack("<I", 0x7FC00000)
    multi = len(dtypes) > 1
    out = []
    for v, t in zip(values, dtypes):
        if t == "string":
            b = v.encode("utf-8")
            out.append((struct.pack("<I", len(b)) if multi else b"") + b)
        elif t == "bool":
            out.append(b"\x01" if v else b"\x00")
        else:
            out.append(struct.pack(_FIXED[t][0], v))
    return b"".join(out)


def decode_key(key: bytes, dtypes: Sequence[str], histogram: bool = False) -> tuple:
    """Encoded key bytes -> tuple of Python values (floats keep their bits)."""
    if histogram and len(key) == 0 and dtypes[0] != "string":
        return (None,)
    if len(dtypes) == 1 and dtypes[0] == "string":
        return (key.decode("utf-8"),)
    out, pos, multi = [], 0, len(dtypes) > 1
    for t in dtypes:
        if t == "string":
            n = struct.unpack_from("<I", key, pos)[0] if multi else len(key) - pos
            pos += 4 if multi else 0
            out.append(key[pos:pos + n].decode("utf-8"))
            pos += n
        elif t == "bool":
            out.append(key[pos] != 0)
            pos += 1
        else:
            fmt, w = _FIXED[t]
            out.append(struct.unpack_from(fmt, key, pos)[0])
            pos += w
    return tuple(out)


# ---------------------------------------------------------------- device table
class FrequencyTable:
    """A dq_freq handle: device-resident (group key -> count) table plus numRows.

    `schema` is the batch schema handed to `consume` (defaults to the key columns alone);
    `histogram=True` is Histogram's NULL-as-"NullValue" grouping (DQ_FREQ_NULL_AS_KEY);
    `few_only=True` groups with the few-groups kernel alone (DQ_FREQ_FEW_ONLY): a batch with more
    distinct keys than it holds raises DeequAmdError with status DQ_ERR_SPACE."""

    def __init__(self, key_columns: Sequence[str], schema: Dict[str, str], histogram: bool = False,
                 device: Optional[int] = None, few_only: bool = False):
        from .engine import current_device
        self.key_columns = list(key_columns)
        self.schema = dict(schema)
        self.names = list(self.schema.keys())
        self.dtypes = [self.schema[c] for c in self.key_columns]
        self.histogram = histogram
        self.device = current_device() if device is None else device
        ctx = L.Context.get(self.device)
        idx = (ctypes.c_int32 * len(self.key_columns))(*[self.names.index(c) for c in self.key_columns])
        types = (ctypes.c_int32 * len(self.names))(*[L.TYPE_CODES[self.schema[n]] for n in self.names])
        h = ctypes.c_void_p()
        flags = (L.DQ_FREQ_NULL_AS_KEY if histogram else 0) | (L.DQ_FREQ_FEW_ONLY if few_only else 0)
        L.check(L.lib().dq_freq_create(ctx.handle, idx, len(self.key_columns), types, len(self.names), flags,
                                       ctypes.byref(h)))
        self.handle = h

    @classmethod
    def like(cls, other: "FrequencyTable") -> "FrequencyTable":
        """An empty table with the same key columns (and a key-only schema)."""
        return cls(other.key_columns, {c: t for c, t in zip(other.key_columns, other.dtypes)},
                   other.histogram, other.device)

    def reserve(self, rows: int) -> None:
        """Size the staging for `rows` rows about to be consumed (optional)."""
        L.check(L.lib().dq_freq_reserve(self.handle, int(rows)))

    def expect_groups(self, groups: int) -> None:
        """Hint: at most about `groups` groups (optional; picks the LDS-aggregating path)."""
        L.check(L.lib().dq_freq_expect_groups(self.handle, int(groups)))

    def consume(self, batch) -> None:
        from .arrow import ArrowBatch
        from .table import dq_columns
        if isinstance(batch, ArrowBatch):  # the Arrow C Data Interface entry point
            schema, array = batch.c_structs(self.names)
            L.check(L.lib().dq_freq_consume_arrow(self.handle, ctypes.byref(schema), ctypes.byref(array), 0))
            return
        cols = dq_columns(batch, self.names)
        L.check(L.lib().dq_freq_consume(self.handle, cols, len(self.names), batch.num_rows))

    def summary(self) -> L.DqFreqSummary:
        s = L.DqFreqSummary()
        L.check(L.lib().dq_freq_get_summary(self.handle, ctypes.byref(s)))
        return s

    @property
    def num_rows(self) -> int:
        return self.summary().num_rows

    def export_flat(self, device: bool = False):
        """Every group as flat columns, in slot order (dq_freq_export_flat): (counts int64[n],
        key offsets int64[n + 1], encoded key bytes uint8) -- numpy arrays, or with `device` torch
        tensors on this table's GPU.  No per-group object is made."""
        n, kb = ctypes.c_int64(), ctypes.c_int64()
        st = L.lib().dq_freq_export_flat(self.handle, None, None, None, 0, 0, 0, ctypes.byref(n), ctypes.byref(kb))
        if st != L.DQ_ERR_SPACE:
            L.check(st)
        if device:
            import torch
            counts = torch.empty(max(1, n.value), dtype=torch.int64, device=self.torch_device)
            offs = torch.empty(n.value + 1, dtype=torch.int64, device=self.torch_device)
            blob = torch.empty(max(1, kb.value), dtype=torch.uint8, device=self.torch_device)
            ptrs = (counts.data_ptr(), offs.data_ptr(), blob.data_ptr())
        else:
            counts = np.empty(max(1, n.value), dtype=np.int64)
            offs = np.empty(n.value + 1, dtype=np.int64)
            blob = np.empty(max(1, kb.value), dtype=np.uint8)
            ptrs = (counts.ctypes.data, offs.ctypes.data, blob.ctypes.data)
        got_n, got_k = ctypes.c_int64(), ctypes.c_int64()
        L.check(L.lib().dq_freq_export_flat(self.handle, ptrs[0], ptrs[1], ptrs[2], n.value, kb.value,
                                            L.DQ_FLAT_DEVICE if device else 0, ctypes.byref(got_n), ctypes.byref(got_k)))
        return counts[:got_n.value], offs[:got_n.value + 1], blob[:got_k.value]

    def import_flat(self, counts, offsets, blob, num_rows: int = 0) -> None:
        """FrequenciesAndNumRows.sum of flat groups (dq_freq_import_flat): numpy arrays or device
        tensors on this table's GPU; duplicate keys add up."""
        n = len(counts)
        if len(offsets) != n + 1:
            raise ValueError("offsets must hold one more value than counts")
        if hasattr(counts, "data_ptr"):
            import torch
            for name, t in (("counts", counts), ("offsets", offsets), ("blob", blob)):
                if not hasattr(t, "data_ptr") or not t.is_cuda or t.device != self.torch_device:
                    raise ValueError("import_flat: %s must be a tensor on %s (got %s)"
                                     % (name, self.torch_device, getattr(t, "device", type(t).__name__)))
            # the library reads int64 counts / offsets and uint8 bytes (Arrow string offsets are
            # often int32): convert rather than let it misread the buffers
            c = counts.to(torch.int64).contiguous()
            o = offsets.to(torch.int64).contiguous()
            b = blob.to(torch.uint8).contiguous()
            L.check(L.lib().dq_freq_import_flat(self.handle, c.data_ptr(), o.data_ptr(), b.data_ptr() if b.numel() else None,
                                                n, int(num_rows), L.DQ_FLAT_DEVICE))
            return
        c = np.ascontiguousarray(counts, dtype=np.int64)
        o = np.ascontiguousarray(offsets, dtype=np.int64)
        b = np.ascontiguousarray(blob, dtype=np.uint8)
        L.check(L.lib().dq_freq_import_flat(self.handle, c.ctypes.data, o.ctypes.data, b.ctypes.data if len(b) else None,
                                            n, int(num_rows), 0))

    def to_arrow(self, strings: Optional[bool] = None, count_column: Optional[str] = None):
        """The state's DataFrame as an Arrow table: the grouping columns + the count column, built
        from the flat export with array operations only.  `strings` (default: a Histogram table)
        casts the key to string as the reference's Histogram state holds it (Histogram.scala:63-66)."""
        import pyarrow as pa
        from .keycols import decode_columns
        strings = self.histogram if strings is None else strings
        counts, offs, blob = self.export_flat()
        cols = decode_columns(offs, blob, self.dtypes, self.histogram, strings=strings)
        name = count_column or ("count" if self.histogram else COUNT_COL)
        return pa.Table.from_arrays(cols + [pa.array(counts, type=pa.int64())], names=list(self.key_columns) + [name])

    def export(self) -> Tuple[np.ndarray, List[bytes]]:
        """Every group: (counts int64[n], encoded keys), in slot order (a list of byte strings:
        the small-state convenience; export_flat / to_arrow carry large states)."""
        counts, offs, blob = self.export_flat()
        raw = blob.tobytes()
        o = offs.tolist()
        return counts, [raw[o[i]:o[i + 1]] for i in range(len(counts))]

    def top(self, n: int) -> Tuple[np.ndarray, List[bytes]]:
        """Groups whose count is at least the n-th largest count (ties at the cut included),
        count descending then encoded key ascending."""
        cap_g, cap_k = max(16, 2 * n), max(4096, 64 * n)
        while True:
            groups = (L.DqFreqGroup * cap_g)()
            keys = ctypes.create_string_buffer(cap_k)
            got, kb = ctypes.c_int64(), ctypes.c_int64()
            st = L.lib().dq_freq_top(self.handle, n, groups, cap_g, keys, cap_k, ctypes.byref(got),
                                     ctypes.byref(kb))
            if st == L.DQ_ERR_SPACE:
                cap_g, cap_k = max(cap_g, got.value), max(cap_k, kb.value)
                continue
            L.check(st)
            return _unpack_groups(groups, got.value, keys.raw)

    def lookup(self, key: bytes) -> int:
        """Count of the group with this encoded key (0 if there is none)."""
        out = ctypes.c_int64()
        buf = ctypes.create_string_buffer(key, max(1, len(key)))
        L.check(L.lib().dq_freq_lookup(self.handle, buf, len(key), ctypes.byref(out)))
        return int(out.value)

    def import_groups(self, counts: Sequence[int], keys: Sequence[bytes], num_rows: int) -> None:
        """FrequenciesAndNumRows.sum for the given groups (GroupingAnalyzers.scala:128-148)."""
        lens = np.fromiter((len(k) for k in keys), dtype=np.int64, count=len(keys))
        offs = np.zeros(len(keys) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        blob = np.frombuffer(b"".join(keys), dtype=np.uint8)
        self.import_flat(np.asarray(counts, dtype=np.int64).reshape(len(keys)), offs, blob, num_rows)

    # ---- multi-GPU key-hash exchange (deequ_amd/distributed.py)
    WIRE_PACKED_BYTES = 16  # sizeof(dq_freq_wire_packed): a key that packs into one word
    WIRE_BYTES = 32         # sizeof(dq_freq_wire): any other key

    @classmethod
    def part_bytes(cls, packed: int, general: int) -> int:
        return cls.WIRE_PACKED_BYTES * int(packed) + cls.WIRE_BYTES * int(general)

    def partition_sizes(self, n_parts: int) -> Tuple[List[int], List[int], List[int]]:
        """(packed groups, other groups, long-key bytes) per owner part (dq_freq_partition sizing)."""
        pp, pg, pk = (ctypes.c_int64 * n_parts)(), (ctypes.c_int64 * n_parts)(), (ctypes.c_int64 * n_parts)()
        st = L.lib().dq_freq_partition(self.handle, n_parts, None, 0, None, 0, pp, pg, pk)
        if st not in (L.DQ_OK, L.DQ_ERR_SPACE):
            L.check(st)
        return list(pp), list(pg), list(pk)

    def partition_into(self, n_parts: int, parts, keys) -> Tuple[List[int], List[int], List[int]]:
        """Scatter the groups by owner into device byte tensors `parts` (per part: its packed
        records, then its other records, each in slice order) and `keys` (long-key bytes)."""
        pp, pg, pk = (ctypes.c_int64 * n_parts)(), (ctypes.c_int64 * n_parts)(), (ctypes.c_int64 * n_parts)()
        L.check(L.lib().dq_freq_partition(self.handle, n_parts, parts.data_ptr(), parts.numel(), keys.data_ptr(),
                                          keys.numel(), pp, pg, pk))
        return list(pp), list(pg), list(pk)

    def import_parts(self, parts, packed: Sequence[int], general: Sequence[int], keys, key_bytes: Sequence[int],
                     num_rows: int = 0) -> None:
        """Merge the received parts (laid out one after the other in device tensors, as
        partition_into writes each) into this table, every slice once."""
        n = len(packed)
        arr = lambda v: (ctypes.c_int64 * max(1, n))(*[int(x) for x in v])  # noqa: E731
        L.check(L.lib().dq_freq_import_parts(self.handle, n, parts.data_ptr(), arr(packed), arr(general),
                                             keys.data_ptr(), arr(key_bytes), int(num_rows)))

    def import_wire(self, groups, n: int, keys, key_bytes: int, num_rows: int = 0) -> None:
        """Merge `n` general wire groups (dq_freq_wire, any order) held in device tensors."""
        L.check(L.lib().dq_freq_import_wire(self.handle, groups.data_ptr(), n, keys.data_ptr(), key_bytes,
                                            int(num_rows)))

    def count_histogram(self, n_bins: int = 1 << 16) -> Tuple[np.ndarray, np.ndarray]:
        """(hist[c] = #groups with count c for c < n_bins, sorted counts >= n_bins)."""
        hist = np.zeros(n_bins, dtype=np.int64)
        cap = 16
        while True:
            big = np.zeros(cap, dtype=np.int64)
            n_big = ctypes.c_int64()
            st = L.lib().dq_freq_count_histogram(
                self.handle, hist.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n_bins,
                big.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap, ctypes.byref(n_big))
            if st == L.DQ_ERR_SPACE:
                cap = max(cap * 2, n_big.value)
                continue
            L.check(st)
            return hist, big[:n_big.value].copy()

    @property
    def torch_device(self):
        import torch
        return torch.device("cuda", self.device)

    def paths(self) -> Dict[str, int]:
        """Which group-by paths this table's groupings took (dq_diag_freq_paths; tests)."""
        out = (ctypes.c_int64 * 14)()
        L.check(L.lib().dq_diag_freq_paths(self.handle, out))
        return {"slots": out[0], "partition_runs": out[1], "slice_bits": out[2], "sort_records": out[3],
                "packed_runs": out[4], "small_runs": out[5], "wait_timeouts": out[6],
                "import_coarse_runs": out[7], "import_skipped_runs": out[8], "hashed_runs": out[9],
                "hashed_inserts": out[10], "compacted": out[11], "uuid_runs": out[12], "raw16_runs": out[13]}

    def merge_from(self, other: "FrequencyTable") -> None:
        """self += other, device to device."""
        L.check(L.lib().dq_freq_merge(self.handle, other.handle))

    def close(self) -> None:
        if getattr(self, "handle", None):
            L.lib().dq_freq_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_GROUP_DTYPE = np.dtype([("count", "<i8"), ("key_offset", "<i8"), ("key_len", "<i4"), ("reserved", "<i4")])
COUNT_COL = "com_amazon_deequ_dq_metrics_count"  # Analyzer.scala:363-364


def _unpack_groups(groups, n: int, raw: bytes) -> Tuple[np.ndarray, List[bytes]]:
    g = np.frombuffer(groups, dtype=_GROUP_DTYPE, count=n)
    offs, lens = g["key_offset"].tolist(), g["key_len"].tolist()
    return g["count"].copy(), [raw[o:o + m] for o, m in zip(offs, lens)]


def compute_frequencies(data, grouping_columns: Sequence[str], histogram: bool = False) -> "FrequenciesAndNumRows":
    """FrequencyBasedAnalyzer.computeFrequencies over every batch of `data` (one pass); over a
    ShardedTable, the key-hash exchanged table of the whole dataset (collective)."""
    from .distributed import compute_frequencies_distributed, is_sharded
    if is_sharded(data):
        return compute_frequencies_distributed(data.local, grouping_columns, histogram, group=data.group)
    schema = data.schema
    table = FrequencyTable(grouping_columns, {c: schema[c] for c in schema}, histogram)
    table.reserve(data.count())
    for batch in data.batches():
        table.consume(batch)
    return FrequenciesAndNumRows(table)


def summary_from_histogram(hist: np.ndarray, big: np.ndarray, num_rows: int) -> L.DqFreqSummary:
    """dq_freq_summary of a (summed) count-of-counts histogram: the same fixed-order arithmetic
    as a single table's summary, so sharded and whole-table metrics agree bit for bit."""
    hist = np.ascontiguousarray(hist, dtype=np.int64)
    big = np.ascontiguousarray(np.sort(np.asarray(big, dtype=np.int64)))
    out = L.DqFreqSummary()
    L.check(L.lib().dq_freq_summary_from_histogram(
        hist.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(hist),
        big.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)) if len(big) else None, len(big), int(num_rows),
        ctypes.byref(out)))
    return out


# ---------------------------------------------------------------- the state
class FrequenciesAndNumRows(State):
    """FrequenciesAndNumRows(frequencies, numRows) (GroupingAnalyzers.scala:124-157), with the
    frequencies held in HBM."""

    def __init__(self, table: FrequencyTable):
        self.table = table
        self._summary = None

    @property
    def columns(self) -> List[str]:
        return self.table.key_columns

    @property
    def numRows(self) -> int:
        return self.summary().num_rows

    def summary(self) -> L.DqFreqSummary:
        if self._summary is None:
            self._summary = self.table.summary()
        return self._summary

    def sum(self, other: "FrequenciesAndNumRows") -> "FrequenciesAndNumRows":
        """Null-safe outer join adding counts (GroupingAnalyzers.scala:128-148)."""
        if not isinstance(other, FrequenciesAndNumRows):
            raise TypeError("cannot sum FrequenciesAndNumRows with %s" % type(other).__name__)
        a, b = self, other
        if a.table.histogram and b.table.histogram and a.table.dtypes != b.table.dtypes:
            # Histogram states persisted by Spark deequ (or by HdfsStateProvider) are keyed by the
            # column cast to string (Histogram.scala:63-66); a freshly computed one keeps the
            # column's type on the device.  Sum them over string keys, as the reference does.
            a, b = a.as_string_keys(), b.as_string_keys()
        if b.table.dtypes != a.table.dtypes or b.table.histogram != a.table.histogram:
            raise ValueError("frequency states over different key columns cannot be summed")
        self, other = a, b
        out = FrequencyTable.like(self.table)
        out.merge_from(self.table)
        out.merge_from(other.table)
        return FrequenciesAndNumRows(out)

    __add__ = sum

    def as_string_keys(self) -> "FrequenciesAndNumRows":
        """A Histogram state keyed by its values cast to string (Spark's Cast to StringType, NULL
        -> "NullValue", Histogram.scala:63-66, 108): the form the reference persists."""
        if not self.table.histogram or self.table.dtypes == ["string"]:
            return self
        arrow = self.table.to_arrow(strings=True)
        return FrequenciesAndNumRows.from_arrow(arrow, self.columns, ["string"], self.numRows, histogram=True)

    def frequencies(self, raw: bool = False) -> Dict:
        """{key tuple: count} on the host (decoded Python values), or with `raw` the encoded
        key bytes -- the exact group identity (decoded floats conflate 0.0 and -0.0).  A dict
        of every group: for large states use to_arrow() / table.export_flat()."""
        counts, keys = self.table.export()
        if raw:
            return {k: int(c) for k, c in zip(keys, counts.tolist())}
        return {decode_key(k, self.table.dtypes, self.table.histogram): int(c)
                for k, c in zip(keys, counts.tolist())}

    def to_arrow(self, strings: Optional[bool] = None):
        """The state's frequencies DataFrame as an Arrow table (see FrequencyTable.to_arrow)."""
        return self.table.to_arrow(strings)

    @staticmethod
    def from_arrow(table, columns: Sequence[str], dtypes: Sequence[str], numRows: int,
                   histogram: bool = False, count_column: Optional[str] = None) -> "FrequenciesAndNumRows":
        """A device state from an Arrow table of the grouping columns + a count column (the
        last column unless named), e.g. a state persisted by Spark deequ: encoded with array
        operations and merged on the device (dq_freq_import_flat; duplicate keys add up)."""
        from .keycols import encode_columns
        names = list(table.column_names)
        ci = names.index(count_column) if count_column else len(names) - 1
        keys = [table.column(i) for i in range(len(names)) if i != ci]
        counts = table.column(ci)
        counts = counts.combine_chunks() if hasattr(counts, "combine_chunks") else counts
        t = FrequencyTable(columns, dict(zip(columns, dtypes)), histogram)
        offs, blob = encode_columns(keys, dtypes, histogram)
        t.import_flat(np.asarray(counts.to_numpy(zero_copy_only=False), dtype=np.int64), offs, blob, numRows)
        return FrequenciesAndNumRows(t)

    @staticmethod
    def from_frequencies(columns: Sequence[str], dtypes: Sequence[str], frequencies: Dict[tuple, int],
                         numRows: int, histogram: bool = False) -> "FrequenciesAndNumRows":
        """Build a device state from host groups (e.g. a state persisted by Spark deequ)."""
        t = FrequencyTable(columns, dict(zip(columns, dtypes)), histogram)
        keys = [encode_key(k, dtypes, histogram) for k in frequencies]
        t.import_groups(list(frequencies.values()), keys, numRows)
        return FrequenciesAndNumRows(t)

    def metricValue(self):
        raise NotImplementedError("frequency metrics are computed by the analyzers")

    def __eq__(self, o):
        return (isinstance(o, FrequenciesAndNumRows) and o.columns == self.columns
                and o.numRows == self.numRows and o.frequencies(raw=True) == self.frequencies(raw=True))

    __hash__ = None

    def __repr__(self):
        s = self.summary()
        return "FrequenciesAndNumRows(columns=%s, groups=%d, numRows=%d)" % (
            ",".join(self.columns), s.num_groups, s.num_rows)
