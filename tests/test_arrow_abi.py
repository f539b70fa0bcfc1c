"""The Arrow C Data Interface boundary (include/deequ_amd.h: dq_arrow_columns, dq_plan_consume_arrow,
dq_freq_consume_arrow) on the CPU: pyarrow exports record batches into ctypes-allocated
ArrowSchema / ArrowArray structs -- as the JVM's org.apache.arrow.c.Data would -- and
dq_arrow_columns (pure host code) maps them onto dq_columns.  Checked: every accepted format,
sliced batches (struct offset + child offset), NULL-free validity, empty strings, and every
rejection the header documents (SURVEY §8(b) eligibility)."""
import ctypes

import numpy as np
import pyarrow as pa
import pytest

from deequ_amd import _lib as L
from deequ_amd.arrow import ArrowBatch, ArrowTable, _Exported, arrow_columns


def _addr(buf):
    return None if buf is None else buf.address


def _batch():
    return pa.record_batch({
        "b": pa.array([True, None, False, True, True, False, None, True, False, True], pa.bool_()),
        "i8": pa.array([1, 2, None, -4, 5, 6, 7, 8, 9, -10], pa.int8()),
        "i16": pa.array(list(range(10)), pa.int16()),
        "i32": pa.array([None] * 3 + list(range(7)), pa.int32()),
        "i64": pa.array([2 ** 40 + k for k in range(10)], pa.int64()),
        "f32": pa.array([0.5 * k for k in range(10)], pa.float32()),
        "f64": pa.array([None, 1.5, 2.5, None, 4.5, 5.5, 6.5, 7.5, 8.5, 9.5], pa.float64()),
        "s": pa.array(["a", "bb", None, "", "dddd", "é", "x", None, "yy", "zzz"], pa.string()),
    })


def test_formats_and_buffers_map_one_to_one():
    batch = _batch()
    types, cols, n_rows, keep = arrow_columns(batch)
    assert n_rows == 10
    assert types == [L.TYPE_CODES[t] for t in ("bool", "int8", "int16", "int32", "int64", "float32", "float64",
                                                  "string")]
    for k, (name, col) in enumerate(zip(batch.schema.names, cols)):
        arr = batch.column(name)
        bufs = arr.buffers()
        assert col.length == 10 and col.offset == arr.offset == 0 and col.flags == 0, name
        assert (col.validity or None) == (_addr(bufs[0]) if arr.null_count else None), name
        if name == "s":
            assert col.offsets == _addr(bufs[1]) and col.values == _addr(bufs[2])
        else:
            assert col.values == _addr(bufs[1]) and not col.offsets, name


@pytest.mark.parametrize("start,length", [(0, 10), (3, 5), (7, 3), (1, 0), (9, 1)])
def test_sliced_batch_offsets(start, length):
    batch = _batch().slice(start, length)
    types, cols, n_rows, keep = arrow_columns(batch)
    assert n_rows == length
    for name, col in zip(batch.schema.names, cols):
        # a sliced RecordBatch exports as a struct of offset-0 length-n children, or as children
        # carrying the offset: either way row r of the batch is slot (col.offset + r)
        arr = batch.column(name)
        assert col.offset == arr.offset, name
        assert col.length == length


def test_struct_offset_is_added_to_child_offsets():
    """A sliced StructArray exported as a bare array: the struct's offset applies to every child."""
    sa = pa.StructArray.from_arrays([pa.array(np.arange(20, dtype=np.int64)), pa.array(["k%d" % i for i in range(20)])],
                                    names=["x", "y"]).slice(4, 9)
    e = _Exported.__new__(_Exported)
    e.schema, e.array = L.ArrowSchema(), L.ArrowArray()
    sa._export_to_c(ctypes.addressof(e.array), ctypes.addressof(e.schema))
    try:
        types = (ctypes.c_int32 * 2)()
        cols = (L.DqColumn * 2)()
        n, rows = ctypes.c_int(), ctypes.c_int64()
        L.check(L.lib().dq_arrow_columns(ctypes.byref(e.schema), ctypes.byref(e.array), 0, types, cols, 2,
                                         ctypes.byref(n), ctypes.byref(rows)))
        assert (n.value, rows.value) == (2, 9)
        assert e.array.offset + e.array.children[0].contents.offset == cols[0].offset == 4
        assert cols[1].offset == 4
        vals = np.frombuffer((ctypes.c_int64 * 20).from_address(cols[0].values), dtype=np.int64)
        assert vals[cols[0].offset] == 4
    finally:
        pa.Array._import_from_c(ctypes.addressof(e.array), ctypes.addressof(e.schema))


def test_single_array_is_a_one_column_batch():
    arr = pa.array([1.0, None, 3.0], pa.float64()).slice(1)
    e = _Exported.__new__(_Exported)
    e.schema, e.array = L.ArrowSchema(), L.ArrowArray()
    arr._export_to_c(ctypes.addressof(e.array), ctypes.addressof(e.schema))
    try:
        types = (ctypes.c_int32 * 1)()
        cols = (L.DqColumn * 1)()
        n, rows = ctypes.c_int(), ctypes.c_int64()
        L.check(L.lib().dq_arrow_columns(ctypes.byref(e.schema), ctypes.byref(e.array), 0, types, cols, 1,
                                         ctypes.byref(n), ctypes.byref(rows)))
        assert (n.value, rows.value, types[0], cols[0].offset) == (1, 2, L.TYPE_CODES["float64"], 1)
    finally:
        pa.Array._import_from_c(ctypes.addressof(e.array), ctypes.addressof(e.schema))


def _status(batch, max_cols=16, flags=0):
    ab = ArrowBatch(batch)
    schema, array = ab.c_structs(batch.schema.names)
    types = (ctypes.c_int32 * 16)()
    cols = (L.DqColumn * 16)()
    n, rows = ctypes.c_int(), ctypes.c_int64()
    st = L.lib().dq_arrow_columns(ctypes.byref(schema), ctypes.byref(array), flags, types, cols, max_cols,
                                  ctypes.byref(n), ctypes.byref(rows))
    ab.close()
    return st, n.value


@pytest.mark.parametrize("arr", [
    pa.array(["a", "b", "a"]).dictionary_encode(),
    pa.array(["a", "b"], pa.large_string()),
    pa.array([[1], [2, 3]], pa.list_(pa.int64())),
    pa.array([1, 2], pa.decimal128(10, 2)),
    pa.array([1, 2], pa.date32()),
    pa.array([1, 2], pa.uint64()),
    pa.array([b"x", b"y"], pa.binary()),
])
def test_off_path_formats_are_unsupported(arr):
    st, _ = _status(pa.record_batch({"c": arr}))
    assert st == L.DQ_ERR_UNSUPPORTED
    assert L.lib().dq_last_error()


def test_struct_level_nulls_are_unsupported():
    sa = pa.StructArray.from_arrays([pa.array([1, 2, 3], pa.int64())], names=["x"],
                                    mask=pa.array([False, True, False]))
    schema, array = L.ArrowSchema(), L.ArrowArray()
    sa._export_to_c(ctypes.addressof(array), ctypes.addressof(schema))
    try:
        types = (ctypes.c_int32 * 1)()
        cols = (L.DqColumn * 1)()
        n, rows = ctypes.c_int(), ctypes.c_int64()
        st = L.lib().dq_arrow_columns(ctypes.byref(schema), ctypes.byref(array), 0, types, cols, 1,
                                      ctypes.byref(n), ctypes.byref(rows))
        assert st == L.DQ_ERR_UNSUPPORTED
    finally:
        pa.Array._import_from_c(ctypes.addressof(array), ctypes.addressof(schema))


def test_too_many_columns_reports_the_count():
    st, n = _status(_batch(), max_cols=3)
    assert st == L.DQ_ERR_SPACE and n == 8


def test_released_and_malformed_structs_are_invalid():
    ab = ArrowBatch(_batch())
    schema, array = ab.c_structs(ab.batch.schema.names)
    types = (ctypes.c_int32 * 16)()
    cols = (L.DqColumn * 16)()
    n, rows = ctypes.c_int(), ctypes.c_int64()
    call = lambda s, a, fl=0: L.lib().dq_arrow_columns(ctypes.byref(s), ctypes.byref(a), fl, types, cols, 16,  # noqa: E731
                                                      ctypes.byref(n), ctypes.byref(rows))
    assert call(schema, array) == L.DQ_OK
    assert call(schema, array, 0x80) == L.DQ_ERR_INVALID  # unknown flag
    child = array.children[1].contents
    saved = child.n_buffers
    child.n_buffers = 3
    assert call(schema, array) == L.DQ_ERR_INVALID
    child.n_buffers = saved
    saved = child.length
    child.length = 4  # shorter than the batch
    assert call(schema, array) == L.DQ_ERR_INVALID
    child.length = saved
    released = L.ArrowArray.from_buffer_copy(array)
    released.release = None
    assert call(schema, released) == L.DQ_ERR_INVALID
    assert call(schema, array) == L.DQ_OK
    ab.close()


def test_arrow_table_partitions_and_schema():
    tbl = pa.Table.from_batches([_batch(), _batch().slice(2, 5)])
    at = ArrowTable(tbl)
    assert [p.num_rows for p in at.batches()] == [10, 5]
    assert at.count() == 15
    assert list(at.schema.values()) == ["bool", "int8", "int16", "int32", "int64", "float32", "float64", "string"]
    with pytest.raises(L.UnsupportedOnGpu):
        ArrowTable(pa.table({"d": pa.array([1], pa.decimal128(5, 1))})).schema
