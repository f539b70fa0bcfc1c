"""The columnar key codec (deequ_amd/keycols.py) against the per-key codec (encode_key /
decode_key) on CPU: flat encoded keys <-> Arrow columns, for every key type, several columns,
Histogram NULLs and the Histogram string cast.  The device side of the flat path
(dq_freq_export_flat / dq_freq_import_flat) is checked in tests/test_gpu_state_scale.py."""
import math
import struct

import numpy as np
import pyarrow as pa
import pytest

from deequ_amd.frequencies import decode_key, encode_key
from deequ_amd.javafmt import spark_cast_to_string
from deequ_amd.keycols import concat_flat, decode_columns, encode_columns

RNG = np.random.default_rng(5)


def _values(t, n):
    if t == "string":
        return ["".join(chr(c) for c in RNG.integers(32, 0x3000, RNG.integers(0, 20))) for _ in range(n)]
    if t == "bool":
        return [bool(x) for x in RNG.integers(0, 2, n)]
    if t in ("float32", "float64"):
        v = [float(x) for x in RNG.normal(0, 1e3, n)]
        v[:4] = [-0.0, 0.0, float("inf"), 1.0e7]
        if t == "float32":
            v = [struct.unpack("<f", struct.pack("<f", x))[0] for x in v]
        return v
    lo, hi = {"int8": (-128, 128), "int16": (-2 ** 15, 2 ** 15), "int32": (-2 ** 31, 2 ** 31),
              "int64": (-2 ** 63, 2 ** 63)}[t]
    return [int(x) for x in RNG.integers(lo, hi, n, dtype=np.int64 if t != "int64" else np.int64)] if t != "int64" \
        else [int(x) for x in RNG.integers(-2 ** 62, 2 ** 62, n)] + [-2 ** 63, 2 ** 63 - 1]


def _flat(keys):
    offs = np.zeros(len(keys) + 1, dtype=np.int64)
    np.cumsum([len(k) for k in keys], out=offs[1:])
    return offs, np.frombuffer(b"".join(keys), dtype=np.uint8)


def _same(a, b):
    if isinstance(a, float):
        return (math.isnan(a) and math.isnan(b)) or (a == b and math.copysign(1, a) == math.copysign(1, b))
    return a == b


TYPES = ["string", "bool", "int8", "int16", "int32", "int64", "float32", "float64"]


@pytest.mark.parametrize("t", TYPES)
def test_single_column_roundtrip(t):
    vals = _values(t, 300)
    keys = [encode_key((v,), [t]) for v in vals]
    offs, blob = _flat(keys)
    (col,) = decode_columns(offs, blob, [t])
    got = col.to_pylist()
    assert all(_same(g, v) for g, v in zip(got, vals))
    offs2, blob2 = encode_columns([col], [t])
    assert np.array_equal(offs2, offs) and bytes(blob2) == b"".join(keys)


@pytest.mark.parametrize("dtypes", [["string", "int32", "string"], ["float64", "bool", "string"],
                                    ["int64", "int8"], ["string", "string"], ["bool", "float32", "int16", "string"]])
def test_multi_column_roundtrip(dtypes):
    n = 257
    cols = [_values(t, n + 2)[:n] for t in dtypes]
    keys = [encode_key(row, dtypes) for row in zip(*cols)]
    offs, blob = _flat(keys)
    arrs = decode_columns(offs, blob, dtypes)
    for a, want in zip(arrs, cols):
        assert all(_same(g, v) for g, v in zip(a.to_pylist(), want))
    rows = list(zip(*[a.to_pylist() for a in arrs]))
    assert [decode_key(k, dtypes) for k in keys] == rows or all(
        all(_same(x, y) for x, y in zip(r1, r2)) for r1, r2 in zip([decode_key(k, dtypes) for k in keys], rows))
    offs2, blob2 = encode_columns(arrs, dtypes)
    assert np.array_equal(offs2, offs) and bytes(blob2) == b"".join(keys)


def test_multi_column_in_chunks(monkeypatch):
    import deequ_amd.keycols as K
    monkeypatch.setattr(K, "_CHUNK", 7)  # several chunks, a ragged last one
    dtypes = ["string", "int64"]
    cols = [_values("string", 50), _values("int64", 50)[:50]]
    keys = [encode_key(r, dtypes) for r in zip(*cols)]
    offs, blob = _flat(keys)
    arrs = decode_columns(offs, blob, dtypes)
    assert [a.to_pylist() for a in arrs] == cols
    offs2, blob2 = encode_columns(arrs, dtypes)
    assert np.array_equal(offs2, offs) and bytes(blob2) == b"".join(keys)


@pytest.mark.parametrize("t", TYPES)
def test_histogram_keys_and_string_cast(t):
    """Histogram tables: NULL is the empty key of a non-string column ("NullValue" for strings);
    the persisted form casts the value to string as Spark does (Histogram.scala:63-66)."""
    vals = _values(t, 100) + [None, None]
    keys = [encode_key((v,), [t], histogram=True) for v in vals]
    offs, blob = _flat(keys)
    (col,) = decode_columns(offs, blob, [t], histogram=True)
    want = ["NullValue" if v is None else v for v in vals] if t == "string" else vals
    assert all(_same(g, v) for g, v in zip(col.to_pylist(), want))
    (s,) = decode_columns(offs, blob, [t], histogram=True, strings=True)
    cast = ["NullValue" if v is None else (v if t == "string" else spark_cast_to_string(v, t)) for v in vals]
    assert s.to_pylist() == cast
    offs2, blob2 = encode_columns([col], [t], histogram=True)
    assert np.array_equal(offs2, offs) and bytes(blob2) == b"".join(keys)


def test_histogram_nan_canonical():
    col = pa.array([float("nan"), struct.unpack("<d", struct.pack("<Q", 0xFFF8000000000001))[0], 1.0])
    offs, blob = encode_columns([col], ["float64"], histogram=True)
    keys = [bytes(blob[offs[i]:offs[i + 1]]) for i in range(3)]
    assert keys[0] == keys[1] == encode_key((float("nan"),), ["float64"], histogram=True)


def test_grouping_states_reject_nulls():
    with pytest.raises(ValueError):
        encode_columns([pa.array(["a", None])], ["string"])
    with pytest.raises(ValueError):
        encode_columns([pa.array([1, None]), pa.array(["x", "y"])], ["int64", "string"])


def test_sliced_and_large_string_columns():
    base = pa.array(["x%d" % i for i in range(100)])
    sl = base.slice(13, 40)
    offs, blob = encode_columns([sl], ["string"])
    assert bytes(blob) == "".join("x%d" % i for i in range(13, 53)).encode()
    offs2, blob2 = encode_columns([sl.cast(pa.large_string())], ["string"])
    assert np.array_equal(offs, offs2) and bytes(blob) == bytes(blob2)
    chunked = pa.chunked_array([base.slice(0, 10), base.slice(10, 90)])
    offs3, blob3 = encode_columns([chunked], ["string"])
    assert len(offs3) == 101 and bytes(blob3) == "".join("x%d" % i for i in range(100)).encode()


def test_offsets_not_from_zero_and_concat():
    keys = [b"ab", b"", b"cde"]
    offs, blob = _flat(keys)
    shifted = np.concatenate([np.zeros(5, np.uint8), blob])
    (col,) = decode_columns(offs + 5, shifted, ["string"])
    assert col.to_pylist() == ["ab", "", "cde"]
    c, o, b = concat_flat([(np.array([1, 2, 3]), offs + 5, shifted), (np.array([4]), np.array([0, 1]), np.array([120], np.uint8))])
    assert c.tolist() == [1, 2, 3, 4] and o.tolist() == [0, 2, 2, 5, 6] and bytes(b) == b"abcdex"
