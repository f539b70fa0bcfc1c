"""dq_plan_create_packed -- the analyzer list as the JVM serializes it (include/deequ_amd.h;
INTEGRATION.md's GpuPlanEncoder).  CPU: the decoder's bounds checks run before any device work,
so truncated, trailing or inconsistent blobs are rejected here; a well-formed blob gets as far as
dq_plan_create's own argument check (no context on this host).  GPU: a packed plan produces the
same states, byte for byte, as the struct-built plan."""
import ctypes
import struct

import pytest

import deequ_amd as d
from deequ_amd import _lib as L
from deequ_amd.engine import PACKED_MAGIC, op_spec_for, pack_ops

SCHEMA = {"i": "int64", "f": "float64", "s": "string", "b": "bool"}


def _specs():
    an = [d.Size(), d.Completeness("i", "b"), d.Compliance("c", "i >= 0 AND s IN ('x', 'y''z')"), d.Sum("f", "s = 'q'"),
          d.ApproxCountDistinct("s"), d.Correlation("i", "f"), d.Maximum("f", "COALESCE(i, 0) > 2")]
    return an, [op_spec_for(a, SCHEMA) for a in an]


def _create(blob, ctx=None):
    types = (ctypes.c_int32 * 4)(*[L.TYPE_CODES[t] for t in SCHEMA.values()])
    h = ctypes.c_void_p()
    st = L.lib().dq_plan_create_packed(ctx, blob, len(blob), types, 4, ctypes.byref(h))
    return st, L.lib().dq_last_error().decode(), h


def test_packed_layout():
    _, specs = _specs()
    blob = pack_ops(specs)
    magic, version, n = struct.unpack_from("<III", blob)
    assert (magic, version, n) == (PACKED_MAGIC, 1, len(specs))
    # a well-formed blob is decoded completely and reaches dq_plan_create (which wants a context)
    st, msg, _ = _create(blob)
    assert st == L.DQ_ERR_INVALID and "NULL argument" in msg


@pytest.mark.parametrize("cut", [0, 4, 11, 12, 20, 40, -30, -1])
def test_truncated_blob_is_invalid(cut):
    _, specs = _specs()
    blob = pack_ops(specs)
    st, msg, _ = _create(blob[:cut] if cut else b"")
    assert st == L.DQ_ERR_INVALID
    assert "NULL argument" not in msg, msg


def test_trailing_bytes_and_bad_headers_are_invalid():
    _, specs = _specs()
    blob = pack_ops(specs)
    assert "trailing" in _create(blob + b"\0")[1]
    assert "magic" in _create(b"XXXX" + blob[4:])[1]
    assert "version" in _create(blob[:4] + struct.pack("<I", 2) + blob[8:])[1]
    # an op claiming more instructions than the blob holds
    bad = bytearray(blob)
    struct.pack_into("<i", bad, 12 + 12, 1000)  # op 0: n_pred
    assert _create(bytes(bad))[0] == L.DQ_ERR_INVALID


@pytest.mark.gpu
def test_packed_plan_equals_struct_plan(gpu):
    import numpy as np
    from deequ_amd.engine import Plan
    rng = np.random.default_rng(2)
    n = 5000
    table = d.Table.from_pydict({
        "i": ("int64", [None if rng.random() < 0.1 else int(x) for x in rng.integers(-5, 9, n)]),
        "f": ("float64", [float(x) for x in rng.normal(0, 1, n)]),
        "s": ("string", [["x", "y'z", "q", None][int(k)] for k in rng.integers(0, 4, n)]),
        "b": ("bool", [bool(x) for x in rng.integers(0, 2, n)])})
    an, specs = _specs()
    ref = Plan(specs, SCHEMA)
    ref.consume(table)
    want = bytes(ref.finish_raw())
    ref.close()
    ctx = L.Context.get(d.current_device())
    st, msg, h = _create(pack_ops(specs), ctx.handle)
    assert st == L.DQ_OK, msg
    try:
        from deequ_amd.table import dq_columns
        cols = dq_columns(table, list(SCHEMA))
        L.check(L.lib().dq_plan_consume(h, cols, 4, n))
        out = (L.DqState * len(specs))()
        L.check(L.lib().dq_plan_finish(h, out, len(specs)))
        assert bytes(out) == want
    finally:
        L.lib().dq_plan_destroy(h)
