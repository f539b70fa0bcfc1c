"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the oracle's C restatement (dq_oracle.c).

Used by tests/ (large-size parity) and bench.py's cpu_baseline leg; never by the product.
"""
import ctypes
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libdq_oracle.so")


class ColState(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_int64), ("n_sel", ctypes.c_int64), ("pm", ctypes.c_int64),
                ("pn", ctypes.c_int64), ("isum", ctypes.c_int64), ("fsum", ctypes.c_double),
                ("n", ctypes.c_double), ("avg", ctypes.c_double), ("m2", ctypes.c_double),
                ("vmin", ctypes.c_double), ("vmax", ctypes.c_double), ("imin", ctypes.c_int64),
                ("imax", ctypes.c_int64)]


OPS = {"=": 0, "!=": 1, "<": 2, "<=": 3, ">": 4, ">=": 5}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            raise ImportError("oracle C library not built (make -C oracle)")
        l = ctypes.CDLL(_PATH)
        l.dqo_time_c2.restype = ctypes.c_double
        l.dqo_time_c2.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ColState)]
        l.dqo_scan.restype = ctypes.c_int
        l.dqo_scan.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                               ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                               ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                               ctypes.c_int, ctypes.POINTER(ColState)]
        l.dqo_time_c2_hll.restype = ctypes.c_double
        l.dqo_time_c2_hll.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        l.dqo_time_c2_hll_for.restype = ctypes.c_double
        l.dqo_time_c2_hll_for.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_double, ctypes.POINTER(ctypes.c_int)]
        l.dqo_gen_c2.restype = None
        l.dqo_gen_c2.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]
        l.dqo_hll_registers.restype = None
        l.dqo_hll_registers.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p]
        l.dqo_hll_registers_mt.restype = None
        l.dqo_hll_registers_mt.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int]
        l.dqo_xxh64.restype = ctypes.c_uint64
        l.dqo_xxh64.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64]
        _lib = l
    return _lib


def time_c2_scan(rows: int, threads: int, hll: bool = True, min_secs: float = 0.0):
    """(seconds, passes): timed passes of the Spark-semantics scan over one C2 sample of `rows`
    rows on `threads` threads (data generation excluded), repeated until `min_secs` have been
    spent (one pass by default); with `hll`, the 8 columns' HLL registers in the timed region."""
    out = (ColState * 8)()
    regs = (ctypes.c_uint8 * (8 * 512))() if hll else None
    passes = ctypes.c_int(0)
    secs = lib().dqo_time_c2_hll_for(rows, threads, out, regs, float(min_secs), ctypes.byref(passes))
    if secs < 0:
        raise MemoryError("oracle could not allocate the C2 sample")
    return secs, passes.value


def gen_c2(rows: int, col: int, seed: int = 42):
    """The C2 column `col` as (values, validity bitmap) numpy arrays."""
    vals = np.empty(rows, dtype=np.int64 if col < 4 else np.float64)
    bm = np.zeros((rows + 7) // 8 + 8, dtype=np.uint8)
    lib().dqo_gen_c2(0, rows, seed, col, vals.ctypes.data, bm.ctypes.data)
    return vals, bm


def scan(columns, preds, parts: int = 1):
    """columns: list of (values ndarray int64/float64, validity bitmap or None);
    preds: list of (op, literal, as_f64) or None.  Returns ColState per column (Spark
    semantics, `parts` partitions merged in order)."""
    n = len(columns)
    rows = len(columns[0][0])
    types = (ctypes.c_int * n)(*[5 if c[0].dtype == np.int64 else 7 for c in columns])
    vals = (ctypes.c_void_p * n)(*[c[0].ctypes.data for c in columns])
    valid = (ctypes.c_void_p * n)(*[(c[1].ctypes.data if c[1] is not None else None) for c in columns])
    op = (ctypes.c_int * n)(*[(OPS[p[0]] if p else -1) for p in preds])
    as_f = (ctypes.c_int * n)(*[(1 if p and p[2] else 0) for p in preds])
    li = (ctypes.c_int64 * n)(*[(int(p[1]) if p and not p[2] else 0) for p in preds])
    lf = (ctypes.c_double * n)(*[(float(p[1]) if p else 0.0) for p in preds])
    out = (ColState * n)()
    rc = lib().dqo_scan(rows, n, types, vals, valid, op, as_f, li, lf, parts, out)
    if rc != 0:
        raise RuntimeError("dqo_scan failed")
    return list(out)


def hll_registers(kind: str, values, validity=None, offsets=None):
    code = {"int64": 5, "int32": 4, "float64": 7, "string": 8}[kind]
    regs = np.zeros(512, dtype=np.uint8)
    lib().dqo_hll_registers(code, len(values) if offsets is None else len(offsets) - 1,
                            values.ctypes.data, None if offsets is None else offsets.ctypes.data,
                            None if validity is None else validity.ctypes.data, regs.ctypes.data)
    return regs


def hll_registers_int64(values, validity, threads: int = 1):
    """The 512 HLL registers (uint8) of an int64 column (Spark hashLong, seed 42), NULL rows
    skipped (validity: LSB-first bitmap or None), on `threads` threads (register max merge)."""
    v = np.ascontiguousarray(values, dtype=np.int64)
    bm = None if validity is None else np.ascontiguousarray(validity, dtype=np.uint8)
    regs = np.zeros(512, dtype=np.uint8)
    lib().dqo_hll_registers_mt(5, len(v), v.ctypes.data, None if bm is None else bm.ctypes.data,
                               regs.ctypes.data, int(threads))
    return regs
