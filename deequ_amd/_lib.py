"""ctypes binding of the deequ_amd C-ABI (include/deequ_amd.h).

The shared library is built in-tree (`deequ_amd/libdeequ_amd.so`, see
`deequ_amd/csrc/Makefile` / `__graft_entry__.build()`).  There is no fallback: if the
library is missing, importing the compute entry points raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_int, c_int32, c_int64, c_size_t,
                    c_uint8, c_uint64, c_void_p)

# DEEQU_AMD_LIB points at another build of the same library (A/B kernel experiments in one run)
LIB_PATH = os.environ.get("DEEQU_AMD_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libdeequ_amd.so")

# ---------------------------------------------------------------- enums (mirror the header)
DQ_OK, DQ_ERR_INVALID, DQ_ERR_UNSUPPORTED, DQ_ERR_DEVICE, DQ_ERR_OOM, DQ_ERR_STATE, DQ_ERR_SPACE = range(7)

DQ_T_BOOL, DQ_T_INT8, DQ_T_INT16, DQ_T_INT32, DQ_T_INT64, DQ_T_FLOAT32, DQ_T_FLOAT64, DQ_T_UTF8 = range(1, 9)
DQ_COL_DEVICE = 0x1

(DQ_OP_SIZE, DQ_OP_COMPLETENESS, DQ_OP_COMPLIANCE, DQ_OP_SUM, DQ_OP_MEAN, DQ_OP_STDDEV,
 DQ_OP_MINIMUM, DQ_OP_MAXIMUM, DQ_OP_APPROX_COUNT_DISTINCT, DQ_OP_DATATYPE, DQ_OP_MIN_LENGTH,
 DQ_OP_MAX_LENGTH, DQ_OP_CORRELATION) = range(1, 14)

DQ_P_COLUMN, DQ_P_LIT_INT, DQ_P_LIT_FLOAT, DQ_P_LIT_NULL, DQ_P_COALESCE, DQ_P_LIT_STRING = 1, 2, 3, 4, 5, 6
DQ_P_CAST_DOUBLE = 7
DQ_P_CAST = 8  # arg = target dq_type (TYPE_CODES)
DQ_P_EQ, DQ_P_NE, DQ_P_LT, DQ_P_LE, DQ_P_GT, DQ_P_GE, DQ_P_EQ_NULLSAFE = 10, 11, 12, 13, 14, 15, 16
DQ_P_IS_NULL, DQ_P_IS_NOT_NULL = 20, 21
DQ_P_AND, DQ_P_OR, DQ_P_NOT, DQ_P_TRUE, DQ_P_FALSE = 30, 31, 32, 33, 34
DQ_CMP_AS_INT64, DQ_CMP_AS_FLOAT64 = 0, 1

DQ_HLL_NUM_WORDS = 52
DQ_FREQ_NULL_AS_KEY = 0x1
DQ_FREQ_FEW_ONLY = 0x2
DQ_FLAT_DEVICE = 0x1

TYPE_CODES = {
    "bool": DQ_T_BOOL, "int8": DQ_T_INT8, "int16": DQ_T_INT16, "int32": DQ_T_INT32,
    "int64": DQ_T_INT64, "float32": DQ_T_FLOAT32, "float64": DQ_T_FLOAT64, "string": DQ_T_UTF8,
}


class DqColumn(Structure):
    _fields_ = [("type", c_int32), ("flags", c_int32), ("length", c_int64), ("offset", c_int64),
                ("validity", c_void_p), ("values", c_void_p), ("offsets", c_void_p)]


class DqPredInsn(Structure):
    _fields_ = [("opcode", c_int32), ("arg", c_int32), ("i64", c_int64), ("f64", c_double)]


class DqPredicate(Structure):
    _fields_ = [("code", POINTER(DqPredInsn)), ("n_insns", c_int32), ("strings_len", c_int32),
                ("strings", c_void_p)]


class DqOp(Structure):
    _fields_ = [("kind", c_int32), ("column", c_int32), ("column2", c_int32), ("reserved", c_int32),
                ("predicate", DqPredicate), ("where", DqPredicate)]


class DqState(Structure):
    _fields_ = [("kind", c_int32), ("has_value", c_int32), ("num_matches", c_int64),
                ("count", c_int64), ("sum", c_double), ("n", c_double), ("avg", c_double),
                ("m2", c_double), ("value", c_double), ("words", c_int64 * DQ_HLL_NUM_WORDS),
                ("y_avg", c_double), ("ck", c_double), ("x_mk", c_double), ("y_mk", c_double)]


DQ_FEW_MAX_GROUPS = 1024


class DqFewResult(Structure):
    _fields_ = [("ok", c_int32), ("n_groups", c_int32), ("n_nulls", c_int64),
                ("completeness", DqState), ("hll", DqState), ("dtype", DqState)]


class DqFreqSummary(Structure):
    _fields_ = [("num_rows", c_int64), ("num_groups", c_int64), ("num_unique", c_int64),
                ("grouped_rows", c_int64), ("entropy", c_double)]


class DqFreqWire(Structure):
    _fields_ = [("ctrl", c_uint64), ("count", c_int64), ("k0", c_uint64), ("k1", c_uint64)]


class DqFreqGroup(Structure):
    _fields_ = [("count", c_int64), ("key_offset", c_int64), ("key_len", c_int32),
                ("reserved", c_int32)]


class ArrowSchema(Structure):
    """struct ArrowSchema of the Arrow C Data Interface (include/deequ_amd.h)."""


ArrowSchema._fields_ = [("format", c_char_p), ("name", c_char_p), ("metadata", c_char_p), ("flags", c_int64),
                        ("n_children", c_int64), ("children", POINTER(POINTER(ArrowSchema))),
                        ("dictionary", POINTER(ArrowSchema)), ("release", c_void_p), ("private_data", c_void_p)]


class ArrowArray(Structure):
    """struct ArrowArray of the Arrow C Data Interface."""


ArrowArray._fields_ = [("length", c_int64), ("null_count", c_int64), ("offset", c_int64), ("n_buffers", c_int64),
                       ("n_children", c_int64), ("buffers", POINTER(c_void_p)),
                       ("children", POINTER(POINTER(ArrowArray))), ("dictionary", POINTER(ArrowArray)),
                       ("release", c_void_p), ("private_data", c_void_p)]


# measurement entry points (include/deequ_amd_diag.h; not part of the drop-in boundary)
DIAG_SIGNATURES = {
    "dq_diag_hash_rate": (c_int, [c_int, c_int, c_int, POINTER(c_double)]),
    "dq_diag_freq_paths": (c_int, [c_void_p, POINTER(c_int64)]),
    "dq_diag_freq_test_flags": (c_int, [c_void_p, c_int32]),
    "dq_diag_parse_double": (c_int, [c_char_p, c_int64, POINTER(c_double), POINTER(c_int32)]),
    "dq_diag_table_hash": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "dq_diag_key_pack": (c_int, [c_char_p, c_int32, POINTER(c_uint64), c_char_p, POINTER(c_int32), POINTER(c_int32)]),
    "dq_diag_uuid_pack": (c_int, [c_char_p, c_int32, POINTER(c_uint64), c_char_p, POINTER(c_int32)]),
    "dq_diag_eval_predicate": (c_int, [POINTER(DqPredicate), POINTER(DqColumn), c_int, c_int64, c_void_p]),
}


# every symbol include/deequ_amd.h declares, with its ctypes signature
SIGNATURES = {
    "dq_last_error": (c_char_p, []),
    "dq_abi_version": (c_int, []),
    "dq_device_count": (c_int, [POINTER(c_int)]),
    "dq_release_cached_memory": (c_int, [c_int]),
    "dq_ctx_create": (c_int, [c_int, c_int, POINTER(c_void_p)]),
    "dq_ctx_destroy": (c_int, [c_void_p]),
    "dq_plan_create": (c_int, [c_void_p, POINTER(DqOp), c_int, POINTER(c_int32), c_int, POINTER(c_void_p)]),
    "dq_plan_destroy": (c_int, [c_void_p]),
    "dq_plan_create_packed": (c_int, [c_void_p, c_char_p, c_size_t, POINTER(c_int32), c_int, POINTER(c_void_p)]),
    "dq_op_supported": (c_int, [POINTER(DqOp), POINTER(c_int32), c_int]),
    "dq_plan_consume": (c_int, [c_void_p, POINTER(DqColumn), c_int, c_int64]),
    "dq_plan_finish": (c_int, [c_void_p, POINTER(DqState), c_int]),
    "dq_plan_reset": (c_int, [c_void_p]),
    "dq_host_register": (c_int, [c_void_p, c_size_t]),
    "dq_host_unregister": (c_int, [c_void_p]),
    "dq_arrow_columns": (c_int, [POINTER(ArrowSchema), POINTER(ArrowArray), c_int, POINTER(c_int32),
                                 POINTER(DqColumn), c_int, POINTER(c_int), POINTER(c_int64)]),
    "dq_plan_consume_arrow": (c_int, [c_void_p, POINTER(ArrowSchema), POINTER(ArrowArray), c_int]),
    "dq_freq_consume_arrow": (c_int, [c_void_p, POINTER(ArrowSchema), POINTER(ArrowArray), c_int]),
    "dq_plan_op_status": (c_int, [c_void_p, c_int]),
    "dq_plan_stream": (c_void_p, [c_void_p]),
    "dq_state_merge": (c_int, [POINTER(DqState), POINTER(DqState), POINTER(DqState)]),
    "dq_state_metric": (c_int, [POINTER(DqState), POINTER(c_double)]),
    "dq_hll_count": (c_double, [POINTER(c_int64)]),
    "dq_hll_merge": (None, [POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    "dq_hll_words_to_bytes": (None, [POINTER(c_int64), POINTER(c_uint8)]),
    "dq_hll_words_from_bytes": (None, [POINTER(c_uint8), POINTER(c_int64)]),
    "dq_xxh64": (c_uint64, [c_void_p, c_size_t, c_uint64]),
    "dq_freq_create": (c_int, [c_void_p, POINTER(c_int32), c_int, POINTER(c_int32), c_int, c_int,
                               POINTER(c_void_p)]),
    "dq_freq_destroy": (c_int, [c_void_p]),
    "dq_freq_reset": (c_int, [c_void_p]),
    "dq_freq_consume": (c_int, [c_void_p, POINTER(DqColumn), c_int, c_int64]),
    "dq_freq_get_summary": (c_int, [c_void_p, POINTER(DqFreqSummary)]),
    "dq_freq_size": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64)]),
    "dq_freq_export": (c_int, [c_void_p, POINTER(DqFreqGroup), c_int64, c_void_p, c_int64,
                               POINTER(c_int64)]),
    "dq_freq_reserve": (c_int, [c_void_p, c_int64]),
    "dq_freq_expect_groups": (c_int, [c_void_p, c_int64]),
    "dq_freq_lookup": (c_int, [c_void_p, c_void_p, c_int64, POINTER(c_int64)]),
    "dq_freq_top": (c_int, [c_void_p, c_int, POINTER(DqFreqGroup), c_int64, c_void_p, c_int64,
                            POINTER(c_int64), POINTER(c_int64)]),
    "dq_freq_merge": (c_int, [c_void_p, c_void_p]),
    "dq_freq_import": (c_int, [c_void_p, POINTER(DqFreqGroup), c_int64, c_void_p, c_int64]),
    "dq_freq_export_flat": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int,
                                    POINTER(c_int64), POINTER(c_int64)]),
    "dq_freq_import_flat": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int]),
    "dq_cast_utf8": (c_int, [c_void_p, POINTER(DqColumn), c_int64, c_int32, c_void_p, c_void_p, POINTER(c_int64)]),
    "dq_cast_utf8_batch": (c_int, [c_void_p, c_int32, POINTER(DqColumn), c_int64, POINTER(c_int32),
                                   POINTER(c_void_p), POINTER(c_void_p)]),
    "dq_profile_few_strings": (c_int, [c_void_p, c_int32, POINTER(DqColumn), c_int64, POINTER(DqFewResult),
                                       c_void_p, c_void_p, c_void_p]),
    "dq_profile_string_groups": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int,
                                         POINTER(DqState), POINTER(DqState)]),
    "dq_freq_partition": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_void_p, c_int64, POINTER(c_int64),
                                  POINTER(c_int64), POINTER(c_int64)]),
    "dq_freq_import_parts": (c_int, [c_void_p, c_int, c_void_p, POINTER(c_int64), POINTER(c_int64), c_void_p,
                                     POINTER(c_int64), c_int64]),
    "dq_freq_import_wire": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int64]),
    "dq_freq_count_histogram": (c_int, [c_void_p, POINTER(c_int64), c_int64, POINTER(c_int64), c_int64,
                                        POINTER(c_int64)]),
    "dq_freq_summary_from_histogram": (c_int, [POINTER(c_int64), c_int64, POINTER(c_int64), c_int64, c_int64,
                                               POINTER(DqFreqSummary)]),
    "dq_group_unique_id": (c_int, [POINTER(c_uint8)]),
    "dq_group_create": (c_int, [c_void_p, c_int, c_int, POINTER(c_uint8), POINTER(c_void_p)]),
    "dq_group_destroy": (c_int, [c_void_p]),
    "dq_group_allgather_merge": (c_int, [c_void_p, POINTER(DqState), c_int]),
    "dq_states_merge_ranks": (c_int, [POINTER(DqState), c_int, c_int, POINTER(DqState)]),
    "dq_group_freq_exchange": (c_int, [c_void_p, c_void_p, c_void_p, POINTER(c_int64)]),
    "dq_group_freq_summary": (c_int, [c_void_p, c_void_p, c_int64, POINTER(DqFreqSummary)]),
    "dq_group_freq_top": (c_int, [c_void_p, c_void_p, c_int, POINTER(DqFreqGroup), c_int64, c_void_p, c_int64,
                                  POINTER(c_int64), POINTER(c_int64)]),
}

_lib = None


class DeequAmdError(RuntimeError):
    """A non-OK dq_status from the C-ABI (message from dq_last_error)."""

    def __init__(self, status: int, message: str):
        super().__init__("deequ_amd status %d: %s" % (status, message))
        self.status = status


class UnsupportedOnGpu(DeequAmdError):
    """DQ_ERR_UNSUPPORTED: the reference would run this analyzer on Spark instead."""


def lib():
    """Load libdeequ_amd.so (raises if it has not been built -- there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("deequ_amd native library not built: %s (run "
                              "`python -c 'import __graft_entry__ as g; g.build()'`)" % LIB_PATH)
        # PyTorch-ROCm bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Only one
        # HIP runtime can live in a process; whichever is loaded first serves everyone, and
        # torch cannot run on a newer one.  So when torch is installed, let it load its runtime
        # first and bind this library to that same runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in list(SIGNATURES.items()) + list(DIAG_SIGNATURES.items()):
            if name in DIAG_SIGNATURES and os.environ.get("DEEQU_AMD_LIB") and not hasattr(l, name):
                continue  # (an older A/B build may lack a newer diagnostic export)
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def check(status: int):
    if status != DQ_OK:
        msg = lib().dq_last_error().decode("utf-8", "replace")
        if status == DQ_ERR_UNSUPPORTED:
            raise UnsupportedOnGpu(status, msg)
        raise DeequAmdError(status, msg)


def device_count() -> int:
    n = c_int(0)
    check(lib().dq_device_count(ctypes.byref(n)))
    return n.value


class Context:
    """One dq_ctx per (process, device); created lazily."""

    _by_device = {}

    def __init__(self, device: int):
        self.device = device
        h = c_void_p()
        check(lib().dq_ctx_create(device, 0, ctypes.byref(h)))
        self.handle = h

    @classmethod
    def get(cls, device: int = 0) -> "Context":
        if device not in cls._by_device:
            cls._by_device[device] = Context(device)
        return cls._by_device[device]
