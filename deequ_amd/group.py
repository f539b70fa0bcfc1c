"""dq_group: the C-ABI's RCCL communicator (include/deequ_amd.h, csrc/dq_group.inc).

The Python engine shards with torch.distributed (deequ_amd.distributed); this wrapper exposes the
torch-free route a JVM driver takes through JNI -- group id from rank 0, one dq_group per
process/GPU, the rank-ordered state fold and the key-hash exchange -- so it can be tested from
Python on the same states and tables.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

from . import _lib as L

ID_BYTES = 128


def unique_id() -> bytes:
    buf = (ctypes.c_uint8 * ID_BYTES)()
    L.check(L.lib().dq_group_unique_id(buf))
    return bytes(buf)


def merge_ranks(gathered, n_ranks: int, n_ops: int):
    """dq_states_merge_ranks (host only): rank-ordered Analyzers.merge of n_ranks state blocks."""
    out = (L.DqState * max(1, n_ops))()
    L.check(L.lib().dq_states_merge_ranks(gathered, n_ranks, n_ops, out))
    return out


class DqGroup:
    def __init__(self, n_ranks: int, rank: int, uid: bytes, device: Optional[int] = None):
        from .engine import current_device
        self.device = current_device() if device is None else device
        self.ctx = L.Context.get(self.device)
        self.n_ranks, self.rank = n_ranks, rank
        ident = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        L.check(L.lib().dq_group_create(self.ctx.handle, n_ranks, rank, ident, ctypes.byref(h)))
        self.handle = h

    def allgather_merge(self, states, n_ops: int):
        """In place: this rank's states become the whole dataset's (collective)."""
        L.check(L.lib().dq_group_allgather_merge(self.handle, states, n_ops))
        return states

    def freq_exchange(self, local) -> Tuple[object, int]:
        """(the table of the keys this rank owns, the dataset's numRows) (collective)."""
        owned = type(local).like(local)
        rows = ctypes.c_int64()
        L.check(L.lib().dq_group_freq_exchange(self.handle, local.handle, owned.handle, ctypes.byref(rows)))
        return owned, rows.value

    def freq_summary(self, owned, num_rows: int) -> L.DqFreqSummary:
        s = L.DqFreqSummary()
        L.check(L.lib().dq_group_freq_summary(self.handle, owned.handle, int(num_rows), ctypes.byref(s)))
        return s

    def freq_top(self, owned, n: int):
        """Histogram's top-n over the dataset from the owned tables (collective): (counts, keys),
        count descending then key ascending, ties at the cut kept -- FrequencyTable.top's
        contract over the union of the ranks' rows."""
        from .frequencies import _unpack_groups
        cap_g, cap_k = max(16, 2 * n), max(4096, 64 * n)
        while True:
            groups = (L.DqFreqGroup * cap_g)()
            keys = ctypes.create_string_buffer(cap_k)
            got, kb = ctypes.c_int64(), ctypes.c_int64()
            st = L.lib().dq_group_freq_top(self.handle, owned.handle, int(n), groups, cap_g, keys, cap_k,
                                           ctypes.byref(got), ctypes.byref(kb))
            if st == L.DQ_ERR_SPACE:  # (the same sizes on every rank: every rank retries)
                cap_g, cap_k = max(cap_g, got.value), max(cap_k, kb.value)
                continue
            L.check(st)
            return _unpack_groups(groups, got.value, keys.raw)

    def close(self) -> None:
        if self.handle:
            L.lib().dq_group_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


__all__ = ["DqGroup", "merge_ranks", "unique_id"]
