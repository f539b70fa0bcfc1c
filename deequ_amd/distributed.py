"""Multi-GPU merge of plan states: one process per GPU, rows sharded across ranks.

The reference's only exchange on this path is Spark's final aggregation: partial states of
every partition are collected and combined with the aggregate's merge, which deequ's
`State.sum` mirrors (AnalysisRunner.scala:313; Analyzer.scala:34-48).  Here each rank scans
its own row shard, then the ranks exchange their POD states (a few KB: 488 B per analyzer)
with ONE all-gather -- RCCL over xGMI when the tensors live on the GPU (`nccl` backend), gloo
on CPU -- and every rank folds them in rank order with the C-ABI's `dq_state_merge`.  The
fixed order makes the fp64 merges (Welford, sums) deterministic; counts and HLL registers
(per-register max) are order independent anyway.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib as L

STATE_BYTES = ctypes.sizeof(L.DqState)


def merge_raw(a: L.DqState, b: L.DqState) -> L.DqState:
    out = L.DqState()
    L.check(L.lib().dq_state_merge(ctypes.byref(a), ctypes.byref(b), ctypes.byref(out)))
    return out


def allgather_merge(states, n_ops: int, group=None, device: Optional[int] = None):
    """All-gather `states` (ctypes DqState array) across the process group and return the
    rank-ordered merge (a new DqState array).  `device` = GPU index for the nccl backend,
    None for a CPU (gloo) group."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    raw = np.frombuffer(ctypes.string_at(ctypes.addressof(states), n_ops * STATE_BYTES), dtype=np.uint8)
    dev = torch.device("cuda", device) if device is not None else torch.device("cpu")
    mine = torch.from_numpy(raw.copy()).to(dev)
    gathered = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine, group=group)
    blobs = [g.cpu().numpy().tobytes() for g in gathered]
    out = (L.DqState * max(1, n_ops))()
    for i in range(n_ops):
        acc = L.DqState.from_buffer_copy(blobs[0], i * STATE_BYTES)
        for r in range(1, world):
            acc = merge_raw(acc, L.DqState.from_buffer_copy(blobs[r], i * STATE_BYTES))
        out[i] = acc
    return out
