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


# ---------------------------------------------------------------- sharded datasets
class ShardedTable:
    """A dataset spread over the ranks of a process group: rank r holds the row shard `local`
    (a Table / PartitionedTable / ArrowTable), the dataset is the union of all shards -- the
    contiguous row ranges of SURVEY §8(e), as Spark's partitions are spread over executors.

    Every entry point that takes data (AnalysisRunner, ColumnProfiler, run_scan,
    compute_frequencies) accepts a ShardedTable and is then COLLECTIVE: every rank calls it with
    the same analyzers, scans only its own shard on its own GPU, and gets the metrics of the
    whole dataset.  Scan states meet in one all-gather folded in rank order (merge_scan_results),
    frequency tables in the key-hash all-to-all (exchange_frequencies)."""

    def __init__(self, local, group=None):
        self.local = local
        self.group = group

    @property
    def schema(self):
        return self.local.schema

    def batches(self):
        return self.local.batches()

    def count(self) -> int:
        """Rows of this rank's shard (what the local staging is sized for)."""
        return self.local.count()

    @property
    def num_rows(self) -> int:
        return self.count()

    def global_count(self) -> int:
        """Rows of the whole dataset (collective)."""
        import torch
        import torch.distributed as dist
        n = torch.tensor([self.local.count()], dtype=torch.int64)
        if _comm_device(self.group) == "cuda":
            n = n.to(_cuda_device())
        dist.all_reduce(n, op=dist.ReduceOp.SUM, group=self.group)
        return int(n.item())

    def with_local(self, local) -> "ShardedTable":
        return ShardedTable(local, self.group)


def is_sharded(data) -> bool:
    return isinstance(data, ShardedTable)


def _cuda_device() -> int:
    from .engine import current_device
    return current_device()


def merge_scan_results(local, error, kinds, group=None):
    """The fused scan's results of every rank -> the whole dataset's (collective).

    `local` = this rank's list of DqState / OpUnsupported (None if its scan raised `error`).
    First every rank learns every rank's outcome (one all_gather_object of a few bytes): if any
    rank's aggregation failed, every rank raises -- the all-fail scope of
    AnalysisRunner.scala:320-323 over the whole dataset.  Then the POD states meet in ONE
    all-gather and fold in rank order (allgather_merge); an op unsupported on any rank's shard is
    unsupported for the dataset (the per-op scope of :340-353)."""
    import torch.distributed as dist
    from .engine import OpUnsupported
    n = len(kinds)
    world = dist.get_world_size(group)
    unsup = [] if local is None else [i for i, r in enumerate(local) if isinstance(r, OpUnsupported)]
    outcome = (None if error is None else "%s: %s" % (type(error).__name__, error), unsup)
    outcomes = [None] * world
    dist.all_gather_object(outcomes, outcome, group=group)
    for r, (err, _) in enumerate(outcomes):
        if err is not None:
            if error is not None:
                raise error
            raise L.DeequAmdError(L.DQ_ERR_STATE, "the fused scan failed on rank %d: %s" % (r, err))
    arr = (L.DqState * max(1, n))()
    for i in range(n):
        if isinstance(local[i], OpUnsupported):
            arr[i] = L.DqState()
            arr[i].kind = kinds[i]  # an empty state: the identity of Analyzers.merge
        else:
            arr[i] = local[i]
    merged = allgather_merge(arr, n, group=group,
                             device=_cuda_device() if _comm_device(group) == "cuda" else None)
    out = [L.DqState.from_buffer_copy(merged[i]) for i in range(n)]
    for r, (_, bad) in enumerate(outcomes):
        for i in bad:
            out[i] = OpUnsupported(L.UnsupportedOnGpu(
                L.DQ_ERR_UNSUPPORTED, "rank %d's shard held input the GPU cannot evaluate exactly for this op" % r))
    return out


def agree(error: Optional[BaseException], what: str, group=None) -> None:
    """Every rank learns whether any rank's local step failed (collective), before the next data
    collective: a failed rank re-raises its own error, the others raise naming the step, so no
    rank is left blocked in a collective its peer never enters (the all-fail scope of
    AnalysisRunner.scala:320-323 over the ranks)."""
    failed = allreduce_flag(error is not None, group)
    if error is not None:
        raise error
    if failed:
        raise L.DeequAmdError(L.DQ_ERR_STATE, "%s failed on another rank" % what)


def allreduce_flag(flag: bool, group=None) -> bool:
    """True on every rank if `flag` is true on any rank (collective)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if flag else 0], dtype=torch.int64)
    if _comm_device(group) == "cuda":
        t = t.to(_cuda_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(t.item())


# ---------------------------------------------------------------- frequency family
# The one real exchange step of the path.  Spark shuffles partial group counts by
# key hash into `spark.sql.shuffle.partitions` and finishes the aggregate per partition
# (GroupingAnalyzers.scala:67-72).  Here every rank groups its own row shard on its GPU, then:
#   1. partitions its table by owner rank (dq_freq_partition, a device scatter),
#   2. exchanges the partitions with ONE all-to-all of wire groups -- 16 B for keys that pack
#      into one word (decimal ids), 32 B for others -- (+ one for long-key bytes): RCCL over xGMI
#      with the nccl backend, gloo on host copies otherwise,
#   3. merges what it received into the table of the keys it owns (dq_freq_import_parts: every
#      part arrives in slice order, so each slice is merged once, in LDS, from all parts).
# Owners then hold disjoint keys: the metrics need only an all-reduce of the count-of-counts
# histograms (integers, exact), and Histogram's top-N an all-gather of per-owner top-N.

def _comm_device(group):
    import torch
    import torch.distributed as dist
    return "cuda" if dist.get_backend(group) == "nccl" else "cpu"


def _comm_tensor_device(group, table):
    """Where a collective's tensors live: the table's GPU for an nccl (RCCL) group, else host."""
    import torch
    return table.torch_device if _comm_device(group) == "cuda" else torch.device("cpu")


def _to(t, device):
    return t if t.device.type == device.type else t.to(device)


def _allgather_var(t, group=None):
    """All-gather a 1-D tensor whose length differs per rank (tensor collectives only: the
    lengths, then the tensors padded to the longest); returns every rank's tensor, trimmed."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(1, max(ns))
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    if t.numel():
        pad[:t.numel()] = t
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return [b[:k] for b, k in zip(bufs, ns)]


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def exchange_frequencies(table, group=None, stats: Optional[dict] = None):
    """Key-hash all-to-all of a local FrequencyTable; returns the table of the keys this rank
    owns (numRows 0: the global numRows is the all-reduce of the local ones).  `stats` (a dict)
    receives this rank's exchange cost: bytes sent / received over the all-to-all and the
    milliseconds of the partition, the all-to-all and the owner-side import."""
    import time
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = table.torch_device
    comm = dev if _comm_device(group) == "cuda" else torch.device("cpu")
    part_p, part_g, part_k, err = [0] * world, [0] * world, [0] * world, None
    t0 = time.perf_counter()
    try:
        part_p, part_g, part_k = table.partition_sizes(world)
        nbytes = sum(table.part_bytes(p, g) for p, g in zip(part_p, part_g))
        send_g = torch.empty(max(16, nbytes), dtype=torch.uint8, device=dev)
        send_k = torch.empty(max(8, sum(part_k)), dtype=torch.uint8, device=dev)
        if nbytes:
            table.partition_into(world, send_g, send_k)
    except Exception as e:  # noqa: BLE001 -- agreed on below, then re-raised
        err = e
    agree(err, "partitioning the frequency table by owner", group)
    _sync(dev)
    t1 = time.perf_counter()
    sizes = torch.tensor([[p, g, k] for p, g, k in zip(part_p, part_g, part_k)], dtype=torch.int64).reshape(-1).to(comm)
    recv_sizes = torch.empty_like(sizes)
    dist.all_to_all_single(recv_sizes, sizes, group=group)
    recv = recv_sizes.cpu().reshape(world, 3).tolist()
    in_g = [table.part_bytes(p, g) for p, g in zip(part_p, part_g)]
    out_g = [table.part_bytes(r[0], r[1]) for r in recv]
    in_k, out_k = list(part_k), [r[2] for r in recv]
    recv_g = torch.empty(max(16, sum(out_g)), dtype=torch.uint8, device=comm)
    recv_k = torch.empty(max(8, sum(out_k)), dtype=torch.uint8, device=comm)
    sg = _to(send_g, comm)
    sk = _to(send_k, comm)
    dist.all_to_all_single(recv_g[:sum(out_g)], sg[:sum(in_g)], out_g, in_g, group=group)
    dist.all_to_all_single(recv_k[:sum(out_k)], sk[:sum(in_k)], out_k, in_k, group=group)
    if comm.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()  # the library reads them on its own stream
    recv_g, recv_k = _to(recv_g, dev), _to(recv_k, dev)
    t2 = time.perf_counter()
    owned, err = None, None
    try:
        owned = type(table).like(table)
        owned.import_parts(recv_g, [r[0] for r in recv], [r[1] for r in recv], recv_k, [r[2] for r in recv], 0)
    except Exception as e:  # noqa: BLE001
        err = e
    try:
        agree(err, "merging the received frequency parts", group)
    except Exception:
        if owned is not None:  # (a half-built table, or one another rank's failure orphans)
            owned.close()
        raise
    _sync(dev)
    t3 = time.perf_counter()
    rank = dist.get_rank(group)
    _LAST_EXCHANGE.clear()
    _LAST_EXCHANGE.update({"bytes_sent": int(sum(in_g) + sum(in_k)),
                      "bytes_sent_remote": int(sum(in_g) + sum(in_k) - in_g[rank] - in_k[rank]),
                      "bytes_received": int(sum(out_g) + sum(out_k)),
                      "partition_ms": (t1 - t0) * 1e3, "alltoall_ms": (t2 - t1) * 1e3, "import_ms": (t3 - t2) * 1e3,
                      "exchange_ms": (t3 - t0) * 1e3})
    if stats is not None:
        stats.update(_LAST_EXCHANGE)
    return owned


_LAST_EXCHANGE: dict = {}


def last_exchange_stats() -> dict:
    """This rank's cost of the last key-hash exchange (exchange_frequencies' stats): bench.py
    reports it beside the C4 step time at N > 1."""
    return dict(_LAST_EXCHANGE)


class DistributedFrequencies:
    """FrequenciesAndNumRows of the union of every rank's rows (GroupingAnalyzers.scala:124-157),
    held as the keys each rank owns after the exchange.  Collective: every rank calls the same
    methods in the same order."""

    def __init__(self, owned, num_rows: int, group=None, exchange: Optional[dict] = None):
        self.owned = owned
        self.group = group
        self._num_rows = int(num_rows)
        self._summary = None
        self.table = _DistributedTableView(self)
        self.exchange = exchange or {}  # this rank's exchange cost (exchange_frequencies' stats)

    @property
    def columns(self):
        return self.owned.key_columns

    @property
    def numRows(self) -> int:
        return self._num_rows

    def summary(self):
        if self._summary is None:
            import torch
            import torch.distributed as dist
            from .frequencies import summary_from_histogram
            hist, big = self.owned.count_histogram()
            dev = _comm_tensor_device(self.group, self.owned)
            h = torch.from_numpy(hist).to(dev)
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            # the counts above the histogram's range: a variable-length tensor gather
            bigs = _allgather_var(torch.from_numpy(np.ascontiguousarray(big, dtype=np.int64)).to(dev), self.group)
            all_big = np.sort(np.concatenate([b.cpu().numpy() for b in bigs])) if bigs else np.zeros(0, np.int64)
            self._summary = summary_from_histogram(h.cpu().numpy(), all_big, self._num_rows)
        return self._summary

    def gather_arrays(self, dst: Optional[int] = None):
        """Every owner's groups as flat arrays -- (counts int64, key lengths int32, key bytes uint8),
        owners in rank order -- from each owner's flat export (dq_freq_export_flat; straight
        into device tensors for an nccl group) gathered with tensor collectives: no per-group
        Python object anywhere.  On every rank (dst None) or only on rank `dst` (the others get
        None).  Collective."""
        import torch
        import torch.distributed as dist
        world = dist.get_world_size(self.group)
        dev = _comm_tensor_device(self.group, self.owned)
        counts, offs, blob = self.owned.export_flat(device=dev.type == "cuda")
        if dev.type != "cuda":
            counts, offs, blob = (torch.from_numpy(np.ascontiguousarray(a)) for a in (counts, offs, blob))
        lens = (offs[1:] - offs[:-1]).to(torch.int32)
        size = torch.tensor([counts.numel(), blob.numel()], dtype=torch.int64, device=dev)
        sizes = [torch.empty_like(size) for _ in range(world)]
        dist.all_gather(sizes, size, group=self.group)
        sizes = [tuple(int(v) for v in t.cpu().tolist()) for t in sizes]
        mg, mk = max(1, max(g for g, _ in sizes)), max(1, max(k for _, k in sizes))

        def padded(t, n):
            out = torch.zeros(n, dtype=t.dtype, device=dev)
            if t.numel():
                out[:t.numel()] = t
            return out
        mine = [padded(counts, mg), padded(lens, mg), padded(blob, mk)]
        out = []
        rank = dist.get_rank(self.group)
        for t in mine:
            if dst is None:
                bufs = [torch.empty_like(t) for _ in range(world)]
                dist.all_gather(bufs, t, group=self.group)
            else:
                bufs = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
                dist.gather(t, bufs, dst=dst, group=self.group)
            out.append(bufs)
        if dst is not None and rank != dst:
            return None
        cs = np.concatenate([out[0][r][:sizes[r][0]].cpu().numpy() for r in range(world)])
        ls = np.concatenate([out[1][r][:sizes[r][0]].cpu().numpy() for r in range(world)])
        kb = np.concatenate([out[2][r][:sizes[r][1]].cpu().numpy() for r in range(world)])
        return cs, ls, kb

    def to_arrow(self, strings: Optional[bool] = None, dst: Optional[int] = None):
        """The whole dataset's frequencies DataFrame as an Arrow table (gather_arrays, then the
        columnar key codec); on every rank or only on `dst`.  Collective."""
        import pyarrow as pa
        from .keycols import decode_columns
        got = self.gather_arrays(dst)
        if got is None:
            return None
        cs, ls, kb = got
        offs = np.zeros(len(ls) + 1, dtype=np.int64)
        np.cumsum(ls, out=offs[1:])
        o = self.owned
        strings = o.histogram if strings is None else strings
        cols = decode_columns(offs, kb, o.dtypes, o.histogram, strings=strings)
        name = "count" if o.histogram else "com_amazon_deequ_dq_metrics_count"
        return pa.Table.from_arrays(cols + [pa.array(cs, type=pa.int64())], names=list(o.key_columns) + [name])

    def frequencies(self, raw: bool = False, dst: Optional[int] = None):
        """Every group of the dataset ({key: count}), gathered as flat arrays (gather_arrays): on
        every rank, or only on rank `dst` (the others get {}).  Collective."""
        from .frequencies import decode_key
        got = self.gather_arrays(dst)
        if got is None:
            return {}
        cs, ls, kb = got
        ends = np.cumsum(ls, dtype=np.int64)
        raw_bytes = kb.tobytes()
        out = {}
        for c, e, n in zip(cs.tolist(), ends.tolist(), ls.tolist()):
            k = raw_bytes[e - n:e]
            out[k if raw else decode_key(k, self.owned.dtypes, self.owned.histogram)] = c
        return out


class _DistributedTableView:
    """What Histogram.computeMetricFrom reads from `state.table`: dtypes and top(n)."""

    def __init__(self, state: DistributedFrequencies):
        self._s = state
        self.dtypes = state.owned.dtypes
        self.key_columns = state.owned.key_columns
        self.histogram = state.owned.histogram

    def top(self, n: int):
        """Union of every owner's top-n (owners hold disjoint keys), cut at the n-th largest
        count with the ties kept -- the contract of FrequencyTable.top."""
        import torch
        counts, keys = self._s.owned.top(n)
        dev = _comm_tensor_device(self._s.group, self._s.owned)
        lens = np.array([len(k) for k in keys], dtype=np.int64)
        blob = np.frombuffer(b"".join(keys), dtype=np.uint8)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        g_counts = _allgather_var(t(np.asarray(counts, dtype=np.int64)), self._s.group)
        g_lens = _allgather_var(t(lens), self._s.group)
        g_blob = _allgather_var(t(blob), self._s.group)
        items = []
        for c, ln, b in zip(g_counts, g_lens, g_blob):
            raw = b.cpu().numpy().tobytes()
            ends = np.cumsum(ln.cpu().numpy())
            items += [(int(ci), raw[e - m:e]) for ci, e, m in zip(c.cpu().tolist(), ends.tolist(), ln.cpu().tolist())]
        items.sort(key=lambda ck: (-ck[0], ck[1]))
        if len(items) > n:
            cut = items[n - 1][0]
            items = [ck for ck in items if ck[0] >= cut]
        return np.array([c for c, _ in items], dtype=np.int64), [k for _, k in items]

    def lookup(self, key: bytes) -> int:
        """Count of one encoded key over the whole dataset (its owner holds it; collective)."""
        import torch
        import torch.distributed as dist
        t = torch.tensor([self._s.owned.lookup(key)], dtype=torch.int64)
        if _comm_device(self._s.group) == "cuda":
            t = t.to(self._s.owned.torch_device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self._s.group)
        return int(t.item())

    def export(self):
        """(counts, keys) of every group of the dataset, on every rank (collective)."""
        cs, ls, kb = self._s.gather_arrays()
        ends = np.cumsum(ls, dtype=np.int64)
        raw_bytes = kb.tobytes()
        return cs, [raw_bytes[e - n:e] for e, n in zip(ends.tolist(), ls.tolist())]


def compute_frequencies_distributed(data, grouping_columns, histogram: bool = False, group=None,
                                    table_factory=None):
    """FrequencyBasedAnalyzer.computeFrequencies over the union of every rank's shard `data`."""
    import torch
    import torch.distributed as dist
    from .frequencies import FrequencyTable
    make = table_factory or FrequencyTable
    schema = data.schema
    local, n_local, err = None, 0, None
    try:
        local = make(grouping_columns, {c: schema[c] for c in schema}, histogram)
        for batch in data.batches():
            local.consume(batch)
        n_local = local.summary().num_rows
    except Exception as e:  # noqa: BLE001 -- every rank fails together (agree)
        err = e
    stats: dict = {}
    try:  # the local table is closed on every exit (another rank's failure raises here too)
        agree(err, "the frequency group-by", group)
        owned = exchange_frequencies(local, group, stats)
    finally:
        if local is not None:
            local.close()
    n = torch.tensor([n_local], dtype=torch.int64)
    if _comm_device(group) == "cuda":
        n = n.to(owned.torch_device)
    dist.all_reduce(n, op=dist.ReduceOp.SUM, group=group)
    return DistributedFrequencies(owned, int(n.item()), group, stats)
