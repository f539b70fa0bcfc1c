"""Multi-rank frequency family (deequ_amd/distributed.py) on CPU with gloo, world sizes 2 and 3.

Each rank groups its own row shard, the ranks exchange their groups by owner with one
all-to-all (16-B packed wire groups for digit keys, 32-B for others, + long-key bytes), and the metrics come from the all-reduced
count-of-counts histogram.  The GPU table is replaced by tests/fake_freq.py (same methods and
wire format) because these CPU tests run no GPU compute; tests/test_gpu_distributed.py runs the
same orchestration on the real dq_freq tables.  Expected values: the oracle over the whole table.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 2400


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _keys(lo, hi):
    out = []
    for i in range(lo, hi):
        if i % 13 == 0:
            out.append(None)
        elif i % 5 == 0:
            out.append("a-rather-long-grouping-key-%03d" % (i % 17))  # > 16 B: key-byte path
        elif i % 3 == 0:
            out.append("%d" % ((i * 104729) % 997))  # digit keys: 16-B packed wire records
        else:
            out.append("k%d" % ((i * 7919) % 611))
    return out


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    import deequ_amd as d
    from deequ_amd.distributed import compute_frequencies_distributed
    from fake_freq import FakeFrequencyTable
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    lo, hi = rank * N // world, (rank + 1) * N // world
    shard = d.Table.from_pydict({"key": ("string", _keys(lo, hi))})
    out = {}
    for hist in (False, True):
        st = compute_frequencies_distributed(shard, ["key"], histogram=hist, table_factory=FakeFrequencyTable)
        s = st.summary()
        counts, keys = st.table.top(7)
        freqs = st.frequencies(raw=True)
        at0 = st.frequencies(raw=True, dst=0)  # gathered on rank 0 only
        assert at0 == (freqs if rank == 0 else {})
        ec, ek = st.table.export()
        assert dict(zip(ek, ec.tolist())) == freqs
        out[hist] = dict(num_rows=st.numRows, groups=s.num_groups, unique=s.num_unique,
                         grouped=s.grouped_rows, entropy=s.entropy,
                         top=list(zip(counts.tolist(), keys)), freqs=freqs)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_equals_whole_table(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    keys = _keys(0, N)
    whole = O.frequencies_state({"key": O.OColumn("string", keys)}, ["key"])
    want = {(k,): c for (k,), c in whole.frequencies.items()}
    for r in range(world):
        got = results[r][False]
        assert got == results[0][False]  # every rank holds the same global answer
        assert got["num_rows"] == N
        assert got["groups"] == len(want)
        assert got["unique"] == sum(1 for c in want.values() if c == 1)
        assert got["grouped"] == sum(want.values())
        assert abs(got["entropy"] - O.entropy_exact(whole)) <= 1e-12 * O.entropy_exact(whole)
        assert {k.decode(): c for k, c in got["freqs"].items()} == {k[0]: c for k, c in want.items()}
        cut = sorted(want.values(), reverse=True)[6]
        assert sorted(c for c, _ in got["top"]) == sorted(c for c in want.values() if c >= cut)
        # Histogram grouping: NULL is the "NullValue" group
        h = results[r][True]
        nulls = sum(1 for k in keys if k is None)
        assert h["groups"] == len(want) + 1 and h["grouped"] == N
        assert {k.decode(): c for k, c in h["freqs"].items()}["NullValue"] == nulls


def _persist_worker(rank, world, port, q, directory):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    import deequ_amd as d
    from deequ_amd.distributed import compute_frequencies_distributed
    from deequ_amd.state_provider import HdfsStateProvider
    from fake_freq import FakeFrequencyTable
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    lo, hi = rank * N // world, (rank + 1) * N // world
    shard = d.Table.from_pydict({"key": ("string", _keys(lo, hi))})
    prov = HdfsStateProvider(os.path.join(directory, "st"))
    out = {}
    for name, hist in (("u", False), ("h", True)):
        st = compute_frequencies_distributed(shard, ["key"], histogram=hist, table_factory=FakeFrequencyTable)
        an = d.Histogram("key") if hist else d.Uniqueness(["key"])
        prov.persist(an, st)
        try:  # a second write without allowOverwrite fails on every rank
            prov.persist(an, st)
            out[name] = "no error"
        except FileExistsError:
            out[name] = "exists"
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_state_persisted_per_owner(tmp_path):
    """HdfsStateProvider over a frequency state held by 2 ranks: each rank writes the part of the
    groups it owns (part-00000, part-00001), nobody gathers the table; the parts together are
    the whole table's state (StateProvider.scala:222-240 layout), disjoint by key."""
    import pyarrow.parquet as pq
    import struct
    from deequ_amd.state_provider import HdfsStateProvider, scala_string_hash
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_persist_worker, args=(r, world, port, q, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(results[r] == {"u": "exists", "h": "exists"} for r in range(world)), results
    import deequ_amd as d
    keys = _keys(0, N)
    whole = O.frequencies_state({"key": O.OColumn("string", keys)}, ["key"])
    for an, want in ((d.Uniqueness(["key"]), {k[0]: c for k, c in whole.frequencies.items()}),
                     (d.Histogram("key"), None)):
        base = str(tmp_path / "st") + "-%d" % scala_string_hash(str(an), 42)
        parts = sorted(os.listdir(base + "-frequencies.pqt"))
        assert parts == ["part-00000.snappy.parquet", "part-00001.snappy.parquet"]
        seen = {}
        for part in parts:
            t = pq.ParquetFile(os.path.join(base + "-frequencies.pqt", part)).read()
            for k, c in zip(t.column(0).to_pylist(), t.column(1).to_pylist()):
                assert k not in seen  # owners hold disjoint keys
                seen[k] = c
        with open(base + "-num_rows.bin", "rb") as f:
            assert struct.unpack(">q", f.read())[0] == N
        if want is None:  # Histogram: NULL is the "NullValue" group
            want = {k[0]: c for k, c in whole.frequencies.items()}
            want["NullValue"] = sum(1 for k in keys if k is None)
        assert seen == want


class _FailingTable:
    """A table factory whose consume raises on rank 1 only."""

    def __init__(self, *a, **k):
        import torch.distributed as dist
        from fake_freq import FakeFrequencyTable
        self._t = FakeFrequencyTable(*a, **k)
        self._fail = dist.get_rank() == 1

    def consume(self, batch):
        if self._fail:
            raise ValueError("-injected-consume-failure-")
        self._t.consume(batch)

    def __getattr__(self, name):
        return getattr(self._t, name)


def _failing_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    import deequ_amd as d
    from deequ_amd.distributed import compute_frequencies_distributed
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shard = d.Table.from_pydict({"key": ("string", _keys(rank * 100, rank * 100 + 100))})
    try:
        compute_frequencies_distributed(shard, ["key"], table_factory=_FailingTable)
        out = "no error"
    except Exception as e:  # noqa: BLE001
        out = "%s: %s" % (type(e).__name__, e)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_group_by_failure_on_one_rank_fails_every_rank():
    """a rank whose local group-by raises must not leave its peers blocked in the
    all-to-all -- every rank raises (the failed one its own error)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert "-injected-consume-failure-" in results[1], results
    assert "failed on another rank" in results[0], results
