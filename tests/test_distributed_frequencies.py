"""Multi-rank frequency family (deequ_amd/distributed.py) on CPU with gloo, world sizes 2 and 3.

Each rank groups its own row shard, the ranks exchange their groups by owner with one
all-to-all (32-B wire groups + long-key bytes), and the metrics come from the all-reduced
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
        out[hist] = dict(num_rows=st.numRows, groups=s.num_groups, unique=s.num_unique,
                         grouped=s.grouped_rows, entropy=s.entropy,
                         top=list(zip(counts.tolist(), keys)), freqs=st.frequencies(raw=True))
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
