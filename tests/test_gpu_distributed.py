"""The multi-rank frequency exchange on the real GPU tables: 2 ranks (gloo for the host-side
collectives, both ranks on cuda:0 -- the one-GPU box cannot run RCCL between two ranks on one
device), each grouping its own shard with dq_freq, partitioning it with dq_freq_partition and
merging the received parts with dq_freq_import_parts (digit keys travel as 16-B packed records).  Bit-exact against the oracle over the
whole table (frequencies, #groups, #unique, top-N); entropy within 1e-12 relative."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import pyoracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 60000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spec(lo, hi):
    rng = np.random.default_rng(5)
    a = rng.integers(0, 9000, N)
    keys = [None if i % 17 == 0 else ("long-key-%020d" % a[i] if i % 3 == 0 else
                                      ("%d" % a[i] if i % 3 == 1 else "k%d" % a[i]))
            for i in range(N)]
    ints = [None if i % 11 == 0 else int(a[i] % 500) for i in range(N)]
    return keys[lo:hi], ints[lo:hi]


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import deequ_amd as d
    from deequ_amd.distributed import compute_frequencies_distributed
    d.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    lo, hi = rank * N // world, (rank + 1) * N // world
    keys, ints = _spec(lo, hi)
    shard = d.Table.from_pydict({"key": ("string", keys), "i": ("int64", ints)})
    out = {}
    for cols, hist in ((["key"], False), (["i"], False), (["key"], True), (["key", "i"], False)):
        st = compute_frequencies_distributed(shard, cols, histogram=hist)
        s = st.summary()
        counts, top_keys = st.table.top(10)
        out[(tuple(cols), hist)] = dict(num_rows=st.numRows, groups=s.num_groups, unique=s.num_unique,
                                        grouped=s.grouped_rows, entropy=s.entropy,
                                        top=sorted(counts.tolist()), freqs=st.frequencies(raw=True))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_exchange_matches_oracle(gpu):
    from deequ_amd.frequencies import encode_key
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    keys, ints = _spec(0, N)
    otable = {"key": O.OColumn("string", keys), "i": O.OColumn("int64", ints)}
    for (cols, hist), got in results[0].items():
        assert results[1][(cols, hist)] == got
        dtypes = ["string" if c == "key" else "int64" for c in cols]
        if hist:
            ostate = O.histogram_state(otable, cols[0])
            want = {encode_key([k[0] if k[0] != "NullValue" else None], dtypes, True): c
                    for k, c in ostate.frequencies.items()}
        else:
            ostate = O.frequencies_state(otable, list(cols))
            want = {encode_key(list(k), dtypes): c for k, c in ostate.frequencies.items()}
        assert got["num_rows"] == N
        assert got["freqs"] == want
        assert got["groups"] == len(want)
        assert got["unique"] == sum(1 for c in want.values() if c == 1)
        assert got["grouped"] == sum(want.values())
        cut = sorted(want.values(), reverse=True)[9]
        assert got["top"] == sorted(c for c in want.values() if c >= cut)
        if not hist:
            e = O.entropy_exact(ostate)
            assert abs(got["entropy"] - e) <= 1e-12 * e
