"""Wall-clock spans of one C4 bench step's host stages (the GPU idles ~1.8 ms between steps in
the kernel trace): table creation, each consume, summary, top, lookup, destruction, and the
step boundary itself (the previous step's context dropped).  Usage:
python tools/r05_c4_spans.py > gpurun_out/r05_c4_spans.txt"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import deequ_amd as d  # noqa: E402
from deequ_amd import frequencies as F  # noqa: E402

d.set_device(0)
data = bench.make_c4_batches(1_000_000_000, 125_000_000, 201_500_000, 0, 0)
an = [d.Uniqueness(["key"]), d.Distinctness(["key"]), d.Entropy("key"), d.CountDistinct(["key"]), d.Histogram("key")]
spans = []


def wrap(cls, name):
    f = getattr(cls, name)

    def g(*a, **k):
        s = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            spans.append((s, time.perf_counter(), name))
    setattr(cls, name, g)


for name in ("__init__", "consume", "summary", "top", "lookup", "close", "count_histogram"):
    if hasattr(F.FrequencyTable, name):
        wrap(F.FrequencyTable, name)
wrap(F, "compute_frequencies")


def step():
    return d.AnalysisRunner.onData(data).addAnalyzers(an).run()


out = step()
torch.cuda.synchronize()
for k in range(3):
    spans.clear()
    t0 = time.perf_counter()
    out = None
    t_drop = time.perf_counter()
    out = step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("step %d: drop %.3f ms, step %.3f ms, trailing sync %.3f ms" % (k, (t_drop - t0) * 1e3, (t1 - t_drop) * 1e3,
                                                                        (t2 - t1) * 1e3))
    for s, e, n in spans:
        print("  %8.3f -> %8.3f  %7.3f ms  %s" % ((s - t0) * 1e3, (e - t0) * 1e3, (e - s) * 1e3, n))
