"""Host-side profile (cProfile) of one C5 / C4 / C1 bench step, to find where the wall time
between kernels goes.  Usage: python tools/prof_host.py c5|c4|c1 > gpurun_out/host_c5.txt"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import deequ_amd as d  # noqa: E402

wl = sys.argv[1]
d.set_device(0)
if wl == "c5":
    from deequ_amd.profiles import ColumnProfilerRunner
    data = bench.make_c5_table(100_000_000, 0, 0)

    def step():
        return ColumnProfilerRunner().onData(data).run()
elif wl == "c4":
    data = bench.make_c4_batches(1_000_000_000, 125_000_000, 201_500_000, 0, 0)
    an = [d.Uniqueness(["key"]), d.Distinctness(["key"]), d.Entropy("key"), d.CountDistinct(["key"]),
          d.Histogram("key")]

    def step():
        return d.AnalysisRunner.onData(data).addAnalyzers(an).run()
else:
    data = bench.make_c1_table(10_000_000, 0, 0)
    an = bench.c1_analyzers()

    def step():
        return d.AnalysisRunner.onData(data).addAnalyzers(an).run()

step()
torch.cuda.synchronize()
t0 = time.perf_counter()
step()
torch.cuda.synchronize()
print("unprofiled step %.2f ms" % ((time.perf_counter() - t0) * 1e3))
pr = cProfile.Profile()
pr.enable()
step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr, stream=sys.stdout)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(30)
