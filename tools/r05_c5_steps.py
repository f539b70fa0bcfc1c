"""Wall time of each of N consecutive C5 profiler steps (a drift over steps shows up here, not
in an average).  Usage: python tools/r05_c5_steps.py [N] > gpurun_out/r05_c5_steps.txt"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import deequ_amd as d  # noqa: E402
from deequ_amd.profiles import ColumnProfilerRunner  # noqa: E402

d.set_device(0)
data = bench.make_c5_table(100_000_000, 0, 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
if os.environ.get("GC_MODE") == "freeze":
    import gc
    gc.collect()
    gc.freeze()
elif os.environ.get("GC_MODE") == "log":
    import gc

    def _cb(phase, info, t=[0.0]):
        if phase == "start":
            t[0] = time.perf_counter()
        elif info.get("generation") == 2:
            print("  gc gen2 %.2f ms, %d collected" % ((time.perf_counter() - t[0]) * 1e3, info.get("collected", 0)))
    gc.callbacks.append(_cb)
out = None
for k in range(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    out = ColumnProfilerRunner().onData(data).run()
    torch.cuda.synchronize()
    print("step %2d %.2f ms  torch reserved %.2f GB" % (k, (time.perf_counter() - t0) * 1e3,
                                                       torch.cuda.memory_reserved() / 1e9), flush=True)
