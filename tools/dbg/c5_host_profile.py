"""Host-side profile of one C5 ColumnProfilerRunner step (cProfile + wall vs GPU time)."""
import cProfile
import pstats
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402
from deequ_amd.profiles import ColumnProfilerRunner  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
table = bench.make_c5_table(rows, 0, 0)
ColumnProfilerRunner().onData(table).run()
torch.cuda.synchronize()
t0 = time.perf_counter()
ColumnProfilerRunner().onData(table).run()
torch.cuda.synchronize()
print("step s", time.perf_counter() - t0)
pr = cProfile.Profile()
pr.enable()
ColumnProfilerRunner().onData(table).run()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(40)
st.sort_stats("tottime").print_stats(25)
