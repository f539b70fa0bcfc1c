"""Debug probe: the C4 key column through one FrequencyTable, sizes given on the command line,
with the library's materialize trace (DQ_FREQ_DEBUG=1) on stderr."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
os.environ.setdefault("DQ_FREQ_DEBUG", "1")
import torch  # noqa: E402

import bench  # noqa: E402
from deequ_amd.frequencies import FrequencyTable  # noqa: E402

for rows in [int(x) for x in sys.argv[1:]]:
    data = bench.make_c4_batches(rows, min(rows, 125_000_000), 201_500_000, 0, 0)
    for hist in (False, True):
        t = FrequencyTable(["key"], {"key": "string"}, histogram=hist) if hist else FrequencyTable(["key"], {"key": "string"})
        t0 = time.time()
        for part in data.parts:
            t.consume(part)
        s = t.summary()
        print("rows %d hist %s: groups %d unique %d  %.3f s" % (rows, hist, s.num_groups, s.num_unique,
                                                                time.time() - t0), flush=True)
