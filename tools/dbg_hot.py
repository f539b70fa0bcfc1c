"""Debug: the hot-key int64 group-by on each path, count mismatches vs numpy."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deequ_amd as d
from deequ_amd.frequencies import FrequencyTable
d.set_device(0)
rng = np.random.default_rng(13)
n = 4_000_000
vals = rng.integers(0, 300_000, n)
vals[rng.random(n) < float(os.environ.get("HOT", "0.5"))] = 987_654_321
u, c = np.unique(vals, return_counts=True)
want = dict(zip(u.tolist(), c.tolist()))
t = FrequencyTable(["v"], {"v": "int64"})
t.consume(d.Table({"v": d.Column.from_numpy(vals, None, "int64")}))
counts, keys = t.export()
got = {int.from_bytes(k, "little", signed=True): int(x) for k, x in zip(keys, counts.tolist())}
bad = [k for k in want if got.get(k) != want[k]]
s = t.summary()
from collections import Counter
dup = Counter(keys)
nd = sum(1 for k, v in dup.items() if v > 1)
hotk = (987654321).to_bytes(8, "little")
print("num_groups", s.num_groups, "exported", len(keys), "dup_keys", nd, "sum_counts", int(counts.sum()), "n", n,
      "hot_slots", dup.get(hotk), "hot_total", int(sum(int(c) for k, c in zip(keys, counts.tolist()) if k == hotk)))
print("paths", t.paths(), "groups", len(got), "want", len(want), "bad", len(bad),
      "missing_rows", sum(want.values()) - sum(got.values()), "hot", got.get(987654321), want.get(987654321))
