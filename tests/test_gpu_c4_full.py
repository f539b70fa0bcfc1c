"""C4 at its real size (1e9 rows, 12-digit keys from a 2.015e8-key domain, 1% NULL,
125M-row batches -- the 2^29-slot, 2^18-slice regime of the partition path): bench.py's C4 step,
then its metrics checked against torch.unique(return_counts=True) over the same integer ids on the
device -- an independent sort-based group-by (bench.py c4_verify).  CountDistinct, Uniqueness,
Distinctness, Histogram's NULL bin and bin count exactly; Entropy within 1e-12 relative; every
Histogram detail bin's count and the detail bins' count multiset exactly."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("keys", ["digits", "alnum", "uuid", "pair", "pair64"])
def test_c4_full_size_against_torch_unique(gpu, keys):
    """digits: 12-digit keys (packed 8-byte records); alnum: 'k' + 11 digits -- keys that are not
    digit strings, staged as 16-byte records from the first batch (the pack probe); uuid: the ids'
    36-character UUID text, and pair: the two-column key (id // 1000, 8 digits of id % 1000) -- the
    hashed records of long and composite keys (round 6), the isPrimaryKey / hasUniqueness shape
    (Check.scala:140-230); pair64: the same pair as (int64, int64), 16-byte-key records."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c4", "--c4-verify", "--steps", "1",
           "--warmup", "0", "--c4-keys", keys]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, PYTHONUNBUFFERED="1"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    v = line["verify"]
    print("\n[c4 full %s] %s" % (keys, json.dumps(v)))
    assert v["ok"], v
    assert v["groups"] > 180_000_000
    if not keys.startswith("pair"):  # (a composite key has no Histogram)
        assert v["detail_bins"] >= 999
