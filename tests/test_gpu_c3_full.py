"""C3's whole job (64 int64 columns x 1e9 rows, the reference's one data.agg,
AnalysisRunner.scala:313): one plan over 8 consumes of 125M-row batches, column 0's 52 HLL
words compared bit for bit with the oracle's registers of all 8 batches (dq_oracle.c, max-merged
as DeequHyperLogLogPlusPlusUtils.merge does).  The estimate is the reference's own: a register
of rank >= 32 adds 2^-(m - 32) through Java's Int shift (StatefulHyperloglogPlus.scala:222),
so ~9.5e8 distinct values can estimate far lower -- the test prints those registers."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c3_whole_job_registers_against_oracle(gpu):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c3", "--c3-batches", "8", "--c3-verify",
           "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, PYTHONUNBUFFERED="1"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    job = line["full_job"]
    v = job["verify"]
    print("\n[c3 full job] rows %d, estimate %s, %s" % (job["rows_per_gpu"], job["column0_estimate"], json.dumps(v)))
    assert job["rows_per_gpu"] == 1_000_000_000
    assert v["words_equal"], v
    assert job["column0_estimate"] == v["estimate_oracle"]
