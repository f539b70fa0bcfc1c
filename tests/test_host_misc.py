"""Host-only behaviour that no GPU test reaches: analyzer identity across processes, and the
test-only publish hook being absent from the production library."""
import os
import pickle
import subprocess
import sys

import deequ_amd as d

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_analyzer_hash_not_pickled():
    a = d.Completeness("c")
    hash(a)  # memoised in the instance
    assert "_dq_hash" in a.__dict__
    b = pickle.loads(pickle.dumps(a))
    assert "_dq_hash" not in b.__dict__
    assert b == a and hash(b) == hash(a)


def test_analyzer_pickle_across_hash_seeds():
    """An analyzer pickled in a process with another str-hash salt still finds its metric in a
    dict keyed by locally built analyzers (AnalyzerContext.metricMap)."""
    blob = subprocess.check_output(
        [sys.executable, "-c",
         "import pickle, sys; sys.path.insert(0, %r); import deequ_amd as d\n"
         "xs = [d.Completeness('c'), d.Mean('c'), d.Compliance('r', 'c > 0'), d.Histogram('c')]\n"
         "[hash(x) for x in xs]\n"
         "sys.stdout.buffer.write(pickle.dumps(xs))" % ROOT],
        env=dict(os.environ, PYTHONHASHSEED="12345"))
    remote = pickle.loads(blob)
    local = {d.Completeness("c"): 1, d.Mean("c"): 2, d.Compliance("r", "c > 0"): 3, d.Histogram("c"): 4}
    assert [local[x] for x in remote] == [1, 2, 3, 4]
