"""C1 (BASELINE.json configs[0]): the reference's own CPU-runnable case, an
AnalysisRunner over the `Item` table (examples/entities.scala:19-25) with Size, Completeness of
all five columns, Compliance("numViews >= 0") and Mean/StdDev/Min/Max(numViews).

The GPU run goes through the AnalysisRunner mirror and is checked metric by metric against the
oracle on the same seeded rows: bit-exact for the counts, Compliance, Min/Max; fp64 Mean/StdDev
within 1e-12 relative of the exact value.  Also the five-row table of examples/BasicExample
.scala:28-33 through the same suite."""
import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from helpers import exact_moments, oracle_table, product_table, rel_err

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12


def c1_spec(n: int, seed: int = 1):
    """C1 rows: id = 0..n-1; productName "Thingy <id>", description and
    priority in {high, low}, each 5% NULL; numViews uniform int64 in [-1e3, 1e6), 5% NULL."""
    rng = np.random.default_rng(seed)

    def nulls(vals):
        m = rng.random(n) < 0.05
        return [None if k else v for v, k in zip(vals, m)]

    ids = list(range(n))
    return {
        "id": ["int64", ids],
        "productName": ["string", nulls(["Thingy %d" % i for i in ids])],
        "description": ["string", nulls(["item %d description" % (i * 7919 % 100003) for i in ids])],
        "priority": ["string", nulls([("high", "low")[k] for k in rng.integers(0, 2, n)])],
        "numViews": ["int64", nulls(rng.integers(-1000, 1_000_000, n).tolist())],
    }


def c1_analyzers():
    return ([d.Size()] + [d.Completeness(c) for c in ("id", "productName", "description", "priority", "numViews")]
            + [d.Compliance("numViews non-negative", "numViews >= 0"), d.Mean("numViews"),
               d.StandardDeviation("numViews"), d.Minimum("numViews"), d.Maximum("numViews")])


def _check(spec):
    ot, pt = oracle_table(spec), product_table(spec)
    analyzers = c1_analyzers()
    ctx = d.AnalysisRunner.onData(pt).addAnalyzers(analyzers).run()
    views = [v for v in spec["numViews"][1] if v is not None]
    for a in analyzers:
        got = ctx.metric(a)
        name = type(a).__name__
        if name == "Size":
            exp = O.size_state(ot).metric_value()
        elif name == "Completeness":
            exp = O.completeness_state(ot, a.column).metric_value()
        elif name == "Compliance":
            exp = O.compliance_state(ot, a.predicate).metric_value()
        elif name == "Minimum":
            exp = O.min_state(ot, "numViews").metric_value()
        elif name == "Maximum":
            exp = O.max_state(ot, "numViews").metric_value()
        else:
            n, mean, m2 = exact_moments(views)
            exp = float(mean) if name == "Mean" else float((m2 / n) ** 0.5)
            assert rel_err(got.value.get(), exp) <= REL_TOL, (a, got, exp)
            continue
        assert got.value.get() == exp, (a, got, exp)


def test_c1_item_table(gpu):
    _check(c1_spec(30_000))


def test_basic_example_items(gpu):
    # examples/BasicExample.scala:28-33
    spec = {
        "id": ["int64", [1, 2, 3, 4, 5]],
        "productName": ["string", ["Thingy A", "Thingy B", None, "Thingy D", "Thingy E"]],
        "description": ["string", ["awesome thing.", "available at http://thingb.com", None,
                                   "checkout https://thingd.ca", None]],
        "priority": ["string", ["high", None, "low", "low", "high"]],
        "numViews": ["int64", [0, 0, 5, 10, 12]],
    }
    _check(spec)
