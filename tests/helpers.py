"""Shared test helpers: build the same table for the oracle and for deequ_amd, and
construct matching analyzers on both sides."""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Optional

import numpy as np

import pyoracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def known_answers():
    with open(os.path.join(GOLDEN, "reference_known_answers.json")) as f:
        return json.load(f)


def oracle_table(spec: Dict[str, list]) -> O.OTable:
    return {name: O.OColumn(dtype, list(values)) for name, (dtype, values) in spec.items()}


def product_table(spec: Dict[str, list]):
    from deequ_amd import Table
    return Table.from_pydict({name: (dtype, list(values)) for name, (dtype, values) in spec.items()})


def product_analyzer(name: str, args: List):
    import deequ_amd as d
    return getattr(d, name)(*args)


FREQ_ANALYZERS = ("Uniqueness", "Distinctness", "CountDistinct", "UniqueValueRatio", "Entropy",
                  "MutualInformation")


def _columns(args) -> List[str]:
    return [args[0]] if isinstance(args[0], str) else list(args[0])


def oracle_state(name: str, args: List, table: O.OTable):
    if name in FREQ_ANALYZERS:
        return O.frequencies_state(table, _columns(args))
    if name == "Histogram":
        return O.histogram_state(table, args[0])
    if name == "Size":
        return O.size_state(table, *args)
    if name == "Compliance":
        return O.compliance_state(table, args[1], *args[2:])
    fn = {"Completeness": O.completeness_state, "Sum": O.sum_state, "Mean": O.mean_state,
          "StandardDeviation": O.stddev_state, "Minimum": O.min_state, "Maximum": O.max_state,
          "ApproxCountDistinct": O.approx_count_distinct_state, "MinLength": O.min_length_state,
          "MaxLength": O.max_length_state, "Correlation": O.correlation_state}[name]
    return fn(table, *args)


def oracle_metric(state, name: str = None, args: List = None) -> object:
    """The metric the reference would report: a float, "empty" (EmptyStateException),
    "failure" (another failure) or, for Histogram, {"bins", "values"}."""
    if name in FREQ_ANALYZERS:
        try:
            v = {"Uniqueness": O.uniqueness_metric, "Distinctness": O.distinctness_metric,
                 "CountDistinct": O.count_distinct_metric, "UniqueValueRatio": O.unique_value_ratio_metric,
                 "Entropy": O.entropy_metric}[name](state) if name != "MutualInformation" else \
                O.mutual_information_metric(state, _columns(args), _columns(args))
        except ValueError:
            return "failure"
        return "empty" if v is None else v
    if name == "Histogram":
        h = O.histogram_metric(state, *([args[2]] if len(args) > 2 else []))
        return {"bins": h["number_of_bins"], "values": h["values"]}
    if state is None:
        return "empty"
    v = state.metric_value()
    return "nan" if v != v else v


def histogram_matches(got: dict, expected: dict) -> bool:
    """Known-answer histogram expectations: bins plus the key set or the number of values."""
    if got["bins"] != expected["bins"]:
        return False
    if "keys" in expected and sorted(got["values"]) != sorted(expected["keys"]):
        return False
    if "n_values" in expected and len(got["values"]) != expected["n_values"]:
        return False
    return True


def random_table(rng: np.random.Generator, n: int, null_frac: float, dtypes=None):
    """Seeded table with one column per dtype (plus string keys).  Returns (spec) usable by
    both oracle_table and product_table."""
    dtypes = dtypes or ["int8", "int16", "int32", "int64", "float32", "float64", "bool", "string"]
    spec = {}
    for t in dtypes:
        if t == "bool":
            vals = rng.integers(0, 2, n).astype(bool).tolist()
        elif t == "string":
            vals = ["k%d" % v for v in rng.integers(0, max(1, n // 3 + 1), n)]
        elif t in ("float32", "float64"):
            arr = rng.normal(1e3, 1e2, n)
            if t == "float32":
                arr = arr.astype(np.float32).astype(np.float64)
            vals = arr.tolist()
        else:
            info = np.iinfo(t)
            lo, hi = (int(info.min), int(info.max)) if t != "int64" else (-2 ** 40, 2 ** 40)
            vals = rng.integers(lo, hi, n, endpoint=True).tolist()
        if null_frac > 0:
            mask = rng.random(n) < null_frac
            vals = [None if m else v for v, m in zip(vals, mask)]
        spec["c_" + t] = [t, vals]
    return spec


def exact_sum(vals) -> float:
    return math.fsum(float(v) for v in vals)


def exact_moments(vals):
    """(n, mean, m2) of the values (as doubles), exact up to the final rounding."""
    from fractions import Fraction
    fr = [Fraction(float(v)) for v in vals]
    n = len(fr)
    if n == 0:
        return 0, None, None
    mean = sum(fr) / n
    m2 = sum((x - mean) ** 2 for x in fr)
    return n, float(mean), float(m2)


def rel_err(a: float, b: float) -> float:
    if a == b:
        return 0.0
    if math.isnan(a) and math.isnan(b):
        return 0.0
    return abs(a - b) / max(abs(b), 1e-300)
