"""Key and string bytes at the very end of a utf8 heap (round 4).

The group-by's fused stage and few-groups kernels read each key as ONE unaligned 16-byte buffer
load at min(offset, heap_end - 16), and the profiler's string pass and string -> number cast read
24 bytes at min(offset, heap_end - 24): a buffer load's range check is per dword counted from the
load's own offset, so a load reaching past the heap would zero whole dwords -- key bytes
included.  A key starting in the heap's last 16 (24) bytes is shifted down in registers; a heap
smaller than the window goes to an exact path.  Checked here bit-exact against plain Python
counting and the oracle: the last keys of a batch of every length 0..15 ending exactly at the heap
end, heaps of 1, 15, 16, 17, 23, 24 and 25 bytes, NULLs last, on every group-by path."""
import collections

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd.frequencies import FrequencyTable
from helpers import oracle_table, product_table

pytestmark = pytest.mark.gpu

PATHS = {
    "partition": {"DQ_FREQ_PART_MIN": "1", "DQ_FREQ_PATH": "sorted"},
    "partition16": {"DQ_FREQ_PART_MIN": "1", "DQ_FREQ_PATH": "sorted", "DQ_FREQ_PACK": "0"},
    "default": {},
    "small": {},
}


def _tails(n_body, tail, digits):
    """n_body keys, then `tail` (the keys at the heap's end)."""
    rng = np.random.default_rng(len(tail) * 7 + n_body)
    body = [("%d" % v) if digits else ("k%d" % v) for v in rng.integers(0, 3000, n_body)]
    return body + list(tail)


def _cases():
    digits_tail = ["1" * ln if ln else "" for ln in range(16)] + ["9876543210", "0", "42"]
    other_tail = ["x" * ln for ln in range(16)] + ["abc", "k9"]
    return [
        ("digits_tail", _tails(20000, digits_tail, True)),
        ("other_tail", _tails(20000, other_tail, False)),
        ("null_last", _tails(20000, ["123", None, "77", None], True)),
        ("tiny1", ["7"]),
        ("tiny15", ["12345", "", "6789", "012345"]),
        ("heap16", ["12345678", "87654321"]),
        ("heap17", ["1234567812345678", "9"]),
        ("heap23", ["abcdefghijk", "lmnopqrstuvw"]),
        ("heap24", ["123456789012", "345678901234"]),
        ("heap25", ["1234567890123", "456789012345"]),
    ]


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("name,keys", _cases(), ids=[c[0] for c in _cases()])
def test_group_by_keys_at_heap_end(gpu, monkeypatch, path, name, keys):
    for k, v in PATHS[path].items():
        monkeypatch.setenv(k, v)
    for hist in (False, True):
        t = FrequencyTable(["key"], {"key": "string"}, histogram=hist)
        if path == "small":
            t.expect_groups(min(len(set(keys)) + 1, 900))
        t.consume(d.Table.from_pydict({"key": ("string", keys)}))
        counts, got_keys = t.export()
        got = dict(zip(got_keys, counts.tolist()))
        want = collections.Counter()
        for k in keys:
            if k is None:
                if hist:
                    want[b"NullValue"] += 1
            else:
                want[k.encode()] += 1
        assert got == dict(want), (path, name, hist)
        assert t.paths()["wait_timeouts"] == 0
        t.close()


@pytest.mark.parametrize("name,keys", _cases(), ids=[c[0] for c in _cases()])
def test_string_pass_at_heap_end(gpu, name, keys):
    """DataType + ApproxCountDistinct (the fused string pass) and the string -> long / double
    casts of the profiler on the same columns: equal to the oracle."""
    spec = {"s": ["string", keys]}
    table, ot = product_table(spec), oracle_table(spec)
    prov = d.InMemoryStateProvider()
    an = [d.DataType("s"), d.ApproxCountDistinct("s")]
    d.AnalysisRunner.onData(table).addAnalyzers(an).saveStatesWith(prov).run()
    assert prov.load(an[0]).counts() == O.datatype_state(ot, "s", None), name
    assert prov.load(an[1]).words == O.approx_count_distinct_state(ot, "s", None).words, name
    import math
    import struct
    from deequ_amd.profiles import cast_string_column
    from test_gpu_profiles import _spark_to_long
    col = d.Column.from_pylist(keys, "string")
    assert cast_string_column(col, "int64").to_pylist() == [None if k is None else _spark_to_long(k) for k in keys]
    for k, g in zip(keys, cast_string_column(col, "float64").to_pylist()):
        want = None if k is None else O.java_parse_double(k)
        if want is None or g is None:
            assert want is None and g is None, (name, k, g)
        elif math.isnan(want):
            assert math.isnan(g), (name, k)
        else:
            assert struct.pack("<d", g) == struct.pack("<d", want), (name, k, g, want)
