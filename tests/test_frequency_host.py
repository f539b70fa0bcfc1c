"""Host-side pieces of the frequency family (no GPU): key codec, Java string casts, analyzer
preconditions and names.  Preconditions run before any device work, as in the reference."""
import math
import random

import numpy as np
import pytest

import deequ_amd as d
import pyoracle as O
from deequ_amd.frequencies import decode_key, encode_key
from deequ_amd.javafmt import java_double_to_string, java_float_to_string, spark_cast_to_string
from deequ_amd.metrics import (IllegalAnalyzerParameterException, NoColumnsSpecifiedException,
                               NumberOfSpecifiedColumnsException)
from helpers import product_table


@pytest.mark.parametrize("dtypes,key", [
    (["string"], ("héllo",)), (["int8"], (-5,)), (["int16"], (-300,)), (["int32"], (2 ** 31 - 1,)),
    (["int64"], (-2 ** 63,)), (["float64"], (-0.0,)), (["float32"], (1.5,)), (["bool"], (True,)),
    (["string", "int32", "string"], ("a", 7, "")), (["float64", "bool", "string"], (2.5, False, "x" * 40)),
])
def test_key_codec_roundtrip(dtypes, key):
    enc = encode_key(key, dtypes)
    got = decode_key(enc, dtypes)
    assert len(got) == len(key)
    for g, k in zip(got, key):
        assert g == k and (not isinstance(k, float) or math.copysign(1, g) == math.copysign(1, k))


def test_key_codec_layout():
    assert encode_key((1,), ["int32"]) == b"\x01\x00\x00\x00"
    assert encode_key(("ab", 1), ["string", "int8"]) == b"\x02\x00\x00\x00ab\x01"
    assert encode_key((None,), ["string"], histogram=True) == b"NullValue"
    assert encode_key((None,), ["int64"], histogram=True) == b""
    assert decode_key(b"", ["int64"], histogram=True) == (None,)
    nan_bits = encode_key((float("nan"),), ["float64"], histogram=True)
    assert nan_bits == (0x7FF8000000000000).to_bytes(8, "little")


def test_java_string_casts_match_oracle_restatement():
    rnd = random.Random(3)
    specials = [0.0, -0.0, 1.0, 1e7, 9999999.999, 1e-3, 9.999e-4, 5e-324, 1.7976931348623157e308,
                float("nan"), float("inf"), -float("inf"), 0.1, 100.0, 2 ** 53]
    for x in specials + [rnd.uniform(-1e12, 1e12) for _ in range(3000)] + \
            [rnd.lognormvariate(0, 30) for _ in range(3000)]:
        assert java_double_to_string(x) == O.java_double_to_string(x), x
        if not abs(x) < 3e38:
            continue
        f = float(np.float32(x))
        assert java_float_to_string(f) == O.java_double_to_string(f, single=True), f


def test_java_string_known_values():
    # Java's Double.toString / Float.toString outputs (JLS / JDK documentation examples)
    assert java_double_to_string(1.0) == "1.0"
    assert java_double_to_string(1e7) == "1.0E7"
    assert java_double_to_string(0.001) == "0.001"
    assert java_double_to_string(1e-4) == "1.0E-4"
    assert java_double_to_string(5e-324) == "4.9E-324"
    assert java_double_to_string(1.7976931348623157e308) == "1.7976931348623157E308"
    assert java_float_to_string(float(np.float32(0.1))) == "0.1"
    assert java_float_to_string(float(np.float32(1.4e-45))) == "1.4E-45"
    assert java_float_to_string(float(np.float32(3.4028235e38))) == "3.4028235E38"
    assert spark_cast_to_string(2147483647, "int32") == "2147483647"
    assert spark_cast_to_string(True, "bool") == "true"


def test_analyzer_names_and_entities():
    assert str(d.Uniqueness("att1")) == "Uniqueness(List(att1))"
    assert str(d.Uniqueness(["a", "b"])) == "Uniqueness(List(a, b))"
    assert str(d.Entropy("att1")) == "Entropy(att1)"
    assert str(d.MutualInformation("a", "b")) == "MutualInformation(List(a, b))"
    assert d.Uniqueness("att1") == d.Uniqueness(["att1"])
    assert d.Uniqueness(["a", "b"]).entity == d.Entity.Mutlicolumn
    assert d.Uniqueness(["a"]).entity == d.Entity.Column
    assert d.MutualInformation("a", "b") == d.MutualInformation(["a", "b"])
    assert len({d.CountDistinct("x"), d.CountDistinct(["x"])}) == 1


def test_precondition_failures_need_no_device():
    table = product_table({"att1": ["string", ["a"]], "att2": ["string", ["b"]]})
    m = d.Distinctness([]).calculate(table)
    assert isinstance(m.value.exception, NoColumnsSpecifiedException)
    assert str(m.value.exception) == "At least one column needs to be specified!"
    m = d.MutualInformation(["att2"]).calculate(table)
    assert isinstance(m.value.exception, NumberOfSpecifiedColumnsException)
    assert str(m.value.exception) == \
        "2 columns have to be specified! Currently, columns contains only 1 column(s): att2!"
    m = d.Histogram("att1", maxDetailBins=1001).calculate(table)
    assert isinstance(m.value.exception, IllegalAnalyzerParameterException)
    assert m.flatten()[0].name == "Histogram.bins"
    m = d.Uniqueness("nope").calculate(table)
    assert type(m.value.exception).__name__ == "NoSuchColumnException"
    assert m.instance == "nope"
