"""The GPU path against the reference's own known answers (tests/golden/
reference_known_answers.json): per analyzer (`calculate`), all analyzers of a table in ONE
fused pass (`AnalysisRunner`), and state merge == union (`Analyzers.merge` and a two-batch
PartitionedTable)."""
import pytest

import deequ_amd as d
from deequ_amd.metrics import EmptyStateException, Failure, Success
from deequ_amd.states import merge
from helpers import histogram_matches, known_answers, product_analyzer, product_table

pytestmark = pytest.mark.gpu

KA = known_answers()


def _check(metric, expected, source):
    if isinstance(expected, dict):  # Histogram
        assert metric.value.isSuccess, (source, metric)
        dist = metric.value.get()
        got = {"bins": dist.numberOfBins, "values": dist.values}
        assert histogram_matches(got, expected), (source, got)
        return
    if expected == "empty":
        assert isinstance(metric.value, Failure), (source, metric)
        assert isinstance(metric.value.exception, EmptyStateException), (source, metric)
    elif expected == "nan":
        assert metric.value.isSuccess and metric.value.get() != metric.value.get(), (source, metric)
    else:
        assert metric.value == Success(expected), (source, metric)


@pytest.mark.parametrize("case", KA["cases"], ids=[c["id"] for c in KA["cases"]])
def test_known_answer_calculate(gpu, case):
    table = product_table(KA["tables"][case["table"]])
    analyzer = product_analyzer(case["analyzer"], case["args"])
    _check(analyzer.calculate(table), case["expected"], case["source"])


def test_known_answers_in_one_fused_run_per_table(gpu):
    by_table = {}
    for c in KA["cases"]:
        by_table.setdefault(c["table"], []).append(c)
    for tname, cases in by_table.items():
        table = product_table(KA["tables"][tname])
        analyzers = [product_analyzer(c["analyzer"], c["args"]) for c in cases]
        ctx = d.AnalysisRunner.onData(table).addAnalyzers(analyzers).run()
        for a, c in zip(analyzers, cases):
            _check(ctx.metric(a), c["expected"], c["source"])


@pytest.mark.parametrize("case", KA["merge_cases"], ids=[c["id"] for c in KA["merge_cases"]])
def test_known_answer_state_merge(gpu, case):
    ta = product_table(KA["tables"][case["table_a"]])
    tb = product_table(KA["tables"][case["table_b"]])
    a = product_analyzer(case["analyzer"], case["args"])
    merged = merge(a.computeStateFrom(ta), a.computeStateFrom(tb))
    _check(a.computeMetricFrom(merged), case["expected"], case["source"])
    # two batches through one plan == the union
    _check(a.calculate(d.PartitionedTable([ta, tb])), case["expected"], case["source"])


def test_empty_state_message(gpu):
    table = product_table(KA["tables"]["dfNullColumns"])
    m = d.Mean("numericCol").calculate(table)
    assert str(m.value.exception) == (
        "Empty state for analyzer Mean(numericCol,None), all input values were NULL.")


def test_precondition_failures(gpu):
    table = product_table(KA["tables"]["dfFull"])
    assert isinstance(d.Mean("att1").calculate(table).value.exception, d.WrongColumnTypeException)
    assert isinstance(d.Completeness("someMissingColumn").calculate(table).value.exception,
                      d.NoSuchColumnException)
    assert d.Completeness("someMissingColumn").calculate(table).value.isFailure
    # MinLength / MaxLength need a string column (AnalyzerTests.scala:519-522, 537-540)
    numeric = product_table(KA["tables"]["dfNumeric"])
    for a in (d.MinLength("att1"), d.MaxLength("att1")):
        assert isinstance(a.calculate(numeric).value.exception, d.WrongColumnTypeException)
    assert isinstance(d.Correlation("item", "att1").calculate(numeric).value.exception,
                      d.WrongColumnTypeException)


def test_incremental_with_state_provider(gpu):
    """algebraic_states_example.md: persist states, then aggregate with more data."""
    store = d.InMemoryStateProvider()
    analyzers = [d.Size(), d.ApproxCountDistinct("id"), d.Completeness("productName"),
                 d.Completeness("description")]
    first = d.AnalysisRunner.onData(product_table(KA["tables"]["items"])).addAnalyzers(
        analyzers).saveStatesWith(store).run()
    assert [first.metric(a).value.get() for a in analyzers] == [3.0, 3.0, 1.0, 0.6666666666666666]
    second = d.AnalysisRunner.onData(product_table(KA["tables"]["itemsMore"])).addAnalyzers(
        analyzers).aggregateWith(store).run()
    assert [second.metric(a).value.get() for a in analyzers] == [5.0, 5.0, 1.0, 0.4]
