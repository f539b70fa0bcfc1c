"""Writes tests/golden/reference_known_answers.json.

Every entry transcribes one known answer of the REFERENCE's own test-suite or docs: the
fixture table's values (FixtureSupport.scala, NullHandlingTests.scala, examples) and the
asserted metric, with the reference file:line it comes from.  Values only -- no reference
code.  The oracle (tests/test_oracle_golden.py) and the GPU path
(tests/test_gpu_known_answers.py) are both checked against this file.

    python tests/golden/make_known_answers.py
"""
import json
import math
import os

T = "src/test/scala/com/amazon/deequ/"
M = "src/main/scala/com/amazon/deequ/"

# --------------------------------------------------------------------------- fixture tables
TABLES = {
    # FixtureSupport.getDfMissing (utils/FixtureSupport.scala:45-62)
    "dfMissing": {
        "item": ["string", ["1", "2", "3", "4", "5", "6", "7", "8", "9", "10", "11", "12"]],
        "att1": ["string", ["a", "b", None, "a", "a", None, None, "b", "a", None, None, None]],
        "att2": ["string", ["f", "d", "f", None, "f", "d", "d", None, "f", None, "f", "d"]],
    },
    # getDfFull (:64-73)
    "dfFull": {
        "item": ["string", ["1", "2", "3", "4"]],
        "att1": ["string", ["a", "a", "a", "b"]],
        "att2": ["string", ["c", "c", "c", "d"]],
    },
    # getDfWithNumericValues (:137-148) -- att1..att3 are Scala Ints (IntegerType)
    "dfNumeric": {
        "item": ["string", ["1", "2", "3", "4", "5", "6"]],
        "att1": ["int32", [1, 2, 3, 4, 5, 6]],
        "att2": ["int32", [0, 0, 0, 5, 6, 7]],
        "att3": ["int32", [0, 0, 0, 4, 6, 7]],
    },
    # getDfWithNumericFractionalValues (:150-160)
    "dfFractional": {
        "item": ["string", ["1", "2", "3", "4", "5", "6"]],
        "att1": ["float64", [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]],
        "att2": ["float64", [0.0, 0.0, 0.0, 5.0, 6.0, 7.0]],
    },
    # getDfWithUniqueColumns (:198-211) -- every column is a string
    "dfUnique": {
        "unique": ["string", ["1", "2", "3", "4", "5", "6"]],
        "nonUnique": ["string", ["0", "0", "0", "5", "6", "7"]],
        "nonUniqueWithNulls": ["string", ["3", "3", "3", None, None, None]],
        "uniqueWithNulls": ["string", ["1", "2", None, "3", "4", "5"]],
        "onlyUniqueWithOtherNonUnique": ["string", ["5", "6", "7", "0", "0", "0"]],
        "halfUniqueCombinedWithNonUnique": ["string", ["0", "0", "0", "4", "5", "6"]],
    },
    # IncrementalAnalyzerTest.initialData / deltaData (analyzers/IncrementalAnalyzerTest.scala:243-260)
    "incrInitial": {
        "item": ["string", ["1", "2", "3"]],
        "att1": ["string", ["a", None, "b"]],
        "count": ["int32", [12, 12, 12]],
    },
    "incrDelta": {
        "item": ["string", ["4", "5"]],
        "att1": ["string", ["b", None]],
        "count": ["int32", [12, 12]],
    },
    # NullHandlingTests.dataWithNullColumns (analyzers/NullHandlingTests.scala:32-53)
    "dfNullColumns": {
        "stringCol": ["string", [None] * 8],
        "numericCol": ["float64", [None] * 8],
        "numericCol2": ["float64", [None] * 8],
        "numericCol3": ["float64", [1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0]],
    },
    # examples/algebraic_states_example.md:10-14 (Item rows) and :55-58 (more data)
    "items": {
        "id": ["int64", [1, 2, 3]],
        "productName": ["string", ["Thingy A", "Thingy B", "Thing C"]],
        "description": ["string", ["awesome thing.", "available tomorrow", None]],
        "priority": ["string", ["high", "low", None]],
        "numViews": ["int64", [0, 0, 5]],
    },
    "itemsMore": {
        "id": ["int64", [4, 5]],
        "productName": ["string", ["Thingy D", "Thingy E"]],
        "description": ["string", [None, None]],
        "priority": ["string", ["low", "high"]],
        "numViews": ["int64", [10, 12]],
    },
    # getDfWithConditionallyUninformativeColumns (:226-233)
    "dfUninformative": {
        "att1": ["int32", [1, 2, 3]],
        "att2": ["int32", [0, 0, 0]],
    },
    # getDfWithConditionallyInformativeColumns (:235-242)
    "dfInformative": {
        "att1": ["int32", [1, 2, 3]],
        "att2": ["int32", [4, 5, 6]],
    },
    # getDfWithVariableStringLengthValues (:259-268)
    "dfStringLengths": {"att1": ["string", ["", "a", "bb", "ccc", "dddd"]]},
    # getDfEmpty (:26-33)
    "dfEmpty": {"column1": ["string", []], "column2": ["string", []]},
    # ---- DataType fixtures (AnalyzerTests.scala:294-420)
    "dfNegative": {  # getDfWithNegativeNumbers (:75-84)
        "item": ["string", ["1", "2", "3", "4"]],
        "att1": ["string", ["-1", "-2", "-3", "-4"]],
        "att2": ["string", ["-1.0", "-2.0", "-3.0", "-4.0"]],
    },
    "dfFracInt": {"item": ["string", ["1", "2"]], "att1": ["string", ["1.0", "1"]]},  # :110-117
    "dfFracStr": {"item": ["string", ["1", "2"]], "att1": ["string", ["1.0", "a"]]},  # :119-126
    "dfIntStr": {"item": ["string", ["1", "2"]], "att1": ["string", ["1", "a"]]},  # :128-135
    # getDfWithNumericValues.att1 cast to FloatType / StringType (AnalyzerTests.scala:321-334)
    "dfNumericCasts": {
        "att1_float": ["float32", [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]],
        "att1_str": ["string", ["1", "2", "3", "4", "5", "6"]],
    },
    # getDfWithNumericFractionalValues.att1 cast to StringType (:336-343)
    "dfFractionalStr": {"att1_str": ["string", ["1.0", "2.0", "3.0", "4.0", "5.0", "6.0"]]},
    "dfBool": {"item": ["string", ["1", "2"]], "att1": ["string", ["true", "false"]]},  # :392-402
    "dfBoolNull": {"item": ["string", ["1", "2", "3", "4"]],  # :404-420
                   "att1": ["string", ["true", "false", None, "2.0"]]},
    # ---- ColumnProfiler fixtures (profiles/ColumnProfilerTest.scala)
    # getDfCompleteAndInCompleteColumns (utils/FixtureSupport.scala:86-97)
    "dfCompleteIncomplete": {
        "item": ["string", ["1", "2", "3", "4", "5", "6"]],
        "att1": ["string", ["a", "b", "a", "a", "b", "a"]],
        "att2": ["string", ["f", "d", None, "f", None, "f"]],
    },
    "profBool": {"attribute": ["bool", [True, True, True, False, False, None]]},  # :228-253
    "profInt": {"attribute": ["int32", [2147483647, 2147483647, 2147483647, 2, 2, None]]},  # :255-280
    "profLong": {"attribute": ["int64", [1, 1, 1, 2, 2, None]]},  # :282-307
    "profDouble": {"attribute": ["float64", [1.0, 1.0, 1.0, 2.0, 2.0, None]]},  # :309-334
    "profFloat": {"attribute": ["float32", [1.0, 1.0, 1.0, 2.0, 2.0, None]]},  # :336-361
    "profShort": {"attribute": ["int16", [1, 1, 1, 2, 2, None]]},  # :363-400
}

A = "analyzers/AnalyzerTests.scala"
C = "checks/CheckTest.scala"
EMPTY = "empty"  # the metric is a Failure(EmptyStateException)
H_FULL = -(0.75 * math.log(0.75) + 0.25 * math.log(0.25))  # AnalyzerTests.scala:135-136
NH = T + "analyzers/NullHandlingTests.scala"
INC = T + "analyzers/IncrementalAnalyzerTest.scala"

CASES = [
    # (id, table, analyzer, args, expected, source)
    ("size_missing", "dfMissing", "Size", [], 12.0, T + A + ":36-37"),
    ("size_full", "dfFull", "Size", [], 4.0, T + A + ":38-39"),
    ("completeness_att1", "dfMissing", "Completeness", ["att1"], 0.5, T + A + ":48-49"),
    ("completeness_att2", "dfMissing", "Completeness", ["att2"], 0.75, T + A + ":50-51"),
    ("completeness_where", "dfMissing", "Completeness", ["att1", "item IN ('1', '2')"], 1.0, T + A + ":68-72"),
    ("compliance_gt3", "dfNumeric", "Compliance", ["rule1", "att1 > 3"], 3.0 / 6, T + A + ":173-174"),
    ("compliance_gt2", "dfNumeric", "Compliance", ["rule2", "att1 > 2"], 4.0 / 6, T + A + ":175-176"),
    ("compliance_where", "dfNumeric", "Compliance", ["rule1", "att2 = 0", "att1 < 4"], 1.0, T + A + ":180-184"),
    ("mean", "dfNumeric", "Mean", ["att1"], 3.5, T + A + ":424-428"),
    ("mean_where", "dfNumeric", "Mean", ["att1", "item != '6'"], 3.0, T + A + ":434-438"),
    ("stddev", "dfNumeric", "StandardDeviation", ["att1"], 1.707825127659933, T + A + ":440-444"),
    ("minimum", "dfNumeric", "Minimum", ["att1"], 1.0, T + A + ":450-454"),
    ("maximum", "dfNumeric", "Maximum", ["att1"], 6.0, T + A + ":460-464"),
    ("maximum_where", "dfNumeric", "Maximum", ["att1", "item != '6'"], 5.0, T + A + ":466-471"),
    ("sum", "dfNumeric", "Sum", ["att1"], 21.0, T + A + ":478-481"),
    ("acd_strings", "dfUnique", "ApproxCountDistinct", ["uniqueWithNulls"], 5.0, T + A + ":543-548"),
    ("acd_int", "dfNumeric", "ApproxCountDistinct", ["att1"], 6.0, T + "analyzers/AnalysisTest.scala:91-92"),
    ("stddev_analysis", "dfNumeric", "StandardDeviation", ["att1"], 1.707825127659933, T + "analyzers/AnalysisTest.scala:87-88"),
    ("frac_mean", "dfFractional", "Mean", ["att1"], 3.5, T + "checks/CheckTest.scala:427-431 (same values)"),
    ("frac_stddev", "dfFractional", "StandardDeviation", ["att1"], 1.707825127659933, T + "checks/CheckTest.scala:429"),
    ("null_size", "dfNullColumns", "Size", [], 8.0, T + "analyzers/NullHandlingTests.scala:60,99"),
    ("null_completeness", "dfNullColumns", "Completeness", ["stringCol"], 0.0, T + "analyzers/NullHandlingTests.scala:61,100"),
    ("null_mean", "dfNullColumns", "Mean", ["numericCol"], EMPTY, T + "analyzers/NullHandlingTests.scala:63,102"),
    ("null_stddev", "dfNullColumns", "StandardDeviation", ["numericCol"], EMPTY, T + "analyzers/NullHandlingTests.scala:64,104"),
    ("null_min", "dfNullColumns", "Minimum", ["numericCol"], EMPTY, T + "analyzers/NullHandlingTests.scala:65,105"),
    ("null_max", "dfNullColumns", "Maximum", ["numericCol"], EMPTY, T + "analyzers/NullHandlingTests.scala:66,106"),
    ("null_sum", "dfNullColumns", "Sum", ["numericCol"], EMPTY, T + "analyzers/NullHandlingTests.scala:74,113"),
    ("null_acd", "dfNullColumns", "ApproxCountDistinct", ["stringCol"], 0.0, T + "analyzers/NullHandlingTests.scala:119"),
    ("items_size", "items", "Size", [], 3.0, M + "examples/algebraic_states_example.md:45-52"),
    ("items_acd", "items", "ApproxCountDistinct", ["id"], 3.0, M + "examples/algebraic_states_example.md:49"),
    ("items_completeness_name", "items", "Completeness", ["productName"], 1.0, M + "examples/algebraic_states_example.md:50"),
    ("items_completeness_desc", "items", "Completeness", ["description"], 0.6666666666666666, M + "examples/algebraic_states_example.md:51"),
    ("incr_size_initial", "incrInitial", "Size", [], 3.0, T + "analyzers/IncrementalAnalyzerTest.scala:45"),
    ("incr_size_delta", "incrDelta", "Size", [], 2.0, T + "analyzers/IncrementalAnalyzerTest.scala:46"),
    ("incr_compliance_initial", "incrInitial", "Compliance", ["att1", "att1 = 'b'"], 0.3333333333333333, T + "analyzers/IncrementalAnalyzerTest.scala:73"),
    ("incr_compliance_delta", "incrDelta", "Compliance", ["att1", "att1 = 'b'"], 0.5, T + "analyzers/IncrementalAnalyzerTest.scala:74"),
    ("incr_completeness_initial", "incrInitial", "Completeness", ["att1"], 0.6666666666666666, T + "analyzers/IncrementalAnalyzerTest.scala:92"),
    ("incr_completeness_delta", "incrDelta", "Completeness", ["att1"], 0.5, T + "analyzers/IncrementalAnalyzerTest.scala:93"),
    ("empty_size", "dfEmpty", "Size", [], 0.0, T + "analyzers/runners/AnalysisRunnerTests.scala (Size of an empty frame is 0)"),
    ("empty_completeness", "dfEmpty", "Completeness", ["column1"], EMPTY, T + "analyzers/NullHandlingTests.scala (sum over zero rows is NULL)"),
    # ---- frequency family (GroupingAnalyzers.scala and the analyzers built on it)
    ("uniq_missing_att1", "dfMissing", "Uniqueness", [["att1"]], 0.0, T + A + ":83-84"),
    ("uniq_missing_att2", "dfMissing", "Uniqueness", [["att2"]], 0.0, T + A + ":85-86"),
    ("uniq_full_att1", "dfFull", "Uniqueness", [["att1"]], 0.25, T + A + ":89-90"),
    ("uniq_full_att2", "dfFull", "Uniqueness", [["att2"]], 0.25, T + A + ":91-92"),
    ("uniq_unique", "dfUnique", "Uniqueness", [["unique"]], 1.0, T + A + ":98-99"),
    ("uniq_unique_with_nulls", "dfUnique", "Uniqueness", [["uniqueWithNulls"]], 5 / 6.0, T + A + ":100-101"),
    ("uniq_multi_unique_nonunique", "dfUnique", "Uniqueness", [["unique", "nonUnique"]], 1.0, T + A + ":102-103"),
    ("uniq_multi_with_nulls", "dfUnique", "Uniqueness", [["unique", "nonUniqueWithNulls"]], 3 / 6.0, T + A + ":104-106"),
    ("uniq_multi_only_unique", "dfUnique", "Uniqueness", [["nonUnique", "onlyUniqueWithOtherNonUnique"]], 1.0, T + A + ":107-109"),
    ("entropy_att1", "dfFull", "Entropy", ["att1"], H_FULL, T + A + ":133-136"),
    ("entropy_att2", "dfFull", "Entropy", ["att2"], H_FULL, T + A + ":137-139"),
    ("mi_full", "dfFull", "MutualInformation", [["att1", "att2"]], H_FULL, T + A + ":148-152"),
    ("mi_uninformative", "dfUninformative", "MutualInformation", [["att1", "att2"]], 0.0, T + A + ":154-157"),
    ("mi_same_column", "dfFull", "MutualInformation", [["att1", "att1"]], H_FULL, T + A + ":159-168 (== Entropy(att1))"),
    ("countdistinct_unique_with_nulls", "dfUnique", "CountDistinct", [["uniqueWithNulls"]], 5.0, T + A + ":560-565"),
    ("countdistinct_att1", "dfNumeric", "CountDistinct", [["att1"]], 6.0, T + "analyzers/AnalysisTest.scala:80,93-94"),
    ("distinctness_item", "dfFull", "Distinctness", [["item"]], 1.0, T + "analyzers/AnalysisTest.scala:38,49"),
    ("uniq_full_multi", "dfFull", "Uniqueness", [["att1", "att2"]], 0.25, T + "analyzers/AnalysisTest.scala:40,51"),
    ("distinctness_att1", "dfFull", "Distinctness", [["att1"]], 0.5, T + "repository/AnalysisResultSerdeTest.scala:202,229-230"),
    ("null_countdistinct", "dfNullColumns", "CountDistinct", [["stringCol"]], 0.0, NH + ":117"),
    ("null_entropy", "dfNullColumns", "Entropy", ["stringCol"], EMPTY, NH + ":121"),
    ("null_mi", "dfNullColumns", "MutualInformation", [["numericCol", "numericCol2"]], EMPTY, NH + ":122"),
    ("null_mi3", "dfNullColumns", "MutualInformation", [["numericCol", "numericCol3"]], EMPTY, NH + ":123"),
    ("incr_uniq_initial", "incrInitial", "Uniqueness", [["att1"]], 0.6666666666666666, INC + ":121"),
    ("incr_uniq_delta", "incrDelta", "Uniqueness", [["att1"]], 0.5, INC + ":122"),
    ("incr_uniq_multi_initial", "incrInitial", "Uniqueness", [["att1", "count"]], 0.6666666666666666, INC + ":143"),
    ("incr_uniq_multi_delta", "incrDelta", "Uniqueness", [["att1", "count"]], 0.5, INC + ":144"),
    # Histogram: expected = number of bins + the reported keys (or only their number)
    ("hist_missing", "dfMissing", "Histogram", ["att1"], {"bins": 3, "keys": ["NullValue", "a", "b"]}, T + A + ":203-215"),
    ("hist_numeric", "dfNumeric", "Histogram", ["att2"], {"bins": 4, "n_values": 4}, T + A + ":217-227"),
    ("hist_top2", "dfMissing", "Histogram", ["att1", None, 2], {"bins": 3, "keys": ["NullValue", "a"]}, T + A + ":249-261"),
    # MinLength / MaxLength (AnalyzerTests.scala:506-540, CheckTest.scala:443-452)
    ("minlength_att1", "dfStringLengths", "MinLength", ["att1"], 0.0, T + A + ":506-510"),
    ("minlength_where", "dfStringLengths", "MinLength", ["att1", "att1 != ''"], 1.0, T + A + ":512-517"),
    ("maxlength_att1", "dfStringLengths", "MaxLength", ["att1"], 4.0, T + A + ":524-528"),
    ("maxlength_where", "dfStringLengths", "MaxLength", ["att1", "att1 != 'dddd'"], 3.0, T + A + ":530-535"),
    ("null_minlength", "dfNullColumns", "MinLength", ["stringCol"], EMPTY, NH + ":69,109"),
    ("null_maxlength", "dfNullColumns", "MaxLength", ["stringCol"], EMPTY, NH + ":70,110"),
    # Correlation (AnalyzerTests.scala:637-655, CheckTest.scala:433-440): "nan" = Double.NaN
    ("corr_uninformative", "dfUninformative", "Correlation", ["att1", "att2"], "nan", T + A + ":637-642"),
    ("corr_informative", "dfInformative", "Correlation", ["att1", "att2"], 1.0, T + A + ":643-650"),
    ("corr_commutative", "dfInformative", "Correlation", ["att2", "att1"], 1.0, T + A + ":651-654"),
    ("null_corr", "dfNullColumns", "Correlation", ["numericCol", "numericCol2"], EMPTY, NH + ":93,124"),
    ("null_corr3", "dfNullColumns", "Correlation", ["numericCol", "numericCol3"], EMPTY, NH + ":125"),
    # ApproxCountDistinct with a `where` filter: `unique < 4` on a STRING column is Spark's
    # implicit string -> double cast (PromoteStrings); the GPU path evaluates it on the device
    ("acd_where_string_cast", "dfUnique", "ApproxCountDistinct", ["uniqueWithNulls", "unique < 4"], 2.0, T + A + ":551-558"),
    # where-filtered checks (CheckTest.scala:174-290): the Compliance analyzers their checks build
    # (Check.satisfies / isLessThan... -> Constraint.complianceConstraint, Constraint.scala:265-279)
    # and the metric each check's assertion pins: the default `_ == 1.0` or the custom `_ == 0.5`
    ("check_satisfies_where", "dfNumeric", "Compliance", ["rule1", "att1 < att2", "att1 > 3"], 1.0, T + C + ":174-190"),
    ("check_satisfies_where_half", "dfNumeric", "Compliance", ["rule3", "att2 > 0", "att1 > 0"], 0.5, T + C + ":180-190"),
    ("check_lt", "dfNumeric", "Compliance", ["att1 is less than att2", "att1 < att2"], 0.5, T + C + ":192-211"),
    ("check_le", "dfNumeric", "Compliance", ["att1 is less than or equal to att3", "att1 <= att3"], 0.5, T + C + ":213-234"),
    ("check_gt", "dfNumeric", "Compliance", ["att2 is greater than att1", "att2 > att1"], 0.5, T + C + ":236-255"),
    ("check_ge", "dfNumeric", "Compliance", ["att3 is greater than or equal to att1", "att3 >= att1"], 0.5, T + C + ":257-278"),
    ("check_lt_where_item", "dfNumeric", "Compliance", ["att1 is less than att2", "att1 < att2", "item > 3"], 1.0, T + C + ":193-194,207 (where on the string column item)"),
    ("check_le_where_item", "dfNumeric", "Compliance", ["att1 is less than or equal to att3", "att1 <= att3", "item > 3"], 1.0, T + C + ":215-216,229"),
    ("check_gt_where_item", "dfNumeric", "Compliance", ["att2 is greater than att1", "att2 > att1", "item > 3"], 1.0, T + C + ":238-239,251"),
    ("check_ge_where_item", "dfNumeric", "Compliance", ["att3 is greater than or equal to att1", "att3 >= att1", "item > 3"], 1.0, T + C + ":260-261,273"),
    # FilterableCheckTest.scala:31-34 (plumbing only: the analyzers a filtered check builds)
    ("filterable_completeness_where", "dfMissing", "Completeness", ["att1", "item = '1'"], 1.0, T + "checks/FilterableCheckTest.scala:31-34 (Completeness with where)"),
]

# Known answers that need the union of two tables (state merge == union):
MERGE_CASES = [
    # (id, table_a, table_b, analyzer, args, expected, source)
    ("items_merge_size", "items", "itemsMore", "Size", [], 5.0, M + "examples/algebraic_states_example.md:74-80"),
    ("items_merge_acd", "items", "itemsMore", "ApproxCountDistinct", ["id"], 5.0, M + "examples/algebraic_states_example.md:76"),
    ("items_merge_name", "items", "itemsMore", "Completeness", ["productName"], 1.0, M + "examples/algebraic_states_example.md:77"),
    ("items_merge_desc", "items", "itemsMore", "Completeness", ["description"], 0.4, M + "examples/algebraic_states_example.md:78"),
    ("incr_size_merged", "incrInitial", "incrDelta", "Size", [], 5.0, T + "analyzers/IncrementalAnalyzerTest.scala:47"),
    ("incr_compliance_merged", "incrInitial", "incrDelta", "Compliance", ["att1", "att1 = 'b'"], 0.4, T + "analyzers/IncrementalAnalyzerTest.scala:75"),
    ("incr_completeness_merged", "incrInitial", "incrDelta", "Completeness", ["att1"], 0.6, T + "analyzers/IncrementalAnalyzerTest.scala:94"),
    ("incr_uniq_merged", "incrInitial", "incrDelta", "Uniqueness", [["att1"]], 0.2, INC + ":123"),
    ("incr_uniq_multi_merged", "incrInitial", "incrDelta", "Uniqueness", [["att1", "count"]], 0.2, INC + ":145"),
]


# DataType known answers: expected DataTypeHistogram (numNull, numFractional, numIntegral,
# numBoolean, numString) -- the distribution's absolute counts
DT = "analyzers/AnalyzerTests.scala"
DATATYPE_CASES = [
    ("dt_string_fallback", "dfFull", "att1", [0, 0, 0, 0, 4], T + DT + ":294-299"),
    ("dt_integral", "dfNumeric", "att1", [0, 0, 6, 0, 0], T + DT + ":301-305"),
    ("dt_integral_negative", "dfNegative", "att1", [0, 0, 4, 0, 0], T + DT + ":307-311"),
    ("dt_fractional_negative", "dfNegative", "att2", [0, 4, 0, 0, 0], T + DT + ":313-318"),
    ("dt_fractional_float", "dfNumericCasts", "att1_float", [0, 6, 0, 0, 0], T + DT + ":321-327"),
    ("dt_integral_string", "dfNumericCasts", "att1_str", [0, 0, 6, 0, 0], T + DT + ":329-334"),
    ("dt_fractional_string", "dfFractionalStr", "att1_str", [0, 6, 0, 0, 0], T + DT + ":336-343"),
    ("dt_frac_and_int", "dfFracInt", "att1", [0, 1, 1, 0, 0], T + DT + ":352-360"),
    ("dt_frac_and_string", "dfFracStr", "att1", [0, 1, 0, 0, 1], T + DT + ":362-370"),
    ("dt_int_and_string", "dfIntStr", "att1", [0, 0, 1, 0, 1], T + DT + ":372-380"),
    ("dt_numeric_and_null", "dfUnique", "uniqueWithNulls", [1, 0, 5, 0, 0], T + DT + ":382-390"),
    ("dt_boolean", "dfBool", "att1", [0, 0, 0, 2, 0], T + DT + ":392-402"),
    ("dt_boolean_null_frac", "dfBoolNull", "att1", [1, 1, 0, 2, 0], T + DT + ":404-420"),
    ("dt_all_null", "dfNullColumns", "stringCol", [8, 0, 0, 0, 0], NH + ":72-73,112-113"),
]

# ColumnProfiler known answers (profiles/ColumnProfilerTest.scala).  `expect` holds only the
# fields the reference test asserts; dataType ids: 0 Unknown 1 Fractional 2 Integral 3 Boolean 4 String.
PT = T + "profiles/ColumnProfilerTest.scala"
_ATT2_COUNTS = {"Boolean": 0, "Fractional": 0, "Integral": 0, "Unknown": 2, "String": 4}
PROFILE_CASES = [
    ("prof_standard", "dfCompleteIncomplete", ["att2"], 1, {}, "att2",
     dict(kind="standard", completeness=2.0 / 3.0, approx=2, dataType=4, inferred=True,
          typeCounts=_ATT2_COUNTS, histogram=None), PT + ":52-76"),
    ("prof_predefined_type", "dfCompleteIncomplete", ["item"], 1, {"item": 4}, "item",
     dict(kind="standard", completeness=1.0, approx=6, dataType=4, inferred=False, typeCounts={},
          histogram=None), PT + ":78-97"),
    ("prof_other_predefined", "dfCompleteIncomplete", ["att2"], 1, {"item": 4}, "att2",
     dict(kind="standard", completeness=2.0 / 3.0, approx=2, dataType=4, inferred=True,
          typeCounts=_ATT2_COUNTS, histogram=None), PT + ":99-121"),
    ("prof_numeric_string", "dfCompleteIncomplete", ["item"], 1, {}, "item",
     dict(kind="numeric", completeness=1.0, approx=6, dataType=2, inferred=True,
          typeCounts={"Boolean": 0, "Fractional": 0, "Integral": 6, "Unknown": 0, "String": 0},
          histogram=None, mean=3.5, maximum=6.0, minimum=1.0, sum=21.0, stdDev=1.707825127659933),
     PT + ":124-159"),
    ("prof_numeric", "dfFractional", ["att1"], 1, {}, "att1",
     dict(kind="numeric", completeness=1.0, approx=6, dataType=1, inferred=False, typeCounts={},
          histogram=None, mean=3.5, maximum=6.0, minimum=1.0, sum=21.0, stdDev=1.707825127659933),
     PT + ":162-196"),
    ("prof_string_histogram", "dfCompleteIncomplete", ["att2"], 10, {}, "att2",
     dict(kind="standard", completeness=2.0 / 3.0, approx=2, dataType=4, inferred=True,
          typeCounts=_ATT2_COUNTS,
          histogram={"bins": 3, "values": {"d": [1, 0.16666666666666666], "f": [3, 0.5],
                                           "NullValue": [2, 0.3333333333333333]}}), PT + ":200-226"),
] + [
    ("prof_hist_" + name, table, None, 120, {}, "attribute",
     dict(histogram_values={k: [c, c / 6.0] for k, c in vals.items()}), PT + lines)
    for name, table, vals, lines in (
        ("boolean", "profBool", {"true": 3, "false": 2, "NullValue": 1}, ":228-253"),
        ("int", "profInt", {"2147483647": 3, "2": 2, "NullValue": 1}, ":255-280"),
        ("long", "profLong", {"1": 3, "2": 2, "NullValue": 1}, ":282-307"),
        ("double", "profDouble", {"1.0": 3, "2.0": 2, "NullValue": 1}, ":309-334"),
        ("float", "profFloat", {"1.0": 3, "2.0": 2, "NullValue": 1}, ":336-361"),
        ("short", "profShort", {"1": 3, "2": 2, "NullValue": 1}, ":363-400"))
]


def main():
    # the Completeness(att2) initial case is the reference's own 4/6 computed on att2
    out = {
        "tables": TABLES,
        "cases": [dict(id=c[0], table=c[1], analyzer=c[2], args=c[3], expected=c[4], source=c[5])
                  for c in CASES],
        "merge_cases": [dict(id=c[0], table_a=c[1], table_b=c[2], analyzer=c[3], args=c[4],
                             expected=c[5], source=c[6]) for c in MERGE_CASES],
        "datatype_cases": [dict(id=c[0], table=c[1], column=c[2], expected=c[3], source=c[4])
                           for c in DATATYPE_CASES],
        "profile_cases": [dict(id=c[0], table=c[1], restrict=c[2], threshold=c[3], predefined=c[4],
                               column=c[5], expect=c[6], source=c[7]) for c in PROFILE_CASES],
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_known_answers.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=False)
    print("wrote", path, len(CASES), "cases +", len(MERGE_CASES), "merge cases")


if __name__ == "__main__":
    main()
