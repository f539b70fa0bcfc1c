import sys, os
sys.path.insert(0, os.getcwd())
import deequ_amd as d
from deequ_amd.profiles import cast_string_column
d.set_device(0)
for vals in (["1e3"], ["1E-3"], ["2e1", "1e3", "3.5e2"], ["1.5", "1e3"], ["10e0"], ["1e+3"], ["1.0e22"]):
    try:
        print(vals, cast_string_column(d.Column.from_pylist(vals, "string"), "float64").to_pylist())
    except Exception as e:
        print(vals, "ERR", e)
