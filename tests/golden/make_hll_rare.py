"""Writes tests/golden/hll_rare_values.json: int64 / int32 values whose Spark XXH64 (seed 42)
lands on the rare branches of the device HLL slot (hll_slot in deequ_amd/csrc/dq_internal.h).

  rare1: bits 54..32 of the hash are zero -> the rank is not decided by the hash's high word;
  rare2: bits 54..23 are zero            -> the high word of w = (x << 9) | 256 is zero (pw > 32).

The values come from tests/golden/hll_rare_search.c (brute force, about 30 s single-threaded);
this script compiles and runs it with gcc and records its output.  Test-fixture generator only.
"""
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "search")
        subprocess.check_call(["gcc", "-O3", "-o", exe, os.path.join(HERE, "hll_rare_search.c")])
        out = subprocess.check_output([exe, "0", str(1 << 34)], text=True)
    rows = [line.split() for line in out.splitlines() if line.strip()]
    fixture = {
        "source": "tests/golden/hll_rare_search.c via make_hll_rare.py",
        "int64": [{"kind": k, "value": int(v)} for k, w, v in rows if w == "8"],
        "int32": [{"kind": k, "value": int(v)} for k, w, v in rows if w == "4"],
    }
    with open(os.path.join(HERE, "hll_rare_values.json"), "w") as f:
        json.dump(fixture, f, indent=1)


if __name__ == "__main__":
    main()
