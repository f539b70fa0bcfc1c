"""Host-side profile (cProfile) of one C5 / C4 / C1 bench step, to find where the wall time
between kernels goes.  Usage: python tools/prof_host.py c5|c4|c1 > gpurun_out/host_c5.txt"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import deequ_amd as d  # noqa: E402

wl = sys.argv[1]
d.set_device(0)
if wl == "c5":
    from deequ_amd.profiles import ColumnProfilerRunner
    data = bench.make_c5_table(100_000_000, 0, 0)

    def step():
        return ColumnProfilerRunner().onData(data).run()
elif wl == "c4":
    data = bench.make_c4_batches(1_000_000_000, 125_000_000, 201_500_000, 0, 0)
    an = [d.Uniqueness(["key"]), d.Distinctness(["key"]), d.Entropy("key"), d.CountDistinct(["key"]),
          d.Histogram("key")]

    def step():
        return d.AnalysisRunner.onData(data).addAnalyzers(an).run()
else:
    data = bench.make_c1_table(10_000_000, 0, 0)
    an = bench.c1_analyzers()

    def step():
        return d.AnalysisRunner.onData(data).addAnalyzers(an).run()

step()
torch.cuda.synchronize()
t0 = time.perf_counter()
step()
torch.cuda.synchronize()
print("unprofiled step %.2f ms" % ((time.perf_counter() - t0) * 1e3))

if os.environ.get("SPANS") == "1":  # wall-clock spans of the profiler's host stages (one step)
    import threading
    from deequ_amd import engine, profiles, runner
    spans = []

    def wrap(mod, name):
        f = getattr(mod, name)

        def g(*a, **k):
            s = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                spans.append((s, time.perf_counter(), name, threading.current_thread().name))
        setattr(mod, name, g)
    for mod, name in [(profiles, "_extract_generic_statistics"), (profiles, "_cast_numeric_string_columns"),
                      (profiles, "compute_histograms"), (profiles, "_create_profiles"),
                      (profiles, "_extract_numeric_statistics"), (profiles, "cast_string_column"),
                      (profiles, "_few_group_strings"), (profiles, "_few_group_metrics"),
                      (profiles, "cast_string_columns"),
                      (engine, "run_scan_raw"), (engine, "_scan_local"), (engine, "op_supported")]:
        wrap(mod, name)
    R = runner.AnalysisRunner
    for name in ("doAnalysisRun", "_runScanningAnalyzers"):
        f = getattr(R, name)

        def mk(f, name):
            def g(*a, **k):
                s = time.perf_counter()
                try:
                    return f(*a, **k)
                finally:
                    spans.append((s, time.perf_counter(), name, threading.current_thread().name))
            return staticmethod(g)
        setattr(R, name, mk(f, name))
    for _ in range(2):
        spans.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        print("step %.2f ms" % ((t1 - t0) * 1e3))
        agg = {}
        for s, e, n, th in spans:
            if n in ("op_supported", "cast_string_column"):
                a = agg.setdefault(n, [0, 0.0])
                a[0] += 1
                a[1] += e - s
                continue
            print("  %8.2f -> %8.2f  %7.2f ms  %-32s %s" % ((s - t0) * 1e3, (e - t0) * 1e3, (e - s) * 1e3, n, th))
        for n, (c, t) in agg.items():
            print("  %s: %d calls, %.2f ms" % (n, c, t * 1e3))
    sys.exit(0)
pr = cProfile.Profile()
pr.enable()
step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr, stream=sys.stdout)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(30)
