"""Benchmark: analyzer-suite scan, 1B rows x 8 numeric columns per GPU (BASELINE.json config 2).

Workload: per rank 1e9 rows x 8 columns, Bernoulli(0.05) NULLs per
column; i0..i3 int64 uniform in [-2^30, 2^32), f0,f1 fp64 uniform in [0, 1e6), f2,f3 fp64
N(1e3, 1e2).  Analyzers (65, the north star's "full scan-shareable + HLL suite"): Size + per
column Completeness, Compliance (c >= 0 for ints, c > 5e5 / c > 1e3 for floats), Sum, Mean,
StandardDeviation, Minimum, Maximum, ApproxCountDistinct -- all in ONE fused pass per step
(every column is read once), as AnalysisRunner.runScanningAnalyzers fuses them.

A step = reset the plan, scan the device-resident batch (the fused gfx950 kernels), pull the
65 states to the host and -- on N > 1 GPUs -- all-gather them over RCCL and merge them in rank
order (State.sum), i.e. the whole job including the final merge.  Inputs are resident in HBM
before timing starts.  Weak scaling: every rank owns its own 1e9-row shard.

Prints ONE JSON line (rank 0) with `roofline` (fused scan pass vs the 8 TB/s HBM peak, timed
with HIP events on the plan's stream) and `cpu_baseline` (the oracle's C restatement of the
same Spark semantics on a bounded sample, on the host cores; rank 0, N = 1 only).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)
BYTES_PER_ROW = 8 * (8 + 1.0 / 8)  # 8 columns x (8 B value + 1 validity bit) = 65 B


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="process-group backend for N > 1: nccl (= RCCL over xGMI, the measured path) or gloo "
                        "(host collectives: the multi-rank path rehearsed on a one-GPU box, ranks sharing cuda:0)")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=int, default=1_000_000_000, help="rows per GPU")
    p.add_argument("--cpu-sample-rows", type=int, default=256_000_000)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="0 = every CPU this process may use (sched_getaffinity, capped by OMP_NUM_THREADS: "
                        "the GPU box's host share for one GPU)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--e2e-batch-rows", type=int, default=62_500_000,
                   help="host-resident C2 batch streamed to 1e9 rows for the PCIe-inclusive rate (0 = skip)")
    p.add_argument("--no-side-passes", action="store_true",
                   help="skip the scan_without_hll pass (profiler runs: the kernel trace then "
                        "holds only the headline launches)")
    p.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4", "c5"],
                   help="c2 = the headline scan (default); c3 = HLL on 64 columns; c4 = group-by")
    p.add_argument("--c1-rows", type=int, default=10_000_000, help="rows per GPU")
    p.add_argument("--c3-columns", type=int, default=64)
    p.add_argument("--c3-type", default="int64", choices=["int64", "utf8"],
                   help="C3 main run (int64) or its string variant (16-char lowercase hex of a u64)")
    p.add_argument("--c3-rows", type=int, default=125_000_000, help="rows per GPU (one batch)")
    p.add_argument("--c3-batches", type=int, default=1,
                   help="> 1: also run the whole C3 job, one plan over this many batches (8 = 1e9 rows)")
    p.add_argument("--c3-verify", action="store_true",
                   help="with --c3-batches: column 0's registers of the whole job against the oracle (untimed)")
    p.add_argument("--c4-rows", type=int, default=1_000_000_000, help="rows per GPU")
    p.add_argument("--c4-batch", type=int, default=125_000_000, help="rows per string batch")
    p.add_argument("--c4-distinct", type=int, default=201_500_000)
    p.add_argument("--c4-keys", default="digits", choices=["digits", "alnum", "uuid", "pair", "pair64"],
                   help="C4 key text: 12 decimal digits (packs into one word: 8-byte records), 'k' + 11 "
                        "digits (not a digit string: the 16-byte record path, after the packed staging gives up), "
                        "uuid (36-character UUID text of the same ids: 128-bit records, isPrimaryKey's "
                        "shape), pair (a two-column key (int64 id / 1000, 8-digit id % 1000): 20 encoded "
                        "bytes, the hashed record path; Uniqueness / Distinctness / UniqueValueRatio / "
                        "CountDistinct of the pair) or pair64 (the same pair as (int64, int64): 16 encoded "
                        "bytes, the 16-byte-key records)")
    p.add_argument("--c4-verify", action="store_true",
                   help="after timing, check the C4 metrics against torch.unique over the integer ids on the "
                        "device (an independent sort-based group-by; 1 rank); adds `verify` to the line")
    p.add_argument("--c5-rows", type=int, default=100_000_000, help="rows per GPU")
    return p.parse_args()


def make_c2_table(rows: int, rank: int, device: int):
    """Synthetic C2 batch generated directly in HBM (chunked to bound temporaries)."""
    import torch
    import deequ_amd as d

    dev = torch.device("cuda", device)
    gen = torch.Generator(device=dev)
    chunk = 1 << 26
    shifts = (2 ** torch.arange(8, device=dev, dtype=torch.int32)).to(torch.int32)
    cols = {}
    for k in range(8):
        name = ("i%d" % k) if k < 4 else ("f%d" % (k - 4))
        gen.manual_seed(42 + 1000 * rank + k)
        if k < 4:
            vals = torch.empty(rows, dtype=torch.int64, device=dev)
        else:
            vals = torch.empty(rows, dtype=torch.float64, device=dev)
        nbytes = (rows + 7) // 8
        valid = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
        for s in range(0, rows, chunk):
            e = min(rows, s + chunk)
            m = e - s
            if k < 4:
                vals[s:e] = torch.randint(-2 ** 30, 2 ** 32, (m,), generator=gen, device=dev, dtype=torch.int64)
            elif k < 6:
                vals[s:e] = torch.rand(m, generator=gen, device=dev, dtype=torch.float64) * 1e6
            else:
                vals[s:e] = torch.randn(m, generator=gen, device=dev, dtype=torch.float64) * 1e2 + 1e3
            bits = (torch.rand(m, generator=gen, device=dev) >= 0.05)
            pad = (-m) % 8
            if pad:
                bits = torch.cat([bits, torch.zeros(pad, dtype=torch.bool, device=dev)])
            packed = (bits.view(-1, 8).to(torch.int32) * shifts).sum(1).to(torch.uint8)
            valid[s // 8: s // 8 + packed.numel()] = packed
        dtype = "int64" if k < 4 else "float64"
        cols[name] = d.Column(dtype, rows, vals, valid, device=True)
    torch.cuda.synchronize(dev)
    return d.Table(cols)


def c2_analyzers():
    import deequ_amd as d
    out = [d.Size()]
    preds = {"i0": "i0 >= 0", "i1": "i1 >= 0", "i2": "i2 >= 0", "i3": "i3 >= 0",
             "f0": "f0 > 5e5", "f1": "f1 > 5e5", "f2": "f2 > 1e3", "f3": "f3 > 1e3"}
    for c in ["i0", "i1", "i2", "i3", "f0", "f1", "f2", "f3"]:
        out += [d.Completeness(c), d.Compliance("%s_rule" % c, preds[c]), d.Sum(c), d.Mean(c),
                d.StandardDeviation(c), d.Minimum(c), d.Maximum(c), d.ApproxCountDistinct(c)]
    return out


def scan_without_hll(table, device: int, steps: int):
    """The same fused pass without the 8 ApproxCountDistinct (57 analyzers), on the same table:
    the HBM-bound side of the kernel next to the headline's VALU-bound one.
    Reported beside the headline, never as `value`."""
    import torch
    import deequ_amd as d
    from deequ_amd.engine import Plan, op_spec_for
    analyzers = [a for a in c2_analyzers() if not isinstance(a, d.ApproxCountDistinct)]
    plan = Plan([op_spec_for(a, table.schema) for a in analyzers], table.schema, device=device)
    stream = torch.cuda.ExternalStream(plan.stream, device=torch.device("cuda", device))
    try:
        ms = []
        for k in range(steps + 1):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            plan.reset()
            ev[0].record(stream)
            plan.consume(table)
            ev[1].record(stream)
            plan.finish_raw()
            if k:  # the first pass warms up
                ms.append(ev[0].elapsed_time(ev[1]))
    finally:
        plan.close()
    kernel_ms = sum(ms) / len(ms)
    achieved = BYTES_PER_ROW * table.num_rows / (kernel_ms * 1e-3) / 1e9
    return {"analyzers": len(analyzers), "kernel_ms": kernel_ms, "achieved": achieved,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS}


def host_ingest(args, device: int):
    """The JNI path's rate: the C2 suite over 1e9 rows that start in HOST memory -- one host batch
    of `e2e_batch_rows` x 8 columns (Arrow layout, 5% NULL) consumed repeatedly through
    dq_plan_consume, whose copies into the two HBM staging slots overlap the previous batch's scan.
    Timed once with pageable buffers and once with the same buffers page-locked
    (dq_host_register).  Reported beside the headline, never as `value` (PCIe-bound, not HBM)."""
    import numpy as np
    import torch
    import deequ_amd as d
    from deequ_amd import _lib
    from deequ_amd.engine import Plan, op_spec_for
    rows = args.e2e_batch_rows
    reps = max(1, (args.rows + rows - 1) // rows)
    rng = np.random.default_rng(42)
    cols = {}
    for k in range(8):
        name = ("i%d" % k) if k < 4 else ("f%d" % (k - 4))
        if k < 4:
            vals = rng.integers(-2 ** 30, 2 ** 32, rows, dtype=np.int64)
        elif k < 6:
            vals = rng.random(rows) * 1e6
        else:
            vals = rng.standard_normal(rows) * 1e2 + 1e3
        bits = np.packbits(rng.random(rows) >= 0.05, bitorder="little")
        cols[name] = d.Column("int64" if k < 4 else "float64", rows, vals, bits)
    table = d.Table(cols)
    analyzers = c2_analyzers()
    plan = Plan([op_spec_for(a, table.schema) for a in analyzers], table.schema, device=device)
    bufs = [b for c in cols.values() for b in (c.values, c.validity)]

    def one_pass():
        plan.reset()
        for _ in range(reps):
            plan.consume(table)
        plan.finish_raw()
    out = {"batch_rows": rows, "batches_per_pass": reps, "rows_per_pass": rows * reps,
           "bytes_per_row": BYTES_PER_ROW}
    try:
        for label in ("pageable", "pinned"):
            if label == "pinned":
                for b in bufs:
                    _lib.check(_lib.lib().dq_host_register(b.ctypes.data, b.nbytes))
            one_pass()  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            one_pass()
            secs = time.perf_counter() - t0
            out[label + "_rows_per_s"] = rows * reps / secs
            out[label + "_pcie_gbs"] = rows * reps * BYTES_PER_ROW / secs / 1e9
    finally:
        for b in bufs:
            _lib.lib().dq_host_unregister(b.ctypes.data)
        plan.close()
    return out


def host_cpu_share() -> int:
    """The host cores this run may use: the CPUs in its affinity mask, capped by OMP_NUM_THREADS
    when the launcher sets it (the GPU box sets 16 per GPU; nproc there counts the whole host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


CPU_BASELINE_SECS = 10.0  # timed CPU work of the baseline (passes over one sample until reached)


def cpu_baseline(sample_rows: int, threads: int):
    """The oracle's C restatement (Spark semantics: sequential per-partition aggregation,
    per-row Welford, partition states merged with State.sum) on `threads` host threads."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import cdq_oracle
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "rows/s", "cores": threads, "kind": "port",
                "sample": "unavailable: %s" % e}
    secs, passes = cdq_oracle.time_c2_scan(sample_rows, threads, min_secs=CPU_BASELINE_SECS)
    rows = sample_rows * passes
    return {"value": rows / secs, "unit": "rows/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "value_per_core": rows / secs / threads,
            "cores_policy": "the CPUs this process may use: affinity mask capped by OMP_NUM_THREADS (the GPU "
                            "pool gives each GPU 16 of the host's %d; os.cpu_count() counts all 8 GPUs' share)"
                            % (os.cpu_count() or 0),
            "sample": "%d passes over one %d-row x 8-col sample (C2 distributions, 5%% NULL), 65 analyzers "
                      "(8 HLL), C restatement of Spark 2.2.2 aggregation (oracle/dq_oracle.c), %d threads, "
                      "%.2f s of CPU work" % (passes, sample_rows, threads, secs)}


def all_host_baseline(sample_rows: int, share: int, share_per_core: float):
    """The same CPU baseline over every host CPU, measured only where the host really grants them.

    The calling thread's affinity mask is widened to all `os.cpu_count()` CPUs (the oracle's
    threads inherit it) and restored afterwards.  The result is reported only when the mask could
    be widened AND the per-core rate stays within 2x of the share's per-core rate; otherwise the
    field says why it is unavailable (a mask the box refuses to widen, or a cgroup CPU quota that
    time-slices the extra threads onto the share's cores: 256 threads on 16 cores measure the
    quota, not the host)."""
    nproc = os.cpu_count() or share
    if nproc <= share:
        return {"value": None, "unavailable": "the host has no CPUs beyond this run's %d" % share}
    try:
        old = os.sched_getaffinity(0)
    except AttributeError:
        return {"value": None, "unavailable": "no affinity interface"}
    try:
        os.sched_setaffinity(0, range(nproc))
        granted = len(os.sched_getaffinity(0))
    except OSError as e:
        granted = len(old)
        why = "affinity mask = %d CPUs (widening to %d refused: %s)" % (granted, nproc, e)
    else:
        why = None
    try:
        if granted <= share:
            return {"value": None, "unavailable": why or "affinity mask = %d CPUs" % granted}
        allc = cpu_baseline(sample_rows, granted)
    finally:
        os.sched_setaffinity(0, old)
    per_core = allc.get("value_per_core")
    if not per_core or per_core < 0.5 * share_per_core:
        return {"value": None, "cores_tried": granted,
                "unavailable": "mask widened to %d CPUs but they measure %.3g rows/s per core against %.3g "
                               "on the %d-CPU share: the extra threads are time-sliced (cgroup CPU quota), "
                               "so no whole-host number was measured" % (granted, per_core or 0.0,
                                                                       share_per_core, share)}
    return {"value": allc["value"], "unit": "rows/s", "cores": granted, "nproc": nproc,
            "value_per_core": per_core, "sample": allc.get("sample")}


# ----------------------------------------------------------------------------- secondary workloads
def _valid_bits(m: int, gen, dev, null_frac: float):
    import torch
    shifts = (2 ** torch.arange(8, device=dev, dtype=torch.int32)).to(torch.int32)
    bits = torch.rand(m, generator=gen, device=dev) >= null_frac
    pad = (-m) % 8
    if pad:
        bits = torch.cat([bits, torch.zeros(pad, dtype=torch.bool, device=dev)])
    return (bits.view(-1, 8).to(torch.int32) * shifts).sum(1).to(torch.uint8)


def make_c3_table(rows: int, n_cols: int, rank: int, device: int, batch: int = 0, into=None):
    """C3: int64 uniform over the 64-bit range (~all distinct), 5% NULL, HBM.
    batch > 0: the batch-th batch of the stream (other seeds), regenerated into `into`'s buffers."""
    import torch
    import deequ_amd as d
    dev = torch.device("cuda", device)
    gen = torch.Generator(device=dev)
    chunk = 1 << 26
    cols = {}
    for k in range(n_cols):
        gen.manual_seed(7000 + 1000 * rank + k + 1_000_000 * batch)
        if into is not None:
            vals, valid = into.columns["h%d" % k].values, into.columns["h%d" % k].validity
        else:
            vals = torch.empty(rows, dtype=torch.int64, device=dev)
            valid = torch.empty((rows + 7) // 8 + 64, dtype=torch.uint8, device=dev)
        for s in range(0, rows, chunk):
            e = min(rows, s + chunk)
            vals[s:e].random_(-2 ** 63, 2 ** 63 - 1, generator=gen)
            packed = _valid_bits(e - s, gen, dev, 0.05)
            valid[s // 8: s // 8 + packed.numel()] = packed
        cols["h%d" % k] = d.Column("int64", rows, vals, valid, device=True)
    torch.cuda.synchronize(dev)
    return into if into is not None else d.Table(cols)


def make_c3_string_table(rows: int, n_cols: int, rank: int, device: int):
    """C3 string variant: 16-char lowercase hex of a uniform u64, 5% NULL, as
    Arrow utf8 (int32 offsets + 16 B of chars per row)."""
    import torch
    import deequ_amd as d
    dev = torch.device("cuda", device)
    gen = torch.Generator(device=dev)
    hexd = torch.tensor(list(b"0123456789abcdef"), dtype=torch.uint8, device=dev)
    shifts = torch.arange(60, -4, -4, dtype=torch.int64, device=dev)
    chunk = 1 << 24
    cols = {}
    for k in range(n_cols):
        gen.manual_seed(9000 + 1000 * rank + k)
        chars = torch.empty(rows * 16 + 16, dtype=torch.uint8, device=dev)
        valid = torch.empty((rows + 7) // 8 + 64, dtype=torch.uint8, device=dev)
        for s in range(0, rows, chunk):
            e = min(rows, s + chunk)
            ids = torch.empty(e - s, dtype=torch.int64, device=dev).random_(-2 ** 63, 2 ** 63 - 1,
                                                                          generator=gen)
            nib = (ids[:, None] >> shifts[None, :]) & 15
            chars[s * 16: e * 16] = hexd[nib].reshape(-1)
            packed = _valid_bits(e - s, gen, dev, 0.05)
            valid[s // 8: s // 8 + packed.numel()] = packed
        offsets = torch.arange(0, 16 * (rows + 1), 16, dtype=torch.int32, device=dev)
        cols["x%d" % k] = d.Column("string", rows, chars, valid, offsets=offsets, device=True)
    torch.cuda.synchronize(dev)
    return d.Table(cols)


def c4_batch_rows(batch: int, keys_kind: str) -> int:
    """Arrow utf8 offsets are int32: one batch holds at most 2^31 - 1 bytes of chars.  36-char
    UUIDs fit 59.6M rows, so the 125M-row default is cut to 50M-row batches for them."""
    width = {"uuid": 36, "pair": 8, "pair64": 0}.get(keys_kind, 12)
    if batch * width >= 2 ** 31:
        return 50_000_000 if width * 50_000_000 < 2 ** 31 else (2 ** 31 - 1) // width
    return batch


def c4_valid_ids(rows: int, batch: int, distinct: int, rank: int, device: int):
    """The integer ids behind make_c4_batches' non-NULL keys, regenerated from the same generator
    sequence (the keys are their 12-digit decimals), concatenated on the device."""
    import torch
    dev = torch.device("cuda", device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7 + 1000 * rank)
    out = []
    for b0 in range(0, rows, batch):
        m = min(batch, rows - b0)
        sub = 1 << 24
        for s in range(0, m, sub):
            e = min(m, s + sub)
            keys = torch.randint(0, distinct, (e - s,), generator=gen, device=dev, dtype=torch.int64)
            valid = torch.rand(e - s, generator=gen, device=dev) >= 0.01  # as _valid_bits draws them
            out.append(keys[valid])
    return torch.cat(out)


def c4_verify(args, metrics, dist_metric, analyzers):
    """The C4 metrics against torch.unique(return_counts=True) over the same ids on the device:
    CountDistinct, Uniqueness, Distinctness exactly, Entropy within 1e-12 (same count-of-counts
    summation order), Histogram's NULL bin and number of bins exactly, and every detail bin's
    count plus the detail bins' count multiset (the top counts; ties at the cut are broken by key)."""
    import math
    import numpy as np
    import torch
    ids = c4_valid_ids(args.c4_rows, c4_batch_rows(args.c4_batch, args.c4_keys), args.c4_distinct, 0,
                       torch.cuda.current_device())
    n_valid = int(ids.numel())
    u, c = torch.unique(ids, sorted=True, return_counts=True)
    del ids
    n = float(args.c4_rows)
    groups, unique = int(u.numel()), int((c == 1).sum())
    hist = torch.bincount(c).cpu().tolist()
    ent = 0.0
    for k in range(1, len(hist)):  # dq_freq_api.inc summary_from_hist's order and terms
        if hist[k]:
            ent += float(hist[k]) * (-(k / n) * math.log(k / n))
    got = {str(a): v for a, v in metrics.items()}
    out = {"n_valid": n_valid, "groups": groups, "unique": unique,
           "count_distinct_ok": got[str(analyzers[3])] == float(groups),
           "uniqueness_ok": got[str(analyzers[0])] == unique / n,
           "distinctness_ok": got[str(analyzers[1])] == groups / n,
           "entropy_rel_err": abs(got[str(analyzers[2])] - ent) / ent}
    if dist_metric is None:  # pair keys: the pair's metrics only (UniqueValueRatio in place of Entropy)
        del out["entropy_rel_err"]
        out["unique_value_ratio_ok"] = got[str(analyzers[2])] == unique / groups
        out["ok"] = all(out[k] for k in out if k.endswith("_ok"))
        return out
    uh, ch = u.cpu().numpy(), c.cpu().numpy()
    vals = {k: v.absolute for k, v in dist_metric.values.items()}
    nonnull = {k: a for k, a in vals.items() if k != "NullValue"}
    # (alnum keys: 'k' + the id's last 11 digits -- the first digit of a 12-digit id below 1e11 is
    # always 0, so the map is one to one)
    idx = np.array([int(k[1:]) if args.c4_keys == "alnum" else uuid_to_id(k) if args.c4_keys == "uuid" else int(k)
                    for k in nonnull], dtype=np.int64)
    cnt = np.array(list(nonnull.values()), dtype=np.int64)
    pos = np.clip(np.searchsorted(uh, idx), 0, len(uh) - 1)
    out["detail_bins"] = len(nonnull)
    out["detail_counts_ok"] = bool(np.all(uh[pos] == idx) and np.all(ch[pos] == cnt))
    out["detail_multiset_ok"] = bool(np.array_equal(np.sort(cnt)[::-1], np.sort(ch)[::-1][:len(cnt)]))
    out["null_bin_ok"] = vals.get("NullValue", 0) == args.c4_rows - n_valid
    out["number_of_bins_ok"] = dist_metric.numberOfBins == groups + (1 if n_valid < args.c4_rows else 0)
    out["ok"] = all(out[k] for k in out if k.endswith("_ok")) and out["entropy_rel_err"] <= 1e-12
    return out


# UUID text of an id (--c4-keys uuid): the 32 hex digits of x = id * A + B and y = (id ^ C) * D
# (mod 2^64), as 8-4-4-4-12.  x is a bijection of the id, so the keys group exactly as the ids.
_UUID_A, _UUID_B = 0x9E3779B97F4A7C15, 0x632BE59BD9B4E019
_UUID_C, _UUID_D = 0x5DEECE66D, 0xC2B2AE3D27D4EB4F


def _s64(v: int) -> int:
    v %= 2 ** 64
    return v - 2 ** 64 if v >= 2 ** 63 else v


def _uuid_chars(ids, dev):
    """(n, 36) uint8 UUID text of int64 ids (torch int64 arithmetic wraps mod 2^64)."""
    import torch
    x = ids * _s64(_UUID_A) + _s64(_UUID_B)
    y = (ids ^ _UUID_C) * _s64(_UUID_D)
    sh = torch.arange(60, -4, -4, dtype=torch.int64, device=dev)
    nib = torch.cat([(x[:, None] >> sh[None, :]) & 15, (y[:, None] >> sh[None, :]) & 15], dim=1)
    hexd = torch.where(nib < 10, nib + 48, nib + 87).to(torch.uint8)  # 0-9, a-f
    dash = torch.full((ids.numel(), 1), ord("-"), dtype=torch.uint8, device=dev)
    return torch.cat([hexd[:, :8], dash, hexd[:, 8:12], dash, hexd[:, 12:16], dash, hexd[:, 16:20], dash,
                      hexd[:, 20:32]], dim=1)


def uuid_to_id(key: str) -> int:
    """The id behind a --c4-keys uuid key (inverting x = id * A + B mod 2^64)."""
    x = int(key.replace("-", "")[:16], 16)
    return ((x - _UUID_B) * pow(_UUID_A, -1, 2 ** 64)) % 2 ** 64


def make_c4_batches(rows: int, batch: int, distinct: int, rank: int, device: int, keys_kind: str = "digits"):
    """C4: a string key = 12-digit zero-padded decimal of a uniform int in [0, distinct), 1% NULL,
    as Arrow utf8 batches of `batch` rows (int32 offsets cap one batch at 2 GiB of chars).
    alnum: the first digit replaced by 'k' (same groups, keys that are not digit strings); uuid:
    the id's 36-character UUID text; pair: two columns a = id // 1000 (int64, NULL where the key is)
    and b = the 8 digits of id % 1000 (utf8).  The ids are the same draws in every case."""
    import torch
    import deequ_amd as d
    dev = torch.device("cuda", device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7 + 1000 * rank)
    pow10 = torch.tensor([10 ** (11 - i) for i in range(12)], dtype=torch.int64, device=dev)
    width = {"uuid": 36, "pair": 8, "pair64": 0}.get(keys_kind, 12)
    batch = c4_batch_rows(batch, keys_kind)
    parts = []
    for b0 in range(0, rows, batch):
        m = min(batch, rows - b0)
        chars = torch.empty(m * width + 16, dtype=torch.uint8, device=dev)
        valid = torch.empty((m + 7) // 8 + 64, dtype=torch.uint8, device=dev)
        avals = torch.empty(m, dtype=torch.int64, device=dev) if keys_kind in ("pair", "pair64") else None
        bvals = torch.empty(m, dtype=torch.int64, device=dev) if keys_kind == "pair64" else None
        sub = 1 << 24
        for s in range(0, m, sub):
            e = min(m, s + sub)
            keys = torch.randint(0, distinct, (e - s,), generator=gen, device=dev, dtype=torch.int64)
            if keys_kind == "uuid":
                chars[s * width: e * width] = _uuid_chars(keys, dev).reshape(-1)
            elif keys_kind == "pair":
                avals[s:e] = keys // 1000
                chars[s * width: e * width] = _strings_from_ints(keys % 1000, 8, b"", dev)
            elif keys_kind == "pair64":
                avals[s:e] = keys // 1000
                bvals[s:e] = keys % 1000
            else:
                digits = (keys[:, None] // pow10[None, :]) % 10 + 48
                if keys_kind == "alnum":
                    digits[:, 0] = ord("k")
                chars[s * 12: e * 12] = digits.to(torch.uint8).reshape(-1)
            packed = _valid_bits(e - s, gen, dev, 0.01)
            valid[s // 8: s // 8 + packed.numel()] = packed
        offsets = torch.arange(0, width * (m + 1), width, dtype=torch.int32, device=dev) if width else None
        if keys_kind == "pair64":
            parts.append(d.Table({"a": d.Column("int64", m, avals, valid, device=True),
                                  "b": d.Column("int64", m, bvals, None, device=True)}))
        elif keys_kind == "pair":
            parts.append(d.Table({"a": d.Column("int64", m, avals, valid, device=True),
                                  "b": d.Column("string", m, chars, None, offsets=offsets, device=True)}))
        else:
            parts.append(d.Table({"key": d.Column("string", m, chars, valid, offsets=offsets, device=True)}))
    torch.cuda.synchronize(dev)
    return d.PartitionedTable(parts)


def _comm_dev(args, local: int):
    """allgather_merge's device argument: the GPU for RCCL, None (host tensors) for gloo."""
    return local if args.backend == "nccl" else None


def valu_roofline(device: int, hashes: float, kernel_ms: float):
    """The hash-bound side of an HLL pass ("HLL is additionally checked against the
    VALU int64-multiply rate"): `hashes` XXH64+register updates executed per launch (every row of
    every HLL column -- the kernels hash branch-free, NULL rows included) over the launch time,
    against the rate a register-only kernel (dq_diag_hash_rate, no HBM traffic) sustains on this
    card right now."""
    from deequ_amd import _lib
    peak = ctypes.c_double(0.0)
    if _lib.lib().dq_diag_hash_rate(device, 1, 5, ctypes.byref(peak)) != 0:
        return None
    achieved = hashes / (kernel_ms * 1e-3)
    return {"bound": "valu", "achieved": achieved / 1e9, "peak": peak.value / 1e9,
            "unit": "Ghash/s", "frac": achieved / peak.value, "hashes_per_launch": hashes,
            "peak_source": "dq_diag_hash_rate: Spark XXH64 (5 x 64-bit multiply) + HLL LDS "
                           "update, register-only, measured live"}


def run_c3(args, world, rank, local):
    """HLL++ ApproxCountDistinct on C3 columns: one fused dq_plan, HIP events on its stream."""
    import numpy as np
    import torch
    import deequ_amd as d
    from deequ_amd.distributed import allgather_merge
    from deequ_amd.engine import Plan, op_spec_for
    utf8 = args.c3_type == "utf8"
    table = (make_c3_string_table if utf8 else make_c3_table)(args.c3_rows, args.c3_columns, rank, local)
    analyzers = [d.ApproxCountDistinct(c) for c in table.schema]
    plan = Plan([op_spec_for(a, table.schema) for a in analyzers], table.schema, device=local)
    stream = torch.cuda.ExternalStream(plan.stream, device=torch.device("cuda", local))

    def step(ev=None):
        plan.reset()
        if ev is not None:
            ev[0].record(stream)
        plan.consume(table)
        if ev is not None:
            ev[1].record(stream)
        raw = plan.finish_raw()
        if world > 1:
            raw = allgather_merge(raw, len(analyzers), device=_comm_dev(args, local))
        return raw
    elapsed, kernel_ms, raw = _timed(args, world, step)
    est = d.ApproxCountDistinctState(list(raw[0].words)).metricValue()
    bpr = args.c3_columns * ((4 + 16 + 1.0 / 8) if utf8 else (8 + 1.0 / 8))
    full_job = None
    if args.c3_batches > 1 and not utf8:
        # the whole C3 job: ONE plan over c3_batches batches of the 1e9-row stream (64 x 1e9 int64
        # = 520 GB does not fit 288 GB of HBM, so each batch is regenerated in HBM between its
        # consumes -- untimed); the scans of all batches are timed with HIP events on the plan's stream
        plan.reset()
        scan_ms = 0.0
        oracle_regs = None
        for b in range(args.c3_batches):
            if b > 0:
                make_c3_table(args.c3_rows, args.c3_columns, rank, local, batch=b, into=table)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            plan.consume(table)
            e1.record(stream)
            e1.synchronize()
            scan_ms += e0.elapsed_time(e1)
            if args.c3_verify and world == 1:  # column 0 of this batch through the oracle (untimed)
                c0 = table.columns["h0"]
                regs = _oracle_hll_int64(c0.values[:args.c3_rows].cpu().numpy(),
                                         c0.validity[:(args.c3_rows + 7) // 8].cpu().numpy())
                oracle_regs = regs if oracle_regs is None else np.maximum(oracle_regs, regs)
        fraw = plan.finish_raw()
        if world > 1:
            fraw = allgather_merge(fraw, len(analyzers), device=_comm_dev(args, local))
        rows_job = args.c3_rows * args.c3_batches
        full_job = {"batches": args.c3_batches, "rows_per_gpu": rows_job, "columns": args.c3_columns,
                    "scan_ms": scan_ms, "rows_per_s_per_gpu": rows_job / (scan_ms * 1e-3),
                    "hbm_gbs": bpr * rows_job / (scan_ms * 1e-3) / 1e9,
                    "column0_estimate": d.ApproxCountDistinctState(list(fraw[0].words)).metricValue(),
                    "note": "one plan, %d consumes of %d-row batches regenerated in HBM between them "
                            "(untimed); scan time = sum of the consumes' HIP-event times"
                            % (args.c3_batches, args.c3_rows)}
        if oracle_regs is not None:
            full_job["verify"] = _c3_verify(oracle_regs, list(fraw[0].words))
    rows_total = args.c3_rows * world * args.steps
    achieved = bpr * args.c3_rows / (kernel_ms * 1e-3) / 1e9
    return {
        "metric": "rows/sec & HBM GB/s for ApproxCountDistinct HLL++ (C3)", "value": rows_total / elapsed,
        "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "utf8 (XXH64 of 16 bytes)" if utf8 else "int64 (XXH64)",
        "data": ("synthetic 16-char lowercase hex of a uniform u64" if utf8 else
                 "synthetic int64 uniform over 2^64") + ", 5% NULL, generated in HBM",
        "config": {"workload": "C3: %d rows/GPU x %d %s columns, one HLL plan (one batch of the "
                               "1B-row stream)" % (args.c3_rows, args.c3_columns, "utf8" if utf8 else "int64"),
                   "rows_per_gpu": args.c3_rows, "columns": args.c3_columns},
        "roofline": _step_roofline(bpr * args.c3_rows, kernel_ms / 1e3, "one HLL plan pass (scan kernels, HIP events)",
                                   workload=None if utf8 else "c3", default_size=args.c3_rows == 125_000_000),
        # (the register-only hash-rate probe times the 8-byte hashLong, not 16-byte strings)
        "valu_roofline": None if utf8 else valu_roofline(local, float(args.c3_rows) * args.c3_columns,
                                                         kernel_ms),
        "check": {"column0_estimate": est, "rows_column0": args.c3_rows},
        "full_job": full_job,
    }


def _oracle_hll_int64(values, validity):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cdq_oracle
    return cdq_oracle.hll_registers_int64(values, validity, host_cpu_share())


def _c3_verify(oracle_regs, gpu_words):
    """Column 0 of the whole C3 job: the GPU plan's 52 words against the oracle's registers of
    every batch (max-merged), and the estimate explained register by register: Deequ's count
    adds 1.0 / (1 << m) with Java's Int shift (StatefulHyperloglogPlus.scala:222), whose count is
    taken mod 32 -- a register of rank m >= 32 adds 2^-(m - 32) instead of 2^-m."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    want = O.hll_pack([int(r) for r in oracle_regs])
    regs = O.hll_unpack(gpu_words)
    high = {i: r for i, r in enumerate(regs) if r >= 32}
    z_low = sum(2.0 ** -r for r in regs if r < 32)
    return {"words_equal": [int(w) for w in gpu_words] == want,
            "registers_ge_32": high,
            "register_max": max(regs),
            "estimate_oracle": O.hll_count(want),
            "estimate_without_int_shift": O.HLL_ALPHA_M2 / (z_low + sum(2.0 ** -r for r in high.values()))
            if high else None,
            "z_inverse_terms": {"ranks_below_32": z_low,
                                "ranks_ge_32_java": sum(1.0 / float(O._java_int_shift_one(r)) for r in high.values())}}


def _column_bytes(col) -> float:
    """Arrow bytes of one column: values (utf8: int32 offsets + chars; bool: bits) + validity bits."""
    n = col.length
    valid = n / 8.0 if col.validity is not None else 0.0
    if col.dtype == "string":
        return 4.0 * (n + 1) + float(col.values.numel() - 16) + valid
    if col.dtype == "bool":
        return n / 8.0 + valid
    return float(n * col.values.element_size()) + valid


def kernel_source_digest() -> str:
    """sha256 (16 hex) of the library's sources (deequ_amd/csrc, include/): the build a PMC
    traffic file was collected on must have exactly these kernels for its bytes to be quoted."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "deequ_amd", "csrc", "*")) + glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in files:
        if os.path.isfile(f) and not f.endswith((".o", ".so")):
            h.update(os.path.relpath(f, ROOT).encode())
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def _pmc_traffic(workload: str):
    """HBM bytes per step of `workload` at its default size, from a PMC pass committed under
    profiles/ (tools/pmc_traffic.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of this same bench,
    read = 2 x FETCH_SIZE on gfx950).  Counters cannot be read inside an unprofiled run, so this
    is a COPIED profile value, labelled as such in the line (traffic_source).  Only a file whose
    `kernel_src_digest` equals this tree's kernel_source_digest() is used: traffic measured on
    other kernels is never quoted (None, with the reason in traffic_source)."""
    import glob
    digest = kernel_source_digest()
    base, _, keys = workload.partition("_")  # e.g. "c4_uuid": the c4 workload with --c4-keys uuid
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic_%s*.json" % base)), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:  # noqa: BLE001
            continue
        args = d.get("bench_args", "")
        shape = args.split("--c4-keys", 1)[1].split()[0] if "--c4-keys" in args else ""
        shape = "" if shape == "digits" else shape
        if d.get("workload", base) != base or shape != keys:
            continue  # (another workload, or the same one with another key shape)
        if d.get("kernel_src_digest") == digest:
            return d["hbm_bytes_per_step"], "copied from %s (PMC pass of this bench at its default size, kernel " \
                "sources %s)" % (os.path.relpath(path, ROOT), digest)
    return None, "null: no PMC traffic file in profiles/ was collected on these kernel sources (%s)" % digest


def _step_roofline(bytes_per_step: float, step_s: float, what: str, traffic=None, workload=None,
                   default_size=True):
    achieved = bytes_per_step / step_s / 1e9
    src = None
    if traffic is None and workload and default_size:
        traffic, src = _pmc_traffic(workload)
    out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel_ms": step_s * 1e3,
           "algorithmic_bytes_per_launch": bytes_per_step, "timed_unit": what}
    if src:
        out["traffic_source"] = src
    return out


def run_c4(args, world, rank, local):
    """Uniqueness/Distinctness/Entropy/CountDistinct (one GPU group-by) + Histogram on C4; on N
    GPUs every rank groups its own shard and the tables meet in the key-hash all-to-all."""
    import deequ_amd as d
    from deequ_amd.distributed import ShardedTable
    shard = make_c4_batches(args.c4_rows, args.c4_batch, args.c4_distinct, rank, local, args.c4_keys)
    data = ShardedTable(shard) if world > 1 else shard
    pair = args.c4_keys in ("pair", "pair64")
    if pair:  # a composite key: the pair's frequency analyzers (Check.hasUniqueness / isPrimaryKey shape)
        cols = ["a", "b"]
        analyzers = [d.Uniqueness(cols), d.Distinctness(cols), d.UniqueValueRatio(cols), d.CountDistinct(cols)]
    else:
        analyzers = [d.Uniqueness(["key"]), d.Distinctness(["key"]), d.Entropy("key"),
                     d.CountDistinct(["key"]), d.Histogram("key")]

    def step(ev=None):
        return d.AnalysisRunner.onData(data).addAnalyzers(analyzers).run()
    elapsed, _, ctx = _timed(args, world, step)
    metrics = {str(a): ctx.metric(a).value.get() for a in analyzers[:4]}
    hist = None if pair else ctx.metric(analyzers[4]).value.get()
    verify = None
    if args.c4_verify and world == 1:
        del ctx
        verify = c4_verify(args, {a: metrics[str(a)] for a in analyzers[:4]}, hist, analyzers)
    in_bytes = sum(_column_bytes(c) for b in shard.batches() for c in b.columns.values())
    groups = metrics[str(analyzers[3])] / world  # the groups this rank's share of the table holds
    # input + one write of the final table (8 B hash + 8 B count + 8 B key ref)
    algo = in_bytes + 24.0 * groups
    step_s = elapsed / args.steps
    return {
        "metric": "rows/sec for the frequency family (C4 group-by)",
        "value": args.c4_rows * world * args.steps / elapsed,
        "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "utf8 keys, int64 counts",
        "data": "synthetic %s keys of ids uniform in [0, %d), 1%% NULL, generated in HBM"
                % ({"digits": "12-digit", "alnum": "'k' + 11-digit", "uuid": "36-character UUID",
                    "pair": "(int64, 8-digit utf8) pair", "pair64": "(int64, int64) pair"}[args.c4_keys],
                   args.c4_distinct),
        "config": {"workload": ("C4: %d rows/GPU in %d-row batches; Uniqueness, Distinctness, UniqueValueRatio, "
                                "CountDistinct of the two-column key (a, b), one GPU group-by%s" if pair else
                                "C4: %d rows/GPU in %d-row utf8 batches; Uniqueness, Distinctness, Entropy, "
                                "CountDistinct + Histogram, all from one GPU group-by of the key (the "
                                "reference runs Histogram as a second job)%s")
                               % (args.c4_rows, c4_batch_rows(args.c4_batch, args.c4_keys),
                                  "; key-hash all-to-all over %d ranks" % world if world > 1 else ""),
                   "keys": args.c4_keys},
        "roofline": _step_roofline(algo, step_s, "one whole group-by step per GPU (stage + level-1 partition, "
                                                 "level-2 partition, slice aggregation, top-N), HBM-bound by design",
                                   workload=("c4" if args.c4_keys == "digits" else "c4_" + args.c4_keys)
                                   if world == 1 else None,
                                   default_size=(args.c4_rows, args.c4_batch, args.c4_distinct)
                                   == (1_000_000_000, 125_000_000, 201_500_000)),
        # SURVEY §8(d) C4 asks for the table accesses per row beside the streaming fraction: the
        # partition path moves each staged row's record three times (stage write, level-2 split
        # read + write, aggregation read) -- 8 B for these digit-string keys (packed words), 16 B
        # for other keys -- and touches the HBM table only in whole-slice writes: no per-row table
        # probe (the probes are in LDS).
        "table_access": _c4_table_access(args.c4_keys, groups, args.c4_rows),
        "check": dict(metrics, **({} if pair else {"histogram_bins": hist.numberOfBins})),
        **({"verify": verify} if verify is not None else {}),
        **({"exchange": _exchange_stats(world, local)} if world > 1 else {}),
    }


def _exchange_stats(world: int, local: int):
    """The key-hash exchange of the last timed C4 step (deequ_amd.distributed.last_exchange_stats):
    rank 0's bytes and milliseconds, plus the maximum over ranks of each time (collective)."""
    import torch
    import torch.distributed as dist
    from deequ_amd.distributed import last_exchange_stats
    st = last_exchange_stats()
    keys = ["partition_ms", "alltoall_ms", "import_ms", "exchange_ms"]
    t = torch.tensor([float(st.get(k, 0.0)) for k in keys], dtype=torch.float64)
    if dist.get_backend() == "nccl":
        t = t.to(torch.device("cuda", local))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out = {k: st.get(k) for k in ("bytes_sent", "bytes_sent_remote", "bytes_received")}
    out.update({k: st.get(k) for k in keys})
    out.update({"max_" + k: v for k, v in zip(keys, t.cpu().tolist())})
    out["exchange_bytes"] = st.get("bytes_sent")
    return out


def _c4_table_access(keys: str, groups: float, rows: int):
    """SURVEY §8(d) C4 asks for the table accesses per row beside the streaming fraction.  Digit
    keys (packed 8-B records): written by the row-order stage, read and written by the level-1
    split, read and written by the level-2 split, read by the slice aggregation -- 3 writes + 3
    reads.  Other short keys (16-B records) and canonical UUIDs (16-B records of their 128 bits)
    take one fused stage-and-split kernel: 2 writes + 2 reads.  Composite keys (hashed records)
    take the row-order stage, copy each key's bytes into the key heap once, and re-read a record
    and two keys per row that joins an existing hash group (the exact compare).  Probes are in
    LDS; the table is written once, occupied slots only (compacted); a UUID group's 36-byte text
    is written once per group."""
    slot_bytes = 32.0
    rec = {"digits": 8, "alnum": 16, "uuid": 16, "pair": 16, "pair64": 16}[keys]
    passes = {"digits": (3, 3), "alnum": (2, 2), "uuid": (2, 2), "pair": (3, 3), "pair64": (2, 2)}[keys]
    heap = {"uuid": 40.0}.get(keys, 0.0)
    return {"record_bytes": rec, "record_writes_per_row": passes[0], "record_reads_per_row": passes[1],
            "global_table_probes_per_row": 0,
            "table_bytes_written_per_row": groups * (slot_bytes + heap) / float(rows),
            "table_write": "occupied slots only" + (" + each group's text (40 B)" if heap else ""),
            "key_heap_copy": keys == "pair"}


def _strings_from_ints(ids, width: int, prefix: bytes, dev):
    """utf8 column pieces: `prefix` + the zero-padded decimal digits of `ids` (fixed width)."""
    import torch
    n = ids.numel()
    pw = torch.tensor([10 ** (width - 1 - i) for i in range(width)], dtype=torch.int64, device=dev)
    digits = ((ids[:, None] // pw[None, :]) % 10 + 48).to(torch.uint8)
    if prefix:
        pre = torch.tensor(list(prefix), dtype=torch.uint8, device=dev).expand(n, len(prefix))
        digits = torch.cat([pre, digits], dim=1)
    return digits.reshape(-1)


def make_c5_table(rows: int, rank: int, device: int):
    """C5: 100 columns, 5% NULL each, seed 5: 40 int64, 30 fp64, 10 low-cardinality
    strings (<= 100 categories, "cat_NN"), 10 high-cardinality strings (16 digits), 10 bool."""
    import torch
    import deequ_amd as d
    dev = torch.device("cuda", device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5 + 1000 * rank)
    cols = {}

    def valid():
        return _valid_bits(rows, gen, dev, 0.05)

    for k in range(40):
        v = torch.randint(-10 ** 6, 10 ** 9, (rows,), generator=gen, device=dev, dtype=torch.int64)
        cols["l%02d" % k] = d.Column("int64", rows, v, valid(), device=True)
    for k in range(30):
        v = torch.randn(rows, generator=gen, device=dev, dtype=torch.float64) * 100.0 + 1000.0
        cols["d%02d" % k] = d.Column("float64", rows, v, valid(), device=True)
    for k in range(20):
        low = k < 10
        width = 2 if low else 16
        prefix = b"cat_" if low else b""
        n_cat = 100 if low else 10 ** 15
        step = len(prefix) + width
        chars = torch.empty(rows * step + 16, dtype=torch.uint8, device=dev)
        sub = 1 << 24
        for s0 in range(0, rows, sub):
            e0 = min(rows, s0 + sub)
            ids = torch.randint(0, n_cat, (e0 - s0,), generator=gen, device=dev, dtype=torch.int64)
            chars[s0 * step: e0 * step] = _strings_from_ints(ids, width, prefix, dev)
        offsets = torch.arange(0, step * (rows + 1), step, dtype=torch.int32, device=dev)
        cols[("s%02d" if low else "u%02d") % k] = d.Column("string", rows, chars, valid(), offsets=offsets,
                                                        device=True)
    for k in range(10):
        bits = _valid_bits(rows, gen, dev, 0.5)  # uniform booleans, packed like a bitmap
        cols["b%02d" % k] = d.Column("bool", rows, bits, valid(), device=True)
    torch.cuda.synchronize(dev)
    return d.Table(cols)


def make_c1_table(rows: int, rank: int, device: int):
    """C1 (BASELINE configs[0]): the Item table of examples/entities.scala:19-25,
    seed 1.  id = 0..n-1; productName "Thingy <id>" and description (fixed-width utf8), priority
    "high"/"low" (variable-length utf8), each 5% NULL; numViews uniform int64 in [-1e3, 1e6),
    5% NULL."""
    import torch
    import deequ_amd as d
    dev = torch.device("cuda", device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1 + 1000 * rank)
    ids = torch.arange(rows, dtype=torch.int64, device=dev) + rows * rank

    def fixed(prefix: bytes, width: int, vals):
        step = len(prefix) + width
        chars = torch.cat([_strings_from_ints(vals, width, prefix, dev),
                           torch.zeros(16, dtype=torch.uint8, device=dev)])
        offs = torch.arange(0, step * (rows + 1), step, dtype=torch.int32, device=dev)
        return chars, offs

    cols = {"id": d.Column("int64", rows, ids, None, device=True)}
    chars, offs = fixed(b"Thingy ", 10, ids)
    cols["productName"] = d.Column("string", rows, chars, _valid_bits(rows, gen, dev, 0.05), offsets=offs, device=True)
    chars, offs = fixed(b"item description ", 6, (ids * 7919) % 100003)
    cols["description"] = d.Column("string", rows, chars, _valid_bits(rows, gen, dev, 0.05), offsets=offs, device=True)
    high = torch.randint(0, 2, (rows,), generator=gen, device=dev).bool()
    lens = torch.where(high, 4, 3).to(torch.int32)
    offs = torch.zeros(rows + 1, dtype=torch.int32, device=dev)
    offs[1:] = torch.cumsum(lens, 0)
    words = torch.tensor([list(b"high"), list(b"low\0")], dtype=torch.uint8, device=dev)
    chars = torch.zeros(int(offs[-1]) + 16, dtype=torch.uint8, device=dev)
    j = torch.arange(4, device=dev)
    pos = offs[:-1, None].to(torch.int64) + j[None, :]
    keep = j[None, :] < lens[:, None]
    chars[pos[keep]] = words[(~high).long()][keep]
    cols["priority"] = d.Column("string", rows, chars, _valid_bits(rows, gen, dev, 0.05), offsets=offs, device=True)
    views = torch.randint(-1000, 1_000_000, (rows,), generator=gen, device=dev, dtype=torch.int64)
    cols["numViews"] = d.Column("int64", rows, views, _valid_bits(rows, gen, dev, 0.05), device=True)
    torch.cuda.synchronize(dev)
    return d.Table(cols)


def c1_analyzers():
    import deequ_amd as d
    return ([d.Size()] + [d.Completeness(c) for c in ("id", "productName", "description", "priority", "numViews")]
            + [d.Compliance("numViews non-negative", "numViews >= 0"), d.Mean("numViews"),
               d.StandardDeviation("numViews"), d.Minimum("numViews"), d.Maximum("numViews")])


def run_c1(args, world, rank, local):
    """The reference's CPU-runnable case through the AnalysisRunner mirror: one whole
    AnalysisRunner.onData(...).addAnalyzers(...).run() per step (plan, fused scan, states,
    metrics), every rank on its own 10M-row Item shard."""
    import deequ_amd as d
    from deequ_amd.distributed import ShardedTable
    shard = make_c1_table(args.c1_rows, rank, local)
    data = ShardedTable(shard) if world > 1 else shard  # metrics of the union of the shards
    analyzers = c1_analyzers()

    def step(ev=None):
        return d.AnalysisRunner.onData(data).addAnalyzers(analyzers).run()
    elapsed, _, ctx = _timed(args, world, step)
    metrics = {str(a): ctx.metric(a).value.get() for a in analyzers}
    return {
        "metric": "rows/sec for the C1 AnalysisRunner suite (Item table)",
        "value": args.c1_rows * world * args.steps / elapsed, "unit": "rows/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64 + utf8 validity",
        "data": "synthetic Item table generated in HBM (seed 1, 5% NULL)",
        "config": {"workload": "C1: %d rows/GPU Item(id, productName, description, priority, numViews); "
                               "Size, 5 x Completeness, Compliance(numViews >= 0), Mean/StdDev/Min/Max(numViews) "
                               "through AnalysisRunner" % args.c1_rows},
        "check": metrics,
    }


def run_c5(args, world, rank, local):
    """ColumnProfilerRunner over the C5 table: 3 passes (generic stats + HLL + DataType; numeric
    stats; exact histograms of the low-cardinality columns); on N GPUs every rank profiles its
    shard and the passes' states / tables meet in the collectives of a ShardedTable."""
    from deequ_amd.distributed import ShardedTable
    from deequ_amd.profiles import ColumnProfilerRunner
    shard = make_c5_table(args.c5_rows, rank, local)
    data = ShardedTable(shard) if world > 1 else shard

    def step(ev=None):
        return ColumnProfilerRunner().onData(data).run()
    elapsed, _, profiles = _timed(args, world, step)
    p = profiles.profiles
    n_hist = sum(1 for c in p.values() if c.histogram is not None)
    step_s = elapsed / args.steps
    cols = shard.columns
    # pass 1 reads every column once: Completeness, HLL, DataType and -- for schema-numeric columns
    # -- the statistics too (profiles.py computes them in pass 1's fused scan, never re-reading)
    pass1 = sum(_column_bytes(c) for c in cols.values())
    cast = [n for n, c in cols.items() if c.dtype == "string" and p[n].dataType in (1, 2)]
    rows = args.c5_rows
    # pass 2 reads only the strings pass 1 typed numeric: the cast kernel reads the string column
    # and writes 8 B + a validity bit per row, the statistics scan reads that back
    pass2 = sum(_column_bytes(cols[n]) + 2 * rows * (8 + 1 / 8.0) for n in cast)
    # pass 3 re-reads only the histogram columns pass 1 did not already group: a few-valued
    # string column's histogram is its pass-1 groups (profiles.py _few_group_strings, one GPU)
    few_path = world == 1 and os.environ.get("DEEQU_AMD_PROFILE_FEW", "1") != "0"
    pass3 = sum(_column_bytes(cols[n]) for n, c in p.items()
                if c.histogram is not None and not (few_path and cols[n].dtype == "string"))
    roof = _step_roofline(pass1 + pass2 + pass3, step_s,
                          "one whole profile per GPU (3 passes; bytes = what each pass must read: pass 1 every column once, pass 2 the numeric-typed strings cast + re-scanned, pass 3 the histogram columns pass 1 did not group)",
                          workload="c5" if world == 1 else None, default_size=args.c5_rows == 100_000_000)
    # the same step priced as if every column were read from HBM exactly once (no pass re-reads a
    # column, no cast output written and read back): the bound of a single-pass profiler
    roof["one_read_per_column"] = {"bytes": pass1, "frac": pass1 / step_s / 1e9 / roof["peak"]}
    return {
        "metric": "rows/sec for ColumnProfilerRunner (C5)", "value": args.c5_rows * world * args.steps / elapsed,
        "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int64/fp64/utf8/bool", "data": "synthetic C5 table generated in HBM (seed 5, 5% NULL)",
        "config": {"workload": "C5: %d rows/GPU x 100 columns (40 int64, 30 fp64, 10 low- and 10 high-cardinality "
                               "utf8, 10 bool); ColumnProfilerRunner, 3 passes, KLL off (reference default)"
                               % args.c5_rows},
        "roofline": roof,
        "check": {"columns": len(p), "histograms": n_hist,
                  "s00_distinct": p["s00"].approximateNumDistinctValues,
                  "l00_completeness": p["l00"].completeness, "numRecords": profiles.numRecords},
    }


def _max_over_ranks(x: float) -> float:
    """MAX over the ranks (the job's time), on the device the process group's backend uses."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _timed(args, world, step):
    """W warmup steps, then K timed steps between barriers + device syncs; max over ranks."""
    import torch
    import torch.distributed as dist
    out = None
    for _ in range(args.warmup):
        out = None  # a step's result (e.g. HBM-resident frequency tables) is dropped before the next
        out = step()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    # The process's long-lived objects (torch, the synthetic tables: ~170k tracked objects) go to
    # the garbage collector's permanent generation first: otherwise a generation-2 collection,
    # triggered by whatever a step allocates, traverses them all in the middle of a timed step
    # (measured: one 46 ms pause every ~11 C5 steps).  The work timed is unchanged.
    import gc
    gc.collect()
    gc.freeze()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = None
        out = step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.unfreeze()
    if world > 1:
        elapsed = _max_over_ranks(elapsed)
    try:
        kernel_ms = sum(a.elapsed_time(b) for a, b in events) / len(events)
    except (RuntimeError, ValueError):  # the step did not record the events
        kernel_ms = None
    return elapsed, kernel_ms, out


def _spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N ranks (one process per GPU) through
    torch.distributed.run as a CHILD process -- nothing here has touched the GPU yet -- and
    return its exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        sys.exit(_spawn_ranks(args.gpus))
    if world_env is not None and int(world_env) != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%s: launch one rank per GPU" % (args.gpus, world_env))
    import torch
    import torch.distributed as dist

    import deequ_amd as d
    from deequ_amd.distributed import allgather_merge
    from deequ_amd.engine import Plan, op_spec_for
    from deequ_amd.states import state_from_dq

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":  # a rehearsal of the multi-rank path: ranks may share a GPU
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    d.set_device(local)
    if world > 1 and args.backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif world > 1:
        dist.init_process_group("gloo")
    if args.workload != "c2":
        result = {"c1": run_c1, "c3": run_c3, "c4": run_c4, "c5": run_c5}[args.workload](args, world, rank, local)
        if rank == 0:
            print(json.dumps(result))
        if world > 1:
            dist.destroy_process_group()
        return

    table = make_c2_table(args.rows, rank, local)
    analyzers = c2_analyzers()
    plan = Plan([op_spec_for(a, table.schema) for a in analyzers], table.schema, device=local)
    stream = torch.cuda.ExternalStream(plan.stream, device=torch.device("cuda", local))
    n_ops = len(analyzers)
    n_hll = sum(isinstance(a, d.ApproxCountDistinct) for a in analyzers)

    def step(ev_pair=None):
        plan.reset()
        if ev_pair is not None:
            ev_pair[0].record(stream)
        plan.consume(table)
        if ev_pair is not None:
            ev_pair[1].record(stream)
        raw = plan.finish_raw()
        if world > 1:
            raw = allgather_merge(raw, n_ops, device=_comm_dev(args, local))
        return raw

    for _ in range(args.warmup):
        raw = step()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        raw = step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = _max_over_ranks(elapsed)

    kernel_ms = sum(a.elapsed_time(b) for a, b in events) / len(events)
    states = [state_from_dq(raw[i]) for i in range(n_ops)]
    # sanity: the suite produced every state (5% NULLs -> nothing is empty)
    assert all(s is not None for s in states), "empty state in the benchmark suite"
    assert states[0].numMatches == args.rows * world

    rows_total = args.rows * world * args.steps
    value = rows_total / elapsed
    achieved = BYTES_PER_ROW * args.rows / (kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = (None, None)
    if args.rows == 1_000_000_000 and n_hll == 8:
        traffic, traffic_src = _pmc_traffic("c2")

    result = {
        "metric": "rows/sec & HBM GB/s for analyzer-suite scan, 1B rows x 8 cols, 1/2/4/8 GPUs",
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64+f64",
        "data": "synthetic (C2 distributions generated in HBM, 5% NULL per column)",
        "config": {"workload": "C2: %d rows/GPU x 8 cols (4 int64 + 4 fp64), 65 scan-shareable "
                               "analyzers (incl. 8 ApproxCountDistinct) fused in one pass" % args.rows,
                   "rows_per_gpu": args.rows, "columns": 8, "analyzers": n_ops,
                   "parallelism": "dp%d (row shards, states all-gathered over RCCL)" % world},
        "hbm_gbs": achieved,
        "roofline": dict({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                          "kernel_ms": kernel_ms,
                          "algorithmic_bytes_per_launch": BYTES_PER_ROW * args.rows},
                         **({"traffic_source": traffic_src} if traffic_src else {})),
        "valu_roofline": valu_roofline(local, float(args.rows) * n_hll, kernel_ms) if n_hll else None,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_side_passes:
        result["scan_without_hll"] = scan_without_hll(table, local, args.steps)
        if args.e2e_batch_rows > 0:
            result["host_ingest"] = host_ingest(args, local)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or host_cpu_share()
        result["cpu_baseline"] = cpu_baseline(args.cpu_sample_rows, threads)
        # beside the one-GPU share: every host CPU (nproc), as SURVEY §8(d) states the baseline
        if result["cpu_baseline"].get("value"):
            result["cpu_baseline"]["all_host_cpus"] = all_host_baseline(
                args.cpu_sample_rows, threads, result["cpu_baseline"]["value_per_core"])
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
