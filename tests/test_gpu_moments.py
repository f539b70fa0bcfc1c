"""StandardDeviation / Mean when a wave's moment shift is an outlier.

Both value scans take a wave's Σd, Σd² about a shift c -- the first valid value the wave probes
(dq_scan_fast.hip, dq_scan.hip) -- and form m2 = S2 - S1²/n.  When c is an outlier that
difference cancels (relative rounding ~ eps * S2 / m2), which Spark's per-row CentralMomentAgg
update never does (StandardDeviation.scala:37-44 merge).  The kernels detect it per wave
(moments_cancel, dq_scan_common.h) and redo the chunk about its mean.  These cases put outliers
exactly on the probe rows: row 0, and the first row of every wave (rows = 0 mod 64):

* small tables against the exact rational moments (tests/test_gpu_parity.py's _check_state);
* a `where` that EXCLUDES the outlier the general kernel probed (the shift is taken from valid
  rows regardless of `where`, so without the guard m2 loses every digit);
* 2^28-row device columns (tens of thousands of rows per wave, C2's regime) whose exact moments
  come from integer sums on the GPU (values are integers, or integers / 1024).

Bar: n bit-exact, mean and m2 within 1e-12 of the exact value (north_star)."""
import zlib
from fractions import Fraction

import numpy as np
import pytest

import deequ_amd as d
from helpers import oracle_table, product_table
from test_gpu_parity import _check_state

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12


def _both_kernels(monkeypatch, fn):
    fn()                      # dq_scan_fast_kernel (no where, int64 / fp64)
    monkeypatch.setenv("DQ_SCAN_FAST", "0")
    try:
        fn()                  # dq_scan_values_kernel
    finally:
        monkeypatch.delenv("DQ_SCAN_FAST")


def _stats(col, where=None):
    return [d.Mean(col, where), d.StandardDeviation(col, where), d.Sum(col, where),
            d.Minimum(col, where), d.Maximum(col, where)]


@pytest.mark.parametrize("dtype", ["int64", "float64"])
@pytest.mark.parametrize("layout", ["row0", "every_wave", "every_wave_nulls"])
def test_outlier_on_probe_rows(gpu, monkeypatch, dtype, layout):
    rng = np.random.default_rng(zlib.crc32((dtype + layout).encode()))
    n = 300_000
    if dtype == "int64":
        vals = [int(x) for x in np.rint(rng.normal(0, 1000, n))]
        big = 10 ** 12
    else:
        vals = [float(x) for x in rng.normal(0, 1, n)]
        big = 1e8
    if layout == "row0":
        vals[0] = big
    else:
        for r in range(0, n, 64):
            vals[r] = big if (r // 64) % 3 else -big
    if layout == "every_wave_nulls":
        vals = [None if (r % 64 and rng.random() < 0.05) else v for r, v in enumerate(vals)]
    spec = {"x": [dtype, vals]}
    ot, pt = oracle_table(spec), product_table(spec).to_device(0)

    def run():
        an = _stats("x")
        st = d.run_scan(an, pt)
        for a in an:
            _check_state(a, st[a], ot)
    _both_kernels(monkeypatch, run)


@pytest.mark.parametrize("dtype", ["int64", "float64"])
def test_where_excludes_probed_outlier(gpu, monkeypatch, dtype):
    """The outliers are valid but filtered out by `where`: they never enter the moments, yet
    the general kernel's probe may pick one as its shift."""
    rng = np.random.default_rng(17)
    n = 200_000
    if dtype == "int64":
        vals = [int(x) for x in np.rint(rng.normal(5000, 10, n))]
        big, where = 10 ** 13, "x < 1000000"
    else:
        vals = [float(x) for x in rng.normal(3.0, 0.5, n)]
        big, where = 1e9, "x < 1e6"
    for r in range(0, n, 64):
        vals[r] = big
    spec = {"x": [dtype, vals]}
    ot, pt = oracle_table(spec), product_table(spec).to_device(0)
    an = _stats("x", where)
    st = d.run_scan(an, pt)
    for a in an:
        _check_state(a, st[a], ot)


def _exact_from_ints(k_sum, k2_sum, n, scale):
    """mean, m2 of values k / scale given Σk, Σk² (Python ints)."""
    mean = Fraction(k_sum, n * scale)
    m2 = Fraction(k2_sum * n - k_sum * k_sum, n * scale * scale)
    return float(mean), float(m2)


@pytest.mark.parametrize("dtype", ["int64", "float64"])
def test_outlier_row0_at_scale(gpu, monkeypatch, dtype):
    """2^28 rows, 5 % NULL, one outlier at row 0 (the first probe of wave 0 of block 0)."""
    import torch
    n = 1 << 28
    g = torch.Generator(device="cuda").manual_seed(123)
    k = torch.randint(-4096, 4096, (n,), device="cuda", generator=g, dtype=torch.int64)
    valid = torch.rand(n, device="cuda", generator=g) >= 0.05
    outlier = 10 ** 9
    k[0] = outlier
    valid[0] = True
    scale = 1 if dtype == "int64" else 1024
    kv = torch.where(valid, k, torch.zeros_like(k))
    cnt = int(valid.sum())
    k_sum = int(kv.sum())
    # Σk² without overflow: the bulk fits int64, the outlier's square is added in Python
    kv[0] = 0
    k2_sum = int((kv * kv).sum()) + outlier * outlier
    mean, m2 = _exact_from_ints(k_sum, k2_sum, cnt, scale)
    if dtype == "int64":
        values = k
    else:
        values = k.to(torch.float64) / scale  # exact: |k| < 2^53
    bits = torch.zeros(n // 8, dtype=torch.uint8, device="cuda")
    vb = valid.view(-1, 8).to(torch.uint8)
    for b in range(8):
        bits |= vb[:, b] << b
    col = d.Column(dtype, n, values.contiguous(), bits, device=True)
    t = d.Table({"x": col})
    del kv, vb

    def run():
        sd = d.StandardDeviation("x")
        st = d.run_scan([sd, d.Mean("x")], t)[sd]
        assert st.n == float(cnt)
        assert abs(st.avg - mean) <= REL_TOL * abs(mean), (st.avg, mean)
        assert abs(st.m2 - m2) <= REL_TOL * abs(m2), (st.m2, m2, abs(st.m2 - m2) / m2)
    _both_kernels(monkeypatch, run)
