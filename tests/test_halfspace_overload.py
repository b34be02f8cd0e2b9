"""Sensitivity of the C3 gap rows to one unverifiable detail of the reference: the unqualified
cos(angle1) / sin(angle1) on a float angle in Constraints::FindHalfSpaces
(/root/reference/src/constraints.cpp:182-186). It resolves to ::cos(double) unless some header of
the ROS / Eigen include chain brings the libstdc++ <math.h> wrapper's float overload into the global
namespace; neither can be built here. The oracle and the device kernel assume the double overload
(oracle/f110_oracle.c, csrc/halfspace_kernels.hip); this test measures what the float overload
would change on the committed gap-row fixtures and on the bench's C3 batch (CPU only: the oracle's
half-spaces and exact optima for both overloads). Measured: about 40% of the QPs get
bitwise different half-spaces, no status changes, optima move by at most 9.2e-5 relative (bench
batch) — inside the north star's 1e-4, but not by much."""
import json
import os

import numpy as np
import pytest
from conftest import GOLDEN
from fuzz_cases import screen_fuzz_case

from f110qp import workload


def _both(oracle, x0, ranges, geom):
    B = x0.shape[0]
    hd = np.zeros((B, 2, 3), np.float32)
    hf = np.zeros((B, 2, 3), np.float32)
    for b in range(B):
        rc, l1, l2, _, _ = oracle.find_half_spaces(x0[b].astype(np.float64), ranges[b], *geom)
        rcf, f1, f2, _, _ = oracle.find_half_spaces(x0[b].astype(np.float64), ranges[b], *geom, float_trig=True)
        assert rc == 0 and rcf == 0
        hd[b] = l1, l2
        hf[b] = f1, f2
    return hd, hf


def _compare(oracle, prm, w, hd, hf):
    diff = np.any(hd.view(np.uint32) != hf.view(np.uint32), axis=(1, 2))
    idx = np.where(diff)[0]
    ud, _, sd = oracle.solve_batch(prm, w["x0"][idx], w["u_lin"][idx], w["x_ref"][idx], hd[idx], gap_active=True)
    uf, _, sf = oracle.solve_batch(prm, w["x0"][idx], w["u_lin"][idx], w["x_ref"][idx], hf[idx], gap_active=True)
    ok = (sd == oracle.SOLVED) & (sf == oracle.SOLVED)
    e = np.abs(ud[ok] - uf[ok]).max(axis=(1, 2)) / np.maximum(1.0, np.abs(ud[ok]).max(axis=(1, 2)))
    return diff.mean(), int((sd != sf).sum()), float(e.max()) if ok.any() else 0.0


def _fixture_case(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    if name == "c3_gap_n20":  # tests/golden/make_golden.py case(..., seed=104)
        ranges, *geom = workload.make_scans(96, seed=104)
        return d, {k: d[k] for k in ("x0", "u_lin", "x_ref")}, ranges, geom, 20, {}
    src = str(d["source"])  # screen_fuzz_case(seed, case) QPs [...]
    seed, case = (int(v) for v in src[src.index("(") + 1:src.index(")")].split(","))
    idx = np.array(json.loads(src[src.index("["):]))
    N, dt, B, over, wf, ranges, geom = screen_fuzz_case(seed, case)
    return d, {k: wf[k][idx] for k in ("x0", "u_lin", "x_ref")}, ranges[idx], geom, N, dict(dt=dt, **over)


@pytest.mark.parametrize("name", ["c3_gap_n20", "stiff_gap_n33_dt005", "stiff_gap_n48_dt005"])
def test_overload_sensitivity_on_golden_fixtures(oracle, name):
    d, w, ranges, geom, N, over = _fixture_case(name)
    hd, hf = _both(oracle, w["x0"], ranges, geom)
    np.testing.assert_array_equal(hd, d["halfspace"])  # the fixtures hold the double-overload rows
    frac, nstat, du = _compare(oracle, oracle.params(N, **over), w, hd, hf)
    assert 0.2 < frac < 0.7, frac  # the overload is visible in the rows ...
    assert nstat == 0 and du <= 1e-4, (nstat, du)  # ... but not in the verdicts or beyond 1e-4


def test_overload_sensitivity_on_bench_batch(oracle):
    B = 4096
    w = workload.make_batch(B, 20, seed=1000)
    ranges, *geom = workload.make_scans(B, seed=2000)
    hd, hf = _both(oracle, w["x0"], ranges, geom)
    frac, nstat, du = _compare(oracle, oracle.params(20), w, hd, hf)
    assert 0.2 < frac < 0.7 and nstat == 0 and du <= 1e-4, (frac, nstat, du)
