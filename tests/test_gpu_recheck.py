"""Direct parity evidence for the fp64 Goldfarb-Idnani re-check (csrc/gi64_kernel.h, DESIGN.md 2g
step 5): the test build's F110QP_RECHECK_ALL route sends EVERY QP of a gap-row call through the
re-check alone (no box screen, no fp32 GI), so its own answers — SOLVED ones included — are compared
with the oracle's exact optimum of the reference QP (src/mpc.cpp:208-306, gap rows :249,271 with the
C3 semantic :297-298). Tolerance: the north star's 1e-4 relative on u* and x*, identical statuses.
f110qp_last_recheck_count reports how many QPs a call listed (every QP on this route)."""
import json
import os

import numpy as np
import pytest
from conftest import GOLDEN
from test_gpu_parity import TOL, halfspaces_oracle, rel_err

from f110qp import workload

pytestmark = pytest.mark.gpu

GAP_GOLDEN = ["c3_gap_n20", "stiff_gap_n33_dt005", "stiff_gap_n48_dt005"]


def _route(capi, knob, N, **over):
    knob("F110QP_RECHECK_ALL", 1)
    s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, **over))
    assert s.test_build
    return s


@pytest.mark.parametrize("name", GAP_GOLDEN)
def test_recheck_route_golden_fixtures(capi, knob, name):
    """The committed gap-row fixtures (tests/golden/make_golden.py) through the re-check alone."""
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    N = int(d["horizon"])
    over = json.loads(str(d["params"])) if "params" in d.files else {}
    B = d["x0"].shape[0]
    s = _route(capi, knob, N, **over)
    u, x, st, it = s.solve(d["x0"], d["u_lin"], d["x_ref"], d["halfspace"])
    assert s.last_recheck_count() == B
    s.close()
    np.testing.assert_array_equal(st, d["status"])
    ok = d["status"] == capi.SOLVED
    assert ok.any()
    assert rel_err(u[ok], d["u"][ok]).max() <= TOL
    assert rel_err(x[ok], d["x"][ok]).max() <= TOL


def test_recheck_route_c3_bench_batch(oracle, capi, knob):
    """The bench's own C3 batch (4,096 x N = 20, bench.py seeds) through the re-check alone: every
    QP's status and optimum equal to the oracle's; the same batch on the product path lists none."""
    B, N = 4096, 20
    w = workload.make_batch(B, N, seed=1000)
    ranges, *geom = workload.make_scans(B, seed=2000)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    s = _route(capi, knob, N)
    u, x, st, it, ob, co = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs, objective=True)
    assert s.last_recheck_count() == B
    s.close()
    ur, xr, sr, obr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True,
                                         objective=True)
    np.testing.assert_array_equal(st, sr)
    ok = sr == oracle.SOLVED
    assert ok.all()
    assert rel_err(u, ur).max() <= TOL and rel_err(x, xr).max() <= TOL
    np.testing.assert_allclose(ob, obr, rtol=1e-6, atol=1e-6)
    p = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE), test_build=False)
    p.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    assert p.last_recheck_count() == 0
    p.close()


def test_recheck_route_infeasible_and_non_finite(oracle, capi, knob):
    """The re-check's exact verdicts on its own: an empty feasible set (PRIMAL_INFEASIBLE), a
    violated stage-0 row, non-finite data (NUMERICAL), mixed with feasible QPs."""
    from test_oracle import infeasible_cases

    N, B = 20, 64
    w = workload.make_batch(B, N, seed=12)
    ranges, *geom = workload.make_scans(B, seed=12)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    for i, (x0, h) in enumerate(infeasible_cases()):
        w["x0"][3 + 10 * i] = x0
        w["u_lin"][3 + 10 * i] = [4.5, 0.0]
        hs[3 + 10 * i] = h
    a0, b0, c0 = (float(v) for v in hs[40, 0])
    hs[40, 0, 2] = c0 - (a0 * float(w["x0"][40, 0]) + b0 * float(w["x0"][40, 1]) + c0) - 0.5
    s = _route(capi, knob, N)
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True)
    np.testing.assert_array_equal(st, sr)
    assert st[40] == capi.PRIMAL_INFEASIBLE
    ok = sr == oracle.SOLVED
    assert rel_err(u[ok], ur[ok]).max() <= TOL and rel_err(x[ok], xr[ok]).max() <= TOL
    w["x0"][5, 0] = np.nan
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    s.close()
    assert st[5] == capi.NUMERICAL and np.isnan(u[5]).all()


@pytest.mark.parametrize("N", [5, 33, 48])
def test_recheck_route_horizons(oracle, capi, knob, N):
    """Other variable counts of the re-check (NUM = 16, 80, 96 instantiations)."""
    B = 128
    w = workload.make_batch(B, N, seed=700 + N)
    ranges, *geom = workload.make_scans(B, seed=700 + N)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    s = _route(capi, knob, N)
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    s.close()
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True)
    cmp = sr != oracle.UNCERTIFIED
    np.testing.assert_array_equal(st[cmp], sr[cmp])
    ok = sr == oracle.SOLVED
    assert ok.sum() > B // 2
    assert rel_err(u[ok], ur[ok]).max() <= TOL and rel_err(x[ok], xr[ok]).max() <= TOL
