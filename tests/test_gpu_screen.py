"""The gap-row box screen (f110qp_kernels.hip gap_screen_kernel): AUTO gap calls of >= 1,024 QPs
solve the box-only problem on the lane back end and send to the wave kernel's GI only the QPs
whose box optimum leaves a gap row violated or within the margin. Same contract as
test_gpu_parity.py against the oracle: identical status per QP, and ||u - u*||_inf /
max(1, ||u*||_inf) <= 1e-4 (same for x) for SOLVED.
"""
import numpy as np
import pytest
from test_gpu_parity import check, halfspaces_oracle, rel_err

from f110qp import workload
from fuzz_cases import screen_fuzz_case

pytestmark = pytest.mark.gpu


def _gap_batch(oracle, B, N, seed, **kw):
    w = workload.make_batch(B, N, seed=seed, **kw)
    ranges, *geom = workload.make_scans(B, seed=seed)
    return w, halfspaces_oracle(oracle, w["x0"], ranges, geom)


def test_screen_c3_full_batch(oracle, capi):
    """BASELINE configs[2] (4,096 x N = 20 with gap rows) on the AUTO path, which screens."""
    s = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE))
    assert s.gap_screen(4096)
    s.close()
    w, hs = _gap_batch(oracle, 4096, 20, 2025)
    u, x, st, it = check(oracle, capi, 20, w, hs, gap=True)
    assert (st == capi.SOLVED).mean() > 0.99


@pytest.mark.parametrize("N", [5, 13, 30, 40, 48])
def test_screen_horizons(oracle, capi, N):
    w, hs = _gap_batch(oracle, 1024, N, 600 + N)
    check(oracle, capi, N, w, hs, gap=True)


def test_screen_agrees_with_wave_only(oracle, capi):
    """Screened and unscreened (explicit wave back end) runs of one batch: same statuses, the same
    optimum to the tolerance."""
    N, B = 20, 2048
    w, hs = _gap_batch(oracle, B, N, 91, lateral=0.8)
    out = {}
    for name, be in (("auto", capi.BACKEND_AUTO), ("wave", capi.BACKEND_WAVE)):
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=be))
        out[name] = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
        s.close()
    np.testing.assert_array_equal(out["auto"][2], out["wave"][2])
    ok = out["wave"][2] == capi.SOLVED
    assert rel_err(out["auto"][0][ok], out["wave"][0][ok].astype(np.float64)).max() <= 1e-4


def test_screen_infeasible_and_non_finite(oracle, capi, knob, monkeypatch):
    """Forced on a small batch (F110QP_GAP_SCREEN=1): infeasible wedges (stage-0 rows violated or
    an empty feasible set) and non-finite inputs pass through to GI and keep their statuses."""
    from test_oracle import infeasible_cases

    knob("F110QP_GAP_SCREEN", "1")
    N, B = 20, 96
    w, hs = _gap_batch(oracle, B, N, 12)
    for i, (x0, h) in enumerate(infeasible_cases()):
        w["x0"][3 + 10 * i] = x0
        w["u_lin"][3 + 10 * i] = [4.5, 0.0]
        hs[3 + 10 * i] = h
    a0, b0, c0 = (float(v) for v in hs[40, 0])  # x0 0.5 outside the first half-space: stage-0 row violated
    hs[40, 0, 2] = c0 - (a0 * float(w["x0"][40, 0]) + b0 * float(w["x0"][40, 1]) + c0) - 0.5
    s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE))
    assert s.gap_screen(B)
    s.close()
    u, x, st, it = check(oracle, capi, N, w, hs, gap=True)
    assert st[40] == capi.PRIMAL_INFEASIBLE
    w["x0"][5, 0] = np.nan
    hs[9, 1, 1] = np.inf
    out = {}
    for name, be in (("auto", capi.BACKEND_AUTO), ("wave", capi.BACKEND_WAVE)):
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=be))
        out[name] = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
        s.close()
    st = out["auto"][2]
    # non-finite state: NUMERICAL; a non-finite gap row: the wave kernel's empty-set verdict
    assert st[5] == capi.NUMERICAL and st[9] == capi.PRIMAL_INFEASIBLE
    np.testing.assert_array_equal(st, out["wave"][2])


# The stiff corners at dt = 0.05 (round 4's strict xfails, now plain cases): (1, 1) N = 33,
# q = (10, 17, 0), steering u_des on its upper bound, where the wave kernel's fp32 GI ended at wrong
# points its old multiplier test let through; (2, 1) N = 48, q = (40, 40, 3), u_des on both lower
# bounds, where it could not certify three QPs. The fp64 certificate sends both kinds to the fp64
# GI re-check (gi64_kernel.h).
STIFF_CASES = ((1, 1), (2, 1))


@pytest.mark.parametrize("seed,case", [(s, c) for s in range(3) for c in range(2)])
def test_screen_fuzz_configs_against_oracle(oracle, capi, seed, case):
    """The AUTO gap path at screen sizes (1,024..1,600 QPs) over random corners of the ABI's
    parameter space (horizon, dt, weights incl. zero state weights, u_des on a bound, narrow
    bounds): exact status parity with the oracle (QPs it cannot certify excluded, as in
    test_gpu_parity.test_fuzz_configs_against_oracle), the optimum and objective to tolerance."""
    N, dt, B, over, w, ranges, geom = screen_fuzz_case(seed, case)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, dt=dt, **over))
    assert s.gap_screen(B)
    u, x, st, it, ob, co = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs, objective=True)
    rc = s.last_recheck_count()
    s.close()
    if (seed, case) in STIFF_CASES:  # the fp64 re-check takes what fp32 GI cannot certify here
        assert rc > 0, (seed, case, rc)
    prm = oracle.params(N, dt=dt, **over)
    ur, xr, sr, obr = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True,
                                         objective=True)
    tag = (seed, case, N, dt, B, over)
    cmp = sr != oracle.UNCERTIFIED
    assert (sr == oracle.UNCERTIFIED).sum() <= max(1, 0.02 * B), tag
    np.testing.assert_array_equal(st[cmp], sr[cmp], err_msg=str(tag))
    ok = sr == oracle.SOLVED
    if ok.any():
        assert rel_err(u[ok], ur[ok]).max() <= 1e-4, tag
        assert rel_err(x[ok], xr[ok]).max() <= 1e-4, tag
        np.testing.assert_allclose(ob[ok], obr[ok], rtol=1e-6, atol=1e-6, err_msg=str(tag))


@pytest.mark.parametrize("backend", ["auto", "wave"])
def test_recheck_processes_every_listed_qp(oracle, capi, backend):
    """More QPs than one re-check grid holds go to the fp64 re-check (4,608 walls the fp32 GI finds
    infeasible, mixed with feasible ones): every listed QP is re-checked (the grid-stride loop over
    the device-side count), so the statuses are the oracle's whatever the list order, and two calls
    agree bit for bit."""
    from test_oracle import infeasible_cases

    N, B = 20, 5120
    w = workload.make_batch(B, N, seed=77)
    x0w, wall = infeasible_cases()[0]
    hs = np.zeros((B, 2, 3), np.float32)
    feas = np.arange(B) % 10 == 0  # the wall 1 m ahead: reachable
    for b in range(B):
        w["x0"][b] = x0w
        w["u_lin"][b] = [4.5, 0.0]
        hs[b] = wall
        if feas[b]:
            hs[b, :, 2] = x0w[0] + 1.0
    be = {"auto": capi.BACKEND_AUTO, "wave": capi.BACKEND_WAVE}[backend]
    s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=be))
    u1, x1, st1, _ = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    u2, x2, st2, _ = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    s.close()
    assert (st1[~feas] == capi.PRIMAL_INFEASIBLE).all()
    np.testing.assert_array_equal(st1, st2)
    np.testing.assert_array_equal(np.nan_to_num(u1, nan=7.0), np.nan_to_num(u2, nan=7.0))
    idx = np.r_[np.where(feas)[0][:32], np.where(~feas)[0][:32]]
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"][idx], w["u_lin"][idx], w["x_ref"][idx], hs[idx],
                                    gap_active=True)
    np.testing.assert_array_equal(st1[idx], sr)
    ok = sr == oracle.SOLVED
    assert rel_err(u1[idx][ok], ur[ok]).max() <= 1e-4
