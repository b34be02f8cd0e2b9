"""The interior-point lane kernel for QPs with gap rows (csrc/lane_ipm_kernel.h), selected by an
explicit F110QP_BACKEND_LANE with gap_mode ACTIVE, against the exact oracle through the C ABI.

Same tolerance and status contract as test_gpu_parity.py: identical per-QP status, and
||u - u*||_inf / max(1, ||u*||_inf) <= 1e-4 (same for x) for SOLVED. QPs the interior point does not
polish (infeasible wedges, stalled paths) are handed to the wave kernel's Goldfarb-Idnani loop in
the same call, so the statuses (PRIMAL_INFEASIBLE included) are the wave kernel's.
"""
import numpy as np
import pytest
from test_gpu_parity import check, halfspaces_oracle, rel_err

from f110qp import workload

pytestmark = pytest.mark.gpu


def _lane(capi):
    return dict(backend=capi.BACKEND_LANE)


def test_ipm_is_selected_and_segmented(capi):
    s = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_LANE))
    assert s.backend_info(4096)[0] == capi.BACKEND_LANE
    assert s.lane_segments(4096) == 4
    assert s.lane_segments(1) in (4, 8)
    # beyond the LDS budget the wave kernel keeps the batch
    assert s.backend_info(65536)[0] == capi.BACKEND_WAVE
    s.close()
    s = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE))  # AUTO: wave GI (measured faster)
    assert s.backend_info(4096)[0] == capi.BACKEND_WAVE
    s.close()


def test_ipm_c3_full_batch(oracle, capi):
    """BASELINE configs[2] at its full size on the interior point."""
    B = 4096
    w = workload.make_batch(B, 20, seed=2025)
    ranges, *geom = workload.make_scans(B, seed=2025)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    u, x, st, it = check(oracle, capi, 20, w, hs, gap=True, **_lane(capi))
    assert (st == capi.SOLVED).mean() > 0.99
    # interior-point iterations of the polished QPs (hand-over QPs report GI iterations)
    assert np.median(it[st == capi.SOLVED]) <= 15


@pytest.mark.parametrize("N", [5, 12, 20, 32, 40, 48])
def test_ipm_horizons_gap(oracle, capi, N):
    B = 300
    w = workload.make_batch(B, N, seed=400 + N)
    ranges, *geom = workload.make_scans(B, seed=400 + N)
    check(oracle, capi, N, w, halfspaces_oracle(oracle, w["x0"], ranges, geom), gap=True, **_lane(capi))


def test_ipm_infeasible_and_mixed_batch(oracle, capi):
    """Infeasible wedges go through the hand-over: PRIMAL_INFEASIBLE exactly where the oracle
    proves it, NaN outputs for them, the exact optimum for the rest."""
    from test_oracle import infeasible_cases

    N = 20
    B = 64
    w = workload.make_batch(B, N, seed=5)
    ranges, *geom = workload.make_scans(B, seed=5)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    for i, (x0, h) in enumerate(infeasible_cases()):
        w["x0"][3 + 10 * i] = x0
        w["u_lin"][3 + 10 * i] = [4.5, 0.0]
        hs[3 + 10 * i] = h
    u, x, st, it = check(oracle, capi, N, w, hs, gap=True, **_lane(capi))
    assert (st == capi.PRIMAL_INFEASIBLE).sum() == 2


def test_ipm_non_finite_inputs_are_numerical(oracle, capi):
    N = 20
    B = 48
    w = workload.make_batch(B, N, seed=8)
    ranges, *geom = workload.make_scans(B, seed=8)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    w["x0"][5, 0] = np.nan
    w["x_ref"][9, 3, 1] = np.inf
    s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_LANE))
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    s.close()
    assert st[5] == capi.NUMERICAL and st[9] == capi.NUMERICAL
    assert np.isnan(u[[5, 9]]).all() and np.isnan(x[[5, 9]]).all()
    ok = np.ones(B, bool)
    ok[[5, 9]] = False
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"][ok], w["u_lin"][ok], w["x_ref"][ok], hs[ok],
                                    gap_active=True)
    np.testing.assert_array_equal(st[ok], sr)
    assert rel_err(u[ok], ur).max() <= 1e-4


def test_ipm_objective_matches_oracle(oracle, capi):
    N = 20
    B = 256
    w = workload.make_batch(B, N, seed=31)
    ranges, *geom = workload.make_scans(B, seed=31)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_LANE))
    u, x, st, it, ob, co = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs, objective=True)
    s.close()
    prm = oracle.params(N)
    ur, xr, sr, obr = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True, objective=True)
    np.testing.assert_array_equal(st, sr)
    ok = sr == oracle.SOLVED
    assert np.all(np.abs(ob[ok] - obr[ok]) <= 1e-6 * np.maximum(1.0, np.abs(obr[ok])))
    cr = oracle.tracking_cost(prm, ur, xr, w["x_ref"])
    assert np.all(np.abs(co[ok] - cr[ok]) <= 1e-5 * np.maximum(1.0, cr[ok]))


def test_ipm_agrees_with_wave_gi(capi):
    """Both back ends return the exact optimum of the same QPs: they agree to the tolerance."""
    N = 20
    B = 1024
    w = workload.make_batch(B, N, seed=77, lateral=0.6)
    ranges, amin, ainc, amax = workload.make_scans(B, seed=77)
    hs = np.zeros((B, 2, 3), np.float32)
    for b in range(B):
        hs[b] = capi.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], amin, ainc, amax)
    out = {}
    for name, be in (("lane", capi.BACKEND_LANE), ("wave", capi.BACKEND_WAVE)):
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=be))
        out[name] = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
        s.close()
    np.testing.assert_array_equal(out["lane"][2], out["wave"][2])
    ok = out["wave"][2] == capi.SOLVED
    assert rel_err(out["lane"][0][ok], out["wave"][0][ok].astype(np.float64)).max() <= 1e-4
