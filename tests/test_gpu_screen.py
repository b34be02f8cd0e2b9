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


def test_screen_infeasible_and_non_finite(oracle, capi, monkeypatch):
    """Forced on a small batch (F110QP_GAP_SCREEN=1): infeasible wedges (stage-0 rows violated or
    an empty feasible set) and non-finite inputs pass through to GI and keep their statuses."""
    from test_oracle import infeasible_cases

    monkeypatch.setenv("F110QP_GAP_SCREEN", "1")
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


def test_early_gi_matches_screen_without_it(oracle, capi, monkeypatch):
    """The early GI (predicted-heaviest QPs on the aux stream, concurrently with the box solve)
    changes only when GI starts: the same statuses and optimum as the screen without it
    (F110QP_GAP_EARLY=0), both against the oracle; a small K forces both GI launches to share
    the batch and the re-check list."""
    N, B = 20, 2048
    w, hs = _gap_batch(oracle, B, N, 333, lateral=0.8)
    out = {}
    for name, k in (("off", "0"), ("k16", "16"), ("default", None)):
        if k is None:
            monkeypatch.delenv("F110QP_GAP_EARLY", raising=False)
        else:
            monkeypatch.setenv("F110QP_GAP_EARLY", k)
        out[name] = check(oracle, capi, N, w, hs, gap=True)
    for name in ("k16", "default"):
        np.testing.assert_array_equal(out[name][2], out["off"][2])
        ok = out["off"][2] == capi.SOLVED
        assert rel_err(out[name][0][ok], out["off"][0][ok].astype(np.float64)).max() <= 1e-6


# Known gaps at the stiff corner dt = 0.05, not of the screen (the explicit wave
# back end gives the same answers; tools/screen_case_probe.py SEED CASE):
#   (1, 1) N = 33, q = (10, 17, 0), steering u_des on its upper bound, 1,562 QPs: the wave kernel's
#          GI returns SOLVED for ~6% of the batch with errors up to 3e-2 after 118-214 iterations;
#   (2, 1) N = 48, q = (40, 40, 3), u_des on both lower bounds, 1,283 QPs: 3 QPs the oracle solves
#          stay SOLVED_INACCURATE (GI uncertified, the fp64 re-check does not polish them).
# Kept visible as strict xfails.
FUZZ_KNOWN_GAP = {(1, 1), (2, 1)}


@pytest.mark.parametrize("seed,case", [(s, c) for s in range(3) for c in range(2)])
def test_screen_fuzz_configs_against_oracle(oracle, capi, seed, case, request):
    if (seed, case) in FUZZ_KNOWN_GAP:
        request.applymarker(pytest.mark.xfail(strict=True, reason="stiff-corner GI accuracy gap, DESIGN.md 2h"))
    """The AUTO gap path at screen sizes (1,024..1,600 QPs) over random corners of the ABI's
    parameter space (horizon, dt, weights incl. zero state weights, u_des on a bound, narrow
    bounds): exact status parity with the oracle (QPs it cannot certify excluded, as in
    test_gpu_parity.test_fuzz_configs_against_oracle), the optimum and objective to tolerance."""
    rng = np.random.default_rng(7100 + seed)
    for c in range(case + 1):
        N = int(rng.choice([5, 13, 20, 27, 33, 40, 48]))
        lo0, lo1 = float(rng.uniform(1.0, 3.5)), float(rng.uniform(-0.6, -0.1))
        hi0, hi1 = lo0 + float(rng.uniform(0.3, 2.0)), -lo1 * float(rng.uniform(0.5, 1.5))
        ud = [float(rng.choice([hi0, lo0, 0.5 * (lo0 + hi0)])), float(rng.choice([0.0, hi1, lo1]))]
        q01 = float(rng.choice([0.0, 1.0, 10.0, 40.0]))
        over = dict(q=[q01, q01 if rng.random() < 0.5 else float(rng.uniform(0.5, 20.0)),
                       float(rng.choice([0.0, 0.5, 3.0]))],
                    r=[float(rng.uniform(0.05, 2.0)), float(rng.uniform(0.5, 10.0))], u_des=ud,
                    u_min=[lo0, lo1], u_max=[hi0, hi1])
        dt = float(np.float32(rng.choice([0.005, 0.01, 0.02, 0.05])))
        B = int(rng.integers(1024, 1600))
        w = workload.make_batch(B, N, seed=int(rng.integers(1 << 30)), heading="true",
                                lateral=float(rng.uniform(0.0, 1.5)), steer_range=float(rng.uniform(0.0, 0.8)))
        ranges, amin, ainc, amax = workload.make_scans(B, seed=int(rng.integers(1 << 30)))
        if c < case:
            continue
        hs = halfspaces_oracle(oracle, w["x0"], ranges, (amin, ainc, amax))
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, dt=dt, **over))
        assert s.gap_screen(B)
        u, x, st, it, ob, co = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs, objective=True)
        s.close()
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
