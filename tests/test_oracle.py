"""The CPU oracle against known answers, an independent numpy/scipy pipeline built from the
assembled reference QP, KKT certificates, and the committed golden fixtures."""
import json
import os

import numpy as np
import pytest
from conftest import GOLDEN

from f110qp import workload


def test_linearize_known_answers(oracle):
    # src/model.cpp:30-59, values derived by hand in SURVEY.md §4
    kats = json.load(open(os.path.join(GOLDEN, "linearize_kat.json")))
    for k in kats:
        A, B, C = oracle.linearize(*k["in"])
        assert A[0, 0] == A[1, 1] == A[2, 2] == 1.0
        assert A[2, 0] == A[2, 1] == A[0, 1] == A[1, 0] == 0.0
        for key, v in k["A"].items():
            i, j = map(int, key.split(","))
            assert A[i, j] == pytest.approx(v, abs=1e-12)
        for key, v in k["B"].items():
            i, j = map(int, key.split(","))
            assert B[i, j] == pytest.approx(v, abs=1e-12)
        assert B[0, 1] == B[1, 1] == 0.0
        np.testing.assert_allclose(C, k["C"], atol=1e-12)


def test_simulate_dynamics_matches_workload(oracle):
    # model.cpp:61-75 vs the vectorised generator used for synthetic mini paths
    path = workload.mini_paths(np.array([0.17]))[0]
    s = np.zeros(3)
    for kk in range(1, path.shape[0]):
        s = oracle.simulate_dynamics(s, [4.5, 0.17], 0.01)
        np.testing.assert_allclose(path[kk], s, rtol=0, atol=1e-13)


@pytest.mark.parametrize("N", [1, 5, 20, 30, 40])
def test_dims(oracle, N):
    n, m, nnzP, nnzA = oracle.dims(N)
    assert n == 5 * N + 3 and m == 7 * N + 5  # mpc.cpp:26-29
    assert nnzP == 9 * (N + 1) + 4 * N and nnzA == 26 * N + 9


def _dense(colptr, rowind, val, nrows, ncols):
    M = np.zeros((nrows, ncols))
    for j in range(ncols):
        for p in range(colptr[j], colptr[j + 1]):
            M[rowind[p], j] += val[p]
    return M


def test_assembly_layout(oracle):
    """Appendix A of SURVEY.md: rows/columns of the reference QP (mpc.cpp:208-306)."""
    N = 20
    prm = oracle.params(N)
    w = workload.make_batch(1, N, seed=3)
    hs = np.array([[0.5, -2.0, 1.5], [-1.0, 0.25, 3.0]])
    x0, ul, xr = w["x0"][0].astype(float), w["u_lin"][0].astype(float), w["x_ref"][0].astype(float)
    ns, n, m = 3 * (N + 1), 5 * N + 3, 7 * N + 5
    for gap in (False, True):
        d = oracle.assemble(prm, x0, ul, xr, hs, gap)
        # CSC canonical: sorted unique row indices per column
        for j in range(n):
            rows = d["A_rowind"][d["A_colptr"][j]:d["A_colptr"][j + 1]]
            assert np.all(np.diff(rows) > 0)
        P = _dense(d["P_colptr"], d["P_rowind"], d["P_val"], n, n)
        A = _dense(d["A_colptr"], d["A_rowind"], d["A_val"], m, n)
        np.testing.assert_array_equal(np.diag(P), np.r_[np.tile([10.0, 10.0, 0.0], N + 1), np.tile([0.1, 5.0], N)])
        assert np.count_nonzero(P - np.diag(np.diag(P))) == 0
        Am, Bm, Cm = oracle.linearize(x0[2], ul[0], ul[1])
        np.testing.assert_array_equal(A[0:3, 0:3], -np.eye(3))
        for i in range(1, N + 1):
            np.testing.assert_array_equal(A[3 * i:3 * i + 3, 3 * (i - 1):3 * i], Am)
            np.testing.assert_array_equal(A[3 * i:3 * i + 3, 3 * i:3 * i + 3], -np.eye(3))
            np.testing.assert_array_equal(A[3 * i:3 * i + 3, ns + 2 * (i - 1):ns + 2 * i], Bm)
            np.testing.assert_array_equal(A[ns + 2 * i:ns + 2 * i + 2, 3 * i:3 * i + 3],
                                          [[hs[0, 0], hs[0, 1], 0], [hs[1, 0], hs[1, 1], 0]])
        row0 = A[ns:ns + 2, 0:3]
        if gap:
            np.testing.assert_array_equal(row0, [[hs[0, 0], hs[0, 1], 0], [hs[1, 0], hs[1, 1], 0]])
        else:  # placeholder ones of CreateLinearConstraintMatrix, never updated (mpc.cpp:241,267)
            np.testing.assert_array_equal(row0, np.ones((2, 3)))
        np.testing.assert_array_equal(A[ns + 2 * (N + 1):, ns:], np.eye(2 * N))
        np.testing.assert_array_equal(d["l"][:3], -x0)
        np.testing.assert_array_equal(d["u"][:3], -x0)
        np.testing.assert_array_equal(d["l"][3:ns], np.tile(-Cm, N))
        gl = d["l"][ns:ns + 2 * (N + 1)]
        if gap:
            np.testing.assert_array_equal(gl, np.tile(-hs[:, 2], N + 1))
        else:
            assert np.all(gl == -1e30)
        assert np.all(d["u"][ns:ns + 2 * (N + 1)] == 1e30)
        np.testing.assert_array_equal(d["l"][ns + 2 * (N + 1):], np.tile(np.float32([3.0, -0.43]).astype(float), N))
        np.testing.assert_array_equal(d["u"][ns + 2 * (N + 1):], np.tile(np.float32([4.5, 0.43]).astype(float), N))
        q = d["q"]
        np.testing.assert_array_equal(q[:3 * N], (-np.array([10.0, 10.0, 0.0]) * xr).ravel())
        np.testing.assert_array_equal(q[3 * N:ns], -np.array([10.0, 10.0, 0.0]) * xr[N - 1])  # terminal, mpc.cpp:228
        np.testing.assert_array_equal(q[ns:], np.tile([-0.45, -0.0], N))


def _independent_box_solve(oracle, prm, x0, ul, xr):
    """numpy/scipy pipeline from the assembled sparse QP: eliminate the dynamics rows,
    then bounded least squares (BVLS) on the condensed problem. No oracle solver code."""
    from scipy.optimize import lsq_linear

    N = prm.horizon
    ns, n = 3 * (N + 1), 5 * N + 3
    d = oracle.assemble(prm, x0, ul, xr, None, False)
    P = _dense(d["P_colptr"], d["P_rowind"], d["P_val"], n, n)
    A = _dense(d["A_colptr"], d["A_rowind"], d["A_val"], 7 * N + 5, n)
    E = A[:ns]
    Ex, Eu = E[:, :ns], E[:, ns:]
    G = -np.linalg.solve(Ex, Eu)           # x = G u + f
    f = np.linalg.solve(Ex, d["l"][:ns])
    Z = np.vstack([G, np.eye(2 * N)])
    z0 = np.r_[f, np.zeros(2 * N)]
    H = Z.T @ P @ Z
    g = Z.T @ (P @ z0 + d["q"])
    L = np.linalg.cholesky(H)
    lo, hi = d["l"][ns + 2 * (N + 1):], d["u"][ns + 2 * (N + 1):]
    res = lsq_linear(L.T, -np.linalg.solve(L, g), bounds=(lo, hi), method="bvls", tol=1e-15)
    return res.x.reshape(N, 2)


@pytest.mark.parametrize("N,seed", [(20, 11), (10, 12), (30, 13)])
def test_exact_solve_vs_independent_bvls(oracle, N, seed):
    prm = oracle.params(N)
    w = workload.make_batch(24, N, seed=seed, lateral=0.8)
    for b in range(24):
        r = oracle.solve(prm, w["x0"][b], w["u_lin"][b], w["x_ref"][b])
        assert r["status"] == oracle.SOLVED
        ub = _independent_box_solve(oracle, prm, w["x0"][b].astype(float), w["u_lin"][b].astype(float),
                                    w["x_ref"][b].astype(float))
        np.testing.assert_allclose(r["u"], ub, atol=1e-8)


def _independent_gap_solve(oracle, prm, x0, ul, xr, hs):
    """scipy SLSQP on the condensed form of the assembled sparse QP WITH its gap rows (C3
    semantic): the dynamics rows eliminated from the CSC of oracle.assemble, the box and gap rows
    as linear inequalities on u. No oracle solver code; SLSQP converged to 1e-12 in the objective."""
    from scipy.optimize import minimize

    N = prm.horizon
    ns, n, m = 3 * (N + 1), 5 * N + 3, 7 * N + 5
    d = oracle.assemble(prm, x0, ul, xr, hs, True)
    P = _dense(d["P_colptr"], d["P_rowind"], d["P_val"], n, n)
    A = _dense(d["A_colptr"], d["A_rowind"], d["A_val"], m, n)
    E = A[:ns]
    Ex, Eu = E[:, :ns], E[:, ns:]
    G = -np.linalg.solve(Ex, Eu)
    f = np.linalg.solve(Ex, d["l"][:ns])
    Z = np.vstack([G, np.eye(2 * N)])
    z0 = np.r_[f, np.zeros(2 * N)]
    H = Z.T @ P @ Z
    g = Z.T @ (P @ z0 + d["q"])
    Ar, lo, hi = A[ns:] @ Z, d["l"][ns:] - A[ns:] @ z0, d["u"][ns:] - A[ns:] @ z0
    fin_lo, fin_hi = lo > -1e29, hi < 1e29
    cons = [{"type": "ineq", "fun": lambda u, M=Ar[fin_lo], c=lo[fin_lo]: M @ u - c, "jac": lambda u, M=Ar[fin_lo]: M},
            {"type": "ineq", "fun": lambda u, M=Ar[fin_hi], c=hi[fin_hi]: c - M @ u, "jac": lambda u, M=Ar[fin_hi]: -M}]
    u0 = np.clip(np.linalg.solve(H, -g), np.tile([3.0, -0.43], N), np.tile([4.5, 0.43], N))
    res = minimize(lambda u: 0.5 * u @ H @ u + g @ u, u0, jac=lambda u: H @ u + g, constraints=cons,
                   method="SLSQP", options={"ftol": 1e-14, "maxiter": 1000})
    assert res.success, res.message
    return res.x.reshape(N, 2)


def test_exact_gap_solve_vs_independent_slsqp(oracle):
    """The oracle's exact solve of the gap-row QP (C3 semantic) against an independent general
    QP solve (scipy SLSQP) of the reference's own assembled sparse QP: the two agree to 1e-6
    (SLSQP's accuracy), on instances with active gap rows."""
    N = 20
    prm = oracle.params(N)
    B = 24
    w = workload.make_batch(B, N, seed=1000)
    ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
    active = 0
    for b in range(B):
        rc, l1, l2, _, _ = oracle.find_half_spaces(w["x0"][b], ranges[b], amin, ainc, amax)
        hs = np.array([l1, l2])
        r = oracle.solve(prm, w["x0"][b], w["u_lin"][b], w["x_ref"][b], hs, True)
        assert r["status"] == oracle.SOLVED
        u = _independent_gap_solve(oracle, prm, w["x0"][b].astype(float), w["u_lin"][b].astype(float),
                                   w["x_ref"][b].astype(float), hs)
        np.testing.assert_allclose(r["u"], u, atol=1e-6)
        y = r["y"][3 * (N + 1):3 * (N + 1) + 2 * (N + 1)]
        active += int((np.abs(y) > 1e-9).any())
    assert active >= B // 4  # the sample exercises active gap rows


@pytest.mark.parametrize("gap", [False, True])
def test_kkt_certificate(oracle, gap):
    N = 20
    prm = oracle.params(N)
    B = 64
    w = workload.make_batch(B, N, seed=21 + gap)
    hs = None
    if gap:
        ranges, amin, ainc, amax = workload.make_scans(B, seed=5)
        hs = np.zeros((B, 2, 3))
        for b in range(B):
            rc, l1, l2, _, _ = oracle.find_half_spaces(w["x0"][b], ranges[b], amin, ainc, amax)
            hs[b] = l1, l2
    for b in range(B):
        h = None if hs is None else hs[b]
        r = oracle.solve(prm, w["x0"][b], w["u_lin"][b], w["x_ref"][b], h, gap)
        assert r["status"] == oracle.SOLVED
        res = oracle.kkt_residuals(prm, w["x0"][b], w["u_lin"][b], w["x_ref"][b], r["z"], r["y"], h, gap)
        assert res.max() < 1e-9, res
        # the dynamics are satisfied exactly by x* (equality rows of the reference QP)
        Am, Bm, Cm = oracle.linearize(*w["x0"][b][2:3], *w["u_lin"][b])
        for i in range(N):
            np.testing.assert_allclose(r["x"][i + 1], Am @ r["x"][i] + Bm @ r["u"][i] + Cm, atol=1e-12)


def test_gi_active_set_full_rank(oracle):
    """Gap rows + u_des on the speed bound: the GI active set reaches n = 2N rows (QPs 92, 99,
    160, 214 of this batch). A further row is then dependent by construction; the oracle once
    added it on a rounding-level pivot and overran its n-slot state (heap corruption)."""
    rng = np.random.default_rng(7000)
    N = int(rng.choice([1, 2, 5, 13, 20, 27, 33, 40, 48]))
    lo0, lo1 = float(rng.uniform(1.0, 3.5)), float(rng.uniform(-0.6, -0.1))
    hi0, hi1 = lo0 + float(rng.uniform(0.3, 2.0)), -lo1 * float(rng.uniform(0.5, 1.5))
    ud = [float(rng.choice([hi0, lo0, 0.5 * (lo0 + hi0)])), float(rng.choice([0.0, hi1, lo1]))]
    q01 = float(rng.choice([0.0, 1.0, 10.0, 40.0]))
    over = dict(q=[q01, q01 if rng.random() < 0.5 else float(rng.uniform(0.5, 20.0)), float(rng.choice([0.0, 0.5, 3.0]))],
                r=[float(rng.uniform(0.05, 2.0)), float(rng.uniform(0.5, 10.0))], u_des=ud, u_min=[lo0, lo1],
                u_max=[hi0, hi1])
    dt = float(np.float32(rng.choice([0.005, 0.01, 0.02, 0.05])))
    assert N == 33 and rng.random() < 0.4  # the gap draw of this seed
    B = 256
    w = workload.make_batch(B, N, seed=int(rng.integers(1 << 30)), heading="true",
                            lateral=float(rng.uniform(0.0, 1.5)), steer_range=float(rng.uniform(0.0, 0.8)))
    ranges, amin, ainc, amax = workload.make_scans(B, seed=int(rng.integers(1 << 30)))
    prm = oracle.params(N, dt=dt, **over)
    full = 0
    for b in (92, 99, 160, 214, 0):
        rc, l1, l2, _, _ = oracle.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], amin, ainc, amax)
        h = np.array([l1, l2], np.float32).astype(np.float64)
        args = (prm, w["x0"][b].astype(np.float64), w["u_lin"][b].astype(np.float64), w["x_ref"][b].astype(np.float64), h)
        r = oracle.solve(*args, True)
        assert r["n_active"] <= 2 * N
        full += r["n_active"] == 2 * N
        # feasibility of the assembled QP by an independent LP (HiGHS)
        feasible = _lp_feasible(oracle.assemble(*args, True))
        if feasible:
            assert r["status"] == oracle.SOLVED
            assert oracle.kkt_residuals(*args[:4], r["z"], r["y"], h, True).max() < 1e-8
        else:
            # infeasible; 214 ends GI on a point outside the box: reported uncertified, not SOLVED
            assert r["status"] in (oracle.PRIMAL_INFEASIBLE, oracle.UNCERTIFIED), (b, r["status"])
    assert full >= 3


def _lp_feasible(A):
    import scipy.sparse as sp
    from scipy.optimize import linprog

    n, m = len(A["q"]), len(A["l"])
    Am = sp.csc_matrix((A["A_val"], A["A_rowind"], A["A_colptr"]), shape=(m, n)).toarray()
    fl, fu = A["l"] > -1e29, A["u"] < 1e29
    res = linprog(np.zeros(n), A_ub=np.vstack([Am[fu], -Am[fl]]), b_ub=np.concatenate([A["u"][fu], -A["l"][fl]]),
                  bounds=(None, None), method="highs")
    assert res.status in (0, 2), res.message
    return res.status == 0


def infeasible_cases():
    """(x0, hs) pairs with no feasible input sequence.
    1. a wall 0.5 m ahead along the heading (x <= x0 + 0.5, unit normal): at v >= 3 m/s the
       car covers 0.6 m within 20 steps of 0.01 s -> the later stages are infeasible;
    2. the stage-0 row itself violated (x0 outside the wedge)."""
    x0 = np.array([1.0, 2.0, 0.0])
    wall = np.array([[-1.0, 0.0, x0[0] + 0.5], [-1.0, 0.0, x0[0] + 0.5]])
    behind = np.array([[-1.0, 0.0, 0.7], [0.0, 1.0, -2.0 + 0.5]])
    return [(x0, wall), (x0, behind)]


def test_infeasible_gap_detected(oracle):
    N = 20
    prm = oracle.params(N)
    w = workload.make_batch(1, N, seed=1)
    for x0, hs in infeasible_cases():
        r = oracle.solve(prm, x0, [4.5, 0.0], w["x_ref"][0], hs, True)
        assert r["status"] == oracle.PRIMAL_INFEASIBLE
        assert np.isnan(r["u"]).all()
    # the same wall 1 m ahead is reachable (stop short at v = 3 m/s)
    x0, hs = infeasible_cases()[0]
    hs = hs.copy()
    hs[:, 2] = x0[0] + 1.0
    r = oracle.solve(prm, x0, [4.5, 0.0], w["x_ref"][0], hs, True)
    assert r["status"] == oracle.SOLVED


def _scan(n=1080, fill=1.0):
    amin = np.float32(-np.pi)
    ainc = np.float32(2 * np.pi / n)
    amax = np.float32(amin + ainc * (n - 1))
    return np.full(n, fill, np.float32), amin, ainc, amax


def _window(amin, ainc, n):
    ang = (amin + np.arange(n, dtype=np.float32) * ainc).astype(np.float32)
    lim = np.float32(1.571) / np.float32(1.5)
    return np.where((ang > -lim) & (ang < lim))[0]


def test_find_half_spaces_quirks(oracle, capi):
    """constraints.cpp:116-265 quirks, checked on the oracle and bit-exactly against the
    product's host implementation (f110qp_find_half_spaces)."""
    r, amin, ainc, amax = _scan()
    win = _window(amin, ainc, len(r))
    x0 = np.array([3.0, -4.0, 0.3])

    def both(ranges):
        rc, l1, l2, lo, hi = oracle.find_half_spaces(x0, ranges, amin, ainc, amax)
        if rc == 0:
            p1, p2 = capi.find_half_spaces(x0, ranges, amin, ainc, amax)
            np.testing.assert_array_equal(p1, l1)
            np.testing.assert_array_equal(p2, l2)
        else:
            with pytest.raises(capi.F110QPError):
                capi.find_half_spaces(x0, ranges, amin, ainc, amax)
        return rc, l1, l2, lo, hi

    # a plain gap of 21 beams -> shrunk by buffer=3 on both sides
    g = r.copy()
    g[win[100]:win[121]] = 6.0
    rc, l1, l2, lo, hi = both(g)
    assert rc == 0 and (lo, hi) == (win[100] + 3, win[120] - 3)
    # the wider of two gaps wins; on a tie the earlier one
    g2 = r.copy()
    g2[win[10]:win[20]] = 6.0
    g2[win[50]:win[60]] = 7.0
    rc, _, _, lo, hi = both(g2)
    assert (lo, hi) == (win[10] + 3, win[19] - 3)
    # single-beam gaps are never recorded (stale `hi`): window opens short -> (-1,-1) quirk
    g3 = r.copy()
    g3[win[5]] = 6.0
    g3[win[40]] = 6.0
    rc, _, _, lo, hi = both(g3)
    assert rc == -1 and (lo, hi) == (-1, -1)
    # window opening on a long single beam and nothing else: best stays (0, 0)
    g4 = r.copy()
    g4[win[0]] = 6.0
    rc, _, _, lo, hi = both(g4)
    assert (lo, hi) == (0, 0) and rc == 0
    # gaps outside the +-1.571/1.5 window are ignored
    g5 = r.copy()
    g5[: win[0]] = 9.0
    g5[win[200]:win[230]] = 5.0
    rc, _, _, lo, hi = both(g5)
    assert (lo, hi) == (win[200] + 3, win[229] - 3)
    # a gap narrower than 2*buffer is not shrunk
    g6 = r.copy()
    g6[win[70]:win[75]] = 5.0
    rc, _, _, lo, hi = both(g6)
    assert (lo, hi) == (win[70], win[74])
    # both lines pass through the car position (c chosen from p), normals point into the gap
    assert abs(l1[0] * x0[0] + l1[1] * x0[1] + (l1[2] - 0.5)) < 1e-3
    assert abs(l2[0] * x0[0] + l2[1] * x0[1] + (l2[2] - 0.5)) < 1e-3


def test_find_half_spaces_synthetic_host_equals_oracle(oracle, capi):
    B = 64
    w = workload.make_batch(B, 20, seed=31)
    ranges, amin, ainc, amax = workload.make_scans(B, seed=31)
    for b in range(B):
        rc, l1, l2, lo, hi = oracle.find_half_spaces(w["x0"][b].astype(float), ranges[b], amin, ainc, amax)
        assert rc == 0
        p1, p2 = capi.find_half_spaces(w["x0"][b].astype(float), ranges[b], amin, ainc, amax)
        np.testing.assert_array_equal(p1, l1)
        np.testing.assert_array_equal(p2, l2)


GOLDEN_CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_reproduces_golden(oracle, name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    N = int(d["horizon"])
    gap = bool(d["gap"])
    hs = d["halfspace"] if gap else None
    over = json.loads(str(d["params"])) if "params" in d.files else {}  # stiff-corner fixtures
    u, x, st = oracle.solve_batch(oracle.params(N, **over), d["x0"], d["u_lin"], d["x_ref"], hs, gap_active=gap)
    np.testing.assert_array_equal(st, d["status"])
    np.testing.assert_allclose(u, d["u"], rtol=0, atol=1e-10)
    np.testing.assert_allclose(x, d["x"], rtol=0, atol=1e-10)
    if gap and "scan_geom" in d.files:
        geom = d["scan_geom"]
        for b in range(d["scan_ranges"].shape[0]):
            rc, l1, l2, lo, hi = oracle.find_half_spaces(d["x0"][b].astype(float), d["scan_ranges"][b], *geom)
            assert (lo, hi) == tuple(d["scan_lohi"][b])
            np.testing.assert_array_equal(np.float32([l1, l2]), d["halfspace"][b])


def test_osqp_admm_restatement(oracle):
    """oracle/osqp_admm.c (the CPU baseline, OSQP 0.6 defaults restated) converges to the exact
    optimum when the tolerances are tightened, and solves every QP at the defaults."""
    N, B = 20, 64
    w = workload.make_batch(B, N, seed=41)
    prm = oracle.params(N)
    u, x, st = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"])
    ua, sa, ia = oracle.admm_solve_batch(prm, oracle.admm_settings(), w["x0"], w["u_lin"], w["x_ref"])
    assert (sa == oracle.SOLVED).all() and ia.max() <= 4000
    tight = oracle.admm_settings(eps_abs=1e-10, eps_rel=1e-10, max_iter=200000)
    ua, sa, ia = oracle.admm_solve_batch(prm, tight, w["x0"], w["u_lin"], w["x_ref"])
    assert (sa == oracle.SOLVED).all()
    np.testing.assert_allclose(ua, u, atol=1e-5)
