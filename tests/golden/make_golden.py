"""Regenerate the committed golden fixtures (data only: inputs + expected outputs).

    python tests/golden/make_golden.py

The reference (smitdumore/f110-mpc) ships no tests, fixtures or solver outputs and cannot be
built here, so the expected outputs come from the CPU oracle (oracle/f110_oracle.c): the exact
optimum of the reference's own QP (src/mpc.cpp:208-306), each one certified by a KKT check on
the assembled sparse problem before it is written. Linearize known answers are derived from
src/model.cpp:30-59 by hand and are checked against the oracle here too.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
from f110qp import workload  # noqa: E402
from fuzz_cases import screen_fuzz_case  # noqa: E402

# (theta, v, delta) -> entries, SURVEY.md §4 item 1 (float64 with dt = 0.01f, L = 0.3302f)
LINEARIZE_KAT = [
    {"in": [0.0, 4.5, 0.0], "A": {"0,2": -0.0, "1,2": 0.0449999989942},
     "B": {"0,0": 0.00999999977648, "2,1": 0.136281044237}, "C": [0.0, -0.0, -0.0]},
    {"in": [0.5, 4.5, 0.2], "A": {"0,2": -0.021574148755, "1,2": 0.0394912144024},
     "B": {"0,0": 0.00877582542275, "1,0": 0.00479425527888, "2,0": 0.00613900784812, "2,1": 0.141881017482},
     "C": [0.0107870743775, -0.0197456072012, -0.0283762034965]},
    {"in": [-2.0, 4.5, -0.43], "A": {"0,2": 0.0409183832926, "1,2": -0.018726607226},
     "B": {"0,0": -0.00416146827246, "1,0": -0.00909297406501, "2,0": -0.0138891893311, "2,1": 0.164945478256},
     "C": [0.0818367665851, -0.0374532144521, 0.0709265556502]},
]


def halfspaces(w, seed, B):
    ranges, amin, ainc, amax = workload.make_scans(B, seed=seed)
    hs = np.zeros((B, 2, 3), np.float32)
    lohi = np.zeros((B, 2), np.int32)
    for b in range(B):
        rc, l1, l2, lo, hi = oracle.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], amin, ainc, amax)
        assert rc == 0
        hs[b, 0], hs[b, 1] = l1, l2
        lohi[b] = lo, hi
    return hs, ranges, np.array([amin, ainc, amax], np.float32), lohi


def certify(prm, w, hs, gap, u, st, tol=1e-8):
    for b in range(len(st)):
        if st[b] != oracle.SOLVED:
            continue
        r = oracle.solve(prm, w["x0"][b], w["u_lin"][b], w["x_ref"][b], None if hs is None else hs[b], gap)
        res = oracle.kkt_residuals(prm, w["x0"][b], w["u_lin"][b], w["x_ref"][b], r["z"], r["y"],
                                   None if hs is None else hs[b], gap)
        assert res.max() < tol, (b, res)
        assert np.abs(r["u"] - u[b]).max() == 0.0


def case(name, N, B, seed, gap=False, heading="zero", lateral=0.3):
    w = workload.make_batch(B, N, seed=seed, heading=heading, lateral=lateral)
    prm = oracle.params(N)
    hs = None
    extra = {}
    if gap:
        hs, ranges, geom, lohi = halfspaces(w, seed, B)
        extra = dict(halfspace=hs, scan_ranges=ranges[:8], scan_geom=geom, scan_lohi=lohi[:8])
    u, x, st = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=gap)
    certify(prm, w, hs, gap, u, st)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), horizon=N, gap=int(gap), x0=w["x0"], u_lin=w["u_lin"],
                        x_ref=w["x_ref"], u=u, x=x, status=st, **extra)
    print(name, "B", B, "N", N, "status", dict(zip(*np.unique(st, return_counts=True))))


def stiff_case(name, seed, case_, n_hard=48, n_rand=48):
    """A slice of one screen-size fuzz case (tests/fuzz_cases.py; the round-4 stiff corners at
    dt = 0.05): the n_hard QPs with the most active rows at the oracle's optimum (the long GI chains)
    and n_rand others, QPs the oracle cannot certify left out. The configuration travels with the
    fixture (params: dt, q, r, u_des, u_min, u_max)."""
    N, dt, B, over, w, ranges, geom = screen_fuzz_case(seed, case_)
    hs = np.zeros((B, 2, 3), np.float32)
    for b in range(B):
        rc, l1, l2, _, _ = oracle.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], *geom)
        assert rc == 0
        hs[b] = l1, l2
    prm = oracle.params(N, dt=dt, **over)
    nact = np.zeros(B, np.int64)
    stat = np.zeros(B, np.int64)
    for b in range(B):
        r = oracle.solve(prm, w["x0"][b], w["u_lin"][b], w["x_ref"][b], hs[b], True)
        nact[b], stat[b] = r["n_active"], r["status"]
    cand = np.where(stat != oracle.UNCERTIFIED)[0]
    hard = cand[np.argsort(-nact[cand], kind="stable")[:n_hard]]
    rest = np.setdiff1d(cand, hard)
    rand = np.sort(np.random.default_rng(seed).choice(rest, size=min(n_rand, len(rest)), replace=False))
    idx = np.sort(np.r_[hard, rand])
    ws = {k: np.ascontiguousarray(w[k][idx]) for k in ("x0", "u_lin", "x_ref")}
    hsi = np.ascontiguousarray(hs[idx])
    u, x, st = oracle.solve_batch(prm, ws["x0"], ws["u_lin"], ws["x_ref"], hsi, gap_active=True)
    certify(prm, ws, hsi, True, u, st, tol=1e-5)  # absolute, against dual terms q x_ref ~ 2e3 (q = 40, |x| ~ 50 m)
    params = dict(dt=dt, **over)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), horizon=N, gap=1, x0=ws["x0"], u_lin=ws["u_lin"],
                        x_ref=ws["x_ref"], u=u, x=x, status=st, halfspace=hsi, params=json.dumps(params),
                        source=f"tests/fuzz_cases.py screen_fuzz_case({seed}, {case_}) QPs {idx.tolist()}")
    print(name, "B", len(idx), "N", N, "dt", dt, "status", dict(zip(*np.unique(st, return_counts=True))),
          "max active", int(nact[hard].max()))


def main():
    for k in LINEARIZE_KAT:
        A, B, C = oracle.linearize(*k["in"])
        for key, v in k["A"].items():
            i, j = map(int, key.split(","))
            assert abs(A[i, j] - v) < 1e-12, (k, key)
        for key, v in k["B"].items():
            i, j = map(int, key.split(","))
            assert abs(B[i, j] - v) < 1e-12, (k, key)
        assert np.abs(C - np.array(k["C"])).max() < 1e-12
    with open(os.path.join(HERE, "linearize_kat.json"), "w") as f:
        json.dump(LINEARIZE_KAT, f, indent=1)
    case("c1_single_n20", 20, 1, seed=101)
    case("c2_box_n20", 20, 96, seed=102)
    case("c2_box_n20_heading", 20, 48, seed=103, heading="true", lateral=0.6)
    case("c3_gap_n20", 20, 96, seed=104, gap=True)
    case("box_n30_default_horizon", 30, 48, seed=105)
    case("box_n5", 5, 48, seed=106)
    case("box_n32", 32, 32, seed=107, lateral=0.8)
    stiff_case("stiff_gap_n33_dt005", 1, 1)
    stiff_case("stiff_gap_n48_dt005", 2, 1)


if __name__ == "__main__":
    main()
