"""Parity of the device planning stage (plan_kernels.hip, through the C ABI) with the CPU
oracle (oracle/plan_oracle.c): grids, candidate validity, waypoint / candidate indices, x_ref
and x0 must be bit-identical (integer, index and float32 outputs of the reference's float and
double expressions). Then the end-to-end tick: plan on the device -> QP batch on the device."""
import numpy as np
import pytest

from f110qp import capi, workload

pytestmark = pytest.mark.gpu


def run_plan_dev(cuda, cfg, sc, table, want_grid=True):
    import torch

    B = sc["pose"].shape[0]
    T, P = table.shape[:2]
    G = capi.grid_blocks(cfg)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).to(cuda)  # noqa: E731
    pose, ranges = t(sc["pose"], np.float64), t(sc["ranges"], np.float32)
    tab, wp = t(table, np.float64), t(sc["waypoints"][:, :2], np.float64)
    out = dict(x_ref=torch.empty((B, P, 3), dtype=torch.float32, device=cuda),
               x0=torch.empty((B, 3), dtype=torch.float32, device=cuda),
               best_traj=torch.empty(B, dtype=torch.int32, device=cuda),
               best_global=torch.empty(B, dtype=torch.int32, device=cuda),
               status=torch.empty(B, dtype=torch.int32, device=cuda),
               valid=torch.empty((B, T), dtype=torch.uint8, device=cuda),
               grid=torch.empty((B, G, G), dtype=torch.uint8, device=cuda) if want_grid else None)
    capi.plan_batch_dev(cfg, pose, ranges, sc["angle_min"], sc["angle_inc"], sc["angle_max"], tab, wp, out["x_ref"],
                        out["x0"], out["best_traj"], out["best_global"], out["status"], valid=out["valid"],
                        grid=out["grid"])
    torch.cuda.synchronize()
    return {k: (v.cpu().numpy() if v is not None else None) for k, v in out.items()}


def check_against_oracle(oracle, pp, sc, table, dev, nmax=None):
    B = sc["pose"].shape[0] if nmax is None else nmax
    for b in range(B):
        g, off = oracle.fill_occ_grid(pp, sc["pose"][b], sc["ranges"][b], sc["angle_min"], sc["angle_inc"],
                                      sc["angle_max"])
        if dev["grid"] is not None:
            np.testing.assert_array_equal(dev["grid"][b], g, err_msg=f"grid {b}")
        r = oracle.plan(pp, sc["pose"][b], g, off, table, sc["waypoints"])
        np.testing.assert_array_equal(dev["valid"][b], r["valid"], err_msg=f"valid {b}")
        assert dev["status"][b] == r["status"], b
        assert dev["best_traj"][b] == r["best_traj"], b
        if r["status"] == 0:
            assert dev["best_global"][b] == r["best_global"], b
            np.testing.assert_array_equal(dev["x_ref"][b], r["x_ref"], err_msg=f"x_ref {b}")
        np.testing.assert_array_equal(dev["x0"][b], r["x0"])


def test_plan_matches_oracle_bit_exact(oracle, cuda):
    sc = workload.make_scenes(512, seed=21)
    pp = oracle.plan_params()
    cfg = capi.default_plan_config()
    table = capi.traj_table(cfg)
    dev = run_plan_dev(cuda, cfg, sc, table)
    check_against_oracle(oracle, pp, sc, table, dev)
    assert (dev["status"] == 0).mean() > 0.8 and dev["grid"].sum() > 0


def test_plan_other_parameters(oracle, cuda):
    """Non-default grid (8 m at 0.05 m: 160 x 160 cells, dilation 0.1), 21 candidates of 30
    points, lookahead 2.0."""
    over = dict(size=8, discrete=np.float32(0.05), dilation=np.float32(0.1), lookahead=np.float32(2.0),
                steer_discrete=20, traj_discrete=30)
    sc = workload.make_scenes(128, seed=22)
    pp = oracle.plan_params(**over)
    cfg = capi.default_plan_config(**over)
    table = capi.traj_table(cfg)
    np.testing.assert_array_equal(table, oracle.traj_table(pp))
    dev = run_plan_dev(cuda, cfg, sc, table)
    assert dev["grid"].shape[1] == 160
    check_against_oracle(oracle, pp, sc, table, dev)


def test_plan_edge_scans(oracle, cuda):
    """inf / NaN / zero ranges (x86 cvtt semantics of the float->int cell index), a scan that
    blocks every candidate (status 1: the reference returns before MPC), and a car facing away
    from a short path (status 2: no waypoint ahead)."""
    sc = workload.make_scenes(16, seed=23)
    r = sc["ranges"]
    r[0, ::7] = np.inf
    r[1, ::5] = np.nan
    r[2, :] = 0.0
    r[3, :] = 0.5                      # a ring of obstacles at 0.5 m: nothing is valid
    pose = sc["pose"].copy()
    pp = oracle.plan_params()
    cfg = capi.default_plan_config()
    table = capi.traj_table(cfg)
    dev = run_plan_dev(cuda, cfg, sc, table)
    check_against_oracle(oracle, pp, sc, table, dev)
    assert dev["status"][3] == 1 and np.isnan(dev["x_ref"][3]).all()
    # every waypoint behind the car
    sc2 = dict(sc, waypoints=np.stack([pose[:4, 0] - 30.0, pose[:4, 1]], 1), pose=pose[:4].copy(),
               ranges=np.full((4, sc["ranges"].shape[1]), 10.0, np.float32))
    sc2["pose"][:, 2:] = [0.0, 1.0]    # yaw 0: facing +x, waypoints at -30 m
    dev2 = run_plan_dev(cuda, cfg, sc2, table)
    check_against_oracle(oracle, pp, sc2, table, dev2)
    assert (dev2["status"] == 2).all()


def test_tick_plan_then_qp_on_device(oracle, cuda):
    """The whole control tick on the device (project::OdomCallback's planning branch, then
    MPC::Update): plan -> x_ref[:, :N], x0 -> f110qp_solve_batch_dev, against the oracle's plan
    followed by the oracle's exact solve."""
    import torch

    N = 20
    sc = workload.make_scenes(256, seed=24)
    pp = oracle.plan_params()
    cfg = capi.default_plan_config()
    table = capi.traj_table(cfg)
    dev = run_plan_dev(cuda, cfg, sc, table, want_grid=False)
    ok = dev["status"] == 0
    x0 = torch.from_numpy(dev["x0"][ok]).to(cuda)
    xr = torch.from_numpy(np.ascontiguousarray(dev["x_ref"][ok])).to(cuda)  # whole miniPath (P = 50)
    Bk = int(ok.sum())
    ul = torch.from_numpy(np.tile(np.float32([4.5, 0.0]), (Bk, 1))).to(cuda)  # set_v(4.5) (project.cpp:170)
    uo = torch.empty((Bk, N, 2), device=cuda)
    xo = torch.empty((Bk, N + 1, 3), device=cuda)
    st = torch.empty(Bk, dtype=torch.int32, device=cuda)
    outs = []
    for be in (capi.BACKEND_WAVE, capi.BACKEND_LANE):  # x_ref_points = 50 on both back ends
        s = capi.Solver(capi.default_config(N, x_ref_points=50, backend=be))
        s.solve_dev(x0, ul, xr, None, uo, xo, st)
        torch.cuda.synchronize()
        s.close()
        outs.append((uo.cpu().numpy().astype(np.float64), st.cpu().numpy()))
    x0r, xrr = [], []
    for b in np.nonzero(ok)[0]:
        g, off = oracle.fill_occ_grid(pp, sc["pose"][b], sc["ranges"][b], sc["angle_min"], sc["angle_inc"],
                                      sc["angle_max"])
        r = oracle.plan(pp, sc["pose"][b], g, off, table, sc["waypoints"])
        x0r.append(r["x0"])
        xrr.append(r["x_ref"][:N])
    ur, xref_r, sr = oracle.solve_batch(oracle.params(N), np.array(x0r), np.tile(np.float32([4.5, 0.0]), (Bk, 1)),
                                        np.array(xrr))
    for u, stn in outs:
        assert (stn == sr).all()
        err = np.abs(u - ur).max(axis=(1, 2)) / np.maximum(1.0, np.abs(ur).max(axis=(1, 2)))
        assert err.max() <= 1e-4
