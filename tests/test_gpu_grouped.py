"""Grouped mode (f110qp_solve_grouped[_dev]) on MI355X: one W = H^-1 per scenario.

The candidates of one control tick share the pose and the linearisation point
(src/project.cpp:76-113 checks 31 candidates of one pose; Model::Linearize depends only on
(theta0, v, delta), src/model.cpp:30-59), so they share the condensed Hessian and its inverse.
The grouped path builds that inverse once per group and must return exactly what the per-QP
wave back end returns (bit for bit: the group's W is the W every member would build), and the
exact optimum of the reference QP within the north-star tolerance (oracle, KKT-certified).
"""
import numpy as np
import pytest

from f110qp import workload
from test_gpu_parity import TOL, halfspaces_oracle, rel_err

pytestmark = pytest.mark.gpu


def grouped_case(scen, N, seed, extra=0, heading="zero"):
    g = workload.make_grouped_batch(scen + (1 if extra else 0), N, seed=seed, heading=heading)
    G = g["group_size"]
    B = scen * G + extra
    w = {k: np.ascontiguousarray(g[k][:B]) for k in ("x0", "u_lin", "x_ref")}
    gid = (np.arange(B) // G).astype(np.int32)
    return w, gid, int(gid.max()) + 1


def solve_wave(capi, N, w, hs=None):
    cfg = capi.default_config(N, backend=capi.BACKEND_WAVE,
                              gap_mode=capi.GAP_ACTIVE if hs is not None else capi.GAP_INACTIVE)
    s = capi.Solver(cfg)
    out = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    s.close()
    return out


def solve_grouped(capi, N, w, gid, G, hs=None, backend=None):
    cfg = capi.default_config(N, backend=capi.BACKEND_WAVE if backend is None else backend,
                              gap_mode=capi.GAP_ACTIVE if hs is not None else capi.GAP_INACTIVE)
    s = capi.Solver(cfg)
    out = s.solve_grouped(w["x0"], w["u_lin"], w["x_ref"], gid, G, hs)
    s.close()
    return out


def assert_same(a, b):
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("N", [20, 30, 40])
def test_grouped_bit_identical_to_per_qp(capi, oracle, N):
    w, gid, G = grouped_case(3, N, seed=10 + N, extra=17)
    ref = solve_wave(capi, N, w)
    got = solve_grouped(capi, N, w, gid, G)
    assert_same(got, ref)
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"])
    np.testing.assert_array_equal(got[2], sr)
    assert rel_err(got[0], ur).max() <= TOL and rel_err(got[1], xr).max() <= TOL


def test_grouped_unsorted_ids_mismatch_and_out_of_range(capi, oracle):
    """Ids in any order; members whose linearisation point differs from their group's first
    member, and ids outside [0, G), solve on their own (still exact, still bit-identical)."""
    N = 20
    w, gid, G = grouped_case(4, N, seed=5)
    rng = np.random.default_rng(0)
    perm = rng.permutation(len(gid))
    w = {k: np.ascontiguousarray(v[perm]) for k, v in w.items()}
    gid = gid[perm].copy()
    # 10 members get their own heading / steer (a different linearisation point)
    odd = rng.choice(len(gid), 10, replace=False)
    w["x0"][odd[:5], 2] += np.float32(0.01)
    w["u_lin"][odd[5:], 1] += np.float32(0.02)
    gid[rng.choice(len(gid), 6, replace=False)] = -1
    gid[rng.choice(len(gid), 6, replace=False)] = G + 3
    ref = solve_wave(capi, N, w)
    got = solve_grouped(capi, N, w, gid, G)
    assert_same(got, ref)
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"])
    np.testing.assert_array_equal(got[2], sr)
    assert rel_err(got[0], ur).max() <= TOL


def test_grouped_empty_groups_and_singletons(capi):
    """num_groups larger than the ids used (empty slots) and one-member groups."""
    N = 20
    w = workload.make_batch(70, N, seed=9)
    gid = np.arange(70, dtype=np.int32) * 2  # every group has one member, odd groups are empty
    assert_same(solve_grouped(capi, N, w, gid, 140), solve_wave(capi, N, w))


def test_grouped_gap_rows(capi, oracle):
    """Half-space rows (config C3 semantics) with grouped candidates: every candidate of a
    scenario sees the scenario's scan."""
    N = 20
    w, gid, G = grouped_case(2, N, seed=31, extra=40)
    ranges, *geom = workload.make_scans(G, seed=31)
    hs_g = halfspaces_oracle(oracle, w["x0"][np.searchsorted(gid, np.arange(G))], ranges, geom)
    hs = np.ascontiguousarray(hs_g[gid])
    ref = solve_wave(capi, N, w, hs)
    got = solve_grouped(capi, N, w, gid, G, hs)
    assert_same(got, ref)
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True)
    np.testing.assert_array_equal(got[2], sr)
    ok = sr == oracle.SOLVED
    assert ok.mean() > 0.9 and rel_err(got[0][ok], ur[ok]).max() <= TOL


def test_grouped_device_entry_and_lane_backend(capi, oracle, cuda):
    """Device-pointer entry point (the C4 shard path) == host entry point; the lane back end
    ignores the groups and still returns the exact optimum."""
    import torch

    N = 40
    w, gid, G = grouped_case(4, N, seed=77, extra=8)
    B = len(gid)
    host = solve_grouped(capi, N, w, gid, G)
    t = {k: torch.from_numpy(v).to(cuda) for k, v in w.items()}
    g = torch.from_numpy(gid).to(cuda)
    uo = torch.empty((B, N, 2), dtype=torch.float32, device=cuda)
    xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device=cuda)
    st = torch.empty(B, dtype=torch.int32, device=cuda)
    it = torch.empty(B, dtype=torch.int32, device=cuda)
    s = capi.Solver(capi.default_config(N, backend=capi.BACKEND_WAVE))
    s.solve_grouped_dev(t["x0"], t["u_lin"], t["x_ref"], None, g, G, uo, xo, st, it)
    torch.cuda.synchronize()
    s.close()
    assert_same((uo.cpu().numpy(), xo.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()), host)
    lane = solve_grouped(capi, N, w, gid, G, backend=capi.BACKEND_LANE)
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"])
    np.testing.assert_array_equal(lane[2], sr)
    assert rel_err(lane[0], ur).max() <= TOL and rel_err(lane[1], xr).max() <= TOL


def test_grouped_c4_shard_full_size(capi, oracle):
    """One GPU's shard of config C4 (8,192 x N = 40, 68 scenarios + a partial one), AUTO back
    end: checked against the oracle on a 1,024-QP sample, the rest against the per-QP run."""
    N = 40
    w, gid, G = grouped_case(68, N, seed=4000, extra=32)
    got = solve_grouped(capi, N, w, gid, G, backend=capi.BACKEND_AUTO)
    assert (got[2] == capi.SOLVED).all()
    idx = np.random.default_rng(1).choice(len(gid), 1024, replace=False)
    sub = {k: np.ascontiguousarray(v[idx]) for k, v in w.items()}
    ur, xr, sr = oracle.solve_batch(oracle.params(N), sub["x0"], sub["u_lin"], sub["x_ref"])
    np.testing.assert_array_equal(got[2][idx], sr)
    assert rel_err(got[0][idx], ur).max() <= TOL and rel_err(got[1][idx], xr).max() <= TOL
