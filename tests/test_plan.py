"""CPU tests of the planning stage (F1/F2: candidate table, occupancy grid, collision check,
lookahead waypoint, end-point selection; src/project.cpp:73-152).

The reference ships no planner tests or outputs, so the oracle (oracle/plan_oracle.c) is pinned
here against an independent numpy restatement of the same reference lines, against the numpy
simulate_dynamics rollout, and the device kernel's parallel form of the reference's sequential
float running minimum is checked against the sequential loop itself.
"""
import os

import numpy as np
import pytest

from f110qp import capi, workload

REF_CSV = "/root/reference/csv/skirk.csv"


def test_traj_table_host_oracle_numpy(oracle):
    """Traj_Plan::generate_traj_table (trajectory_planner.cpp:26-72): C ABI == oracle bit for bit,
    and == the numpy simulate_dynamics rollout (model.cpp:61-75) to rounding."""
    pp = oracle.plan_params()
    t_or = oracle.traj_table(pp)
    t_abi = capi.traj_table(capi.default_plan_config())
    np.testing.assert_array_equal(t_abi, t_or)
    T = pp.steer_discrete + 1
    steer = -0.4 + np.arange(T) * (2 * 0.4 / 30)
    t_np = workload.mini_paths(steer, speed=4.5, dt=0.01, points=50)
    np.testing.assert_allclose(t_or, t_np, rtol=0, atol=1e-12)
    assert t_or.shape == (31, 50, 3) and np.all(t_or[:, 0] == 0)
    # the table is symmetric in steer: candidate i mirrors candidate T-1-i
    np.testing.assert_allclose(t_or[:, :, 1], -t_or[::-1, :, 1], atol=1e-12)
    # other params: size follows the params
    t2 = capi.traj_table(capi.default_plan_config(steer_discrete=20, traj_discrete=30))
    assert t2.shape == (21, 30, 3)


def _csv_text(n=37, seed=0):
    rng = np.random.default_rng(seed)
    rows = rng.normal(size=(n, 6)) * [5, 5, 1, 1, 1, 1]
    return "".join(",".join(repr(float(v)) for v in r) + "\n" for r in rows), rows


def test_parse_waypoints_quirks(oracle):
    """Trajectory::ReadCSV (trajectory.cpp:18-55): x = stof(first field), y = stof(rest of the
    line), ori from the previous point, where the predecessor of point 0 is (0u - 1) % n."""
    text, rows = _csv_text()
    a = capi.parse_waypoints(text)
    b = oracle.parse_waypoints(text)
    np.testing.assert_array_equal(a, b)
    assert a.shape == (37, 3)
    np.testing.assert_array_equal(a[:, 0], rows[:, 0].astype(np.float32))
    np.testing.assert_array_equal(a[:, 1], rows[:, 1].astype(np.float32))
    prev = (2 ** 32 - 1) % 37  # unsigned wrap
    x, y = a[:, 0].astype(np.float32), a[:, 1].astype(np.float32)
    assert a[0, 2] == np.float32(np.arctan2(np.float64(y[0] - y[prev]), np.float64(x[0] - x[prev])))
    assert a[5, 2] == np.float32(np.arctan2(np.float64(y[5] - y[4]), np.float64(x[5] - x[4])))


@pytest.mark.skipif(not os.path.exists(REF_CSV), reason="reference checkout not present")
def test_parse_reference_csv(oracle):
    """The reference's own global path (csv/skirk.csv, 500 rows of 6 columns)."""
    text = open(REF_CSV).read()
    a = capi.parse_waypoints(text)
    np.testing.assert_array_equal(a, oracle.parse_waypoints(text))
    assert a.shape == (500, 3)
    assert (2 ** 32 - 1) % 500 == 295  # the wrapped predecessor of point 0


def _cvtt(v):
    v = np.asarray(v, np.float32)
    ok = (v >= np.float32(-2147483648.0)) & (v < np.float32(2147483648.0))
    return np.where(ok, np.trunc(np.where(ok, v, 0)).astype(np.int64), -2147483648)


def np_fill_grid(pose, ranges, amin, ainc, amax, size=10, disc=np.float32(0.1), dil=np.float32(0.15)):
    """Independent numpy float32 restatement of OccGrid::FillOccGrid (occupancy_grid.cpp:55-88)."""
    f = np.float32
    G = int(f(size) / disc)
    px, py, qz, qw = pose
    cur = f(np.arctan2(2 * qw * qz, 1 - 2 * qz * qz))
    o0 = f(px + 0.275 * np.cos(np.float64(cur)))
    o1 = f(py + 0.275 * np.sin(np.float64(cur)))
    ns = int((f(amax) - f(amin)) / f(ainc) + f(1))
    ii = np.arange(ns)
    ang = (f(amin) + (ii.astype(np.float32) * f(ainc))).astype(np.float32) + cur
    ang = ang.astype(np.float32)
    r = ranges[:ns].astype(np.float64)
    cx = (r * np.cos(ang.astype(np.float64))).astype(np.float32) + o0
    cy = (r * np.sin(ang.astype(np.float64))).astype(np.float32) + o1
    offs = []
    o = -dil
    while o <= dil:
        offs.append(o)
        o = f(o + disc)
    grid = np.zeros((G, G), np.uint8)
    for xo in offs:
        for yo in offs:
            col = _cvtt(((cx + xo).astype(np.float32) - o0) / disc + f(G // 2))
            row = _cvtt(((cy + yo).astype(np.float32) - o1) / disc + f(G // 2))
            m = (col >= 0) & (col < G) & (row >= 0) & (row < G)
            grid[row[m], col[m]] = 1
    return grid, np.float32([o0, o1])


def np_plan(pose, grid, off, table, wp, lookahead=np.float32(2.5), disc=np.float32(0.1)):
    """Independent restatement of project.cpp:76-152 + trajectory.cpp:81-126 (sequential)."""
    f = np.float32
    G = grid.shape[0]
    px, py, qz, qw = pose
    s = 2.0 / (qz * qz + qw * qw)
    zz, wz = qz * (qz * s), qw * (qz * s)
    r00, r01, r10, r11 = 1.0 - zz, -wz, wz, 1.0 - zz

    def c2w(x, y):
        x, y = np.float64(f(x)), np.float64(f(y))
        return f(r00 * x + r01 * y + np.float64(f(px))), f(r10 * x + r11 * y + np.float64(f(py)))

    T, P = table.shape[:2]
    valid = np.zeros(T, np.uint8)
    ends = []
    for i in range(T):
        ok = True
        for j in range(P):
            wx, wy = c2w(table[i, j, 0], table[i, j, 1])
            col = int(_cvtt((wx - off[0]) / disc + f(G // 2)))
            row = int(_cvtt((wy - off[1]) / disc + f(G // 2)))
            if not (0 <= row < G and 0 <= col < G) or grid[row, col]:
                ok = False
        valid[i] = ok
        if ok:
            ends.append((i,) + c2w(table[i, -1, 0], table[i, -1, 1]))
    if not ends:
        return valid, -1, -1, 1
    tx = r00 * (-px) + r10 * (-py)
    ty = r01 * (-px) + r11 * (-py)
    mind, closest = np.float32(np.finfo(np.float32).max), -1
    for i in range(wp.shape[0]):
        x, y = np.float64(f(wp[i, 0])), np.float64(f(wp[i, 1]))
        cx, cy = f(r00 * x + r10 * y + tx), f(r01 * x + r11 * y + ty)
        if cx < 0:
            continue
        d = abs(np.sqrt(np.float64(cx) ** 2 + np.float64(cy) ** 2) - np.float64(lookahead))
        if d < np.float64(mind):
            mind, closest = f(d), i
    if closest < 0:
        return valid, -1, -1, 2
    gx, gy = np.float64(f(wp[closest, 0])), np.float64(f(wp[closest, 1]))
    best, bd = -1, np.inf
    for i, ex, ey in ends:
        d = np.sqrt((np.float64(ex) - gx) ** 2 + (np.float64(ey) - gy) ** 2)
        if d < bd:
            bd, best = d, i
    return valid, closest, best, 0


def test_oracle_planner_against_numpy_restatement(oracle):
    sc = workload.make_scenes(24, seed=5)
    pp = oracle.plan_params()
    table = oracle.traj_table(pp)
    statuses = []
    for b in range(24):
        g, off = oracle.fill_occ_grid(pp, sc["pose"][b], sc["ranges"][b], sc["angle_min"], sc["angle_inc"],
                                      sc["angle_max"])
        gn, offn = np_fill_grid(sc["pose"][b], sc["ranges"][b], sc["angle_min"], sc["angle_inc"], sc["angle_max"])
        np.testing.assert_array_equal(off, offn)
        np.testing.assert_array_equal(g, gn)
        r = oracle.plan(pp, sc["pose"][b], g, off, table, sc["waypoints"])
        v, bg, bt, st = np_plan(sc["pose"][b], g, off, table, sc["waypoints"])
        np.testing.assert_array_equal(r["valid"], v)
        assert (r["status"], r["best_global"], r["best_traj"]) == (st, bg, bt)
        statuses.append(st)
        if st == 0:
            # miniPath_: the chosen candidate in the map frame, ori 0 (project.cpp:149-152)
            assert r["x_ref"].shape == (50, 3) and np.all(r["x_ref"][:, 2] == 0)
            assert np.allclose(r["x_ref"][0, :2], sc["pose"][b, :2], atol=1e-5)
    assert statuses.count(0) >= 12 and g.sum() > 100


def _sequential_float_min(d):
    m, idx = np.float32(np.finfo(np.float32).max), -1
    for i, v in enumerate(d):
        if v < np.float64(m):
            m, idx = np.float32(v), i
    return idx


def _parallel_float_min(d):
    """The device kernel's form (plan_kernels.hip): F = min float(d); i0 = first index with
    float(d) = F; answer = last j > i0 with d_j < F, else i0."""
    fd = d.astype(np.float32)
    F = fd.min()
    i0 = int(np.nonzero(fd == F)[0][0])
    later = np.nonzero((np.arange(len(d)) > i0) & (d < np.float64(F)))[0]
    return int(later[-1]) if len(later) else i0


def test_parallel_running_float_minimum_equals_the_sequential_loop():
    """Trajectory::get_best_global_idx keeps its running minimum in a float (trajectory.cpp:88,
    103-107): the answer depends on float rounding and ties. Adversarial arrays full of values
    that round to the same float, both sides of it."""
    rng = np.random.default_rng(0)
    for trial in range(400):
        n = int(rng.integers(1, 60))
        base = np.float64(np.float32(rng.uniform(0.01, 3.0)))
        ulp = np.float64(np.spacing(np.float32(base)))
        d = base + rng.integers(-3, 4, n) * ulp * rng.choice([0.1, 0.25, 0.5, 0.49, 0.51, 1.0], n)
        if trial % 3 == 0:
            d = np.abs(rng.normal(1.0, 1.0, n))
        assert _sequential_float_min(d) == _parallel_float_min(d), d
