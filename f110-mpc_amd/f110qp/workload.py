"""Synthetic tick batches for the f110qp hot path, numpy only.

The reference ships no datasets; its inputs come from the simulator. The generator follows
the reference's own recipe for a candidate trajectory:
  - mini paths: Traj_Plan::generate_traj_table (src/trajectory_planner.cpp:26-72), i.e.
    `traj_discrete`=50 states from (0,0,0) by Model::simulate_dynamics (src/model.cpp:61-75,
    CAR_LENGTH = 0.35) at constant speed and steer, dt = 0.01;
  - car -> world with Transforms::CarPointToWorldPoint (src/transforms.cpp:3-20), as float;
  - ori = 0 for every reference state (src/project.cpp:147), or the true heading;
  - u_lin = (4.5, steer): v is forced to 4.5 before MPC::Update (src/project.cpp:170);
  - half spaces from FindHalfSpaces on a synthetic 1080-beam scan with one guaranteed gap.
All arrays are in the include/f110qp.h layouts (float32, row-major).
"""
from __future__ import annotations

import numpy as np

CAR_LENGTH = 0.35  # src/model.cpp:2
TRAJ_POINTS = 50   # params.yaml:57 traj_discrete
SPEED = 4.5        # params.yaml:46 umax; project.cpp:170


def mini_paths(steer, speed=SPEED, dt=0.01, points=TRAJ_POINTS):
    """Vectorised generate_traj_table rollouts: steer [B] -> car-frame states [B, points, 3]."""
    steer = np.asarray(steer, np.float64).reshape(-1)
    B = steer.shape[0]
    out = np.zeros((B, points, 3))
    s = np.zeros((B, 3))
    for k in range(1, points):  # trajectory_planner.cpp:291-297
        d0 = speed * np.cos(s[:, 2])
        d1 = speed * np.sin(s[:, 2])
        d2 = np.tan(steer) * speed / CAR_LENGTH
        s = s + np.stack([d0, d1, d2], 1) * dt
        out[:, k] = s
    return out


def car_to_world(px, py, pose):
    """CarPointToWorldPoint: rotate by the pose yaw, add the (float) position -> float32."""
    th = pose[:, 2:3].astype(np.float64)
    c, s = np.cos(th), np.sin(th)
    wx = c * px - s * py + pose[:, 0:1].astype(np.float32).astype(np.float64)
    wy = s * px + c * py + pose[:, 1:2].astype(np.float32).astype(np.float64)
    return wx.astype(np.float32), wy.astype(np.float32)


def make_batch(batch: int, horizon: int, seed: int = 0, heading: str = "zero", lateral: float = 0.3,
               steer_range: float = 0.4):
    """Independent ticks (configs C2/C3 of BASELINE.json). Returns dict(x0, u_lin, x_ref)."""
    rng = np.random.default_rng(seed)
    x0 = np.stack([rng.uniform(-50, 50, batch), rng.uniform(-50, 50, batch),
                   rng.uniform(-np.pi, np.pi, batch)], 1).astype(np.float32)
    u_lin = np.stack([np.full(batch, SPEED), rng.uniform(-steer_range, steer_range, batch)], 1).astype(np.float32)
    steer = rng.uniform(-steer_range, steer_range, batch)
    off = rng.uniform(-lateral, lateral, batch)
    path = mini_paths(steer)
    x_ref = _to_ref(path, off, x0, horizon, heading)
    return dict(x0=x0, u_lin=u_lin, x_ref=x_ref)


def _to_ref(path, off, x0, horizon, heading):
    px = path[:, :horizon, 0]
    py = path[:, :horizon, 1] + off[:, None]
    wx, wy = car_to_world(px, py, x0)
    if heading == "zero":
        ori = np.zeros_like(wx)
    else:
        ori = (x0[:, 2:3].astype(np.float64) + path[:, :horizon, 2]).astype(np.float32)
    return np.ascontiguousarray(np.stack([wx, wy, ori], 2), np.float32)


def make_grouped_batch(scenarios: int, horizon: int, seed: int = 0, lanes=(0.0, 0.25, -0.25, 0.5, -0.5, 0.75),
                       steers: int = 20, steer_range: float = 0.4, heading: str = "zero"):
    """Config C4: per scenario one car state and linearisation point shared by
    len(lanes) x steers candidate mini paths (lateral lane offset x steer value)."""
    rng = np.random.default_rng(seed)
    G = len(lanes) * steers
    x0s = np.stack([rng.uniform(-50, 50, scenarios), rng.uniform(-50, 50, scenarios),
                    rng.uniform(-np.pi, np.pi, scenarios)], 1).astype(np.float32)
    uls = np.stack([np.full(scenarios, SPEED), rng.uniform(-steer_range, steer_range, scenarios)], 1).astype(np.float32)
    steer_vals = np.linspace(-steer_range, steer_range, steers)
    st = np.tile(steer_vals, len(lanes))
    off = np.repeat(np.asarray(lanes, np.float64), steers)
    path = mini_paths(st)
    x0 = np.repeat(x0s, G, 0)
    u_lin = np.repeat(uls, G, 0)
    x_ref = _to_ref(np.tile(path, (scenarios, 1, 1)), np.tile(off, scenarios), x0, horizon, heading)
    return dict(x0=x0, u_lin=u_lin, x_ref=x_ref, group_size=G)


SCAN_BEAMS = 1080


def scan_geometry(beams: int = SCAN_BEAMS):
    amin = np.float32(-np.pi)
    ainc = np.float32(2 * np.pi / beams)
    amax = np.float32(amin + ainc * (beams - 1))
    return amin, ainc, amax


def make_scans(batch: int, seed: int = 0, beams: int = SCAN_BEAMS, gap_center=0.6, gap_width=(0.3, 0.9)):
    """Synthetic LaserScans: short returns (1-2.5 m, below follow_gap_thresh = 3,
    params.yaml:49) everywhere except one arc of long returns (4-10 m) near the heading."""
    rng = np.random.default_rng(seed + 7919)
    amin, ainc, amax = scan_geometry(beams)
    ang = amin + ainc * np.arange(beams, dtype=np.float64)
    r = rng.uniform(1.0, 2.5, (batch, beams)).astype(np.float32)
    ctr = rng.uniform(-gap_center, gap_center, batch)
    w = rng.uniform(gap_width[0], gap_width[1], batch)
    m = np.abs(ang[None, :] - ctr[:, None]) < (w[:, None] / 2)
    r[m] = rng.uniform(4.0, 10.0, int(m.sum())).astype(np.float32)
    return r, amin, ainc, amax


def make_stream(batch: int, horizon: int, ticks: int, seed: int = 0, dt: float = 0.01, heading_change_every: int = 0):
    """Config C5: `ticks` consecutive control ticks of `batch` independent cars. Each car keeps
    its mini path (the reference re-plans only near the path end, src/project.cpp:180-188)
    while x0 advances 4.5*dt along the heading per tick; u_lin keeps v = 4.5 and the steer of
    the previous tick. With heading_change_every = k > 0 a tenth of the cars also turn by a
    small angle every k ticks (their linearisation point changes). Returns a list of dicts."""
    base = make_batch(batch, horizon, seed=seed)
    rng = np.random.default_rng(seed + 17)
    x0 = base["x0"].astype(np.float64).copy()
    ticks_out = []
    turners = rng.random(batch) < 0.1
    for t in range(ticks):
        if t > 0:
            x0[:, 0] += SPEED * dt * np.cos(x0[:, 2])
            x0[:, 1] += SPEED * dt * np.sin(x0[:, 2])
            if heading_change_every and t % heading_change_every == 0:
                x0[turners, 2] += rng.uniform(-0.05, 0.05, int(turners.sum()))
        ticks_out.append(dict(x0=x0.astype(np.float32), u_lin=base["u_lin"].copy(), x_ref=base["x_ref"].copy()))
    return ticks_out


def simulate_dynamics(x, u, dt=0.01):
    """Model::simulate_dynamics (src/model.cpp:61-75, CAR_LENGTH = 0.35), vectorised fp64:
    x [B,3] (x, y, ori), u [B,2] (v, steer) -> the state one Euler step later."""
    x = np.asarray(x, np.float64)
    u = np.asarray(u, np.float64)
    d = np.stack([u[:, 0] * np.cos(x[:, 2]), u[:, 0] * np.sin(x[:, 2]), np.tan(u[:, 1]) * u[:, 0] / CAR_LENGTH], 1)
    return x + d * dt


def closed_loop_stream(solve, batch: int, horizon: int, ticks: int, seed: int = 0, dt: float = 0.01,
                       replan_every: int = 5, lateral: float = 0.3, steer_range: float = 0.4):
    """Config C5 as a closed receding-horizon loop (project::OdomCallback's MPC branch,
    src/project.cpp:160-198, driven by a simulated car). Per tick and car:
      - x0 = the car's pose (x, y, GetCarOrientation), so theta0 changes every tick;
      - u_lin = GetNextInput() with v forced to 4.5 (project.cpp:163-170): the steer of the
        previous solution's next input u*_1 (u*_0 is applied first);
      - x_ref = the first N states of the car's current mini path; the path is re-planned from the
        current pose every `replan_every` ticks (the reference re-plans within 1.98 m of the end
        of its 2.2 m mini path, project.cpp:180-188), staggered over the cars;
      - then the plant advances: x0 <- simulate_dynamics(x0, u*_0, dt) (model.cpp:61-75).
    `solve(x0, u_lin, x_ref) -> u [B, N, 2]` is the solver that closes the loop (a GPU back end or
    the oracle). Returns the list of tick dicts (x0, u_lin, x_ref), float32 ABI layouts."""
    rng = np.random.default_rng(seed)
    base = make_batch(batch, horizon, seed=seed, lateral=lateral, steer_range=steer_range)
    x = base["x0"].astype(np.float64)
    ul = base["u_lin"].copy()
    xr = base["x_ref"].copy()
    out = []
    for t in range(ticks):
        if t > 0:
            rp = (np.arange(batch) + t) % replan_every == 0
            n = int(rp.sum())
            if n:
                x0f = x[rp].astype(np.float32)
                path = mini_paths(rng.uniform(-steer_range, steer_range, n))
                xr[rp] = _to_ref(path, rng.uniform(-lateral, lateral, n), x0f, horizon, "zero")
        x0 = x.astype(np.float32)
        tick = dict(x0=x0, u_lin=ul.copy(), x_ref=xr.copy())
        out.append(tick)
        u = np.asarray(solve(tick["x0"], tick["u_lin"], tick["x_ref"]), np.float64)
        ok = np.isfinite(u).all(axis=(1, 2))
        u0 = np.where(ok[:, None], u[:, 0], np.stack([np.full(batch, 0.5), np.zeros(batch)], 1))  # Input(0.5, 0)
        x = simulate_dynamics(x, u0, dt)
        nxt = u[:, 1] if horizon > 1 else u[:, 0]
        ul = np.stack([np.full(batch, SPEED), np.where(ok, nxt[:, 1], ul[:, 1])], 1).astype(np.float32)
    return out


def warm_key_hit_rate(ticks) -> float:
    """Fraction of (car, tick > 0) whose linearisation point bits (theta0, v, steer) equal the
    previous tick's: the wave back end's warm W = H^-1 cache hits exactly then."""
    hits = tot = 0
    for a, b in zip(ticks[:-1], ticks[1:]):
        same = (a["x0"][:, 2].view(np.uint32) == b["x0"][:, 2].view(np.uint32)) & \
               (a["u_lin"].view(np.uint32) == b["u_lin"].view(np.uint32)).all(axis=1)
        hits += int(same.sum())
        tot += same.size
    return hits / max(1, tot)


# ---- planning scenes (pose + LaserScan + global path) for the device planning stage -----------

def track_waypoints(n: int = 500, a: float = 12.0, b: float = 6.0) -> np.ndarray:
    """A closed elliptical global path of n points (x, y as float32 values, like the CSV)."""
    t = np.linspace(0.0, 2 * np.pi, n, endpoint=False)
    return np.stack([a * np.cos(t), b * np.sin(t)], 1).astype(np.float32).astype(np.float64)


def _ray_circles(ox, oy, ang, cx, cy, rad, max_range):
    """Ray casting: ranges [B, R] from origins (ox, oy) [B] along angles [B, R] against circles
    (cx, cy, rad) [B, C]."""
    dx, dy = np.cos(ang), np.sin(ang)                       # [B, R]
    px = cx[:, None, :] - ox[:, None, None]                 # [B, 1, C]
    py = cy[:, None, :] - oy[:, None, None]
    t = px * dx[..., None] + py * dy[..., None]             # projection, [B, R, C]
    d2 = px * px + py * py - t * t
    r2 = (rad * rad)[:, None, :]
    hit = (d2 <= r2) & (t > 0)
    th = t - np.sqrt(np.maximum(r2 - d2, 0.0))
    th = np.where(hit & (th > 0), th, np.inf)
    return np.minimum(th.min(axis=2), max_range)


def make_scenes(batch: int, seed: int = 0, beams: int = SCAN_BEAMS, obstacles: int = 6, waypoints=None,
                max_range: float = 10.0):
    """Scenarios for project::OdomCallback's planning branch: a car near the global path with the
    path heading (+ noise), its 1080-beam 2*pi LaserScan (from the lidar 0.275 m ahead, as
    OccGrid::FillOccGrid assumes, occupancy_grid.cpp:63-64) of the two track walls (circles along
    the path at +-1.6 m) and a few obstacles. Returns dict(pose [B,4] f64 (x, y, qz, qw),
    ranges [B,beams] f32, geometry, waypoints [W,2] f64)."""
    rng = np.random.default_rng(seed)
    wp = track_waypoints() if waypoints is None else np.asarray(waypoints, np.float64)[:, :2]
    W = wp.shape[0]
    k = rng.integers(0, W, batch)
    nxt = wp[(k + 1) % W]
    hd = np.arctan2(nxt[:, 1] - wp[k, 1], nxt[:, 0] - wp[k, 0])
    yaw = hd + rng.uniform(-0.3, 0.3, batch)
    off = rng.uniform(-0.4, 0.4, batch)
    x = wp[k, 0] - np.sin(hd) * off
    y = wp[k, 1] + np.cos(hd) * off
    pose = np.stack([x, y, np.sin(yaw / 2), np.cos(yaw / 2)], 1)
    # walls: circles of radius 0.12 every ~0.25 m along the path, +-1.6 m laterally
    hw = np.arctan2(np.roll(wp[:, 1], -1) - wp[:, 1], np.roll(wp[:, 0], -1) - wp[:, 0])
    wall = np.concatenate([wp + 1.6 * np.stack([-np.sin(hw), np.cos(hw)], 1),
                           wp - 1.6 * np.stack([-np.sin(hw), np.cos(hw)], 1)])
    # only the wall circles within max_range of the car matter
    amin, ainc, amax = scan_geometry(beams)
    ang = yaw[:, None] + (amin + ainc * np.arange(beams, dtype=np.float64))[None, :]
    lx, ly = x + 0.275 * np.cos(yaw), y + 0.275 * np.sin(yaw)
    d = np.hypot(wall[None, :, 0] - lx[:, None], wall[None, :, 1] - ly[:, None])
    near = np.argsort(d, axis=1)[:, :160]
    cx = np.take_along_axis(np.broadcast_to(wall[:, 0], d.shape), near, 1)
    cy = np.take_along_axis(np.broadcast_to(wall[:, 1], d.shape), near, 1)
    rad = np.full(cx.shape, 0.12)
    # obstacles 1-4 m ahead in a +-60 degree cone
    ob_r = rng.uniform(1.0, 4.0, (batch, obstacles))
    ob_a = yaw[:, None] + rng.uniform(-1.0, 1.0, (batch, obstacles))
    cx = np.concatenate([cx, lx[:, None] + ob_r * np.cos(ob_a)], 1)
    cy = np.concatenate([cy, ly[:, None] + ob_r * np.sin(ob_a)], 1)
    rad = np.concatenate([rad, rng.uniform(0.1, 0.35, (batch, obstacles))], 1)
    ranges = _ray_circles(lx, ly, ang, cx, cy, rad, max_range).astype(np.float32)
    return dict(pose=pose, ranges=ranges, angle_min=amin, angle_inc=ainc, angle_max=amax, waypoints=wp)


def drive_stream(ticks: int, seed: int = 0, step: float = 0.09, beams: int = SCAN_BEAMS, obstacles: int = 40,
                 max_range: float = 10.0):
    """A scripted drive for the project node's callbacks: the car follows the elliptical path
    (4.5 m/s x 20 ms per tick = 0.09 m, src/project.cpp:233-235) with a small lateral wobble; the
    world holds the two track walls and `obstacles` static circles beside the path. Returns
    dict(pose [T,4] f64, ranges [T,beams] f32, geometry, waypoints [W,2])."""
    rng = np.random.default_rng(seed)
    wp = track_waypoints()
    W = wp.shape[0]
    seg = np.hypot(*(np.roll(wp, -1, 0) - wp).T)
    s_along = np.concatenate([[0.0], np.cumsum(seg)])
    total = s_along[-1]
    s0 = rng.uniform(0, total)
    s = (s0 + step * np.arange(ticks)) % total
    k = np.searchsorted(s_along, s, side="right") - 1
    frac = (s - s_along[k]) / seg[k]
    nxt = wp[(k + 1) % W]
    base = wp[k] + (nxt - wp[k]) * frac[:, None]
    hd = np.arctan2(nxt[:, 1] - wp[k, 1], nxt[:, 0] - wp[k, 0])
    lat = 0.2 * np.sin(np.arange(ticks) * 0.15)
    x = base[:, 0] - np.sin(hd) * lat
    y = base[:, 1] + np.cos(hd) * lat
    yaw = hd + 0.05 * np.cos(np.arange(ticks) * 0.2)
    pose = np.stack([x, y, np.sin(yaw / 2), np.cos(yaw / 2)], 1)
    hw = np.arctan2(np.roll(wp[:, 1], -1) - wp[:, 1], np.roll(wp[:, 0], -1) - wp[:, 0])
    nrm = np.stack([-np.sin(hw), np.cos(hw)], 1)
    wall = np.concatenate([wp + 1.6 * nrm, wp - 1.6 * nrm])
    oi = rng.integers(0, W, obstacles)
    obst = wp[oi] + nrm[oi] * rng.choice([-0.9, 0.9], obstacles)[:, None]
    cxs = np.concatenate([wall[:, 0], obst[:, 0]])
    cys = np.concatenate([wall[:, 1], obst[:, 1]])
    rads = np.concatenate([np.full(len(wall), 0.12), rng.uniform(0.15, 0.3, obstacles)])
    amin, ainc, amax = scan_geometry(beams)
    ang = yaw[:, None] + (amin + ainc * np.arange(beams, dtype=np.float64))[None, :]
    lx, ly = x + 0.275 * np.cos(yaw), y + 0.275 * np.sin(yaw)
    d = np.hypot(cxs[None, :] - lx[:, None], cys[None, :] - ly[:, None])
    near = np.argsort(d, axis=1)[:, :200]
    ranges = _ray_circles(lx, ly, ang, cxs[near], cys[near], rads[near], max_range).astype(np.float32)
    return dict(pose=pose, ranges=ranges, angle_min=amin, angle_inc=ainc, angle_max=amax, waypoints=wp)
