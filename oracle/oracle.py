"""ctypes wrapper of liboracle.so — the CPU checker (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg import this
module. The product path (``f110-mpc_amd/``) never does: it must fail loudly when its HIP
library is missing instead of falling back to anything here.

Every function restates a reference routine (paths relative to the reference repo root):
  linearize             src/model.cpp:30-59
  simulate_dynamics     src/model.cpp:61-75
  find_half_spaces      src/constraints.cpp:116-265
  assemble              src/mpc.cpp:26-29,208-340
  solve / solve_batch   OSQP's role at src/mpc.cpp:81-142, solved exactly (see f110_oracle.c)
  traj_table            src/trajectory_planner.cpp:26-72
  fill_occ_grid         src/occupancy_grid.cpp:55-88
  plan                  src/project.cpp:73-152, src/trajectory.cpp:81-126
  parse_waypoints       src/trajectory.cpp:18-55
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "liboracle.so")

SOLVED = 1
MAX_ITER = -2
PRIMAL_INFEASIBLE = -3
UNCERTIFIED = -99  # the oracle's own re-check failed: no reference answer for this QP
INFTY = 1e30


class Params(C.Structure):
    _fields_ = [
        ("horizon", C.c_int),
        ("dt", C.c_float),
        ("q", C.c_double * 3),
        ("r", C.c_double * 2),
        ("u_des", C.c_double * 2),
        ("u_min", C.c_float * 2),
        ("u_max", C.c_float * 2),
    ]


class PlanParams(C.Structure):
    _fields_ = [
        ("size", C.c_int),
        ("discrete", C.c_float),
        ("dilation", C.c_float),
        ("lookahead", C.c_float),
        ("speed_max", C.c_double),
        ("steer_max", C.c_double),
        ("steer_discrete", C.c_int),
        ("traj_discrete", C.c_int),
        ("dt", C.c_double),
    ]


class AdmmSettings(C.Structure):
    _fields_ = [
        ("rho", C.c_double),
        ("sigma", C.c_double),
        ("alpha", C.c_double),
        ("eps_abs", C.c_double),
        ("eps_rel", C.c_double),
        ("max_iter", C.c_int),
        ("check_termination", C.c_int),
        ("scaling", C.c_int),
        ("adaptive_rho", C.c_int),
        ("warm_start", C.c_int),
    ]


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int)
        fp = C.POINTER(C.c_float)
        L.f110o_default_params.argtypes = [C.POINTER(Params), C.c_int]
        L.f110o_linearize.argtypes = [C.c_double, C.c_double, C.c_double, C.c_double, dp, dp, dp]
        L.f110o_simulate_dynamics.argtypes = [dp, dp, C.c_double, dp]
        L.f110o_find_half_spaces.argtypes = [dp, fp, C.c_int, C.c_float, C.c_float, C.c_float,
                                             C.c_float, C.c_float, C.c_float, dp, dp, ip, ip]
        L.f110o_find_half_spaces_trig.argtypes = [dp, fp, C.c_int, C.c_float, C.c_float, C.c_float,
                                                  C.c_float, C.c_float, C.c_float, dp, dp, ip, ip, C.c_int]
        L.f110o_assemble.argtypes = [C.POINTER(Params), dp, dp, dp, dp, C.c_int, ip, ip, dp, dp,
                                     ip, ip, dp, dp, dp]
        L.f110o_condense.argtypes = [C.POINTER(Params), dp, dp, dp, dp, dp]
        L.f110o_solve.argtypes = [C.POINTER(Params), dp, dp, dp, dp, C.c_int, dp, dp, dp, dp, dp, ip]
        L.f110o_kkt_residuals.argtypes = [C.POINTER(Params), dp, dp, dp, dp, C.c_int, dp, dp, dp]
        L.f110o_solve_batch.argtypes = [C.POINTER(Params), C.c_int, fp, fp, fp, fp, C.c_int, dp,
                                        dp, ip, C.c_int]
        L.f110o_solve_batch_obj.argtypes = [C.POINTER(Params), C.c_int, fp, fp, fp, fp, C.c_int, dp,
                                            dp, ip, dp, C.c_int]
        if hasattr(L, "f110o_admm_solve_batch"):
            L.f110o_admm_default_settings.argtypes = [C.POINTER(AdmmSettings)]
            L.f110o_admm_solve.argtypes = [C.POINTER(Params), C.POINTER(AdmmSettings), dp, dp, dp,
                                           dp, C.c_int, dp, dp, ip]
            L.f110o_admm_solve_batch.argtypes = [C.POINTER(Params), C.POINTER(AdmmSettings), C.c_int,
                                                 fp, fp, fp, fp, C.c_int, dp, ip, ip, C.c_int]
            L.f110o_tick_latency.argtypes = [C.POINTER(Params), C.POINTER(AdmmSettings), C.c_int, C.c_int,
                                             fp, fp, fp, fp, C.c_int, C.c_int, dp]
        pp = C.POINTER(PlanParams)
        up = C.POINTER(C.c_ubyte)
        L.f110o_default_plan_params.argtypes = [pp]
        L.f110o_grid_blocks.argtypes = [pp]
        L.f110o_traj_table.argtypes = [pp, dp]
        L.f110o_car_orientation.argtypes = [dp]
        L.f110o_car_orientation.restype = C.c_float
        L.f110o_dilation_offsets.argtypes = [pp, fp, C.c_int]
        L.f110o_fill_occ_grid.argtypes = [pp, dp, fp, C.c_int, C.c_float, C.c_float, C.c_float, up, fp]
        L.f110o_plan.argtypes = [pp, dp, up, fp, dp, dp, C.c_int, up, ip, ip, fp, fp]
        L.f110o_parse_waypoints.argtypes = [C.c_char_p, dp, C.c_int]
        for name in ("f110o_num_variables", "f110o_num_constraints", "f110o_nnz_P", "f110o_nnz_A"):
            getattr(L, name).argtypes = [C.c_int]
        _lib = L
    return _lib


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _ptr(a, t=C.c_double):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def params(horizon: int, **over) -> Params:
    p = Params()
    lib().f110o_default_params(C.byref(p), horizon)
    for k, v in over.items():
        if k in ("q", "r", "u_des", "u_min", "u_max"):
            arr = getattr(p, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(p, k, v)
    return p


def linearize(theta, v, delta, dt=np.float32(0.01)):
    A = np.zeros(9)
    B = np.zeros(6)
    Cc = np.zeros(3)
    lib().f110o_linearize(float(theta), float(v), float(delta), float(np.float32(dt)), _ptr(A), _ptr(B), _ptr(Cc))
    return A.reshape(3, 3), B.reshape(3, 2), Cc


def simulate_dynamics(state, inp, dt):
    s = _d(state)
    u = _d(inp)
    out = np.zeros(3)
    lib().f110o_simulate_dynamics(_ptr(s), _ptr(u), float(dt), _ptr(out))
    return out


def find_half_spaces(state, ranges, angle_min, angle_inc, angle_max, thresh=3.0, divider=1.5, buffer=3.0,
                     float_trig=False):
    """float_trig: the float overload of cos / sin at constraints.cpp:182-186 (see f110_oracle.c)."""
    s = _d(state)
    r = np.ascontiguousarray(ranges, dtype=np.float32)
    l1 = np.zeros(3)
    l2 = np.zeros(3)
    lo = C.c_int()
    hi = C.c_int()
    rc = lib().f110o_find_half_spaces_trig(_ptr(s), _ptr(r, C.c_float), len(r), float(angle_min),
                                           float(angle_inc), float(angle_max), float(thresh), float(divider),
                                           float(buffer), _ptr(l1), _ptr(l2), C.byref(lo), C.byref(hi),
                                           int(bool(float_trig)))
    return rc, l1, l2, lo.value, hi.value


def dims(N):
    L = lib()
    return (L.f110o_num_variables(N), L.f110o_num_constraints(N), L.f110o_nnz_P(N), L.f110o_nnz_A(N))


def assemble(prm: Params, x0, u_lin, x_ref, hs=None, gap_active=False):
    """Return dict of CSC arrays exactly as MPC holds them after Update (mpc.cpp:77-80)."""
    N = prm.horizon
    n, m, nnzP, nnzA = dims(N)
    out = dict(P_colptr=np.zeros(n + 1, np.int32), P_rowind=np.zeros(nnzP, np.int32), P_val=np.zeros(nnzP),
               q=np.zeros(n), A_colptr=np.zeros(n + 1, np.int32), A_rowind=np.zeros(nnzA, np.int32),
               A_val=np.zeros(nnzA), l=np.zeros(m), u=np.zeros(m))
    hsa = None if hs is None else _d(hs).reshape(6)
    ip = C.c_int
    lib().f110o_assemble(C.byref(prm), _ptr(_d(x0)), _ptr(_d(u_lin)), _ptr(_d(x_ref).reshape(-1)), _ptr(hsa),
                         int(gap_active), _ptr(out["P_colptr"], ip), _ptr(out["P_rowind"], ip), _ptr(out["P_val"]),
                         _ptr(out["q"]), _ptr(out["A_colptr"], ip), _ptr(out["A_rowind"], ip), _ptr(out["A_val"]),
                         _ptr(out["l"]), _ptr(out["u"]))
    return out


def condense(prm: Params, x0, u_lin, x_ref):
    """Condensed (H, g) of one tick, float64, from an explicit Gamma."""
    N = prm.horizon
    H = np.zeros((2 * N, 2 * N))
    g = np.zeros(2 * N)
    lib().f110o_condense(C.byref(prm), _ptr(_d(x0)), _ptr(_d(u_lin)), _ptr(_d(x_ref).reshape(-1)), _ptr(H), _ptr(g))
    return H, g


def solve(prm: Params, x0, u_lin, x_ref, hs=None, gap_active=False):
    N = prm.horizon
    n, m, _, _ = dims(N)
    u = np.zeros(2 * N)
    x = np.zeros(3 * (N + 1))
    z = np.zeros(n)
    y = np.zeros(m)
    obj = C.c_double()
    na = C.c_int()
    hsa = None if hs is None else _d(hs).reshape(6)
    st = lib().f110o_solve(C.byref(prm), _ptr(_d(x0)), _ptr(_d(u_lin)), _ptr(_d(x_ref).reshape(-1)), _ptr(hsa),
                           int(gap_active), _ptr(u), _ptr(x), _ptr(z), _ptr(y), C.byref(obj), C.byref(na))
    return dict(status=st, u=u.reshape(N, 2), x=x.reshape(N + 1, 3), z=z, y=y, obj=obj.value, n_active=na.value)


def kkt_residuals(prm: Params, x0, u_lin, x_ref, z, y, hs=None, gap_active=False):
    res = np.zeros(3)
    hsa = None if hs is None else _d(hs).reshape(6)
    lib().f110o_kkt_residuals(C.byref(prm), _ptr(_d(x0)), _ptr(_d(u_lin)), _ptr(_d(x_ref).reshape(-1)), _ptr(hsa),
                              int(gap_active), _ptr(_d(z)), _ptr(_d(y)), _ptr(res))
    return res


def solve_batch(prm: Params, x0, u_lin, x_ref, hs=None, gap_active=False, num_threads=0, objective=False):
    """Exact batched solve on float32 ABI-layout inputs. Returns (u[B,N,2], x[B,N+1,3], status[B])
    and, with objective=True, also obj[B] = OSQP's 1/2 z'Pz + q'z at the exact optimum."""
    N = prm.horizon
    x0 = np.ascontiguousarray(x0, np.float32)
    B = x0.shape[0]
    ul = np.ascontiguousarray(u_lin, np.float32)
    xr = np.ascontiguousarray(x_ref, np.float32)
    assert xr.shape == (B, N, 3), xr.shape
    h = None if hs is None else np.ascontiguousarray(hs, np.float32).reshape(B, 6)
    u = np.zeros((B, N, 2))
    x = np.zeros((B, N + 1, 3))
    st = np.zeros(B, np.int32)
    fp = C.c_float
    ob = np.zeros(B) if objective else None
    lib().f110o_solve_batch_obj(C.byref(prm), B, _ptr(x0, fp), _ptr(ul, fp), _ptr(xr, fp), _ptr(h, fp),
                                int(gap_active), _ptr(u), _ptr(x), _ptr(st, C.c_int), _ptr(ob), int(num_threads))
    if objective:
        return u, x, st, ob
    return u, x, st


def tracking_cost(prm: Params, u, x, x_ref):
    """sum_{i=0..N} 1/2|x_i - r_i|_Q^2 + sum_k 1/2|u_k - u_des|_R^2 of solutions u [B,N,2], x [B,N+1,3]
    (r_N = x_ref[N-1], mpc.cpp:228), float64: the `cost` output of f110qp_solve_*_ex, evaluated
    directly (no cancellation against OSQP's constant-free objective)."""
    N = prm.horizon
    xr = np.asarray(x_ref, np.float64)[:, :N]
    r_ext = np.concatenate([xr, xr[:, N - 1:N]], 1)
    q = np.array(prm.q[:])
    r = np.array(prm.r[:])
    ud = np.array(prm.u_des[:])
    return 0.5 * (((np.asarray(x, np.float64) - r_ext) ** 2) * q).sum(axis=(1, 2)) + \
        0.5 * (((np.asarray(u, np.float64) - ud) ** 2) * r).sum(axis=(1, 2))


def select(group, num_groups, cost, status):
    """Per-scenario argmin (the checker of f110qp_select_dev): smallest index among the solved
    members with the minimal cost; -1 / +inf for a scenario without a solved member."""
    winner = np.full(num_groups, -1, np.int64)
    best = np.full(num_groups, np.inf)
    for b in range(len(group)):
        g = int(group[b])
        if 0 <= g < num_groups and status[b] == SOLVED and cost[b] < best[g]:
            best[g] = cost[b]
            winner[g] = b
    return winner, best


def cost_from_obj(prm: Params, obj, x_ref):
    """OSQP's objective plus the constant it drops: obj + 1/2 sum_{i=0..N} r_i'Q r_i + N/2 u_des'R u_des
    (r_i = x_ref[i], r_N = x_ref[N-1], mpc.cpp:221-229) = the tracking cost sum 1/2|x-r|_Q^2 +
    1/2|u-u_des|_R^2 of the solution (the `cost` output of f110qp_solve_*_ex)."""
    N = prm.horizon
    xr = np.asarray(x_ref, np.float64)[:, :N]
    q = np.array(prm.q[:])
    r = np.array(prm.r[:])
    ud = np.array(prm.u_des[:])
    c = 0.5 * (xr ** 2 * q).sum(axis=(1, 2)) + 0.5 * (xr[:, N - 1] ** 2 * q).sum(axis=1)
    return obj + c + 0.5 * N * float((r * ud * ud).sum())


def admm_settings(**over) -> AdmmSettings:
    s = AdmmSettings()
    lib().f110o_admm_default_settings(C.byref(s))
    for k, v in over.items():
        setattr(s, k, v)
    return s


def admm_solve_batch(prm: Params, settings: AdmmSettings, x0, u_lin, x_ref, hs=None, gap_active=False,
                     num_threads=0):
    """OSQP-default ADMM restatement (CPU baseline). Returns (u[B,N,2], status[B], iters[B])."""
    N = prm.horizon
    x0 = np.ascontiguousarray(x0, np.float32)
    B = x0.shape[0]
    ul = np.ascontiguousarray(u_lin, np.float32)
    xr = np.ascontiguousarray(x_ref, np.float32)
    h = None if hs is None else np.ascontiguousarray(hs, np.float32).reshape(B, 6)
    u = np.zeros((B, N, 2))
    st = np.zeros(B, np.int32)
    it = np.zeros(B, np.int32)
    fp = C.c_float
    lib().f110o_admm_solve_batch(C.byref(prm), C.byref(settings), B, _ptr(x0, fp), _ptr(ul, fp), _ptr(xr, fp),
                                 _ptr(h, fp), int(gap_active), _ptr(u), _ptr(st, C.c_int), _ptr(it, C.c_int),
                                 int(num_threads))
    return u, st, it


def tick_latency(prm: Params, settings: AdmmSettings, x0, u_lin, x_ref, ticks: int, exact: bool = False,
                 hs=None, gap_active=False):
    """C1 baseline: `ticks` single-QP solves on the calling thread (one core), instance t % B each;
    returns the wall nanoseconds of every tick (timed inside C) and the number solved."""
    N = prm.horizon
    x0 = np.ascontiguousarray(x0, np.float32)
    B = x0.shape[0]
    ul = np.ascontiguousarray(u_lin, np.float32)
    xr = np.ascontiguousarray(x_ref, np.float32)
    h = None if hs is None else np.ascontiguousarray(hs, np.float32).reshape(B, 6)
    ns = np.zeros(ticks)
    fp = C.c_float
    nsol = lib().f110o_tick_latency(C.byref(prm), C.byref(settings), int(exact), B, _ptr(x0, fp), _ptr(ul, fp),
                                    _ptr(xr, fp), _ptr(h, fp), int(gap_active), int(ticks), _ptr(ns))
    return ns, int(nsol)


# ---- planning stage (plan_oracle.c) ------------------------------------------------------------

def plan_params(**over) -> PlanParams:
    p = PlanParams()
    lib().f110o_default_plan_params(C.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


def traj_table(pp: PlanParams) -> np.ndarray:
    T, P = pp.steer_discrete + 1, pp.traj_discrete
    t = np.zeros((T, P, 3), np.float64)
    lib().f110o_traj_table(C.byref(pp), _ptr(t))
    return t


def dilation_offsets(pp: PlanParams) -> np.ndarray:
    buf = np.zeros(64, np.float32)
    n = lib().f110o_dilation_offsets(C.byref(pp), _ptr(buf, C.c_float), 64)
    return buf[:n].copy()


def fill_occ_grid(pp: PlanParams, pose, ranges, angle_min, angle_inc, angle_max):
    """pose = (x, y, qz, qw) doubles -> (grid [G, G] uint8, occ_offset [2] float32)"""
    G = lib().f110o_grid_blocks(C.byref(pp))
    grid = np.zeros((G, G), np.uint8)
    off = np.zeros(2, np.float32)
    r = np.ascontiguousarray(ranges, np.float32)
    lib().f110o_fill_occ_grid(C.byref(pp), _ptr(_d(pose)), _ptr(r, C.c_float), r.shape[0], angle_min,
                              angle_inc, angle_max, _ptr(grid, C.c_ubyte), _ptr(off, C.c_float))
    return grid, off


def plan(pp: PlanParams, pose, grid, off, table, waypoints):
    """-> dict(status, valid [T] uint8, best_global, best_traj, x_ref [P, 3] f32, x0 [3] f32)"""
    T, P = pp.steer_discrete + 1, pp.traj_discrete
    wp = _d(np.asarray(waypoints)[:, :2])
    valid = np.zeros(T, np.uint8)
    bg, bt = C.c_int(-1), C.c_int(-1)
    xr = np.zeros((P, 3), np.float32)
    x0 = np.zeros(3, np.float32)
    st = lib().f110o_plan(C.byref(pp), _ptr(_d(pose)), _ptr(np.ascontiguousarray(grid, np.uint8), C.c_ubyte),
                          _ptr(np.ascontiguousarray(off, np.float32), C.c_float), _ptr(_d(table)), _ptr(wp),
                          wp.shape[0], _ptr(valid, C.c_ubyte), C.byref(bg), C.byref(bt), _ptr(xr, C.c_float),
                          _ptr(x0, C.c_float))
    return dict(status=st, valid=valid, best_global=bg.value, best_traj=bt.value, x_ref=xr, x0=x0)


def parse_waypoints(text: str, max_n: int = 100000) -> np.ndarray:
    wp = np.zeros((max_n, 3), np.float64)
    n = lib().f110o_parse_waypoints(text.encode(), _ptr(wp), max_n)
    return wp[:n].copy()
