# Host design check (imports the CPU oracle, so it lives under tests/): a float64 numpy model of
# a Mehrotra predictor-corrector interior point on the lane (Riccati) structure for QPs WITH the
# follow-the-gap rows (BASELINE configs[2], C3), run on the bench's C3 batch and compared with the
# exact oracle. Not product code: the kernel is csrc/lane_ipm_kernel.h.
#
# The QP (recentred on x0; mpc.cpp:208-306 with the C3 gap semantic mpc.cpp:297-298):
#   min sum_{i<N} 1/2|x_i - r_i|_Q^2 + 1/2|x_N - r_{N-1}|_Q^2 + sum_i 1/2|u_i - ud|_R^2
#   s.t. x_{i+1} = A x_i + B u_i + C (model.cpp:42-55), x_0 = 0,
#        lb <= u_i <= ub (constraints.cpp:19,21), nu_k' x_{i+1} >= beta_k (k = 0, 1; mpc.cpp:249,271).
# Per stage i the six inequality rows are (u0 - lb0, ub0 - u0, u1 - lb1, ub1 - u1, nu_0'x_{i+1} - beta_0,
# nu_1'x_{i+1} - beta_1), each with a slack s > 0 and a multiplier z > 0. The primal iterate keeps
# x = rollout(u), so every Newton step is the LQ problem in (dx, du) with
#   R~_i = R + diag(Sig_0 + Sig_1, Sig_2 + Sig_3),   Q~_{i+1} = Q + sum_k Sig_{4+k} nu_k nu_k'
# (Sig = z / s) and linear terms grad f - D'z + D'((rc + z rp) / s): one Riccati factorisation per
# iteration, two solves (Mehrotra predictor, corrector) on it.
import sys

import numpy as np

sys.path.insert(0, "f110-mpc_amd")
sys.path.insert(0, "oracle")
sys.path.insert(0, "tests")


def setup(prm, x0, ul, xr, hs):
    B = x0.shape[0]
    N = prm.horizon
    dt = float(np.float32(prm.dt))
    q = np.array(prm.q[:]); r = np.array(prm.r[:]); ud = np.array(prm.u_des[:])
    lb = np.array([float(prm.u_min[0]), float(prm.u_min[1])])
    ub = np.array([float(prm.u_max[0]), float(prm.u_max[1])])
    X0 = x0[:, 0].astype(np.float64); Y0 = x0[:, 1].astype(np.float64); th0 = x0[:, 2].astype(np.float64)
    v = ul[:, 0].astype(np.float64); d = ul[:, 1].astype(np.float64)
    Lw = float(np.float32(0.3302))
    sn, cs = np.sin(th0), np.cos(th0)
    sec2 = 1.0 / np.cos(d) ** 2
    a02 = -v * sn * dt; a12 = v * cs * dt
    A = np.zeros((B, 3, 3)); A[:] = np.eye(3); A[:, 0, 2] = a02; A[:, 1, 2] = a12
    Bm = np.zeros((B, 3, 2)); Bm[:, 0, 0] = cs * dt; Bm[:, 1, 0] = sn * dt
    Bm[:, 2, 0] = np.tan(d) * dt / Lw; Bm[:, 2, 1] = v * sec2 * dt / Lw
    c0r = v * th0 * sn * dt; c1r = -v * th0 * cs * dt; c2 = -d * v * sec2 * dt / Lw
    Cv = np.stack([c0r + a02 * th0, c1r + a12 * th0, c2], 1)
    ref = xr[:, :N].astype(np.float64) - np.stack([X0, Y0, th0], 1)[:, None, :]  # [B,N,3]
    refx = np.concatenate([ref, ref[:, N - 1:N]], 1)  # r_0..r_N, r_N = x_ref[N-1] (mpc.cpp:228)
    nu = np.zeros((B, 2, 3)); nu[:, :, 0] = hs[:, :, 0]; nu[:, :, 1] = hs[:, :, 1]
    beta = -hs[:, :, 2].astype(np.float64) - hs[:, :, 0] * X0[:, None] - hs[:, :, 1] * Y0[:, None]
    nrm = np.linalg.norm(nu, axis=2)  # rows normalised (same feasible set)
    nu = nu / nrm[:, :, None]; beta = beta / nrm
    return dict(B=B, N=N, q=q, r=r, ud=ud, lb=lb, ub=ub, A=A, Bm=Bm, Cv=Cv, refx=refx, nu=nu, beta=beta,
                X0=X0, Y0=Y0, th0=th0)


def rollout(S, u):
    B, N = S["B"], S["N"]
    x = np.zeros((B, N + 1, 3))
    for i in range(N):
        x[:, i + 1] = np.einsum("bij,bj->bi", S["A"], x[:, i]) + np.einsum("bij,bj->bi", S["Bm"], u[:, i]) + S["Cv"]
    return x


def cons(S, u, x):
    """the six inequality values per stage: [B, N, 6] (>= 0 feasible)"""
    c = np.empty(u.shape[:2] + (6,))
    c[..., 0] = u[..., 0] - S["lb"][0]; c[..., 1] = S["ub"][0] - u[..., 0]
    c[..., 2] = u[..., 1] - S["lb"][1]; c[..., 3] = S["ub"][1] - u[..., 1]
    xn = x[:, 1:]
    c[..., 4] = np.einsum("bj,bij->bi", S["nu"][:, 0], xn) - S["beta"][:, 0:1]
    c[..., 5] = np.einsum("bj,bij->bi", S["nu"][:, 1], xn) - S["beta"][:, 1:2]
    return c


def factor(S, sig):
    """Riccati factorisation of the Newton system: K [B,N,2,3], Hinv [B,N,2,2] (P kept implicit)."""
    B, N = S["B"], S["N"]
    A, Bm, nu = S["A"], S["Bm"], S["nu"]
    Q = np.diag(S["q"]); R = np.diag(S["r"])
    K = np.zeros((B, N, 2, 3)); Hi = np.zeros((B, N, 2, 2))
    P = Q[None] + np.einsum("b,bi,bj->bij", sig[:, N - 1, 4], nu[:, 0], nu[:, 0]) \
        + np.einsum("b,bi,bj->bij", sig[:, N - 1, 5], nu[:, 1], nu[:, 1])
    for i in range(N - 1, -1, -1):
        Rt = R[None].repeat(B, 0).copy()
        Rt[:, 0, 0] += sig[:, i, 0] + sig[:, i, 1]
        Rt[:, 1, 1] += sig[:, i, 2] + sig[:, i, 3]
        PB = P @ Bm
        H = Rt + np.transpose(Bm, (0, 2, 1)) @ PB
        X = np.transpose(PB, (0, 2, 1)) @ A
        Hinv = np.linalg.inv(H)
        Ki = -Hinv @ X
        K[:, i] = Ki; Hi[:, i] = Hinv
        if i > 0:
            Qt = Q[None] + np.einsum("b,bi,bj->bij", sig[:, i - 1, 4], nu[:, 0], nu[:, 0]) \
                + np.einsum("b,bi,bj->bij", sig[:, i - 1, 5], nu[:, 1], nu[:, 1])
            Pn = Qt + np.transpose(A, (0, 2, 1)) @ P @ A + np.transpose(X, (0, 2, 1)) @ Ki
            P = 0.5 * (Pn + np.transpose(Pn, (0, 2, 1)))
    return K, Hi


def solve(S, K, Hi, gu, gx):
    """Newton step for linear terms gu [B,N,2] (on u_i), gx [B,N,3] (on x_{i+1}): (du, dx)."""
    B, N = S["B"], S["N"]
    A, Bm = S["A"], S["Bm"]
    k = np.zeros((B, N, 2))
    p = gx[:, N - 1].copy()
    for i in range(N - 1, -1, -1):
        h = gu[:, i] + np.einsum("bji,bj->bi", Bm, p)
        k[:, i] = -np.einsum("bij,bj->bi", Hi[:, i], h)
        if i > 0:
            p = gx[:, i - 1] + np.einsum("bji,bj->bi", A, p) + np.einsum("bji,bj->bi", K[:, i], h)
    du = np.zeros((B, N, 2)); dx = np.zeros((B, N + 1, 3))
    for i in range(N):
        du[:, i] = np.einsum("bij,bj->bi", K[:, i], dx[:, i]) + k[:, i]
        dx[:, i + 1] = np.einsum("bij,bj->bi", A, dx[:, i]) + np.einsum("bij,bj->bi", Bm, du[:, i])
    return du, dx


def dcons(S, du, dx):
    dc = np.empty(du.shape[:2] + (6,))
    dc[..., 0] = du[..., 0]; dc[..., 1] = -du[..., 0]; dc[..., 2] = du[..., 1]; dc[..., 3] = -du[..., 1]
    dc[..., 4] = np.einsum("bj,bij->bi", S["nu"][:, 0], dx[:, 1:])
    dc[..., 5] = np.einsum("bj,bij->bi", S["nu"][:, 1], dx[:, 1:])
    return dc


def lin_terms(S, u, x, w):
    """gu, gx for the D' w pull-back plus the cost gradient: grad f - D' w"""
    gu = (u - S["ud"]) * S["r"]
    gu[..., 0] -= w[..., 0] - w[..., 1]
    gu[..., 1] -= w[..., 2] - w[..., 3]
    gx = (x[:, 1:] - S["refx"][:, 1:]) * S["q"]
    gx -= w[..., 4:5] * S["nu"][:, None, 0] + w[..., 5:6] * S["nu"][:, None, 1]
    return gu, gx


def step_len(v, dv):
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(dv < 0, -v / dv, np.inf)
    return np.minimum(1.0, r.reshape(r.shape[0], -1).min(1))


def stationarity(S, u, x, z):
    """reduced gradient of the Lagrangian (costate backward), inf-norm per QP"""
    B, N = S["B"], S["N"]
    gu, gx = lin_terms(S, u, x, z)
    lam = gx[:, N - 1].copy()
    res = np.zeros(B)
    for i in range(N - 1, -1, -1):
        g = gu[:, i] + np.einsum("bji,bj->bi", S["Bm"], lam)
        res = np.maximum(res, np.abs(g).max(1))
        if i > 0:
            lam = gx[:, i - 1] + np.einsum("bji,bj->bi", S["A"], lam)
    return res


def polish(S, u, x, s, z, rho=1e8, tolp=1e-9, told=1e-9, refine=1, eps_s=0.0, act=None):
    """OSQP-style polish: guess the active rows (z > s), solve the equality-constrained QP on
    them by an augmented Lagrangian with penalty rho (one Riccati factorisation, 1 + refine solves
    on it), verify primal feasibility of the inactive rows and the sign of the active rows'
    multipliers. Returns (u+, x+, z+, ok [B])."""
    c = cons(S, u, x)
    if act is None:
        act = z > s
    sig = np.where(act, rho, 0.0)
    K, Hi = factor(S, sig)
    y = np.where(act, z, 0.0) if POLY0 else np.zeros_like(z)
    for r in range(1 + refine):
        gu, gx = lin_terms(S, u, x, np.where(act, y - rho * c, 0.0))
        du, dx = solve(S, K, Hi, gu, gx)
        u = u + du
        x = rollout(S, u)
        c = cons(S, u, x)
        y = np.where(act, y - rho * c, 0.0)
    scale = np.ones_like(c)
    scale[..., 0] += abs(S["lb"][0]); scale[..., 1] += abs(S["ub"][0])
    scale[..., 2] += abs(S["lb"][1]); scale[..., 3] += abs(S["ub"][1])
    okp = (act | (c >= -tolp * scale)).reshape(c.shape[0], -1).all(1)
    okd = ((y >= -told) | (s <= eps_s)).reshape(c.shape[0], -1).all(1)
    okd &= (~act | (np.abs(c) <= tolp * scale)).reshape(c.shape[0], -1).all(1)
    polish.viol = np.where(act, np.abs(c), 0).reshape(c.shape[0], -1).max(1)
    polish.next_act = (act & (y > 1e-12)) | (~act & (c < -1e-12 * scale))
    return u, x, y, okp & okd


POL = {}
POLY0 = True
PREGUESS = False
SEPSTEP = False
ZINIT = 1.0
ZMODE = 0
PDAS_GAPFIRST = False
NOSOC = False
REUSE = 0
REUSE_LOG = []
FIXSIG = 0.0


def polish_reuse(S, u, x, s, z, K, Hi, sig, nsolve=2, tolp=1e-7, told=1e-7):
    """Polish on the IPM's own factorisation (penalty Sig = z/s per row): active rows (z > s) by
    an augmented Lagrangian with penalty Sig_j and multiplier start z_j, inactive rows as
    proximal terms Sig_j (D_j (w - w_k))^2. Each round is one solve with the same factor."""
    B = S["B"]
    act = z > s
    y = np.where(act, z, 0.0)
    scale = np.ones(act.shape)
    scale[..., 0] += abs(S["lb"][0]); scale[..., 1] += abs(S["ub"][0])
    scale[..., 2] += abs(S["lb"][1]); scale[..., 3] += abs(S["ub"][1])
    ok = np.zeros(B, bool); used = np.full(B, nsolve + 1)
    uu, xx = u.copy(), x.copy()
    for r in range(nsolve):
        c = cons(S, uu, xx)
        gu, gx = lin_terms(S, uu, xx, np.where(act, y - sig * c, 0.0))
        du, dx = solve(S, K, Hi, gu, gx)
        uu = uu + du; xx = rollout(S, uu)
        c = cons(S, uu, xx)
        y = np.where(act, y - sig * c, 0.0)
        okp = (act | (c >= -tolp * scale)).reshape(B, -1).all(1)
        okd = (~act | ((y >= -told) & (np.abs(c) <= tolp * scale))).reshape(B, -1).all(1)
        newly = okp & okd & ~ok
        used[newly] = r + 1
        ok |= okp & okd
    return uu, xx, y, ok, used


def pdas(S, u, x, act, y, max_pass=30, rho=1e8, tolp=1e-9, told=1e-9, eps=1e-12):
    """Primal-dual active set on the penalty/augmented-Lagrangian Riccati: each pass solves the
    equality QP on the guessed rows (one factorisation, two solves), then re-guesses
    act = (act & y > eps) | (~act & c < -eps). Converged when nothing changes and the point
    verifies. Returns (u, x, y, done, passes)."""
    B = S["B"]
    done = np.zeros(B, bool); passes = np.full(B, max_pass)
    scale = np.ones(act.shape)
    scale[..., 0] += abs(S["lb"][0]); scale[..., 1] += abs(S["ub"][0])
    scale[..., 2] += abs(S["lb"][1]); scale[..., 3] += abs(S["ub"][1])
    for k in range(max_pass):
        sig = np.where(act, rho, 0.0)
        K, Hi = factor(S, sig)
        yy = np.where(act, y, 0.0)
        uu, xx = u.copy(), x.copy()
        c = cons(S, uu, xx)
        for r in range(2):
            gu, gx = lin_terms(S, uu, xx, np.where(act, yy - rho * c, 0.0))
            du, dx = solve(S, K, Hi, gu, gx)
            uu = uu + du
            xx = rollout(S, uu)
            c = cons(S, uu, xx)
            yy = np.where(act, yy - rho * c, 0.0)
        okp = (act | (c >= -tolp * scale)).reshape(B, -1).all(1)
        okd = (~act | (yy >= -told)).reshape(B, -1).all(1)
        ok = okp & okd & ~done
        passes[ok] = k + 1
        upd = ~done
        u = np.where(upd[:, None, None], uu, u); x = np.where(upd[:, None, None], xx, x)
        y = np.where(upd[:, None, None], yy, y)
        done |= ok
        if done.all():
            break
        keep = act & (yy > eps)
        add = ~act & (c < -eps * scale)
        if PDAS_GAPFIRST:  # gap rows: add only the earliest newly violated stage of each row
            g = add[..., 4:]
            first = np.argmax(g, axis=1)  # [B, 2]
            has = g.any(1)
            m1 = np.zeros_like(g)
            bi = np.arange(B)[:, None]; ki = np.arange(2)[None, :]
            m1[bi, first, ki] = has
            add[..., 4:] = m1
        nact = keep | add
        act = np.where(done[:, None, None], act, nact)
    return u, x, y, done, passes


def ipm(S, max_it=40, tol=1e-9, tau=0.995, init="lq", s_floor=1.0, verbose=False, pol_mu=0.0, ret_state=False):
    B, N = S["B"], S["N"]
    m = 6 * N
    if init == "lq":  # unconstrained LQ solution as the primal start
        u0 = np.zeros((B, N, 2)); x0 = rollout(S, u0)
        K, Hi = factor(S, np.zeros((B, N, 6)))
        gu, gx = lin_terms(S, u0, x0, np.zeros((B, N, 6)))
        du, dx = solve(S, K, Hi, gu, gx)
        u = u0 + du
    else:
        u = np.broadcast_to(0.5 * (S["lb"] + S["ub"]), (B, N, 2)).copy()
    x = rollout(S, u)
    c = cons(S, u, x)
    s = np.maximum(c, s_floor)
    z = np.ones((B, N, 6)) * ZINIT
    if ZMODE == 1:  # z s = const
        z = ZINIT / s
    done = np.zeros(B, bool); iters = np.full(B, max_it)
    pact = None; pprev = np.zeros(B, bool)
    for it in range(max_it):
        mu = (s * z).reshape(B, -1).sum(1) / m
        rp = c - s
        rpn = np.abs(rp).reshape(B, -1).max(1)
        st = stationarity(S, u, x, z)
        conv = (mu < tol) & (rpn < tol) & (st < tol)
        if pol_mu > 0:
            pa = None
            if PREGUESS and it > 0 and pact is not None:
                pa = np.where(pprev[:, None, None], pact, z > s)
            pu, px, pz, pok = polish(S, u, x, s, z, act=pa, **POL)
            pprev = mu < pol_mu
            pact = polish.next_act
            pok &= mu < pol_mu
            take = pok & ~done
            u = np.where(take[:, None, None], pu, u); x = np.where(take[:, None, None], px, x)
            conv = pok
        conv |= mu < 1e-15  # numerically at the end of the central path
        newly = conv & ~done
        iters[newly] = it
        done |= conv
        if done.all():
            break
        sig = z / s
        K, Hi = factor(S, sig)
        if REUSE:
            pu, px, pz, pok, used = polish_reuse(S, u, x, s, z, K, Hi, sig, nsolve=REUSE)
            REUSE_LOG.append((it, pok.copy(), used.copy()))
        # predictor
        rc = s * z
        gu, gx = lin_terms(S, u, x, z - (rc + z * rp) / s)
        du, dx = solve(S, K, Hi, gu, gx)
        ds = dcons(S, du, dx) + rp
        dz = -(rc + z * ds) / s
        a = np.minimum(step_len(s, ds), step_len(z, dz))
        mua = ((s + a[:, None, None] * ds) * (z + a[:, None, None] * dz)).reshape(B, -1).sum(1) / m
        sigma = (mua / mu) ** 3
        # corrector
        if NOSOC:  # no second-order term: aff + sigma mu cen (one factor, two RHS in one sweep)
            ds = ds * 0.0; dz = dz * 0.0
        if FIXSIG > 0:
            sigma = np.full_like(sigma, FIXSIG)
        rc = s * z + ds * dz - (sigma * mu)[:, None, None]
        gu, gx = lin_terms(S, u, x, z - (rc + z * rp) / s)
        du, dx = solve(S, K, Hi, gu, gx)
        ds = dcons(S, du, dx) + rp
        dz = -(rc + z * ds) / s
        a = tau * np.minimum(step_len(s, ds), step_len(z, dz))
        if verbose:
            with np.errstate(divide="ignore", invalid="ignore"):
                rs = np.where(ds < 0, -s / ds, np.inf); rz = np.where(dz < 0, -z / dz, np.inf)
            for j in range(B):
                if a[j] < 0.5 and not done[j]:
                    js = np.unravel_index(np.argmin(rs[j]), rs[j].shape); jz = np.unravel_index(np.argmin(rz[j]), rz[j].shape)
                    print("   qp", j, "a_s %.2f at %s s %.1e ds %.1e z %.1e" % (rs[j][js], js, s[j][js], ds[j][js], z[j][js]),
                          "| a_z %.2f at %s z %.1e dz %.1e s %.1e" % (rz[j][jz], jz, z[j][jz], dz[j][jz], s[j][jz]), "sigma %.2e" % sigma[j])
        a = np.where(done, 0.0, np.minimum(a, 1.0))
        if SEPSTEP:
            ap = np.where(done, 0.0, tau * step_len(s, ds)); ad = np.where(done, 0.0, tau * step_len(z, dz))
        else:
            ap = ad = a
        u = u + ap[:, None, None] * du
        x = rollout(S, u)
        s = s + ap[:, None, None] * ds
        z = z + ad[:, None, None] * dz
        c = cons(S, u, x)
        if verbose:
            print(it, "mu", " ".join("%.1e" % v for v in mu), "alpha", " ".join("%.2f" % v for v in a), "done", done.astype(int))
    if ret_state:
        return u, x, s, z, done, iters
    return u, x, done, iters


def main():
    import os

    import oracle
    from f110qp import workload
    from test_gpu_parity import halfspaces_oracle

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    w = workload.make_batch(B, N, seed=1000)
    ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, (amin, ainc, amax))
    prm = oracle.params(N)
    S = setup(prm, w["x0"], w["u_lin"], w["x_ref"], hs)
    tol = float(os.environ.get("TOL", "1e-9"))
    for k in ("rho", "tolp", "told", "eps_s"):
        if os.environ.get(k.upper()):
            POL[k] = float(os.environ[k.upper()])
    global POLY0, PREGUESS, SEPSTEP, PDAS_GAPFIRST, NOSOC, FIXSIG
    NOSOC = bool(int(os.environ.get("NOSOC", "0")))
    FIXSIG = float(os.environ.get("FIXSIG", "0"))
    PDAS_GAPFIRST = bool(int(os.environ.get("GAPFIRST", "0")))
    SEPSTEP = bool(int(os.environ.get("SEPSTEP", "0")))
    PREGUESS = bool(int(os.environ.get("PREGUESS", "0")))
    POLY0 = bool(int(os.environ.get("POLY0", "1")))
    if os.environ.get("REFINE"):
        POL["refine"] = int(os.environ["REFINE"])
    kipm = os.environ.get("KIPM")
    if kipm is not None:
        kipm = int(kipm)
        if kipm > 0:
            u, x, s_, z_, _, _ = ipm(S, max_it=kipm, tol=0.0, s_floor=float(os.environ.get("SFLOOR", "0.1")),
                                     ret_state=True)
            act, y = z_ > s_, z_
        else:
            u = np.zeros((B, N, 2)); x = rollout(S, u)
            K, Hi = factor(S, np.zeros((B, N, 6)))
            gu, gx = lin_terms(S, u, x, np.zeros((B, N, 6)))
            du, dx = solve(S, K, Hi, gu, gx)
            u = u + du; x = rollout(S, u)
            act = cons(S, u, x) < 0; y = np.zeros((B, N, 6))
        u, x, y, done, it = pdas(S, u, x, act, y)
        print("pdas after", kipm, "ipm iterations")
    else:
      u, x, done, it = ipm(S, tol=tol, init=os.environ.get("INIT", "lq"), pol_mu=float(os.environ.get("POLMU", "0")),
                         s_floor=float(os.environ.get("SFLOOR", "1.0")), verbose=bool(os.environ.get("V")))
    ur, xr, sr = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True)
    ok = (sr == 1) & done
    eu = np.abs(u - ur).max(axis=(1, 2)) / np.maximum(1, np.abs(ur).max(axis=(1, 2)))
    X = x + np.stack([S["X0"], S["Y0"], S["th0"]], 1)[:, None, :]
    ex = np.abs(X - xr).max(axis=(1, 2)) / np.maximum(1, np.abs(xr).max(axis=(1, 2)))
    print("oracle status", np.unique(sr, return_counts=True))
    print("converged", done.mean(), "iters mean", it[done].mean(), "max", it[done].max(),
          "p99", np.percentile(it[done], 99), "hist", np.bincount(it))
    print("max rel err u", eu[ok].max(), "x", ex[ok].max(), "n > 1e-6", int((eu[ok] > 1e-6).sum()))


if __name__ == "__main__":
    main()
