# Host design check (imports the CPU oracle, so it lives under tests/): a float64 numpy model of
# the lane kernel's Riccati/PDAS with the follow-the-gap rows as stage-local mixed constraints
# (DESIGN.md section 2f), run on the bench's C3 batch and compared with the exact oracle.
# Not product code: the kernel is csrc/lane_kernel.h (GAP instantiation).
#
# Gap row k of stage i+1 (mpc.cpp:249,271,297-298, C3 semantic): nu_k' x_{i+1} >= beta_k with
# nu_k = (a_k, b_k, 0). Through the dynamics (model.cpp:42-51; B[:,1] = (0, 0, b21) so nu_k'B[:,1]
# = 0) it is a constraint on (x_i, u0_i): d_k' x_i + e_k u0_i >= f_k, d_k = A' nu_k,
# e_k = nu_k' B[:,0], f_k = beta_k - nu_k' C. Active, it pins u0_i = kappa' x_i + kappa0.
import sys

import numpy as np

sys.path.insert(0, "f110-mpc_amd")
sys.path.insert(0, "oracle")
sys.path.insert(0, "tests")


def lane_gap_solve(prm, x0, ul, xr, hs, kmax=16, max_pass=60, tol=1e-9, verbose=False, gap_first=False):
    B = x0.shape[0]
    N = prm.horizon
    dt = float(np.float32(prm.dt))
    q = np.array(prm.q[:]); r = np.array(prm.r[:]); ud = np.array(prm.u_des[:])
    lb = np.array([float(prm.u_min[0]), float(prm.u_min[1])])
    ubd = np.array([float(prm.u_max[0]), float(prm.u_max[1])])
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
    ref = xr.astype(np.float64) - np.stack([X0, Y0, th0], 1)[:, None, :]  # [B,N,3]
    Q = np.diag(q); R = np.diag(r)
    # gap rows, recentred
    nu = np.zeros((B, 2, 3)); nu[:, :, 0] = hs[:, :, 0]; nu[:, :, 1] = hs[:, :, 1]
    beta = -hs[:, :, 2].astype(np.float64) - hs[:, :, 0] * X0[:, None] - hs[:, :, 1] * Y0[:, None]
    dk = np.einsum("bji,bkj->bki", A, nu)          # A' nu_k   [B,2,3]
    ek = np.einsum("bkj,bj->bk", nu, Bm[:, :, 0])   # nu_k' B0  [B,2]
    fk = beta - np.einsum("bkj,bj->bk", nu, Cv)     # [B,2]
    AiT = np.linalg.inv(np.transpose(A, (0, 2, 1)))  # A'^-1
    # state: c0 in {0 free, 1 lb, 2 ub, 3 gap0, 4 gap1}, c1 in {0, 1, 2}
    c0 = np.zeros((B, N), int); c1 = np.zeros((B, N), int)
    degen = np.zeros(B, bool)
    jmax_hist = []
    done = np.zeros(B, bool); iters = np.zeros(B, int); conflict = np.zeros(B, int)
    bi = np.arange(B)
    for pas in range(max_pass):
        if (done | degen).all():
            break
        single = pas >= kmax
        # ---- backward
        K = np.zeros((B, N, 2, 3)); k = np.zeros((B, N, 2)); Z0 = np.zeros((B, N, 3)); z0 = np.zeros((B, N))
        P = np.zeros((B, 3, 3)); P[:] = Q
        p = -np.einsum("ij,bj->bi", Q, ref[:, N - 1])
        for i in range(N - 1, -1, -1):
            PA = P @ A; PB = P @ Bm
            g = np.einsum("bij,bj->bi", P, Cv) + p
            Huu = R[None] + np.transpose(Bm, (0, 2, 1)) @ PB
            X = np.transpose(Bm, (0, 2, 1)) @ PA
            Y = Q[None] + np.transpose(A, (0, 2, 1)) @ PA
            h = -(R @ ud)[None] + np.einsum("bji,bj->bi", Bm, g)
            hx = -np.einsum("ij,bj->bi", Q, ref[:, i]) + np.einsum("bji,bj->bi", A, g)
            a0 = c0[:, i].copy(); a1 = c1[:, i].copy()
            Kb = np.zeros((B, 2, 3)); kb = np.zeros((B, 2))
            gi = np.clip(a0 - 3, 0, 1)
            isg = a0 >= 3
            ee = ek[bi, gi]
            Kb[:, 0] = np.where(isg[:, None], -dk[bi, gi] / np.where(isg, ee, 1.0)[:, None], 0.0)
            kb[:, 0] = np.where(a0 == 1, lb[0], np.where(a0 == 2, ubd[0], np.where(isg, fk[bi, gi] / np.where(isg, ee, 1.0), 0.0)))
            kb[:, 1] = np.where(a1 == 1, lb[1], np.where(a1 == 2, ubd[1], 0.0))
            f0 = a0 == 0; f1 = a1 == 0
            M00 = np.where(f0, Huu[:, 0, 0], 1.0); M11 = np.where(f1, Huu[:, 1, 1], 1.0)
            M01 = np.where(f0 & f1, Huu[:, 0, 1], 0.0)
            det = M00 * M11 - M01 * M01
            I = np.zeros((B, 2, 2))
            I[:, 0, 0] = np.where(f0, M11 / det, 0); I[:, 1, 1] = np.where(f1, M00 / det, 0)
            I[:, 0, 1] = I[:, 1, 0] = np.where(f0 & f1, -M01 / det, 0)
            Kf = Kb - I @ (X + Huu @ Kb)
            kf = kb - np.einsum("bij,bj->bi", I, h + np.einsum("bij,bj->bi", Huu, kb))
            Z = Huu @ Kf + X
            z = np.einsum("bij,bj->bi", Huu, kf) + h
            K[:, i] = Kf; k[:, i] = kf; Z0[:, i] = Z[:, 0]; z0[:, i] = z[:, 0]
            Pn = Y + np.transpose(X, (0, 2, 1)) @ Kf + np.transpose(Kf, (0, 2, 1)) @ Z
            P = 0.5 * (Pn + np.transpose(Pn, (0, 2, 1)))
            p = hx + np.einsum("bji,bj->bi", X, kf) + np.einsum("bji,bj->bi", Kf, z)
        # ---- forward
        x = np.zeros((B, 3)); lam = p.copy()
        changed = np.zeros(B, bool); flipped = np.zeros(B, bool); pconf = np.zeros(B, bool)
        gnew = np.zeros((B, 2), bool)
        jmax = np.full(B, -1)
        U = np.zeros((B, N, 2)); Xs = np.zeros((B, N + 1, 3))
        for i in range(N):
            u = np.einsum("bij,bj->bi", K[:, i], x) + k[:, i]
            psi0 = np.einsum("bj,bj->b", Z0[:, i], x) + z0[:, i]
            w = np.einsum("bij,bj->bi", AiT, lam - np.einsum("ij,bj->bi", Q, x - ref[:, i]))
            a0 = c0[:, i].copy(); a1 = c1[:, i].copy()
            isg = a0 >= 3; gi = np.clip(a0 - 3, 0, 1)
            mu_g = np.where(isg, psi0 / np.where(isg, ek[bi, gi], 1.0), 0.0)
            lam = w + mu_g[:, None] * nu[bi, gi] * isg[:, None]
            xn = np.einsum("bij,bj->bi", A, x) + np.einsum("bij,bj->bi", Bm, u) + Cv
            g1 = r[1] * (u[:, 1] - ud[1]) + Bm[:, 2, 1] * lam[:, 2]
            # u0's four candidate rows: value c (>= 0 feasible) and multiplier when active
            cval = np.stack([u[:, 0] - lb[0], ubd[0] - u[:, 0],
                             np.einsum("bj,bj->b", nu[:, 0], xn) - beta[:, 0],
                             np.einsum("bj,bj->b", nu[:, 1], xn) - beta[:, 1]], 1)
            mult = np.stack([psi0, -psi0, psi0 / ek[:, 0], psi0 / ek[:, 1]], 1)
            act_old = np.stack([a0 == 1, a0 == 2, a0 == 3, a0 == 4], 1)
            scale = np.stack([1 + abs(lb[0]) + 0 * psi0, 1 + abs(ubd[0]) + 0 * psi0,
                              1 + np.abs(beta[:, 0]), 1 + np.abs(beta[:, 1])], 1)
            act_new = np.where(act_old, mult > tol, cval < -tol * scale)
            if gap_first:  # at most one NEW gap row per side and pass (the earliest violated stage)
                newg = act_new[:, 2:] & ~act_old[:, 2:]
                act_new[:, 2:] &= ~(newg & gnew)
                gnew |= newg
            nact = act_new.sum(1)
            # more than one row pinning u0: keep the old one if it stays, else the most violated
            viol = np.where(act_new, np.where(act_old, np.inf, -cval / scale), -np.inf)
            pick = np.argmax(viol, 1)
            conflict += nact > 1
            pconf |= nact > 1
            n0 = np.where(nact == 0, 0, pick + 1)
            # u1 box
            n1 = np.where(a1 == 1, np.where(g1 > tol, 1, 0), np.where(a1 == 2, np.where(g1 < -tol, 2, 0),
                          np.where(u[:, 1] < lb[1] - tol, 1, np.where(u[:, 1] > ubd[1] + tol, 2, 0))))
            if single:
                take0 = (n0 != a0) & ~flipped
                c0[:, i] = np.where(take0, n0, a0); flipped |= take0
                take1 = (n1 != a1) & ~flipped
                c1[:, i] = np.where(take1, n1, a1); flipped |= take1
            else:
                c0[:, i] = n0; c1[:, i] = n1
            chg_i = (c0[:, i] != a0) | (c1[:, i] != a1)
            changed |= chg_i
            jmax = np.where(chg_i, i, jmax)
            U[:, i] = u; Xs[:, i + 1] = xn
            x = xn
        degen |= ~done & ~changed & pconf  # a fixed point that needs two rows on one u0
        changed |= pconf
        jmax_hist.append(np.where(changed, jmax, -1))
        newly = ~done & ~changed
        iters[newly] = pas + 1
        done |= ~changed
        if pas == 0:
            U_out = U.copy(); X_out = Xs.copy()
        U_out[newly] = U[newly]; X_out[newly] = Xs[newly]
    X_out = X_out + np.stack([X0, Y0, th0], 1)[:, None, :]
    lane_gap_solve.jmax_hist = jmax_hist
    return U_out, X_out, done, iters, degen


def main():
    import oracle
    from f110qp import workload
    from test_gpu_parity import halfspaces_oracle

    B, N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 20
    w = workload.make_batch(B, N, seed=1000)
    ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, (amin, ainc, amax))
    prm = oracle.params(N)
    import os
    u, x, done, it, conf = lane_gap_solve(prm, w["x0"], w["u_lin"], w["x_ref"], hs,
                                          gap_first=bool(int(os.environ.get("GAP_FIRST", "0"))),
                                          kmax=int(os.environ.get("KMAX", "16")))
    ur, xr, sr = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True)
    ok = (sr == 1) & done
    eu = np.abs(u - ur).max(axis=(1, 2)) / np.maximum(1, np.abs(ur).max(axis=(1, 2)))
    print("oracle status", np.unique(sr, return_counts=True))
    print("converged", done.mean(), "passes mean", it[done].mean(), "max", it[done].max(),
          "p99", np.percentile(it[done], 99), "degenerate (rescue)", int(conf.sum()))
    print("max rel err u (converged & solved)", eu[ok].max() if ok.any() else None,
          "n bad", int((eu[ok] > 1e-6).sum()))
    print("not converged but oracle solved", int(((sr == 1) & ~done).sum()),
          "converged but oracle not solved", int(((sr != 1) & done).sum()))


if __name__ == "__main__":
    main()
