# Host design check (imports the CPU oracle, so it lives under tests/): a numpy model of the wave
# kernel's Goldfarb-Idnani loop (range space, W = H^-1) on the condensed C3 QP, counting GI
# iterations per rule for picking the violated row (steepest edge).
# Rules: 1 W-norm on every row, 2 the round-2 kernel (box 1+|b|, gap |(a,b)|+1), 3 Euclidean,
# 4 W-norm on the gap rows only, 5 = 4 with any violated gap row taken before the box rows (round 4,
# kept: max 34 -> 30 on the C3 batch). Usage: python tests/diag_gi_selection_model.py [B]
import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'f110-mpc_amd'); sys.path.insert(0, 'oracle')
import numpy as np, oracle
from f110qp import workload
from test_gpu_parity import halfspaces_oracle

def condensed(prm, x0, ul, xr, hs):
    N = prm.horizon
    A, Bm, Cc = oracle.linearize(x0[2], ul[0], ul[1], prm.dt)
    X0 = np.array([x0[0], x0[1], x0[2]], float)
    # free response + Gamma, recentred on (x, y)
    xs = np.zeros((N + 1, 3)); xs[0] = [0, 0, x0[2]]
    Cr = Cc + (A - np.eye(3)) @ np.array([x0[0], x0[1], 0.0])  # recentre (x,y)
    for k in range(N):
        xs[k + 1] = A @ xs[k] + Cr
    G = np.zeros((N + 1, 3, 2 * N))
    for k in range(1, N + 1):
        G[k] = A @ G[k - 1]
        G[k][:, 2 * (k - 1):2 * k] += Bm
    q = np.array(prm.q[:]); r = np.array(prm.r[:]); ud = np.array(prm.u_des[:])
    ref = np.asarray(xr, float) - np.array([x0[0], x0[1], 0.0])
    refx = np.concatenate([ref[:N], ref[N - 1:N]], 0)  # r_0..r_N (r_0 unused: x0 fixed)
    H = np.diag(np.tile(r, N)).astype(float)
    g = -np.tile(r * ud, N).astype(float)
    for k in range(1, N + 1):
        Qk = np.diag(q)
        H += G[k].T @ Qk @ G[k]
        g += G[k].T @ Qk @ (xs[k] - refx[k])
    # constraints C u >= b
    rows = []; bs = []
    lb = np.array([prm.u_min[0], prm.u_min[1]], float); ubd = np.array([prm.u_max[0], prm.u_max[1]], float)
    for v in range(2 * N):
        e = np.zeros(2 * N); e[v] = 1; rows.append(e); bs.append(lb[v % 2])
        rows.append(-e); bs.append(-ubd[v % 2])
    for k in range(1, N + 1):
        for h in range(2):
            a, b, c = hs[h]
            beta = -c - a * x0[0] - b * x0[1]
            nrow = a * G[k][0] + b * G[k][1]
            rows.append(nrow); bs.append(beta - (a * xs[k][0] + b * xs[k][1]))
    return H, g, np.array(rows), np.array(bs)

def gi(H, g, Cn, b, rule, gn=1.0):
    n = H.shape[0]
    W = np.linalg.inv(H)
    x = -W @ g
    act = []; mult = []
    it = 0
    if rule == 1:
        cw = np.sqrt(np.einsum('ij,jk,ik->i', Cn, W, Cn))
    elif rule == 3:  # Euclidean norm of each row
        cw = np.linalg.norm(Cn, axis=1)
    elif rule in (4, 5):  # W-norm for gap rows, the kernel's 1+|bound| for box rows
        cw = np.sqrt(np.einsum('ij,jk,ik->i', Cn, W, Cn))
        cw[:4 * (n // 2)] = 1 + np.abs(b[:4 * (n // 2)])
    elif rule == 2:  # the wave kernel's scaling: box 1+|bound|, gap |(a,b)|+1
        cw = np.concatenate([1 + np.abs(b[:4 * (n // 2)]), np.full(len(b) - 4 * (n // 2), gn)])
    else:
        cw = np.ones(len(b))
    while True:
        s = Cn @ x - b
        s[act] = 0
        sc = s / cw
        p = int(np.argmin(sc))
        if sc[p] >= -1e-9 * (1 + np.abs(b[p])):
            return x, it
        if rule == 5:  # gap rows first
            nb = 4 * (n // 2)
            viol = sc < -1e-9 * (1 + np.abs(b))
            if viol[nb:].any():
                p = nb + int(np.argmin(np.where(viol[nb:], sc[nb:], np.inf)))
        np_ = Cn[p]; up = 0.0
        while True:
            it += 1
            if it > 500: return x, it
            if act:
                NA = Cn[act].T
                S = NA.T @ W @ NA
                rr = np.linalg.solve(S, NA.T @ W @ np_)
                z = W @ np_ - W @ NA @ rr
            else:
                rr = np.zeros(0); z = W @ np_
            piv = z @ np_
            t1 = np.inf; k = -1
            for a_ in range(len(act)):
                if rr[a_] > 0 and mult[a_] / rr[a_] < t1: t1 = mult[a_] / rr[a_]; k = a_
            t2 = -(np_ @ x - b[p]) / piv if piv > 1e-12 * (np_ @ W @ np_) else np.inf
            t = min(t1, t2)
            if not np.isfinite(t): return None, it
            mult = [m - t * r_ for m, r_ in zip(mult, rr)]
            up += t
            if np.isfinite(t2): x = x + t * z
            if t2 <= t1:
                act.append(p); mult.append(up); break
            del act[k]; del mult[k]

if __name__ == '__main__':
    B, N = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 20
    w = workload.make_batch(4096, N, seed=1000)
    ranges, amin, ainc, amax = workload.make_scans(4096, seed=2000)
    idx = np.arange(B) if B < 4096 else np.arange(4096)
    hs = halfspaces_oracle(oracle, w['x0'][idx], ranges[idx], (amin, ainc, amax))
    prm = oracle.params(N)
    ur, xr_, sr = oracle.solve_batch(prm, w['x0'][idx], w['u_lin'][idx], w['x_ref'][idx], hs, gap_active=True)
    its = {0: [], 1: [], 2: [], 3: [], 4: [], 5: []}
    for j, bq in enumerate(idx):
        H, g, Cn, b = condensed(prm, w['x0'][bq].astype(float), w['u_lin'][bq].astype(float), w['x_ref'][bq], hs[j].astype(float))
        gn = float(np.hypot(hs[j][0][0], hs[j][0][1])) + 1.0
        for rule in (1, 2, 3, 4, 5):
            x, it = gi(H, g, Cn, b, rule, gn)
            its[rule].append(it)
            if rule >= 4 and x is not None:
                e = np.abs(x - ur[j].reshape(-1)).max()
                assert e < 1e-6, (j, e)
    for rule in (1, 2, 3, 4, 5):
        a = np.array(its[rule]); print('rule', rule, 'mean', a.mean(), 'p99', np.percentile(a, 99), 'max', a.max())

