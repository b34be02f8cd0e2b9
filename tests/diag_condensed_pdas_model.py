# Host design check (imports the CPU oracle, so it lives under tests/): numpy PDAS (HIK) on the
# condensed C3 QP with every row (box + gap) through S_A = N_A' W N_A: passes, active-set sizes
# and singular S_A per QP, vs the oracle; kmax multi-flip passes then single flips.
import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'f110-mpc_amd'); sys.path.insert(0, 'oracle')
import numpy as np, oracle
from f110qp import workload
from test_gpu_parity import halfspaces_oracle
from diag_gi_selection_model import condensed

def pdas(H, g, Cn, b, kmax=16, maxp=60, tol=1e-9):
    W = np.linalg.inv(H); xu = -W @ g
    m = len(b)
    act = np.zeros(m, bool)
    qs = []
    for p in range(maxp):
        A = np.where(act)[0]
        if len(A):
            NA = Cn[A].T
            S = NA.T @ W @ NA
            try:
                mu = np.linalg.solve(S, b[A] - NA.T @ xu)
            except np.linalg.LinAlgError:
                return None, p, qs, 'singular'
            x = xu + W @ NA @ mu
        else:
            mu = np.zeros(0); x = xu
        qs.append(len(A))
        s = Cn @ x - b
        new = act.copy()
        mult = np.zeros(m); mult[A] = mu
        scale = 1 + np.abs(b)
        want = np.where(act, mult > tol, s < -tol * scale)
        if p >= kmax:  # single flip: least index
            diff = np.where(want != act)[0]
            if len(diff): new[diff[0]] = want[diff[0]]
        else:
            new = want
        if (new == act).all():
            return x, p + 1, qs, 'ok'
        act = new
    return x, maxp, qs, 'maxpass'

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = 20
w = workload.make_batch(4096, N, seed=1000)
ranges, amin, ainc, amax = workload.make_scans(4096, seed=2000)
idx = np.arange(B)
hs = halfspaces_oracle(oracle, w['x0'][idx], ranges[idx], (amin, ainc, amax))
prm = oracle.params(N)
ur, xr_, sr = oracle.solve_batch(prm, w['x0'][idx], w['u_lin'][idx], w['x_ref'][idx], hs, gap_active=True)
P = []; Q = []; st = []; bad = 0
for j in range(B):
    H, g, Cn, b = condensed(prm, w['x0'][j].astype(float), w['u_lin'][j].astype(float), w['x_ref'][j], hs[j].astype(float))
    x, p, qs, s = pdas(H, g, Cn, b)
    P.append(p); Q.append(max(qs) if qs else 0); st.append(s)
    if s == 'ok' and np.abs(x - ur[j].reshape(-1)).max() > 1e-6: bad += 1
P = np.array(P); Q = np.array(Q); st = np.array(st)
print('status', {k: int((st == k).sum()) for k in set(st)}, 'wrong', bad)
print('passes mean %.2f p99 %.0f max %d' % (P.mean(), np.percentile(P, 99), P.max()), 'max q', Q.max())
# cost model: GI ~ its * (3k + 350 q) cycles ; PDAS ~ passes * (1.5k + q^2*6 + 150 q)
print('hist', np.bincount(P).tolist())
