# Host diagnostic; it imports the CPU oracle, so it lives under tests/ (test infrastructure).
# Active-row census of the bench C3 batch on the CPU oracle; host only.
import sys, numpy as np
sys.path.insert(0, "f110-mpc_amd"); sys.path.insert(0, ".")
from f110qp import capi, workload
from oracle import oracle
B, N = 4096, 20
w = workload.make_batch(B, N, seed=1000)
ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
hs = np.zeros((B, 2, 3), np.float32)
for b in range(B):
    l1, l2 = capi.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], amin, ainc, amax)
    hs[b, 0] = l1; hs[b, 1] = l2
prm = oracle.params(N)
na = np.zeros(B, int); st = np.zeros(B, int); ngap = np.zeros(B, int); nbox = np.zeros(B, int)
m_dyn = 3 * (N + 1)
for b in range(B):
    r = oracle.solve(prm, w["x0"][b], w["u_lin"][b], w["x_ref"][b], hs[b], gap_active=True)
    na[b] = r["n_active"]; st[b] = r["status"]
    y = r["y"]
    ngap[b] = (np.abs(y[m_dyn:m_dyn + 2 * (N + 1)]) > 1e-9).sum()
    nbox[b] = (np.abs(y[m_dyn + 2 * (N + 1):]) > 1e-9).sum()
np.savez("/tmp/sh/c3.npz", na=na, st=st, ngap=ngap, nbox=nbox, hs=hs)
print("status", np.unique(st, return_counts=True))
print("n_active pct", np.percentile(na, [50, 90, 99, 99.9, 100]))
o = np.argsort(-na)[:10]
for b in o: print(b, na[b], ngap[b], nbox[b], st[b], hs[b].ravel())
