"""Quick GPU-vs-oracle probe (prints per-config error statistics). Debug aid."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle
from f110qp import capi, workload

def run(N, B, gap, seed=1):
    w = workload.make_batch(B, N, seed=seed)
    hs = None
    if gap:
        ranges, amin, ainc, amax = workload.make_scans(B, seed=seed)
        hs = np.zeros((B, 2, 3), np.float32)
        for b in range(B):
            l1, l2 = capi.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], amin, ainc, amax)
            hs[b, 0], hs[b, 1] = l1, l2
    cfg = capi.default_config(N, gap_mode=1 if gap else 0)
    s = capi.Solver(cfg)
    t = time.time()
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    tg = time.time() - t
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=gap)
    ok = (st == 1) & (sr == 1)
    eu = np.abs(u - ur).max(axis=(1, 2)) / np.maximum(1, np.abs(ur).max(axis=(1, 2)))
    ex = np.abs(x - xr).max(axis=(1, 2)) / np.maximum(1, np.abs(xr).max(axis=(1, 2)))
    print(f"N={N} B={B} gap={gap}: gpu status {dict(zip(*np.unique(st, return_counts=True)))} oracle {dict(zip(*np.unique(sr, return_counts=True)))} "
          f"status-agree {(st == sr).mean():.4f} iters mean {it.mean():.2f} max {it.max()} | eu max {np.nanmax(np.where(ok, eu, 0)):.3e} "
          f"ex max {np.nanmax(np.where(ok, ex, 0)):.3e} n>1e-4 {(np.where(ok, eu, 0) > 1e-4).sum()} t {tg*1e3:.1f} ms", flush=True)
    bad = np.where(ok & (eu > 1e-4))[0]
    if len(bad):
        b = bad[0]
        print("  worst", b, "eu", eu[b], "\n  gpu u", u[b, :4].ravel(), "\n  ref u", ur[b, :4].ravel(), flush=True)
    return eu

if __name__ == "__main__":
    for N, B, gap in [(20, 256, False), (20, 1024, False), (5, 256, False), (30, 256, False), (32, 256, False),
                      (20, 512, True), (10, 256, True)]:
        run(N, B, gap)
