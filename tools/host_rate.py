"""PCIe-inclusive rate of the host-pointer entry point (f110qp_solve_batch): wall clock per call
with numpy inputs and outputs in host memory (packed pinned staging, one H2D + one D2H per call
above 64 QPs, zero-copy at or below). Not bench.py's `value` (inputs resident in HBM there).
Usage: python tools/host_rate.py [batch ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402

N = 20
for B in [int(a) for a in sys.argv[1:]] or [1, 64, 1024, 4096, 65536]:
    w = workload.make_batch(B, N, seed=7)
    ctx = capi.Solver(capi.default_config(N))
    for _ in range(3):
        ctx.solve(w["x0"], w["u_lin"], w["x_ref"])
    reps = 50 if B <= 4096 else 10
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        u, x, st, it = ctx.solve(w["x0"], w["u_lin"], w["x_ref"])
        t.append(time.perf_counter() - t0)
    p50 = float(np.median(t))
    print(f"host pointers B={B:6d} N={N}: p50 {p50 * 1e6:9.1f} us/call  {B / p50:.3e} QP/s  "
          f"solved {np.mean(st == 1):.3f}", flush=True)
    ctx.close()
