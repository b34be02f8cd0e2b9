"""One gap QP through the lane interior point (explicit F110QP_BACKEND_LANE) with varying
iteration caps, and with F110QP_IPM_DEBUG=1 (the raw iterate after k iterations, no polish test),
against the oracle. Test infrastructure (imports the oracle).

usage: python tools/ipm_qp_probe.py N B seed index
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "f110-mpc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from f110qp import capi, workload  # noqa: E402
import oracle  # noqa: E402
from test_gpu_parity import halfspaces_oracle  # noqa: E402


def main():
    N, B, seed, b = (int(a) for a in sys.argv[1:5])
    w = workload.make_batch(B, N, seed=seed)
    ranges, *geom = workload.make_scans(B, seed=seed)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    i = np.array([b])
    x0, ul, xr, h = w["x0"][i], w["u_lin"][i], w["x_ref"][i], hs[i]
    ur, _, sr = oracle.solve_batch(oracle.params(N), x0, ul, xr, h, gap_active=True)
    rows = []
    cases = [(0, 30, tol, sig) for tol in ("1e-8", "1e-7", "1e-6") for sig in ("1", "100", "1e4")]
    cases += [(1, k, "1e-8", "100") for k in (10, 14, 17, 20, 30)]
    for dbg, its, tol, sig in cases:
        os.environ["F110QP_IPM_MAXIT"] = str(its)
        os.environ["F110QP_IPM_DEBUG"] = str(dbg)
        os.environ["F110QP_IPM_TOL"] = tol
        os.environ["F110QP_IPM_ACTSIG"] = sig
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_LANE))
        seg = s.lane_segments(1)
        u, x, st, it = s.solve(x0, ul, xr, h)
        s.close()
        rows.append(dict(debug=dbg, maxit=its, tol=tol, act_sig=sig, S=seg, status=int(st[0]), iters=int(it[0]),
                         err=float(np.nanmax(np.abs(u - ur))) if np.isfinite(u).all() else None))
    print(json.dumps(dict(oracle=int(sr[0]), rows=rows)))


if __name__ == "__main__":
    main()
