"""Debug probe: the interior-point lane kernel's iterate after k iterations (F110QP_IPM_DEBUG=1,
F110QP_IPM_MAXIT=k: no polish, every QP returned as it stands) against the fp64 numpy model
(tests/diag_ipm_model.py) run the same k iterations from the same start. Test infrastructure.

usage: python tools/ipm_compare.py [B] [k ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "f110-mpc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from f110qp import capi, workload  # noqa: E402
import oracle  # noqa: E402
import diag_ipm_model as M  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ks = [int(a) for a in sys.argv[2:]] or [0, 1, 2, 3]
    N = 20
    w = workload.make_batch(B, N, seed=1000)
    ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
    hs = np.zeros((B, 2, 3), np.float32)
    for b in range(B):
        rc, l1, l2, _, _ = oracle.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], amin, ainc, amax)
        hs[b] = l1, l2
    prm = oracle.params(N)
    S = M.setup(prm, w["x0"], w["u_lin"], w["x_ref"], hs)
    os.environ["F110QP_IPM_DEBUG"] = "1"
    for rot in ("1", "0"):
        os.environ["F110QP_LANE_ROT"] = rot
        for k in ks:
            os.environ["F110QP_IPM_MAXIT"] = str(k)
            s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_LANE))
            u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
            s.close()
            um, xm, _, _ = M.ipm(S, max_it=k, tol=0.0, init="mid", s_floor=1.0)
            X = xm + np.stack([S["X0"], S["Y0"], S["th0"]], 1)[:, None, :]
            eu = np.abs(u - um).max(axis=(1, 2))
            ex = np.abs(x - X).max(axis=(1, 2))
            print(f"rot={rot} k={k}: |u - model| max {eu.max():.3e} median {np.median(eu):.3e}; "
                  f"|x - model| max {ex.max():.3e}; worst QP {int(np.argmax(eu))}; status {np.unique(st)}", flush=True)


if __name__ == "__main__":
    main()
