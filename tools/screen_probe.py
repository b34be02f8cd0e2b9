"""Status probe of one gap batch on the screened AUTO path and the wave-only path against the
oracle: per mismatching QP its statuses, iterations and whether the screen passed it. Test
infrastructure (imports the oracle).

usage: python tools/screen_probe.py N B seed
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
    N, B, seed = (int(a) for a in sys.argv[1:4])
    w = workload.make_batch(B, N, seed=seed)
    ranges, *geom = workload.make_scans(B, seed=seed)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True)
    out = {}
    for name, be in (("auto", capi.BACKEND_AUTO), ("wave", capi.BACKEND_WAVE)):
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=be))
        out[name] = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
        out[name + "_screen"] = s.gap_screen(B)
        s.close()
    sb = capi.Solver(capi.default_config(N, backend=capi.BACKEND_LANE))
    ub, xb, stb, itb = sb.solve(w["x0"], w["u_lin"], w["x_ref"])
    sb.close()
    bad = np.where((out["auto"][2] != sr) | (out["wave"][2] != sr))[0]
    rows = []
    for b in bad:
        rows.append(dict(b=int(b), oracle=int(sr[b]), auto=int(out["auto"][2][b]), wave=int(out["wave"][2][b]),
                         it_auto=int(out["auto"][3][b]), it_wave=int(out["wave"][3][b]), box_status=int(stb[b]),
                         box_vs_gap_du=float(np.abs(ub[b] - ur[b]).max())))
    print(json.dumps(dict(N=N, B=B, seed=seed, screen=out["auto_screen"], mismatches=rows)))


if __name__ == "__main__":
    main()
