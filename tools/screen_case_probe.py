"""Replays one case of tests/test_gpu_screen.py::test_screen_fuzz_configs_against_oracle and
localises a parity failure: per failing QP the AUTO (screened) result, the explicit wave result,
the box-only lane result against the box-only oracle, and whether the screen passed it.
Test infrastructure (imports the oracle).

usage: python tools/screen_case_probe.py seed case
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "f110-mpc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from f110qp import capi, workload  # noqa: E402
import oracle  # noqa: E402
from test_gpu_parity import halfspaces_oracle, rel_err  # noqa: E402
from fuzz_cases import screen_fuzz_case  # noqa: E402


def main():
    seed, want = int(sys.argv[1]), int(sys.argv[2])
    N, dt, B, over, w, ranges, geom = screen_fuzz_case(seed, want)
    hs = halfspaces_oracle(oracle, w["x0"], ranges, geom)
    prm = oracle.params(N, dt=dt, **over)
    ur, xr, sr = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True)
    ubr, xbr, sbr = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"])
    res = {}
    for name, be, gap in (("auto", capi.BACKEND_AUTO, True), ("wave", capi.BACKEND_WAVE, True),
                          ("lane_box", capi.BACKEND_LANE, False), ("wave_box", capi.BACKEND_WAVE, False)):
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE if gap else capi.GAP_INACTIVE,
                                            backend=be, dt=dt, **over))
        res[name] = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs if gap else None)
        if name == "lane_box":
            res["lane_info"] = (s.backend_info(B), s.lane_segments(B))
        s.close()
    ok = sr == oracle.SOLVED
    ea = rel_err(res["auto"][0], ur)
    ew = rel_err(res["wave"][0], ur)
    elb = rel_err(res["lane_box"][0], ubr)
    ewb = rel_err(res["wave_box"][0], ubr)
    bad = np.where(ok & (ea > 1e-4))[0]
    out = dict(N=N, dt=dt, B=B, over=over, lane_info=res["lane_info"], n_bad=int(len(bad)),
               n_status_mismatch=int(((res["auto"][2] != sr) & (sr != oracle.UNCERTIFIED)).sum()),
               max_err_auto=float(ea[ok].max()), max_err_wave=float(ew[ok].max()),
               max_err_lane_box=float(elb[sbr == 1].max()), max_err_wave_box=float(ewb[sbr == 1].max()),
               n_lane_box_bad=int((elb[sbr == 1] > 1e-4).sum()),
               bad=[dict(b=int(b), err_auto=float(ea[b]), err_wave=float(ew[b]), err_lane_box=float(elb[b]),
                         box_eq_gap=float(np.abs(ubr[b] - ur[b]).max()), it_auto=int(res["auto"][3][b]),
                         it_lane_box=int(res["lane_box"][3][b])) for b in bad[:8]])
    mm = np.where((res["auto"][2] != sr) & (sr != oracle.UNCERTIFIED))[0]
    out["mismatch"] = [dict(b=int(b), st_auto=int(res["auto"][2][b]), st_wave=int(res["wave"][2][b]),
                            st_oracle=int(sr[b]), err_auto=float(ea[b]), err_wave=float(ew[b]),
                            it_auto=int(res["auto"][3][b]), it_wave=int(res["wave"][3][b]))
                       for b in mm[:12]]
    out["status_counts_auto"] = {int(k): int(v) for k, v in zip(*np.unique(res["auto"][2], return_counts=True))}
    out["status_counts_oracle"] = {int(k): int(v) for k, v in zip(*np.unique(sr, return_counts=True))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
