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


def main():
    seed, want = int(sys.argv[1]), int(sys.argv[2])
    rng = np.random.default_rng(7100 + seed)
    for case in range(want + 1):
        N = int(rng.choice([5, 13, 20, 27, 33, 40, 48]))
        lo0, lo1 = float(rng.uniform(1.0, 3.5)), float(rng.uniform(-0.6, -0.1))
        hi0, hi1 = lo0 + float(rng.uniform(0.3, 2.0)), -lo1 * float(rng.uniform(0.5, 1.5))
        ud = [float(rng.choice([hi0, lo0, 0.5 * (lo0 + hi0)])), float(rng.choice([0.0, hi1, lo1]))]
        q01 = float(rng.choice([0.0, 1.0, 10.0, 40.0]))
        over = dict(q=[q01, q01 if rng.random() < 0.5 else float(rng.uniform(0.5, 20.0)),
                       float(rng.choice([0.0, 0.5, 3.0]))],
                    r=[float(rng.uniform(0.05, 2.0)), float(rng.uniform(0.5, 10.0))], u_des=ud,
                    u_min=[lo0, lo1], u_max=[hi0, hi1])
        dt = float(np.float32(rng.choice([0.005, 0.01, 0.02, 0.05])))
        B = int(rng.integers(1024, 1600))
        w = workload.make_batch(B, N, seed=int(rng.integers(1 << 30)), heading="true",
                                lateral=float(rng.uniform(0.0, 1.5)), steer_range=float(rng.uniform(0.0, 0.8)))
        ranges, amin, ainc, amax = workload.make_scans(B, seed=int(rng.integers(1 << 30)))
        if case < want:
            continue
        hs = halfspaces_oracle(oracle, w["x0"], ranges, (amin, ainc, amax))
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
        print(json.dumps(out))


if __name__ == "__main__":
    main()
