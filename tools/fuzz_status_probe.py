"""GPU probe of the status disagreements of tests/test_gpu_parity.py::test_fuzz_configs_against_oracle:
replays the fuzz generator for seeds [a, b), runs the back end the test picks, and records every QP
whose status differs from the oracle's (or that the oracle leaves UNCERTIFIED) with its inputs and
configuration in an npz for host-side analysis. Test infrastructure (imports the oracle).

usage: python tools/fuzz_status_probe.py OUT.npz [seed_lo seed_hi]
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
    out = sys.argv[1]
    lo, hi = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1, 5)
    recs = []
    summary = []
    for seed in range(lo, hi):
        rng = np.random.default_rng(9000 + seed)
        for case in range(4):
            N = int(rng.choice([1, 2, 5, 13, 20, 27, 33, 40, 48]))
            lo0, lo1 = float(rng.uniform(1.0, 3.5)), float(rng.uniform(-0.6, -0.1))
            hi0, hi1 = lo0 + float(rng.uniform(0.3, 2.0)), -lo1 * float(rng.uniform(0.5, 1.5))
            ud = [float(rng.choice([hi0, lo0, 0.5 * (lo0 + hi0)])), float(rng.choice([0.0, hi1, lo1]))]
            q01 = float(rng.choice([0.0, 1.0, 10.0, 40.0]))
            over = dict(q=[q01, q01 if rng.random() < 0.5 else float(rng.uniform(0.5, 20.0)),
                           float(rng.choice([0.0, 0.5, 3.0]))],
                        r=[float(rng.uniform(0.05, 2.0)), float(rng.uniform(0.5, 10.0))], u_des=ud,
                        u_min=[lo0, lo1], u_max=[hi0, hi1])
            dt = float(np.float32(rng.choice([0.005, 0.01, 0.02, 0.05])))
            B = int(rng.integers(1, 400))
            gap = bool(rng.random() < 0.3)
            be = "wave" if (gap or rng.random() < 0.5) else "lane"
            w = workload.make_batch(B, N, seed=int(rng.integers(1 << 30)), heading="true",
                                    lateral=float(rng.uniform(0.0, 1.5)), steer_range=float(rng.uniform(0.0, 0.8)))
            hs = None
            if gap:
                ranges, amin, ainc, amax = workload.make_scans(B, seed=int(rng.integers(1 << 30)))
                hs = halfspaces_oracle(oracle, w["x0"], ranges, (amin, ainc, amax))
            cfg = capi.default_config(N, gap_mode=capi.GAP_ACTIVE if gap else capi.GAP_INACTIVE,
                                      backend=capi.BACKEND_WAVE if be == "wave" else capi.BACKEND_LANE, dt=dt, **over)
            s = capi.Solver(cfg)
            u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
            s.close()
            prm = oracle.params(N, dt=dt, **over)
            ur, xr, sr = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=gap)
            bad = (st != sr) | (sr == oracle.UNCERTIFIED)
            summary.append(dict(seed=seed, case=case, N=N, dt=dt, be=be, gap=gap, B=B,
                                mismatch=int(bad.sum()), pairs=sorted({(int(a), int(b)) for a, b in zip(st[bad], sr[bad])})))
            for b in np.where(bad)[0]:
                recs.append(dict(seed=seed, case=case, index=int(b), N=N, dt=dt, be=be, gap=gap, over=json.dumps(over),
                                 x0=w["x0"][b], u_lin=w["u_lin"][b], x_ref=w["x_ref"][b],
                                 hs=(hs[b] if gap else np.zeros((2, 3), np.float32)), st=int(st[b]), sr=int(sr[b]),
                                 it=int(it[b])))
    for row in summary:
        if row["mismatch"]:
            print(json.dumps(row))
    print("total mismatching QPs", len(recs), "over", len(summary), "cases")
    np.savez(out, recs=np.array([json.dumps({k: (v.tolist() if isinstance(v, np.ndarray) else v)
                                             for k, v in r.items()}) for r in recs]))


if __name__ == "__main__":
    main()
