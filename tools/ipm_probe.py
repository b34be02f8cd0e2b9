"""GPU probe of the interior-point lane kernel (lane_ipm_kernel.h) on the bench's C3 batch:
status and accuracy against the exact oracle, the iteration histogram, and the kernel time of the
lane (interior point + hand-over) and wave (GI) back ends by HIP events. Test infrastructure
(imports the oracle); writes one JSON line per batch size to stdout.

usage: python tools/ipm_probe.py [B ...]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "f110-mpc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from f110qp import capi, workload  # noqa: E402
import oracle  # noqa: E402


def time_debug(B=4096, N=20, ks=(0, 5, 10)):
    """kernel us of k interior-point iterations without the polish (F110QP_IPM_DEBUG)"""
    dev = torch.device("cuda:0")
    w = workload.make_batch(B, N, seed=1000)
    hs = np.tile(np.float32([[1.0, 0.2, 30.0], [-0.3, 1.0, 30.0]]), (B, 1, 1))
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    x0, ul, xrf, hsd = T(w["x0"]), T(w["u_lin"]), T(w["x_ref"]), T(hs.reshape(B, 6))
    os.environ["F110QP_IPM_DEBUG"] = "1"
    res = {}
    for k in ks:
        os.environ["F110QP_IPM_MAXIT"] = str(k)
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_LANE))
        u = torch.empty(B, N, 2, device=dev)
        x = torch.empty(B, N + 1, 3, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        launch = s.prepare_dev(x0, ul, xrf, hsd, u, x, st)
        launch()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            launch()
        e1.record()
        torch.cuda.synchronize()
        res[k] = round(e0.elapsed_time(e1) * 100.0, 1)
        s.close()
    del os.environ["F110QP_IPM_DEBUG"], os.environ["F110QP_IPM_MAXIT"]
    print(json.dumps({"debug_us_by_iters": res}), flush=True)


def main():
    if sys.argv[1:2] == ["time"]:
        time_debug()
        return
    sizes = [int(a) for a in sys.argv[1:]] or [4096]
    N = 20
    dev = torch.device("cuda:0")
    for B in sizes:
        w = workload.make_batch(B, N, seed=1000)
        ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
        t0 = time.time()
        hs = np.zeros((B, 2, 3), np.float32)
        for b in range(B):
            rc, l1, l2, _, _ = oracle.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], amin, ainc, amax)
            hs[b] = l1, l2
        ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=True)
        t_or = time.time() - t0
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        x0, ul, xrf, hsd = T(w["x0"]), T(w["u_lin"]), T(w["x_ref"]), T(hs.reshape(B, 6))
        out = {"B": B, "N": N, "oracle_s": round(t_or, 2)}
        for name, be in (("lane", capi.BACKEND_LANE), ("wave", capi.BACKEND_WAVE)):
            s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=be))
            info = s.backend_info(B)
            segs = s.lane_segments(B)
            u = torch.empty(B, N, 2, device=dev)
            x = torch.empty(B, N + 1, 3, device=dev)
            st = torch.empty(B, dtype=torch.int32, device=dev)
            it = torch.empty(B, dtype=torch.int32, device=dev)
            launch = s.prepare_dev(x0, ul, xrf, hsd, u, x, st, it)
            launch()
            torch.cuda.synchronize()
            uu, ss, ii = u.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()
            ok = (sr == 1) & (ss == 1)
            eu = np.abs(uu - ur).max(axis=(1, 2)) / np.maximum(1, np.abs(ur).max(axis=(1, 2)))
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    launch()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 100.0)  # us per call
            out[name] = dict(backend=info[0], qpw=info[1], segments=segs, us=round(min(ts), 1),
                             status_match=int((ss == sr).sum()), status_hist={int(k): int(v) for k, v in zip(*np.unique(ss, return_counts=True))},
                             max_rel_err_u=float(eu[ok].max()) if ok.any() else None,
                             iters_max=int(ii[ss == 1].max()) if (ss == 1).any() else None,
                             iters_hist=np.bincount(np.clip(ii[ss == 1], 0, 60)).tolist())
            s.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
