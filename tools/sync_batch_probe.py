"""Synchronous call cost at large batches: f110qp_solve_batch_dev_sync (the completion word: every
wave's system-scope fence, then one arrival each) against the asynchronous call plus a stream
synchronize, per batch size (kernel work identical). Prints one JSON line per size.

    python tools/sync_batch_probe.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))


def main():
    import torch

    from f110qp import capi, workload

    for N, B, gap in ((20, 1024, False), (20, 4096, False), (20, 65536, False), (40, 8192, False),
                      (40, 65536, False), (20, 1, True), (20, 256, True), (20, 4096, True)):
        w = workload.make_batch(B, N, seed=1000)
        d = {k: torch.from_numpy(np.ascontiguousarray(w[k])).cuda() for k in ("x0", "u_lin", "x_ref")}
        o = (torch.empty((B, N, 2), device="cuda"), torch.empty((B, N + 1, 3), device="cuda"),
             torch.empty((B,), dtype=torch.int32, device="cuda"))
        st = torch.cuda.Stream()
        hs = None
        if gap:  # the C3 half-spaces: one scan per QP through the device FindHalfSpaces
            ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
            hs = torch.empty((B, 2, 3), dtype=torch.float32, device="cuda")
            capi.find_half_spaces_dev(d["x0"], torch.from_numpy(ranges).cuda(), amin, ainc, amax, hs)
            torch.cuda.synchronize()
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE if gap else capi.GAP_INACTIVE))
        fs = s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], hs, *o, stream=st, sync=True)
        fa = s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], hs, *o, stream=st)
        for _ in range(10):
            fs()
        ts, ta = [], []
        for i in range(60):
            t0 = time.perf_counter()
            fs()
            ts.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            fa()
            st.synchronize()
            ta.append(time.perf_counter() - t0)
        print(json.dumps({"N": N, "B": B, "gap": gap, "dev_sync_p50_us": round(float(np.median(ts)) * 1e6, 1),
                          "async_then_sync_p50_us": round(float(np.median(ta)) * 1e6, 1),
                          "polled": s.sync_signals()}), flush=True)
        s.close()


if __name__ == "__main__":
    main()
