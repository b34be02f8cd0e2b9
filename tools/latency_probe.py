"""Single-QP and small-batch latency of both back ends (BASELINE metric "solve p50 latency"):
for B in a range of small batches and N = 20 / 40, the kernel time by HIP events over back-to-back
launches and the wall time per call (one C call through the prepared launcher + stream sync), for
the wave kernel and the lane back end at every segment count S it can run. Prints one JSON line.

usage: python tools/latency_probe.py [reps]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402
capi.USE_TEST_BUILD = True  # the F110QP_* knobs below are read by the test build only


def run(N, B, be, seg, reps, dev):
    if seg:
        os.environ["F110QP_LANE_SEG"] = str(seg)
    else:
        os.environ.pop("F110QP_LANE_SEG", None)
    w = workload.make_batch(B, N, seed=77 + B)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    x0, ul, xr = T(w["x0"]), T(w["u_lin"]), T(w["x_ref"])
    s = capi.Solver(capi.default_config(N, backend=be))
    got = s.lane_segments(B) if be == capi.BACKEND_LANE else 0
    u = torch.empty(B, N, 2, device=dev)
    x = torch.empty(B, N + 1, 3, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    launch = s.prepare_dev(x0, ul, xr, None, u, x, st, stream=stream)
    for _ in range(20):
        launch()
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == capi.SOLVED).all()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(50):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    k_us = e0.elapsed_time(e1) * 1000.0 / 50
    wall = []
    for _ in range(reps):
        t0 = time.perf_counter()
        launch()
        stream.synchronize()
        wall.append(time.perf_counter() - t0)
    s.close()
    wall = np.sort(np.array(wall) * 1e6)
    return dict(N=N, B=B, backend="lane" if be == capi.BACKEND_LANE else "wave", S=got, kernel_us=round(k_us, 2),
                wall_p50_us=round(float(np.percentile(wall, 50)), 2), wall_p99_us=round(float(np.percentile(wall, 99)), 2))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rows = []
    for N in (20, 40):
        for B in (1, 4, 16, 64, 256, 512, 768, 1024):
            rows.append(run(N, B, capi.BACKEND_WAVE, 0, reps, dev))
            for S in (2, 4, 8):
                if N // S >= 2:
                    rows.append(run(N, B, capi.BACKEND_LANE, S, reps, dev))
            print(json.dumps(rows[-4:]), flush=True)
    print(json.dumps({"latency_rows": rows}))


if __name__ == "__main__":
    main()
