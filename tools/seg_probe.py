"""Fixed cost vs per-pass cost of the lane back end (sequential and partitioned-horizon kernels):
kernel time (HIP events over back-to-back launches) with the pass cap max_iter = 1..8 at a given
batch and horizon, F110QP_LANE_SEG = 1 (sequential) and 0 (auto). A linear fit of time against
min(passes, cap) separates the launch/staging/output cost from one PDAS pass.
Run on the GPU box:  python tools/seg_probe.py [B] [N]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402
capi.USE_TEST_BUILD = True  # the F110QP_* knobs below are read by the test build only

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.cuda.is_available()
capi.load()
w = workload.make_batch(B, N, seed=5, heading="true", lateral=0.6, steer_range=0.4)
dev = torch.device("cuda", 0)
x0 = torch.from_numpy(w["x0"]).to(dev)
ul = torch.from_numpy(w["u_lin"]).to(dev)
xr = torch.from_numpy(w["x_ref"]).to(dev)
uo = torch.empty((B, N, 2), dtype=torch.float32, device=dev)
xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device=dev)
st = torch.empty((B,), dtype=torch.int32, device=dev)
it = torch.empty((B,), dtype=torch.int32, device=dev)
for seg in ("1", "0"):
    os.environ["F110QP_LANE_SEG"] = seg
    rows = []
    for cap in (1, 2, 3, 4, 6, 8, 0):
        # the pass cap is max(max_iter, kmax): cap both (PDAS passes up to the cap, same iterates)
        if cap:
            os.environ["F110QP_LANE_KMAX"] = str(cap)
        else:
            os.environ.pop("F110QP_LANE_KMAX", None)
        s = capi.Solver(capi.default_config(N, backend=capi.BACKEND_LANE, max_iter=cap))
        f = s.prepare_dev(x0, ul, xr, None, uo, xo, st, it)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        K = 50
        e0.record()
        for _ in range(K):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / K * 1e3
        passes = int(it.max().item())
        rows.append((cap, passes, us))
        print(f"seg={seg} S={s.lane_segments(B)} B={B} N={N} max_iter={cap}: max passes {passes} kernel {us:.1f} us", flush=True)
        s.close()
    a = np.array([(p, u) for _, p, u in rows], float)
    k, c = np.polyfit(a[:, 0], a[:, 1], 1)
    print(f"seg={seg}: per pass {k:.2f} us, fixed {c:.2f} us", flush=True)
