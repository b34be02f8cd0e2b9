"""C4 pass structure of the lane kernels: the PDAS pass histogram of the 65,536 x N = 40 batch
and the kernel time under a pass cap (F110QP_LANE_PASSCAP, measurement knob), with the fraction
of QPs converged within the cap. Prints one JSON line.

usage: python tools/c4_pass_probe.py [B]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402
capi.USE_TEST_BUILD = True  # the F110QP_* knobs below are read by the test build only


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    N = 40
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = workload.make_grouped_batch(-(-B // 120), N, seed=0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a[:B])).to(dev)  # noqa: E731
    x0, ul, xr = T(g["x0"]), T(g["u_lin"]), T(g["x_ref"])
    u = torch.empty(B, N, 2, device=dev)
    x = torch.empty(B, N + 1, 3, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    rows = {}
    for cap in (0, 1, 2, 3, 4, 5, 6, 7):
        if cap:
            os.environ["F110QP_LANE_PASSCAP"] = str(cap)
        else:
            os.environ.pop("F110QP_LANE_PASSCAP", None)
        s = capi.Solver(capi.default_config(N))
        launch = s.prepare_dev(x0, ul, xr, None, u, x, st, it, stream=stream)
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            launch()
        e1.record(stream)
        torch.cuda.synchronize()
        sn = st.cpu().numpy()
        r = dict(kernel_us=round(e0.elapsed_time(e1) * 1000.0 / 20, 1), solved=float((sn == capi.SOLVED).mean()),
                 segments=s.lane_segments(B))
        if cap == 0:
            r["pass_hist"] = np.bincount(it.cpu().numpy()).tolist()
            itn = it.cpu().numpy().reshape(-1, 64)
            r["wave_max_pass_hist"] = np.bincount(itn.max(1)).tolist()
        rows[f"cap{cap}"] = r
        s.close()
    print(json.dumps(dict(B=B, N=N, rows=rows)))


if __name__ == "__main__":
    main()
