"""Why does one wave of the partitioned-horizon lane kernel take longer with more QPs in it
(round-5 verdict: N = 20, S = 4, B = 1 10.6 us, B = 4 20.7 us, one wave either way)? Kernel time
(HIP events over back-to-back launches) against the QPs' PDAS pass counts, on the C2 bench batch
(bench.py seeds): (a) single QPs of known pass count, (b) one QP copied 16 times (a full wave of
identical QPs), (c) 16 distinct QPs, (d) prefixes of the batch. If the time depends only on the
wave's maximum pass count, the growth is pass-count divergence, not the number of QPs per wave.

usage: python tools/c2_growth_probe.py   (one JSON line per case, then a fit)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402


def kernel_us(s, w, dev, reps=100):
    B = w["x0"].shape[0]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    x0, ul, xr = T(w["x0"]), T(w["u_lin"]), T(w["x_ref"])
    N = s.horizon
    u = torch.empty(B, N, 2, device=dev)
    x = torch.empty(B, N + 1, 3, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    launch = s.prepare_dev(x0, ul, xr, None, u, x, st, it, stream=stream)
    for _ in range(10):
        launch()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == capi.SOLVED).all()
    return e0.elapsed_time(e1) * 1000.0 / reps, it.cpu().numpy()


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N = 20
    full = workload.make_batch(1024, N, seed=1000)  # the C2 bench batch
    s = capi.Solver(capi.default_config(N, backend=capi.BACKEND_LANE))
    _, its = kernel_us(s, full, dev, reps=5)
    pick = lambda idx: {k: np.ascontiguousarray(full[k][idx]) for k in ("x0", "u_lin", "x_ref")}  # noqa: E731
    rows = []

    def case(name, idx):
        w = pick(np.asarray(idx))
        B = w["x0"].shape[0]
        k, it = kernel_us(s, w, dev)
        r = dict(case=name, B=B, S=s.lane_segments(B), waves=-(-B * s.lane_segments(B) // 64),
                 max_passes=int(it.max()), mean_passes=round(float(it.mean()), 2), kernel_us=round(k, 2))
        rows.append(r)
        print(json.dumps(r), flush=True)

    for p in sorted(set(its.tolist())):
        q = int(np.where(its == p)[0][0])
        case(f"single QP {q} ({p} passes)", [q])
        case(f"QP {q} x16 (one wave of copies)", [q] * 16)
        case(f"QP {q} x4", [q] * 4)
    case("first 4 QPs", range(4))
    case("first 16 QPs", range(16))
    lo = np.where(its == its.min())[0][:16]
    case("16 QPs of the fewest passes", lo)
    hi = np.where(its == its.max())[0][:16]
    case("16 QPs of the most passes", hi)
    for B in (64, 256, 1024):
        case(f"first {B} QPs", range(B))
    s.close()
    X = np.array([[1.0, r["max_passes"]] for r in rows])
    y = np.array([r["kernel_us"] for r in rows])
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    resid = y - X @ coef
    print(json.dumps({"fit": "kernel_us = a + b * max_passes", "a": round(coef[0], 2), "b": round(coef[1], 2),
                      "max_abs_resid_us": round(float(np.abs(resid).max()), 2), "rows": rows}))


if __name__ == "__main__":
    main()
