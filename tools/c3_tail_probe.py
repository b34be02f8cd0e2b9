"""C3 tail probe: is the gap kernel's time its slowest QP's chain? Solves the bench's C3 batch on
the wave back end, takes the QPs with the most GI iterations, and times (HIP events) the wave
kernel on each alone (B = 1), on the 64 heaviest together, and on the whole batch.

usage: python tools/c3_tail_probe.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402


def timed(s, dev, x0, ul, xr, hs, reps=20):
    B = x0.shape[0]
    N = s.horizon
    u = torch.empty(B, N, 2, device=dev)
    x = torch.empty(B, N + 1, 3, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    launch = s.prepare_dev(x0, ul, xr, hs, u, x, st, stream=stream)
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, N = 4096, 20  # the bench's C3 inputs (bench.py: make_batch seed 1000, make_scans seed 2000)
    w = workload.make_batch(B, N, seed=1000)
    ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
    hs_d = torch.empty((B, 2, 3), dtype=torch.float32, device=dev)
    capi.find_half_spaces_dev(torch.from_numpy(w["x0"]).to(dev), torch.from_numpy(ranges).to(dev), amin, ainc,
                              amax, hs_d, stream=torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    hs = hs_d.cpu().numpy()
    s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_WAVE))
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    order = np.argsort(-it, kind="stable")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    rows = {"iters_top": it[order[:16]].tolist(), "iters_hist": np.bincount(it).tolist()}
    rows["full_us"] = timed(s, dev, T(w["x0"]), T(w["u_lin"]), T(w["x_ref"]), T(hs))
    for k in (64, 256, 1024):
        idx = order[:k]
        rows[f"top{k}_us"] = timed(s, dev, T(w["x0"][idx]), T(w["u_lin"][idx]), T(w["x_ref"][idx]), T(hs[idx]))
    rows["single_us"] = []
    for b in order[:6]:
        idx = np.array([b])
        rows["single_us"].append((int(b), int(it[b]), round(timed(s, dev, T(w["x0"][idx]), T(w["u_lin"][idx]),
                                                                   T(w["x_ref"][idx]), T(hs[idx])), 1)))
    s.close()
    # the box screen (f110qp_kernels.hip gap_screen_kernel) replayed on the host from the lane
    # back end's box-only outputs: how many QPs go on to GI
    sb = capi.Solver(capi.default_config(N, backend=capi.BACKEND_LANE))
    ub, xb, stb, itb = sb.solve(w["x0"], w["u_lin"], w["x_ref"])
    sb.close()
    h = hs.astype(np.float64)
    a, bb, c = h[:, :, 0][:, :, None], h[:, :, 1][:, :, None], h[:, :, 2][:, :, None]
    X, Y = xb[:, None, 1:, 0].astype(np.float64), xb[:, None, 1:, 1].astype(np.float64)
    ax, by = a * X, bb * Y
    ok_rows = ax + by + c >= 1e-6 * (1 + np.abs(ax) + np.abs(by) + np.abs(c))
    st0 = (h[:, :, 0] * w["x0"][:, None, 0] + h[:, :, 1] * w["x0"][:, None, 1] >= -h[:, :, 2] - 1e-9).all(1)
    keep = ok_rows.all((1, 2)) & st0 & (stb == capi.SOLVED)
    rows["screen_pass"] = int(keep.sum())
    rows["screen_pass_row_only"] = int(ok_rows.all((1, 2)).sum())
    rows["screen_pass_st0"] = int(st0.sum())
    rows["gi_iters_of_passed_mean"] = float(it[keep].mean()) if keep.any() else None
    rows["gi_iters_of_rest_mean"] = float(it[~keep].mean())
    sa = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE))
    rows["auto_screen"] = sa.gap_screen(B)
    rows["auto_us"] = timed(sa, dev, T(w["x0"]), T(w["u_lin"]), T(w["x_ref"]), T(hs))
    ua, xa, sta, ita = sa.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    sa.close()
    rows["auto_vs_wave_status_equal"] = bool((sta == st).all())
    rows["auto_vs_wave_max_du"] = float(np.abs(ua - u).max())
    rest = ~keep
    rows["rest_us"] = timed(capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_WAVE)),
                            dev, T(w["x0"][rest]), T(w["u_lin"][rest]), T(w["x_ref"][rest]), T(hs[rest]))
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
