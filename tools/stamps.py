"""Per-phase cycle breakdown of the solve kernel from the -DF110QP_STAMPS diagnostic build.
Run:  F110QP_LIB=f110-mpc_amd/lib_stamps/libf110qp.so python tools/stamps.py [B] [N] [gap]
Shares are meaningful, absolute time is not (the stamps forbid some overlap)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
gap = len(sys.argv) > 3 and sys.argv[3] == "gap"
L = capi.load()
assert hasattr(L, "f110qp_read_stamps"), "not a stamps build"
w = workload.make_batch(B, N, seed=1)
hs = None
if gap:
    ranges, amin, ainc, amax = workload.make_scans(B, seed=1)
    hs = np.stack([np.stack(capi.find_half_spaces(w["x0"][b].astype(float), ranges[b], amin, ainc, amax)) for b in range(B)]).astype(np.float32)
s = capi.Solver(capi.default_config(N, gap_mode=1 if gap else 0))
for _ in range(3):
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
buf = np.zeros((B, 16), np.uint64)
L.f110qp_read_stamps.argtypes = [C.c_void_p, C.c_int]
L.f110qp_read_stamps(C.c_void_p(buf.ctypes.data), B)
names = ["inputs+linearize", "gradient g (fp64 scans)", "hessian (closed form)", "sweep inverse", "active set (fp32)",
         "refinement+fp64 check", "outputs", "total", " gi: step1 search", " pdas (box) | gi: W n_p", " gi: v_j gather",
         " gi: tri solves", " gi: z update", " gi: step lengths", " gi: append slot"]
tot = buf[:, 7].astype(float)
print(f"B={B} N={N} gap={gap} iters mean {it.mean():.2f} max {it.max()}")
for i, n in enumerate(names):
    if i >= 8 and buf[:, 15].sum() == 0:
        break
    v = buf[:, i].astype(float)
    print(f"{n:28s} mean {v.mean():9.0f}  max {v.max():9.0f}  share {v.mean() / tot.mean() * 100:5.1f}%")
it_ = buf[:, 15].astype(float)
print(f"per-iteration: gi cycles/iter {(buf[:, 4].astype(float).sum() / max(1, it_.sum())):.0f}")
q = np.percentile(tot, [50, 90, 99, 100])
imax = int(np.argmax(tot))
print(f"total cycles p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} max {q[3]:.0f} (slowest QP: {int(it_[imax])} iterations, "
      f"gi {buf[imax, 4]:.0f}, refine {buf[imax, 5]:.0f}); iteration histogram {np.bincount(it_.astype(int), minlength=8)[:64].tolist()}")
print("slowest QP by phase:", {n.strip(): int(buf[imax, i]) for i, n in enumerate(names)})
