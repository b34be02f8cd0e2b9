"""Per-sweep cycle breakdown of the lane-per-QP kernel from the -DF110QP_STAMPS build.
Run:  F110QP_LIB=f110-mpc_amd/lib_stamps/libf110qp.so python tools/lane_stamps.py [B] [N] [mode] [qpw] [data]
(mode: F110QP_LANE_MODE scratch placement, 0 auto; qpw: F110QP_LANE_QPW QPs per wave, 0 auto;
data: batch (make_batch) or grouped (the C4 candidate sets)). Cycles are per wave (s_memtime)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
if len(sys.argv) > 3:
    os.environ["F110QP_LANE_MODE"] = sys.argv[3]
QPW = int(sys.argv[4]) if len(sys.argv) > 4 else 0
if QPW:
    os.environ["F110QP_LANE_QPW"] = str(QPW)
DATA = sys.argv[5] if len(sys.argv) > 5 else "batch"
from f110qp import capi, workload  # noqa: E402

L = capi.load()
assert hasattr(L, "f110qp_read_lane_stamps"), "not a stamps build"
if DATA == "grouped":
    g = workload.make_grouped_batch(-(-B // 120), N, seed=4000)
    w = {k: np.ascontiguousarray(g[k][:B]) for k in ("x0", "u_lin", "x_ref")}
else:
    w = workload.make_batch(B, N, seed=1)
s = capi.Solver(capi.default_config(N, backend=capi.BACKEND_LANE))
for _ in range(3):
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"])
Lq = QPW
if not Lq:
    Lq = 64
    while Lq > 1 and -(-B // Lq) < 2048:
        Lq //= 2
W = min(4096, -(-B // Lq))
buf = np.zeros((W, 8), np.uint64)
L.f110qp_read_lane_stamps.argtypes = [C.c_void_p, C.c_int]
L.f110qp_read_lane_stamps(C.c_void_p(buf.ctypes.data), W)
b = buf.astype(float)
npass = b[:, 5]
print(f"B={B} N={N} L={Lq} waves={-(-B // Lq)} iters mean {it.mean():.2f} max {it.max()} | passes/wave mean {npass.mean():.2f} max {npass.max():.0f}")
for i, n in enumerate(["setup (stage x_ref, linearize)", "riccati backward", "forward + costate + PDAS", "(unused)", "output"]):
    print(f"{n:32s} mean {b[:, i].mean():9.0f}  max {b[:, i].max():9.0f}  per pass-stage {b[:, i].sum() / max(1, npass.sum()) / N:7.1f}")
print(f"{'total':32s} mean {b[:, 6].mean():9.0f}  max {b[:, 6].max():9.0f}")
