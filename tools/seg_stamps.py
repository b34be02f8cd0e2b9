"""Per-phase cycles of the partitioned-horizon lane kernel (lane_seg_kernel.h) from the stamps build.
Run:  F110QP_LIB=f110-mpc_amd/lib_stamps/libf110qp.so python tools/seg_stamps.py [B] [N]
Per wave (lane 0): setup (staging, linearisation, references, warm start), then summed over the
passes: backward sweep, segment-end recursion, refresh, forward sweep; output sweep; total."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.cuda.is_available()
L = capi.load()
assert hasattr(L, "f110qp_read_seg_stamps"), "not a stamps build"
w = workload.make_batch(B, N, seed=5, heading="true", lateral=0.6, steer_range=0.4)
s = capi.Solver(capi.default_config(N, backend=capi.BACKEND_LANE))
S = s.lane_segments(B)
for _ in range(3):
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"])
W = min(4096, (B * S + 63) // 64)
buf = np.zeros((W, 16), np.uint64)
L.f110qp_read_seg_stamps.argtypes = [C.c_void_p, C.c_int]
L.f110qp_read_seg_stamps(C.c_void_p(buf.ctypes.data), W)
b = buf.astype(float)
tot = b[:, 7]
print(f"B={B} N={N} S={S} waves={W} passes per wave mean {b[:, 6].mean():.2f} max {b[:, 6].max():.0f}")
for i, n in enumerate(["setup", "backward", "segment ends", "refresh", "forward", "output"]):
    print(f"{n:14s} mean {b[:, i].mean():8.0f}  max {b[:, i].max():8.0f}  share {b[:, i].mean() / tot.mean() * 100:5.1f}%")
for i, n in zip(range(8, 16), ["  staging", "  linearize", "  refs to fp64", "  warm + rest", "    rN shfl",
                                "    mask init", "    rest", "  out loop"]):
    print(f"{n:14s} mean {b[:, i].mean():8.0f}  max {b[:, i].max():8.0f}")
np_ = np.maximum(b[:, 6], 1)
print(f"per pass: backward {np.mean(b[:, 1] / np_):.0f}, segment ends {np.mean(b[:, 2] / np_):.0f}, refresh "
      f"{np.mean(b[:, 3] / np_):.0f}, forward {np.mean(b[:, 4] / np_):.0f} cycles; total p50 {np.median(tot):.0f} "
      f"max {tot.max():.0f}")
