"""FindHalfSpaces kernel time vs beams per scan and scans per launch (HIP events, 50 launches)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402

dev = torch.device("cuda", 0)
for B, nr in ((4096, 1080), (4096, 512), (4096, 128), (4096, 64), (1024, 1080), (16384, 1080), (65536, 1080)):
    r, amin, ainc, amax = workload.make_scans(B, seed=1, beams=nr)
    rd = torch.from_numpy(r).to(dev)
    x0 = torch.zeros((B, 3), dtype=torch.float32, device=dev)
    hs = torch.empty((B, 2, 3), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(5):
        capi.find_half_spaces_dev(x0, rd, amin, ainc, amax, hs, stream=s)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(50):
        capi.find_half_spaces_dev(x0, rd, amin, ainc, amax, hs, stream=s)
    b.record(s)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 50 * 1e3
    gbs = B * (nr * 4 + 44) / (us * 1e-6) / 1e9
    print(f"B {B:6d} beams {nr:5d}: {us:7.2f} us  {gbs:7.1f} GB/s")
