"""Multi-process HIP evidence for the C4 split: two ranks (torch.distributed,
gloo, both on GPU 0 of the box) each solve their scenario-aligned shard of a grouped C4-style
batch through the C ABI; the all-gathered result is bit-identical to one process solving the
whole batch (the QPs are independent: no data-path collective, the split changes nothing)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("N,scen,be", [(40, 9, "lane"), (20, 5, "wave")])
def test_two_rank_hip_shards_bit_equal(capi, cuda, tmp_path, N, scen, be):
    import torch

    from f110qp import workload

    backend = {"lane": capi.BACKEND_LANE, "wave": capi.BACKEND_WAVE}[be]
    out = tmp_path / "sharded.npz"
    env = {**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                    "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                    os.path.join(ROOT, "tests", "shard_gpu_worker.py"), str(out), str(N), str(scen), str(backend)],
                   check=True, timeout=180, env=env, cwd=ROOT)
    d = np.load(out)
    assert int(d["world"]) == 2
    g = workload.make_grouped_batch(scen, N, seed=4242)
    B = g["x0"].shape[0]
    s = capi.Solver(capi.default_config(N, device=0, backend=backend))
    dev = torch.device("cuda", 0)
    x0, ul, xr = (torch.from_numpy(np.ascontiguousarray(g[k])).to(dev) for k in ("x0", "u_lin", "x_ref"))
    gid = (torch.arange(B, dtype=torch.int32) // g["group_size"]).to(dev)
    uo = torch.empty((B, N, 2), dtype=torch.float32, device=dev)
    xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    s.solve_grouped_dev(x0, ul, xr, None, gid, scen, uo, xo, st, None)
    torch.cuda.synchronize()
    s.close()
    assert (st.cpu().numpy() == capi.SOLVED).all()
    np.testing.assert_array_equal(d["status"], st.cpu().numpy())
    np.testing.assert_array_equal(d["u"], uo.cpu().numpy())
    np.testing.assert_array_equal(d["x"], xo.cpu().numpy())


@pytest.mark.parametrize("N,scen,be", [(40, 5, "lane"), (40, 5, "wave"), (20, 9, "auto")])
def test_two_rank_select_straddling_scenarios(capi, cuda, tmp_path, N, scen, be):
    """The per-scenario selection across ranks when a scenario straddles
    two GPUs: each rank solves its half (split at a non-multiple of 120) with the cost output and
    selects per global scenario id on the device, the min-loc all-reduce combines the ranks. With
    one kernel on both sides (N = 40: the same lane_seg S, or the wave kernel) the result equals
    one process selecting over the whole batch, bit for bit. N = 20 with AUTO: the whole batch
    (1,080 QPs) runs the segmented lane kernel, each rank's 540 the wave kernel, so the costs agree
    to rounding: best costs to 1e-9 relative, winners wherever the scenario's two best candidates
    are further apart than that (shard.select_sharded)."""
    import torch

    from f110qp import workload

    backend = {"lane": capi.BACKEND_LANE, "wave": capi.BACKEND_WAVE, "auto": capi.BACKEND_AUTO}[be]
    out = tmp_path / "select.npz"
    env = {**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                    "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                    os.path.join(ROOT, "tests", "shard_gpu_worker.py"), str(out), str(N), str(scen), str(backend),
                    "select"], check=True, timeout=180, env=env, cwd=ROOT)
    d = np.load(out)
    assert int(d["world"]) == 2 and int(d["lo1"]) % 120 != 0  # scenario 2 straddles the ranks
    g = workload.make_grouped_batch(scen, N, seed=4242)
    B = g["x0"].shape[0]
    dev = torch.device("cuda", 0)
    x0, ul, xr = (torch.from_numpy(np.ascontiguousarray(g[k])).to(dev) for k in ("x0", "u_lin", "x_ref"))
    gid = (torch.arange(B, dtype=torch.int32) // g["group_size"]).to(dev)
    uo = torch.empty((B, N, 2), dtype=torch.float32, device=dev)
    xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    co = torch.empty(B, dtype=torch.float64, device=dev)
    s = capi.Solver(capi.default_config(N, device=0, backend=backend))
    s.solve_dev(x0, ul, xr, None, uo, xo, st, None, cost=co)
    win = torch.empty(scen, dtype=torch.int32, device=dev)
    best = torch.empty(scen, dtype=torch.float64, device=dev)
    capi.select_dev(gid, scen, co, st, win, best)
    torch.cuda.synchronize()
    s.close()
    if be != "auto":
        np.testing.assert_array_equal(d["winner"], win.cpu().numpy().astype(np.int64))
        np.testing.assert_array_equal(d["best"], best.cpu().numpy())
        return
    s_ = capi.Solver(capi.default_config(N, device=0, backend=backend))
    assert s_.backend_info(B)[0] != s_.backend_info(B // 2)[0]  # different kernels per rank and whole
    s_.close()
    np.testing.assert_allclose(d["best"], best.cpu().numpy(), rtol=1e-9)
    cn, sn, gn = co.cpu().numpy(), st.cpu().numpy(), gid.cpu().numpy()
    for k in range(scen):
        c = np.sort(cn[(gn == k) & (sn == capi.SOLVED)])
        if len(c) > 1 and c[1] - c[0] > 1e-9 * max(1.0, c[0]):
            assert d["winner"][k] == int(win[k])


def test_rccl_min_loc_select_one_rank(capi, cuda, tmp_path):
    """The nccl (= RCCL) process-group path of the selection on the box's one GPU: a world of one
    under torch.distributed.run runs shard.select_sharded's two all_reduce(MIN) on device tensors
    through RCCL (an identity at world size 1), and the result equals the single-process selection.
    The multi-GPU runs of bench.py use the same backend (--dist-backend nccl, the default)."""
    import torch

    from f110qp import workload

    N, scen = 40, 5
    out = tmp_path / "select_rccl.npz"
    env = {**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                    "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                    os.path.join(ROOT, "tests", "shard_gpu_worker.py"), str(out), str(N), str(scen),
                    str(capi.BACKEND_LANE), "select", "nccl"], check=True, timeout=180, env=env, cwd=ROOT)
    d = np.load(out)
    assert int(d["world"]) == 1
    g = workload.make_grouped_batch(scen, N, seed=4242)
    B = g["x0"].shape[0]
    dev = torch.device("cuda", 0)
    x0, ul, xr = (torch.from_numpy(np.ascontiguousarray(g[k])).to(dev) for k in ("x0", "u_lin", "x_ref"))
    gid = (torch.arange(B, dtype=torch.int32) // g["group_size"]).to(dev)
    uo = torch.empty((B, N, 2), dtype=torch.float32, device=dev)
    xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    co = torch.empty(B, dtype=torch.float64, device=dev)
    s = capi.Solver(capi.default_config(N, device=0, backend=capi.BACKEND_LANE))
    s.solve_dev(x0, ul, xr, None, uo, xo, st, None, cost=co)
    win = torch.empty(scen, dtype=torch.int32, device=dev)
    best = torch.empty(scen, dtype=torch.float64, device=dev)
    capi.select_dev(gid, scen, co, st, win, best)
    torch.cuda.synchronize()
    s.close()
    np.testing.assert_array_equal(d["winner"], win.cpu().numpy().astype(np.int64))
    np.testing.assert_array_equal(d["best"], best.cpu().numpy())
