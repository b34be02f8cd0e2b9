"""One rank of the multi-process HIP shard check (tests/test_gpu_shard.py): launched by
torch.distributed.run with the gloo backend; every rank solves its scenario-aligned shard of a
C4-style grouped batch on cuda:0 through the C ABI (f110qp_solve_grouped_dev, the back end given),
the shards are all-gathered over gloo (host tensors), rank 0 writes the global result.
Mode "select" (5th argument): the split is NOT scenario-aligned (scenarios straddle the ranks);
every rank solves its shard with the cost output, runs f110qp_select_dev over the global
scenario ids, and the per-rank winners meet in the min-loc all-reduce (shard.select_sharded)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402
from f110qp.shard import select_sharded, shard_range, solve_sharded  # noqa: E402


def main():
    out_path, N, scen, be = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    mode = sys.argv[5] if len(sys.argv) > 5 else "gather"
    # 6th argument: the process-group backend (gloo: host tensors, ranks may share GPU 0; nccl = RCCL,
    # one GPU per rank: the min-loc all-reduces run on device tensors)
    pgb = sys.argv[6] if len(sys.argv) > 6 else "gloo"
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    dist.init_process_group(pgb, **({"device_id": dev} if pgb == "nccl" else {}))
    g = workload.make_grouped_batch(scen, N, seed=4242)
    G = g["group_size"]
    inputs = {k: torch.from_numpy(np.ascontiguousarray(g[k])) for k in ("x0", "u_lin", "x_ref")}
    solver = capi.Solver(capi.default_config(N, device=0, backend=be))

    def solve_fn(sh):
        B = sh["x0"].shape[0]
        x0, ul, xr = (sh[k].to(dev) for k in ("x0", "u_lin", "x_ref"))
        gid = (torch.arange(B, dtype=torch.int32) // G).to(dev)
        uo = torch.empty((B, N, 2), dtype=torch.float32, device=dev)
        xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        solver.solve_grouped_dev(x0, ul, xr, None, gid, max(1, -(-B // G)), uo, xo, st, None)
        torch.cuda.synchronize(dev)
        return {"u": uo.cpu(), "x": xo.cpu(), "status": st.cpu()}

    if mode == "select":
        world, rank = dist.get_world_size(), dist.get_rank()
        total = inputs["x0"].shape[0]
        lo, hi = shard_range(total, world, rank, 1)
        B = hi - lo
        x0, ul, xr = (inputs[k][lo:hi].to(dev) for k in ("x0", "u_lin", "x_ref"))
        gid = (torch.arange(lo, hi, dtype=torch.int32) // G).to(dev)  # global scenario ids
        uo = torch.empty((B, N, 2), dtype=torch.float32, device=dev)
        xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        co = torch.empty(B, dtype=torch.float64, device=dev)
        solver.solve_dev(x0, ul, xr, None, uo, xo, st, None, cost=co)
        win = torch.empty(scen, dtype=torch.int32, device=dev)
        best = torch.empty(scen, dtype=torch.float64, device=dev)
        capi.select_dev(gid, scen, co, st, win, best)
        torch.cuda.synchronize(dev)
        win = win.cpu().to(torch.int64)
        win = torch.where(win >= 0, win + lo, win)
        if pgb == "nccl":  # device tensors through RCCL
            b, w = select_sharded(best, win.to(dev))
            b, w = b.cpu(), w.cpu()
        else:
            b, w = select_sharded(best.cpu(), win)
        if rank == 0:
            lo1 = shard_range(total, world, 1, 1)[0] if world > 1 else total
            np.savez(out_path, best=b.numpy(), winner=w.numpy(), world=world, lo1=lo1)
        solver.close()
        dist.destroy_process_group()
        return
    out = solve_sharded(solve_fn, inputs, group_align=G)
    if dist.get_rank() == 0:
        np.savez(out_path, u=out["u"].numpy(), x=out["x"].numpy(), status=out["status"].numpy(),
                 world=dist.get_world_size())
    solver.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
