"""Sharding of a global batch over ranks, exercised with world_size 2 over
gloo on the CPU: the gathered sharded result must be bit-identical to the one-process result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from f110qp.shard import shard_range


@pytest.mark.parametrize("total,world,align", [(65536, 8, 120), (1000, 3, 1), (7, 4, 1), (0, 2, 1), (240, 2, 120),
                                               (65536, 1, 120), (121, 2, 120)])
def test_shard_range_partitions(total, world, align):
    owned = []
    prev_hi = 0
    for r in range(world):
        lo, hi = shard_range(total, world, r, align)
        assert lo == prev_hi and lo <= hi
        if hi < total:
            assert hi % align == 0
        owned.append(hi - lo)
        prev_hi = hi
    assert prev_hi == total and sum(owned) == total
    # balanced to within one group
    assert max(owned) - min(owned) <= 2 * align  # one group plus the partial tail group


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "f110-mpc_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist

    import oracle
    from f110qp import workload
    from f110qp.shard import solve_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N = 20
    w = workload.make_grouped_batch(3, N, seed=5, lanes=(0.0, 0.25), steers=5)  # 3 scenarios x 10
    inputs = {k: torch.from_numpy(w[k]) for k in ("x0", "u_lin", "x_ref")}

    def solve_fn(sh):
        if sh["x0"].shape[0] == 0:
            return {"u": torch.zeros((0, N, 2), dtype=torch.float64), "status": torch.zeros(0, dtype=torch.int32)}
        u, x, st = oracle.solve_batch(oracle.params(N), sh["x0"].numpy(), sh["u_lin"].numpy(), sh["x_ref"].numpy())
        return {"u": torch.from_numpy(u), "status": torch.from_numpy(st)}

    out = solve_sharded(solve_fn, inputs, group_align=w["group_size"])
    q.put((rank, out["u"].numpy(), out["status"].numpy()))
    dist.destroy_process_group()


def test_sharded_equals_single_process_gloo():
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle
    from f110qp import workload

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    N = 20
    w = workload.make_grouped_batch(3, N, seed=5, lanes=(0.0, 0.25), steers=5)
    u, x, st = oracle.solve_batch(oracle.params(N), w["x0"], w["u_lin"], w["x_ref"])
    for rank, ug, sg in res:
        np.testing.assert_array_equal(ug, u)
        np.testing.assert_array_equal(sg, st)


def _select_worker(rank, world, port, q):
    """One rank: exact costs of its (unaligned) shard by the CPU oracle, the local per-scenario
    argmin over GLOBAL scenario ids, then the min-loc all-reduce of f110qp.shard.select_sharded."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "f110-mpc_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist

    import oracle
    from f110qp.shard import select_sharded, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N, w, gid, G = _select_batch()
    lo, hi = shard_range(len(gid), world, rank, 1)  # align 1: scenarios straddle the ranks
    prm = oracle.params(N)
    u, x, st = oracle.solve_batch(prm, w["x0"][lo:hi], w["u_lin"][lo:hi], w["x_ref"][lo:hi])
    cost = oracle.tracking_cost(prm, u, x, w["x_ref"][lo:hi])
    win, best = oracle.select(gid[lo:hi], G, cost, st)
    win = np.where(win >= 0, win + lo, -1)
    b, wi = select_sharded(torch.from_numpy(best), torch.from_numpy(win))
    q.put((rank, lo, hi, b.numpy(), wi.numpy()))
    dist.destroy_process_group()


def _select_batch():
    """5 scenarios x 10 candidates; scenario 3 holds two identical candidates (indices 34 and 35,
    a tie the smaller index must win)."""
    from f110qp import workload

    N = 20
    w = workload.make_grouped_batch(5, N, seed=77, lanes=(0.0, 0.25), steers=5)
    for k in ("x0", "u_lin", "x_ref"):
        w[k][35] = w[k][34]
    gid = np.repeat(np.arange(5), 10)
    return N, w, gid, 5


@pytest.mark.parametrize("world", [2, 3])
def test_select_sharded_minloc_gloo(world):
    """Per-scenario selection across ranks whose shards split scenarios (align 1): the min-loc
    all-reduce returns exactly the single-process argmin (cost and global index, ties to the
    smaller index), on every rank."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle

    N, w, gid, G = _select_batch()
    # the split really straddles: some scenario has candidates on two ranks
    bounds = [shard_range(len(gid), world, r, 1) for r in range(world)]
    assert any(lo % 10 != 0 for lo, _ in bounds[1:])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_select_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    prm = oracle.params(N)
    u, x, st = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"])
    cost = oracle.tracking_cost(prm, u, x, w["x_ref"])
    win, best = oracle.select(gid, G, cost, st)
    assert win[3] != 35  # the tie went to index 34 (or a better candidate)
    for rank, lo, hi, b, wi in res:
        np.testing.assert_array_equal(wi, win)
        np.testing.assert_array_equal(b, best)
