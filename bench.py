#!/usr/bin/env python3
"""bench.py — QP solves/s of the f110qp HIP path (BASELINE.json metric) on 1..8 MI355X.

A "step" is one f110qp_solve_batch_dev launch over one batch of synthetic ticks already
resident in HBM (linearise + condense + exact QP solve + (u*, x*) write-back for every QP).
Default workload: BASELINE.json configs[1] = 1,024 independent horizon-20 QPs, box input
constraints. One process per GPU (torch.distributed, RCCL backend); each rank solves its own
batch (weak scaling, no data-path collective: the QPs are independent); the timed region is
bracketed by barrier + synchronize and the max over ranks is reported.

Extra JSON fields: "roofline" (dominant kernel = the solve kernel: algorithmic bytes and
flops per launch / its average duration from HIP events on the launch stream) and
"cpu_baseline" (the CPU oracle timed on a bounded sample on the host cores; rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))

CONFIGS = {
    # name: (batch per GPU, horizon, gap rows active, warm-started stream, description)
    "c2": (1024, 20, False, False, "configs[1]: batch=1024 QPs, horizon=20, box constraints only"),
    "c3": (4096, 20, True, False, "configs[2]: batch=4096 QPs, horizon=20, + half-space gap constraints "
                                  "(FindHalfSpaces of one 1,080-beam scan per QP inside every step)"),
    "c5": (4096, 20, False, True, "configs[4]: batch=4096 QPs, horizon=20, warm-started closed receding-horizon "
                                   "loop (x0 <- simulate_dynamics(x0, u*_0), u_lin = (4.5, steer of u*_1), "
                                   "mini path re-planned every 5 ticks; previous tick's active set seeds the solve)"),
    "c5_cold": (4096, 20, False, False, "configs[4] closed-loop stream solved cold (no warm start), for comparison"),
    "c5_straight": (4096, 20, False, True, "best case, not configs[4]: warm stream whose x0 slides along a fixed "
                                           "heading with fixed u_lin and x_ref (every linearisation key repeats)"),
    "c2_big": (65536, 20, False, False, "throughput: batch=65536 QPs, horizon=20, box constraints"),
    # global batch, sharded over the ranks (strong scaling): 546 scenarios x 120 candidates + 16
    "c4": (65536, 40, False, False, "configs[3]: batch=65536 QPs, horizon=40, 6-lane x 20 mini-trajectory "
                                    "candidate sets (grouped), sharded over the GPUs"),
}
STRONG = {"c4"}
# the whole control tick on the device: planning stage (occupancy grid, collision check of the 31
# candidates, lookahead waypoint, selection; project.cpp:73-152) then the QP of every scenario
CONFIGS["tick"] = (1024, 20, False, False, "control tick x1024 scenarios: device planning stage (1080-beam "
                   "scan -> 100x100 occupancy grid -> 31 candidates -> lookahead waypoint -> x_ref) + QP, N=20")
GROUP = 120  # candidates per scenario in c4 (6 lane offsets x 20 steer values)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 vector (= FP32 MFMA) peak
FP64_PEAK_TFLOPS = 78.6     # MI355X spec FP64 vector; tools/microbench/latency.hip measures the
                            # matching issue rate (one wave64 fp64 FMA per 4 cycles per SIMD)
# fp64 flops per stage and PDAS pass of the sequential Riccati algorithm (lane_kernel.h, ISA count,
# DESIGN.md 4): the algorithmic work of a pass, whatever kernel runs it. fp64_compute is priced on it.
LANE_FLOPS_PER_STAGE = 290
# lane_seg_kernel (partitioned horizon) executes more per stage and pass: the backward stage with the
# segment's closed-loop map (160 fp64 instructions), the feed-forward refresh (16) and the forward
# (35), ~2.5 flops per instruction, plus the S - 1 segment steps (~200 fp64 each) spread per stage.
# That parallel-in-time redundancy is reported as "segmentation_overhead", never counted as work.
SEG_FLOPS_PER_STAGE = 530


def seg_flops_per_stage(S: int, N: int) -> float:
    """fp64 flops the segmented kernel executes per stage and pass (redundancy included)."""
    return SEG_FLOPS_PER_STAGE + 500.0 * (S - 1) / N * S


def bytes_per_qp(N: int, gap: bool, warm: bool = False, backend: str = "wave") -> int:
    """ABI bytes moved per QP: x0, u_lin, x_ref (+ halfspace) in; u*, x*, status, iters out.
    Warm start adds the active masks (read + write; 2 x 64-bit words per 64 variables and side)
    and, for the wave back end, the slot key and one read of the cached W = H^-1 (2N x 2N fp32)
    on a key hit. Scratch traffic of the lane back end is not algorithmic (see "traffic")."""
    inp = 4 * (3 + 2 + 3 * N + (6 if gap else 0))
    out = 4 * (2 * N + 3 * (N + 1) + 1 + 1)
    rows = (2 * N + 63) // 64
    extra = 0
    if warm:
        extra = 2 * 2 * 8 * rows + ((16 + 4 * (2 * N) ** 2) if backend == "wave" else 0)
    return inp + out + extra


def flops_per_qp(N: int, passes: float, pivots: float, gap: bool = False) -> float:
    """Algorithmic flops of the wave kernel (DESIGN.md "Roofline"), n = 2N: closed-form Hessian
    25 n^2, symmetric sweep inverse 2 n^3; box rows: per PDAS pass one product with the swept
    matrix T (2 n^2), per bound entering or leaving the free set one pivot of T (2 n^2), two fp64
    refinement steps (2 n^2 + ~60 n for the fp64 rollout and costate each). Gap rows (GI): per
    iteration 2 n (W n_p) + 2 q^2 (two triangular solves) + 2 n q (z) with q = pivots."""
    n = 2 * N
    base = 25 * n * n + 2 * n ** 3 + 2 * (2 * n * n + 60 * n)
    if gap:
        q = pivots
        return base + 2 * n * n + passes * (2 * n + 2 * q * q + 2 * n * q)
    return base + passes * 2 * n * n + pivots * 2 * n * n


def load_traffic(config: str, batch: int, horizon: int, backend: str):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary of this config
    (tools/profile_round.sh + tools/summarize_profiles.py), only when it was taken on the same
    (config, batch, horizon, back end); None otherwise."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}_{batch}.json")
    if not os.path.exists(path):
        path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception:
        return None
    key = (d.get("config"), d.get("batch"), d.get("horizon"), d.get("backend"))
    return d.get("hbm_bytes_per_launch") if key == (config, batch, horizon, backend) else None


def cpu_threads_default() -> int:
    """Host threads for the throughput baseline: the CPUs this process may run on, capped by
    OMP_NUM_THREADS when the environment sets it (the GPU box sets it to its per-GPU CPU share;
    nproc there reports the whole machine)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _admm_rate(oracle, prm, st, w, hs, gap, threads, seconds, B):
    n = 0
    t0 = time.perf_counter()
    while True:
        _, stat, its = oracle.admm_solve_batch(prm, st, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=gap,
                                               num_threads=threads)
        n += B
        el = time.perf_counter() - t0
        if el >= seconds:
            return n, el, stat, its


def cpu_baseline(config: str, N: int, gap: bool, seconds: float, threads: int, c1_ticks: int,
                 full_threads: int = 0):
    """Time the reference's algorithm on the host cores: oracle/osqp_admm.c, a restatement of
    OSQP 0.6 with the settings MPC::Update uses (defaults + warm start; mpc.cpp:98-133) on the
    reference's own sparse QP (re-scaled and re-factored per tick, as OSQP must when A changes).
    The independent QPs of a batch start cold. Also reports the exact fp64 oracle's rate, and
    BASELINE configs[0] (C1): single horizon-20 QP ticks on ONE core (MPC::Update solves one QP
    per odometry tick, mpc.cpp:133 / project.cpp:188), p50/p99 over c1_ticks ticks, both solvers."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker only: used here for the cpu_baseline leg, never for the GPU value
    from f110qp import workload

    B = 2048
    w = workload.make_batch(B, N, seed=12345)
    hs = None
    if gap:
        hs = _halfspaces_host(w, B)
    prm = oracle.params(N)
    st = oracle.admm_settings()
    oracle.admm_solve_batch(prm, st, w["x0"][:64], w["u_lin"][:64], w["x_ref"][:64],
                            None if hs is None else hs[:64], gap_active=gap, num_threads=threads)
    n, el, stat, its = _admm_rate(oracle, prm, st, w, hs, gap, threads, seconds, B)
    # the same over every CPU this process may run on (all host cores), when the
    # per-GPU share (OMP_NUM_THREADS on the GPU box) is smaller than that
    full = None
    if full_threads > threads:
        # a bigger batch per call (OpenMP team start-up amortised over more QPs) and a sweep of
        # thread counts up to every CPU of the affinity mask: the box is shared with other GPUs'
        # jobs, so the best count is reported with the whole sweep
        Bf = 16384
        wf = workload.make_batch(Bf, N, seed=12346)
        hsf = _halfspaces_host(wf, Bf) if gap else None
        sweep = {}
        for t in sorted({min(full_threads, k) for k in (64, 128, full_threads)}):
            nf, elf, _, _ = _admm_rate(oracle, prm, st, wf, hsf, gap, t, 2.0, Bf)
            sweep[t] = nf / elf
        tb = max(sweep, key=sweep.get)
        full = {"value": sweep[tb], "unit": "QP solves/s", "cores": tb,
                "threads_sweep": {str(k): v for k, v in sweep.items()}, "affinity_cpus": full_threads,
                "sample": f"batches of {Bf} {config} ticks (horizon {N}), >= 2 s per thread count, same solver, "
                          f"OpenMP; best of the sweep reported (the GPU box's CPUs are shared with other jobs)"}
    # the exact solver (the parity oracle) on the same sample, for reference
    n2 = 0
    t1 = time.perf_counter()
    while True:
        oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], hs, gap_active=gap, num_threads=threads)
        n2 += B
        el2 = time.perf_counter() - t1
        if el2 >= max(2.0, seconds / 5):
            break
    # C1: one core, one QP per tick, horizon 20 (configs[0]), timed per tick inside C
    c1 = {}
    if c1_ticks > 0:
        w1 = workload.make_batch(1024, 20, seed=777)
        prm1 = oracle.params(20)
        for name, exact in (("osqp_admm_restatement", False), ("exact_oracle", True)):
            ns, nsol = oracle.tick_latency(prm1, st, w1["x0"], w1["u_lin"], w1["x_ref"], c1_ticks, exact=exact)
            us = ns / 1e3
            c1[name] = {"p50_us": float(np.percentile(us, 50)), "p99_us": float(np.percentile(us, 99)),
                        "mean_us": float(us.mean()), "ticks": int(c1_ticks), "solved": nsol,
                        "qps_one_core": float(1e6 / us.mean())}
        c1["note"] = ("C1 = BASELINE configs[0]: single horizon-20 QP per tick on one core (calling thread), "
                      "wall time of the whole solve per tick; instances cycle over 1,024 seeded ticks")
    out = dict(value=n / el, unit="QP solves/s", cores=threads, kind="port",
                host={"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
                      "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "cpu_model": cpu_model(),
                      "threads_used": threads},
                c1_single_core=c1,
                sample=f"{n} QPs ({n // B} x {B} {config} ticks, horizon {N}) in {el:.1f} s: oracle/osqp_admm.c "
                       f"(OSQP 0.6 defaults restated: Ruiz scaling, rho=0.1 adaptive, sigma=1e-6, alpha=1.6, "
                       f"eps=1e-3, check every 25, banded LDL' KKT) with OpenMP over QPs; mean ADMM iters "
                       f"{float(np.mean(its)):.1f}, solved {float(np.mean(stat == 1)):.3f}",
                exact_oracle_qps=n2 / el2)
    if full is not None:
        out["full_host"] = full
        out["note"] = (f"value/cores = the per-GPU CPU share ({threads} threads = OMP_NUM_THREADS on the GPU box); "
                       f"full_host = the best of a thread sweep up to all {full_threads} CPUs of the affinity mask")
    return out


def measure_latency(capi, solver, cfg, w, hs, N, dev, stream, step, reps=300):
    """p50/p99 wall latency (µs) of one QP solve and of one launch of the configured batch."""
    import torch

    def pct(v):
        v = np.sort(np.asarray(v) * 1e6)
        return {"p50_us": float(np.percentile(v, 50)), "p99_us": float(np.percentile(v, 99)),
                "min_us": float(v[0])}

    one = {k: torch.from_numpy(np.ascontiguousarray(w[k][:1])).to(dev) for k in ("x0", "u_lin", "x_ref")}
    h1 = None if hs is None else hs[:1].contiguous()
    uo = torch.empty((1, N, 2), dtype=torch.float32, device=dev)
    xo = torch.empty((1, N + 1, 3), dtype=torch.float32, device=dev)
    st = torch.empty((1,), dtype=torch.int32, device=dev)
    c1 = type(cfg).from_buffer_copy(cfg)
    c1.warm_start = 0  # a cold solve per call: the latency of one control tick
    c1.x_ref_points = 0
    s1 = capi.Solver(c1)
    dev_t, prep_t, prep_async_t, host_t, batch_t = [], [], [], [], []
    for i in range(reps + 20):
        t0 = time.perf_counter()
        s1.solve_dev(one["x0"], one["u_lin"], one["x_ref"], h1, uo, xo, st, stream=stream)
        stream.synchronize()
        if i >= 20:
            dev_t.append(time.perf_counter() - t0)
    # the same through the prepared launcher: one C call per tick that returns with the answer
    # (f110qp_solve_batch_dev_sync: launch, then wait on the kernel's completion word, or the
    # stream where the call is several kernels; what a C++ caller of the ABI pays), no ctypes
    # argument conversion
    launch1s = s1.prepare_dev(one["x0"], one["u_lin"], one["x_ref"], h1, uo, xo, st, stream=stream, sync=True)
    for i in range(reps + 20):
        t0 = time.perf_counter()
        launch1s()
        if i >= 20:
            prep_t.append(time.perf_counter() - t0)
    # the asynchronous launcher followed by torch's stream synchronize (round-4 measurement)
    launch1 = s1.prepare_dev(one["x0"], one["u_lin"], one["x_ref"], h1, uo, xo, st, stream=stream)
    for i in range(reps + 20):
        t0 = time.perf_counter()
        launch1()
        stream.synchronize()
        if i >= 20:
            prep_async_t.append(time.perf_counter() - t0)
    # the same one-QP call over 64 distinct QPs of the batch (each its own tick, 5 calls each): the
    # latency depends on the QP's PDAS pass count (DESIGN.md 2b'), QP 0 above is one sample of it
    nmix = min(64, int(w["x0"].shape[0]))
    mix = {k: torch.from_numpy(np.ascontiguousarray(w[k][:nmix])).to(dev) for k in ("x0", "u_lin", "x_ref")}
    hmix = None if hs is None else hs[:nmix].contiguous()
    mix_l = [s1.prepare_dev(mix["x0"][i:i + 1], mix["u_lin"][i:i + 1], mix["x_ref"][i:i + 1],
                            None if hmix is None else hmix[i:i + 1], uo, xo, st, stream=stream, sync=True)
             for i in range(nmix)]
    for f in mix_l:
        f()
    mix_t = []
    for rep_ in range(5):
        for f in mix_l:
            t0 = time.perf_counter()
            f()
            mix_t.append(time.perf_counter() - t0)
    # the B = 1 kernel alone (HIP events over back-to-back launches)
    ea = torch.cuda.Event(enable_timing=True)
    eb = torch.cuda.Event(enable_timing=True)
    ea.record(stream)
    for _ in range(50):
        launch1()
    eb.record(stream)
    torch.cuda.synchronize(dev)
    k1_us = ea.elapsed_time(eb) * 1000.0 / 50
    be1, _, _ = s1.backend_info(1)
    seg1 = s1.lane_segments(1) if be1 == capi.BACKEND_LANE else 1
    hx = {k: np.ascontiguousarray(w[k][:1]) for k in ("x0", "u_lin", "x_ref")}
    hh = None if hs is None else hs[:1].cpu().numpy()
    for i in range(reps + 20):
        t0 = time.perf_counter()
        s1.solve(hx["x0"], hx["u_lin"], hx["x_ref"], hh)
        if i >= 20:
            host_t.append(time.perf_counter() - t0)
    polled = s1.sync_signals()
    s1.close()
    for i in range(min(reps, 100) + 5):
        t0 = time.perf_counter()
        step()
        stream.synchronize()
        if i >= 5:
            batch_t.append(time.perf_counter() - t0)
    return {"single_qp_device": pct(prep_t), f"single_qp_device_{nmix}_qps": pct(mix_t),
            "single_qp_device_async_then_sync": pct(prep_async_t),
            "single_qp_device_ctypes": pct(dev_t),
            "single_qp_host_pointers": pct(host_t), "batch_launch": pct(batch_t),
            "single_qp_kernel_us": k1_us,
            "single_qp_polled_calls": polled,
            "single_qp_backend": ("lane" + (f" (S = {seg1})" if seg1 > 1 else "")) if be1 == capi.BACKEND_LANE else "wave",
            "note": "wall clock per call incl. launch + wait for the results: single_qp_device is one C call "
                    "(f110qp_solve_batch_dev_sync: launch + poll of the kernel's completion word in pinned host "
                    "memory, hipStreamSynchronize for multi-kernel gap-row calls) on QP 0 of the batch, "
                    f"_{nmix}_qps the same call over {nmix} distinct QPs of the batch, _async_then_sync the "
                    "asynchronous launcher then torch's stream synchronize, _ctypes with the per-call argument "
                    "conversion; host-pointer path: the kernel reads and writes pinned host memory (zero-copy) and "
                    "the call polls the same completion word"}


def _halfspaces_host(w, B):
    from f110qp import capi, workload

    ranges, amin, ainc, amax = workload.make_scans(B, seed=99)
    hs = np.zeros((B, 2, 3), np.float32)
    for b in range(B):
        l1, l2 = capi.find_half_spaces(w["x0"][b].astype(np.float64), ranges[b], amin, ainc, amax)
        hs[b, 0] = l1
        hs[b, 1] = l2
    return hs


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, argv: list, print_only: bool = False) -> int:
    """`bench.py --gpus N` without a launcher: start N child processes of this script, one per GPU
    (RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1), before this process touches
    the GPU; the children's output passes through (rank 0 prints the JSON line). Returns the exit
    code: 0 only if every rank exited 0."""
    import subprocess

    port = _free_port()
    envs = []
    for i in range(n):
        e = dict(os.environ)
        e.update(RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    cmd = [sys.executable, os.path.abspath(__file__)] + argv
    if print_only:
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        print(json.dumps({"cmd": cmd, "ranks": [{k: e[k] for k in keys} for e in envs]}))
        return 0
    procs = [subprocess.Popen(cmd, env=e) for e in envs]
    codes = [p.wait() for p in procs]
    bad = [(i, c) for i, c in enumerate(codes) if c != 0]
    if bad:
        print(f"bench.py: ranks failed (rank, exit code): {bad}", file=sys.stderr)
        return 1
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override batch per GPU")
    ap.add_argument("--horizon", type=int, default=0, help="override the config's horizon N")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the throughput baseline (0: the affinity CPU count, capped by "
                         "OMP_NUM_THREADS when set)")
    ap.add_argument("--c1-ticks", type=int, default=10000, help="single-core C1 ticks per solver (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-full-host", action="store_true",
                    help="skip the all-CPUs leg of the CPU baseline (the per-GPU share is always timed)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, one GPU per rank); gloo only to rehearse several "
                         "ranks on fewer GPUs (ranks share devices round robin)")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the latency probes (profiling runs: only the config's launches)")
    ap.add_argument("--grouped", default="auto", choices=["auto", "on", "off"],
                    help="grouped solve (one W = H^-1 per 120-candidate scenario, f110qp_solve_grouped_dev); "
                         "auto = on for c4")
    ap.add_argument("--backend", default="auto", choices=["auto", "wave", "lane"],
                    help="solver back end (auto: lane-per-QP for box-only batches >= capi.LANE_MIN_BATCH = 1024 "
                         "at N <= 32, >= capi.LANE_MIN_BATCH_WIDE = 1 at N > 32; f110qp_backend_info)")
    ap.add_argument("--print-launch", action="store_true", help=argparse.SUPPRESS)  # test hook: the rank plan
    args = ap.parse_args()

    # one process per GPU: under torch.distributed.run (WORLD_SIZE set) it must agree with --gpus;
    # without a launcher, --gpus N > 1 starts the N ranks itself (before any GPU call here)
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: refusing to run "
                  f"a different number of ranks than asked for", file=sys.stderr)
            sys.exit(2)
    elif args.gpus > 1:
        argv = [a for a in sys.argv[1:] if a != "--print-launch"]
        sys.exit(launch_ranks(args.gpus, argv, print_only=args.print_launch))
    elif args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gloo = args.dist_backend == "gloo"
    ndev = max(1, torch.cuda.device_count())
    dev = torch.device("cuda", (local % ndev) if world > 1 else 0)
    torch.cuda.set_device(dev)
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def allreduce(v: float, op) -> float:
        """Scalar all-reduce over the ranks (RCCL on the device, or gloo on the host)."""
        t = torch.tensor([v], dtype=torch.float64, device="cpu" if gloo else dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    from f110qp import capi, workload

    Bper, N, gap, warm, desc = CONFIGS[args.config]
    if args.batch:
        Bper = args.batch
    if args.horizon:
        N = args.horizon
    strong = args.config in STRONG
    stream_cfg = args.config.startswith("c5")
    tick_cfg = args.config == "tick"
    if tick_cfg:
        sc = workload.make_scenes(Bper, seed=3000 + rank)
        pcfg = capi.default_plan_config()
        ptab = torch.from_numpy(capi.traj_table(pcfg)).to(dev)
        ppose = torch.from_numpy(sc["pose"]).to(dev)
        pranges = torch.from_numpy(sc["ranges"]).to(dev)
        pwp = torch.from_numpy(np.ascontiguousarray(sc["waypoints"][:, :2])).to(dev)
        P = pcfg.traj_discrete
        pxr = torch.empty((Bper, P, 3), dtype=torch.float32, device=dev)
        px0 = torch.empty((Bper, 3), dtype=torch.float32, device=dev)
        pbt = torch.empty(Bper, dtype=torch.int32, device=dev)
        pbg = torch.empty(Bper, dtype=torch.int32, device=dev)
        pst = torch.empty(Bper, dtype=torch.int32, device=dev)
        w = workload.make_batch(Bper, N, seed=1000 + rank)  # u_lin (v = 4.5, project.cpp:170)
        w["u_lin"][:, 1] = 0.0
    if strong:
        # one global batch of grouped candidates; this rank solves its scenario-aligned shard
        from f110qp import shard
        total = Bper
        lo, hi = shard.shard_range(total, world, rank, GROUP)
        g = workload.make_grouped_batch(-(-total // GROUP), N, seed=4000)
        w = {k: np.ascontiguousarray(g[k][:total][lo:hi]) for k in ("x0", "u_lin", "x_ref")}
        gid_np = (np.arange(lo, hi) // GROUP - lo // GROUP).astype(np.int32)
        Bper = hi - lo
    elif stream_cfg:
        # one tick of the stream per step, all ticks staged in HBM before timing
        nt = args.warmup + args.steps + 20
        if args.config == "c5_straight":
            ticks = workload.make_stream(Bper, N, nt, seed=1000 + rank)
        else:
            # the closed loop is generated once, before timing, by a cold solver of the same back end
            # (its u*_0 drives the simulated car); the timed steps replay the recorded ticks
            gen_cfg = capi.default_config(N, device=dev.index, backend={"auto": capi.BACKEND_AUTO, "wave":
                                          capi.BACKEND_WAVE, "lane": capi.BACKEND_LANE}[args.backend])
            gen = capi.Solver(gen_cfg)
            ticks = workload.closed_loop_stream(lambda a, b_, c: gen.solve(a, b_, c)[0], Bper, N, nt,
                                                seed=1000 + rank)
            gen.close()
        key_hit = workload.warm_key_hit_rate(ticks)
        IT = torch.empty((nt, Bper), dtype=torch.int32, device=dev)
        X0 = torch.from_numpy(np.stack([t["x0"] for t in ticks])).to(dev)
        UL = torch.from_numpy(np.stack([t["u_lin"] for t in ticks])).to(dev)
        XR = torch.from_numpy(np.stack([t["x_ref"] for t in ticks])).to(dev)
        w = ticks[0]
    elif not strong:
        w = workload.make_batch(Bper, N, seed=1000 + rank)
    x0 = torch.from_numpy(w["x0"]).to(dev)
    ul = torch.from_numpy(w["u_lin"]).to(dev)
    xr = torch.from_numpy(w["x_ref"]).to(dev)
    hs = None
    if gap:
        # one 1,080-beam LaserScan per QP, resident in HBM; FindHalfSpaces runs inside every step
        # (MPC::Update calls it per tick, mpc.cpp:75)
        ranges, amin, ainc, amax = workload.make_scans(Bper, seed=2000 + rank)
        rng_d = torch.from_numpy(ranges).to(dev)
        hs = torch.empty((Bper, 2, 3), dtype=torch.float32, device=dev)
    uo = torch.empty((Bper, N, 2), dtype=torch.float32, device=dev)
    xo = torch.empty((Bper, N + 1, 3), dtype=torch.float32, device=dev)
    st = torch.empty((Bper,), dtype=torch.int32, device=dev)
    it = torch.empty((Bper,), dtype=torch.int32, device=dev)
    backend = {"auto": capi.BACKEND_AUTO, "wave": capi.BACKEND_WAVE, "lane": capi.BACKEND_LANE}[args.backend]
    cfg = capi.default_config(N, gap_mode=capi.GAP_ACTIVE if gap else capi.GAP_INACTIVE, device=dev.index,
                              warm_start=int(warm), backend=backend,
                              x_ref_points=(pcfg.traj_discrete if tick_cfg else 0))
    grouped = (args.grouped == "on") or (args.grouped == "auto" and strong)
    if grouped:
        if not strong:  # independent ticks: every QP its own group (measures the prepare overhead)
            gid_np = np.arange(Bper, dtype=np.int32)
        gid = torch.from_numpy(gid_np).to(dev)
        ngroups = int(gid_np.max()) + 1
    solver = capi.Solver(cfg)
    # the launch this call makes, as the library resolves it (back end, QPs per wave, scratch)
    eff, lane_qpw, lane_scr = solver.backend_info(Bper, grouped)
    be_name = "lane" if eff == capi.BACKEND_LANE else "wave"
    lane_seg = solver.lane_segments(Bper) if be_name == "lane" else 1
    lane_starts = solver.lane_starts(Bper) if be_name == "lane" else 1
    if be_name == "lane":
        dtype = "fp64" if lane_scr in (1, 3) else "fp64 (fp32 Riccati-gain scratch in " + (
            "LDS)" if lane_scr == 2 else "HBM)")
    else:
        dtype = "fp32 (fp64 refinement and re-check)"
    stream = torch.cuda.current_stream(dev)
    tick = [0]

    def plan_step():
        capi.plan_batch_dev(pcfg, ppose, pranges, sc["angle_min"], sc["angle_inc"], sc["angle_max"], ptab, pwp,
                            pxr, px0, pbt, pbg, pst, stream=stream)

    def hs_step():
        capi.find_half_spaces_dev(x0, rng_d, amin, ainc, amax, hs, stream=stream)

    # the static-buffer steps go through a prepared launcher: one C call per step, as a C++
    # caller of the ABI would make (Python argument marshalling is not part of the solve)
    fast = None
    if not (tick_cfg or stream_cfg):
        fast = (solver.prepare_grouped_dev(x0, ul, xr, hs, gid, ngroups, uo, xo, st, it, stream=stream) if grouped
                else solver.prepare_dev(x0, ul, xr, hs, uo, xo, st, it, stream=stream))

    def step():
        if gap:
            hs_step()
        if fast is not None:
            fast()
        elif tick_cfg:
            plan_step()
            # scenarios without a valid candidate keep NaN x_ref and come back non-solved,
            # as MPC::Update is skipped for them in the reference (project.cpp:117-121)
            solver.solve_dev(px0, ul, pxr, hs, uo, xo, st, it, stream=stream)
        elif stream_cfg:
            t = tick[0] % X0.shape[0]  # the latency probe after the timed region wraps around
            tick[0] += 1
            solver.solve_dev(X0[t], UL[t], XR[t], hs, uo, xo, st, IT[t], stream=stream)
        elif grouped:
            solver.solve_grouped_dev(x0, ul, xr, hs, gid, ngroups, uo, xo, st, it, stream=stream)
        else:
            solver.solve_dev(x0, ul, xr, hs, uo, xo, st, it, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if warm:
        solver.warm_hits()  # zero the warm-start counters: the timed steps' own are read below
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # what the warm start did in the timed steps (f110qp_warm_hits: device counters of the lane back
    # ends; the wave back end reports none)
    warm_eff = None
    if warm:
        wt_calls, wt_hits = solver.warm_hits()
        warm_eff = {"calls_moving_warm_state": wt_calls, "calls": args.steps, "qps_seeded": wt_hits,
                    "hit_rate": wt_hits / float(Bper * args.steps),
                    "note": "counted on the device; a QP is seeded when its slot key (theta0, v, steer bits) "
                            "repeats; the closed loop's theta0 moves every tick, so its solves are cold solves"
                            if be_name == "lane" else "wave back end: not counted"}
    if world > 1:
        el = allreduce(el, dist.ReduceOp.MAX)

    # solver statistics of the last step (all steps solve the same batch); streams: every timed tick
    stn = st.cpu().numpy()
    itn = IT[args.warmup:args.warmup + args.steps].cpu().numpy() if stream_cfg else it.cpu().numpy()
    solved = float((stn == capi.SOLVED).mean())

    # dominant kernel duration: HIP events on the launch stream around back-to-back launches
    # (the queue stays full, so host launch overhead is not counted; rocprofv3 --stats agrees)
    KEV = 20 if not stream_cfg else 18
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    step()
    a.record(stream)
    for _ in range(KEV):
        step()
    b.record(stream)
    torch.cuda.synchronize(dev)
    kms = a.elapsed_time(b) / KEV  # ms per launch
    plan_ms = None
    hs_ms = None
    if gap:  # the FindHalfSpaces kernel alone, same stream
        a.record(stream)
        for _ in range(20):
            hs_step()
        b.record(stream)
        torch.cuda.synchronize(dev)
        hs_ms = a.elapsed_time(b) / 20
        kms = kms - hs_ms  # the QP kernel of the step
    if tick_cfg:  # the planning kernel alone, same stream
        a.record(stream)
        for _ in range(20):
            plan_step()
        b.record(stream)
        torch.cuda.synchronize(dev)
        plan_ms = a.elapsed_time(b) / 20
        kms = kms - plan_ms  # the QP kernel(s) of the step

    # per-QP latency: single-QP solves (B = 1) through the device entry point (launch + sync)
    # and through the host-pointer entry point (H2D + launch + D2H), plus the per-launch
    # distribution of the configured batch; rank 0 only, outside the timed region
    latency = None
    if rank == 0 and not args.no_latency:
        latency = measure_latency(capi, solver, cfg, w, hs, N, dev, stream, step)

    if strong:
        total_qps = int(round(allreduce(float(Bper), dist.ReduceOp.SUM) if world > 1 else Bper)) * args.steps
    else:
        total_qps = Bper * world * args.steps
    value = total_qps / el
    ms_per_step = el / args.steps * 1e3
    bpq = bytes_per_qp(N, gap, warm, be_name)
    # active-set size ~ iterations for an add-only run; use iterations as the upper bound
    seg_overhead = None
    if be_name == "lane":
        # Riccati + forward + adjoint sweeps: (active-set changes + 1) passes over N stages, priced at
        # the sequential algorithm's flops (the segmented kernel's redundancy is reported apart)
        fpq = LANE_FLOPS_PER_STAGE * N * (float(itn.mean()) + 1.0)
        if lane_seg > 1 and not gap:
            seg_overhead = {"executed_flops_per_stage_pass": seg_flops_per_stage(lane_seg, N),
                            "algorithmic_flops_per_stage_pass": LANE_FLOPS_PER_STAGE,
                            "ratio": seg_flops_per_stage(lane_seg, N) / LANE_FLOPS_PER_STAGE,
                            "note": "parallel-in-time redundancy of the partitioned horizon (closed-loop map "
                                    "per stage, S - 1 segment steps); not counted in fp64_compute"}
        cpeak, cname = FP64_PEAK_TFLOPS, "fp64_compute"
    else:
        # pivots >= bounds active at the solution (each entered the active set once)
        un = uo.cpu().numpy()
        lo = np.float32([cfg.u_min[0], cfg.u_min[1]])
        hi = np.float32([cfg.u_max[0], cfg.u_max[1]])
        n_act = float(((np.abs(un - lo) < 1e-6) | (np.abs(un - hi) < 1e-6)).sum(axis=(1, 2)).mean())
        fpq = flops_per_qp(N, float(itn.mean()), n_act, gap)
        cpeak, cname = FP32_PEAK_TFLOPS, "fp32_compute"
    achieved_gbs = bpq * Bper / (kms * 1e-3) / 1e9
    achieved_tf = fpq * Bper / (kms * 1e-3) / 1e12
    # the PMC summary's back-end key (tools/summarize_profiles.py KERNELS): the partitioned-horizon
    # kernel is "lane_seg"
    prof_be = be_name if be_name == "wave" else ("lane_seg" if lane_seg > 1 else "lane")
    traffic = load_traffic(args.config, Bper, N, prof_be)

    out = {
        "metric": f"QP solves/s (horizon={N}, nx=3 reference model, nu=2)",
        "value": value,
        "unit": "QP solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (seeded; SURVEY.md 8(d) recipe: simulate_dynamics mini paths)",
        "config": {
            "workload": desc,
            "batch_per_gpu": Bper,
            "global_batch": total_qps // args.steps,
            "horizon": N,
            "gap_rows": bool(gap),
            "warm_start": bool(warm),
            "backend": {"wave": "wave-per-QP (condensed, PDAS/GI)",
                        "lane": "lane-per-QP box screen (Riccati/PDAS fp64) + wave GI for the QPs it does not "
                                "clear" if gap else "lane-per-QP (Riccati/PDAS fp64)"}[be_name]
                       + (" grouped: one W = H^-1 per scenario" if grouped and be_name == "wave" else ""),
            **({"lane_qps_per_wave": lane_qpw, "lane_scratch": capi.SCRATCH_NAMES[lane_scr],
                "lane_segments": lane_seg, "lane_pdas_starts": lane_starts}
               if be_name == "lane" else {}),
            "parallelism": f"independent QP shards x{world} (no collective)"
                           + (f", scenario-aligned ({GROUP}) split of one global batch" if strong else ""),
            "solved_fraction": solved,
            **({"step": "f110qp_find_half_spaces_dev (one 1,080-beam scan per QP) + f110qp_solve_batch_dev",
                "halfspace_kernel_ms": hs_ms,
                "halfspace_roofline": {"bound": "hbm", "bytes_per_scan": 4 * (ranges.shape[1] + 3 + 6 + 2),
                                       "achieved_gbs": 4 * (ranges.shape[1] + 11) * Bper / (hs_ms * 1e-3) / 1e9,
                                       "peak_gbs": HBM_PEAK_GBS,
                                       "frac": 4 * (ranges.shape[1] + 11) * Bper / (hs_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}}
               if gap else {}),
            **({"plan_kernel_ms": plan_ms, "planned_fraction": float((pst.cpu().numpy() == 0).mean()),
                "step": "f110qp_plan_batch_dev + f110qp_solve_batch_dev (x_ref_points = 50)"} if tick_cfg else {}),
            "mean_active_set_iters": float(itn.mean()),
            "max_active_set_iters": int(itn.max()),
            **({"warm_key_hit_rate": key_hit,
                "stream": "closed loop" if args.config != "c5_straight" else "straight (best case)"}
               if stream_cfg else {}),
            **({"warm_effective": warm_eff} if warm_eff is not None else {}),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": {"wave": "f110qp::solve_kernel",
                       "lane": ("f110qp::lane_kernel" if lane_seg == 1 else
                                f"f110qp::lane_seg_kernel<{lane_seg}> (partitioned horizon)")
                               + (" box screen + the wave kernel's GI over its list" if gap else
                                  " (the only launch of the step)")}[be_name],
            "kernel_ms_per_launch": kms,
            "algorithmic_bytes_per_qp": bpq,
            cname: {"achieved": achieved_tf, "peak": cpeak, "unit": "TFLOP/s",
                    "frac": achieved_tf / cpeak, "flops_per_qp": fpq},
            **({"segmentation_overhead": seg_overhead} if seg_overhead else {}),
            "note": ("lane kernel: fp64 VALU-issue and scratch-latency bound (Riccati sweeps, 64 QPs per "
                     "wave); traffic = PMC HBM bytes incl. the Riccati scratch" if be_name == "lane" and lane_seg == 1 else
                     f"partitioned-horizon lane kernel: one QP per {lane_seg} lanes"
                     + (" x 2 PDAS starts (twin: the first to converge answers)" if lane_starts == 2 else "")
                     + ", latency-bound by the slowest QP's PDAS passes x (N/S stages + S-1 segment steps); "
                     "scratch in LDS, HBM = inputs/outputs"
                     if be_name == "lane" else
                     "wave kernel: latency-bound (serial active-set chain per wave); neither HBM nor FP32 "
                     "peak binds"),
        },
    }
    if latency is not None:
        out["latency"] = latency
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(args.config, N, gap, args.cpu_seconds,
                                               args.cpu_threads or cpu_threads_default(), args.c1_ticks,
                                               full_threads=0 if args.no_full_host else len(os.sched_getaffinity(0)))
        except Exception as e:  # the baseline must never take the GPU number down
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    solver.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
