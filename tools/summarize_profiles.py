"""Summarise tools/profile_round.sh output into profiles/<round>/ and profiles/pmc_<config>.json.

For each config: the kernel-stats CSV of the trace pass is copied; the PMC passes give
FETCH_SIZE and WRITE_SIZE (KB per dispatch) of the dominant kernel, averaged over its
dispatches, reported raw (see MI355X_MICROARCH.md: gfx950 FETCH_SIZE under-reports wide
coalesced streams by 2x; these kernels' reads are narrow gathers, so no correction is applied).
Usage: python tools/summarize_profiles.py r02 c2 c4 c4_8192 ... (a name <config>_<batch> is the
config run at that batch, profiled with PROF_NAME=<name> tools/profile_round.sh <config> --batch <batch>)
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"wave": "solve_kernel", "lane": "lane_kernel", "lane_seg": "lane_seg_kernel"}


def find(pattern):
    m = sorted(glob.glob(pattern, recursive=True))
    return m[0] if m else None


def pmc_per_dispatch(path, counter, kname):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kname not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return (sum(vals.values()) / len(vals), len(vals)) if vals else (None, 0)


def main():
    rnd = sys.argv[1]
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for c in sys.argv[2:]:
        base = os.path.join(ROOT, "gpurun_out", f"prof_{c}")
        bench = json.load(open(os.path.join(base, "bench_trace.json")))
        be = "lane" if bench["config"]["backend"].startswith("lane") else "wave"
        if be == "lane" and bench["config"].get("lane_segments", 1) > 1:
            be = "lane_seg"
        kname = KERNELS[be]
        ks = find(os.path.join(base, "trace", "**", "*kernel_stats.csv"))
        if ks:
            shutil.copy(ks, os.path.join(dst, f"{c}_kernel_stats.csv"))
            with open(ks) as f:
                rows = [r for r in csv.DictReader(f) if kname in r["Name"]]
            avg_us = float(rows[0]["AverageNs"]) / 1e3 if rows else None
        else:
            avg_us = None
        shutil.copy(os.path.join(base, "bench_trace.json"), os.path.join(dst, f"{c}_bench_under_rocprof.json"))
        fetch, nf = pmc_per_dispatch(find(os.path.join(base, "fetch", "**", "*counter_collection.csv")), "FETCH_SIZE", kname)
        write, nw = pmc_per_dispatch(find(os.path.join(base, "write", "**", "*counter_collection.csv")), "WRITE_SIZE", kname)
        for sub, name in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
            src = find(os.path.join(base, sub, "**", "*counter_collection.csv"))
            if src:
                shutil.copy(src, os.path.join(dst, f"{c}_pmc_{sub}.csv"))
        B = bench["config"]["batch_per_gpu"]
        hbm = (fetch + write) * 1024 if fetch is not None and write is not None else None
        out = {
            "config": c.split("_")[0] if c.split("_")[-1].isdigit() else c,
            "batch": B,
            "horizon": bench["config"]["horizon"],
            "backend": be,
            "kernel": f"f110qp::{kname} (config {c}: {B} QPs, N={bench['config']['horizon']}, {bench['config']['backend']})",
            "passes": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --no-cpu --config {c} --steps 20",
            "rocprof_avg_kernel_us": avg_us,
            "bench_hip_event_kernel_us": bench["roofline"]["kernel_ms_per_launch"] * 1e3,
            "fetch_size_kb_per_launch": fetch,
            "write_size_kb_per_launch": write,
            "dispatches": [nf, nw],
            "hbm_bytes_per_launch": hbm,
            "hbm_bytes_per_qp": hbm / B if hbm else None,
            "algorithmic_bytes_per_qp": bench["roofline"]["algorithmic_bytes_per_qp"],
            "note": "FETCH_SIZE/WRITE_SIZE are KB (x1024), summed over the kernel's dispatches and averaged; raw. MI355X_MICROARCH.md: gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads and other widths are uncalibrated; these kernels read with 4-B (x_ref staging) and 4/8-B (scratch) lanes, so the read share may be under-reported by up to 2x.",
        }
        json.dump(out, open(os.path.join(ROOT, "profiles", f"pmc_{c}.json"), "w"), indent=1)
        print(c, json.dumps(out))


if __name__ == "__main__":
    main()
