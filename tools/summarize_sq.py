"""Summarise tools/sq_pass.sh runs into profiles/<round>/sq_<name>.json: per dispatch of the
dominant kernel (name substring), the SQ counters summed over the device and averaged over the
dispatches, and the derived shares: active / parked (s_waitcnt) / issue-stalled fractions of the
wave cycles, VALU instructions per wave and per active-VALU cycle, LDS issue stalls. SQ_*CYCLES
count quad-cycles (MI355X_MICROARCH.md), which cancels in the fractions.
Usage: python tools/summarize_sq.py r04 NAME:KERNEL_SUBSTRING ...
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rnd = sys.argv[1]
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for spec in sys.argv[2:]:
        name, kname = spec.split(":", 1)
        files = sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"sq_{name}", "pmc", "**", "*counter_collection.csv"),
                                 recursive=True))
        if not files:
            print(name, "no counter file")
            continue
        per = {}
        kernel = None
        waves = {}
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                if kname not in row.get("Kernel_Name", ""):
                    continue
                kernel = row["Kernel_Name"]
                d = row["Dispatch_Id"]
                per.setdefault(d, {})
                c = row["Counter_Name"]
                per[d][c] = per[d].get(c, 0.0) + float(row["Counter_Value"])
                waves[d] = int(row.get("Grid_Size", 0) or 0) // max(1, int(row.get("Workgroup_Size", 64) or 64))
        if not per:
            print(name, "kernel not found")
            continue
        keys = sorted({k for v in per.values() for k in v})
        avg = {k: sum(v.get(k, 0.0) for v in per.values()) / len(per) for k in keys}
        nw = max(1, sum(waves.values()) // max(1, len(waves)))
        wc = avg.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        out = {
            "kernel": kernel, "dispatches": len(per), "waves_per_dispatch": nw, "counters_avg_per_dispatch": avg,
            "active_frac": avg.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "parked_waitcnt_frac": avg.get("SQ_WAIT_ANY", 0.0) / wc,
            "issue_stall_frac": avg.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "valu_active_frac": avg.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
            "lds_issue_stall_frac": avg.get("SQ_WAIT_INST_LDS", 0.0) / wc,
            "valu_insts_per_wave": avg.get("SQ_INSTS_VALU", 0.0) / nw,
            "lds_insts_per_wave": avg.get("SQ_INSTS_LDS", 0.0) / nw,
            "wave_cycles_per_wave_x4": 4.0 * wc / nw,
            "source": os.path.relpath(files[0], ROOT),
            "note": "fractions of SQ_WAVE_CYCLES (quad-cycles cancel); per-wave values divide the device sums by the "
                    "dispatch's waves (grid / 64)",
        }
        json.dump(out, open(os.path.join(dst, f"sq_{name}.json"), "w"), indent=1)
        print(name, json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()
                                if k not in ("counters_avg_per_dispatch", "source", "note")}))


if __name__ == "__main__":
    main()
