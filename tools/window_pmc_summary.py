"""Slow-window study, counter side: per dispatch of step_lean_kernel in a rocprofv3 --pmc
run of tools/probe_window_spread.py (counters GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES,
SQ_BUSY_CYCLES, SQ_WAVES), the duration, the GPU-active cycles per microsecond (the clock
summed over the XCDs) and the waves' cycles; the slow launches (> 1.05 x the median
duration) against the rest.  A clock dip would show as fewer active cycles per us in the
slow launches; the same cycles per us with more wave cycles means the waves themselves
took longer (memory-side stalls).  One JSON object.

    python tools/window_pmc_summary.py <pmc dir>/..._counter_collection.csv [--out x.json]
"""
import argparse
import collections
import csv
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--out")
    a = ap.parse_args()
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(a.csv)):
        if "step_lean" not in r["Kernel_Name"]:
            continue
        d = by[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ids = sorted(by)
    du = np.array([by[i]["dur_us"] for i in ids])
    gui = np.array([by[i]["GRBM_GUI_ACTIVE"] for i in ids])
    wav = np.array([by[i]["SQ_WAVE_CYCLES"] for i in ids])
    slow = du > 1.05 * np.median(du)
    clk = gui / du
    out = {
        "dispatches": len(ids), "slow_dispatches": int(slow.sum()),
        "dur_us_p10_p50_p90": [float(np.percentile(du, p)) for p in (10, 50, 90)],
        "gui_active_cycles_per_us_p10_p50_p90": [float(np.percentile(clk, p)) for p in (10, 50, 90)],
        "gui_active_cycles_per_us_slow_vs_rest": [float(clk[slow].mean()), float(clk[~slow].mean())],
        "corr_duration_gui_active": float(np.corrcoef(du, gui)[0, 1]),
        "corr_duration_wave_cycles": float(np.corrcoef(du, wav)[0, 1]),
        "slow_over_rest": {"duration": float(du[slow].mean() / du[~slow].mean()),
                           "gui_active": float(gui[slow].mean() / gui[~slow].mean()),
                           "wave_cycles": float(wav[slow].mean() / wav[~slow].mean())},
    }
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
