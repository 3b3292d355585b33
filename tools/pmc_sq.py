"""Per env-tick SQ counters of the K-tick kernel from a rocprofv3 --pmc pass of bench.py
(one wave per env: per-wave counters are per env).  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_*
count quad-cycles (MI355X_MICROARCH.md, s_memtime row); instruction counts are per wave.

    python tools/pmc_sq.py gpurun_out/<tag>/pmc_sq --ticks 20 --out profiles/<tag>_pmc_sq.json
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--kernel", default="step_lean_kernel")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    per = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            d = per.setdefault(key, {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = [d for d in per.values() if d.get("SQ_WAVES")]
    out = {"kernel": a.kernel, "dispatches": len(rows), "ticks_per_launch": a.ticks, "per_wave_per_tick": {}}
    for c in sorted({c for d in rows for c in d}):
        if c == "SQ_WAVES":
            continue
        vals = [d[c] / d["SQ_WAVES"] / a.ticks for d in rows if c in d]
        if vals:
            out["per_wave_per_tick"][c] = statistics.median(vals)
    pw = out["per_wave_per_tick"]
    if "SQ_WAIT_ANY" in pw and "SQ_WAVE_CYCLES" in pw:
        out["wait_any_frac"] = pw["SQ_WAIT_ANY"] / pw["SQ_WAVE_CYCLES"]
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
