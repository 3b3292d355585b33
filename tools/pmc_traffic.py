"""Turn the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into the per-launch
HBM traffic figure bench.py reports as roofline.traffic (profiles/heist_step_traffic.json).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 128-B requests at
64 B, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Counters
are in KB (rocprofv3 derived metrics).  Only the step kernel's dispatches are used
(step_kernel for one tick per launch; step_lean_kernel / step_multi_kernel for K ticks).

    python tools/pmc_traffic.py gpurun_out/<tag>/pmc_fetch gpurun_out/<tag>/pmc_write [--envs 4096]
"""
import argparse
import csv
import glob
import json
import os
import statistics

KERNELS = ("step_kernel",)


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in KERNELS) and r["Counter_Name"] == counter:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--workload", default="architect", help="bench.py --layouts of the profiled command")
    ap.add_argument("--profile", default=None, help="run tag the passes come from (e.g. r02a)")
    ap.add_argument("--ticks", type=int, default=1, help="ticks per launch (bench.py --ticks-per-launch)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    global KERNELS
    # K-tick launches: the lean one-wave kernel (20 x 20 at one wave per env), else the generic one
    KERNELS = ("step_lean_kernel", "step_multi_kernel") if a.ticks > 1 else ("step_kernel",)
    if a.out is None:
        a.out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                             "heist_step_multi_traffic.json" if a.ticks > 1 else "heist_step_traffic.json")
    fetch = per_dispatch(a.fetch_dir, "FETCH_SIZE")
    write = per_dispatch(a.write_dir, "WRITE_SIZE")
    f_kb, w_kb = statistics.median(fetch), statistics.median(write)
    fetch_b = 2 * f_kb * 1024.0
    write_b = w_kb * 1024.0
    out = {"kernel": "heist::" + KERNELS[0], "envs": a.envs, "workload": a.workload, "ticks_per_launch": a.ticks,
           "profile": a.profile or os.path.basename(os.path.dirname(os.path.abspath(a.fetch_dir))), "dispatches": [len(fetch), len(write)],
           "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
           "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
           "hbm_bytes_per_launch": fetch_b + write_b,
           "hbm_bytes_per_tick": (fetch_b + write_b) / a.ticks,
           "hbm_bytes_per_env_step": (fetch_b + write_b) / a.ticks / a.envs,
           "note": "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B); Infinity-Cache hits are "
                   "counted by these memory-side counters"}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
