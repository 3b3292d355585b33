"""Summarise a rocprofv3 --pmc counter_collection.csv: median per counter over the
dispatches of kernels whose name matches a regex.  Usage:
    python tools/pmc_summary.py <counter_collection.csv> <kernel-regex> [out.json] [--modes N_MODES PER_MODE]
With --modes the matching dispatches are split by order into N_MODES modes cycling in
blocks of PER_MODE (tools/probe_multi_modes.py), and medians are per mode."""
import collections
import csv
import json
import re
import sys


def main():
    args = sys.argv[1:]
    modes = None
    if "--modes" in args:
        i = args.index("--modes")
        modes = (int(args[i + 1]), int(args[i + 2]))
        args = args[:i] + args[i + 3:]
    path, rx = args[0], re.compile(args[1])
    rows = collections.defaultdict(dict)
    with open(path) as f:
        for r in csv.DictReader(f):
            if rx.search(r["Kernel_Name"]):
                key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(rows))
                rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    groups = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, d in enumerate(sorted(rows)):
        m = (k // modes[1]) % modes[0] if modes else 0
        for c, v in rows[d].items():
            groups[m][c].append(v)
    med = {m: {c: sorted(v)[len(v) // 2] for c, v in sorted(g.items())} for m, g in groups.items()}
    out = {"kernel_regex": args[1], "stat": "median over dispatches",
           "counters": med.get(0, {}) if not modes else None,
           "modes": {str(m): v for m, v in sorted(med.items())} if modes else None,
           "dispatches": len(rows)}
    txt = json.dumps(out, indent=1)
    print(txt)
    if len(args) > 2:
        with open(args[2], "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
