"""Summarise a rocprofv3 --pmc counter_collection.csv: median per counter over the
dispatches of kernels whose name matches a regex.  Usage:
    python tools/pmc_summary.py <counter_collection.csv> <kernel-regex> [out.json]"""
import collections
import csv
import json
import re
import sys


def main():
    path, rx = sys.argv[1], re.compile(sys.argv[2])
    agg = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if rx.search(r["Kernel_Name"]):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"kernel_regex": sys.argv[2], "stat": "median over dispatches",
           "counters": {k: sorted(v)[len(v) // 2] for k, v in sorted(agg.items())},
           "dispatches": {k: len(v) for k, v in sorted(agg.items())}}
    txt = json.dumps(out, indent=1)
    print(txt)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
