"""Per-probe-mode PMC summary: rocprofv3 --pmc counter CSV of tools/probe_step_modes.py,
whose step_kernel dispatches come in blocks of 55 (5 warm-up + 50 timed) cycling through
the probe modes 0..9 for 5 rounds.  Prints, per mode, the median of each counter over its
dispatches, divided by SQ_WAVES where that makes a per-wave figure.
    python tools/pmc_modes.py <counter_collection.csv> [out.json]"""
import collections
import csv
import json
import sys

MODES = (0, 1, 2, 3, 4, 5, 6, 7, 8, 9)
PER_MODE = 55


def main():
    rows = collections.defaultdict(dict)
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            if "step_kernel" in r["Kernel_Name"]:
                rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(rows)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, d in enumerate(ids):
        mode = MODES[(k // PER_MODE) % len(MODES)]
        for c, v in rows[d].items():
            agg[mode][c].append(v)
    out = {}
    for m in MODES:
        med = {c: sorted(v)[len(v) // 2] for c, v in agg[m].items()}
        waves = med.get("SQ_WAVES", 0) or 1
        out[str(m)] = {"dispatches": len(agg[m].get("SQ_WAVES", [])),
                       "per_wave": {c: round(v / waves, 1) for c, v in med.items() if c != "SQ_WAVES"},
                       "SQ_WAVES": waves}
    txt = json.dumps({"n_dispatch": len(ids), "modes": out}, indent=1)
    print(txt)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
