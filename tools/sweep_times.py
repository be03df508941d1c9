"""Summarise a rocprofv3 kernel trace (or --pmc counter collection) in
dispatch order: one line per kernel dispatch of the last build (name, ms or
counter value), then totals per kernel.  Measurement tool.
usage: python tools/sweep_times.py <rocprofv3 -d dir> [--pmc COUNTER]
"""
import csv
import glob
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").replace("srt::(anonymous namespace)::", "")
    return n.split("(")[0]


def main():
    d = sys.argv[1]
    pmc = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--pmc" else None
    if pmc:
        f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
        rows = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != pmc:
                continue
            k = int(r["Dispatch_Id"])
            rows[k] += float(r["Counter_Value"])
            names[k] = short(r["Kernel_Name"])
        seq = [(names[k], rows[k]) for k in sorted(rows)]
        unit = pmc
    else:
        f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
        rs = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        seq = [(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in rs]
        unit = "ms"
    tot = defaultdict(lambda: [0, 0.0])
    for n, x in seq:
        tot[n][0] += 1
        tot[n][1] += x
    for n, (c, x) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"TOTAL {n}: {c} dispatches, {x:.3f} {unit}")
    sweeps = [(n, x) for n, x in seq if "sweep" in n]
    print("sweeps:", " ".join(f"{x:.3f}" for _, x in sweeps))


if __name__ == "__main__":
    main()
