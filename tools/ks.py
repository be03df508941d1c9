"""Compact per-kernel summary of a rocprofv3 kernel_stats CSV.
usage: python tools/ks.py <run_kernel_stats.csv> [top]"""
import csv
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("srt::", "")
    base = n.split("(")[0]
    return base.replace("unsigned short", "u16").replace("unsigned int", "u32")


rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:top]:
    print(f"{short(r['Name'])[:64]:64s} {int(r['Calls']):6d} {float(r['TotalDurationNs']) / 1e6:9.3f} ms "
          f"avg {float(r['AverageNs']) / 1e3:9.2f} us")
