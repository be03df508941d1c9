"""Per-kernel PMC totals from rocprofv3 SQLite results (one or more --pmc
passes), with per-dispatch averages.  Measurement tool.
usage: python tools/pmc_summary.py gpurun_out/<pass dir> [...]
"""
import collections
import glob
import sqlite3
import sys


def short(name):
    n = name.split("namespace)::")[-1] if "namespace)::" in name else name
    return n.split("(")[0]


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in sys.argv[1:]:
        db = glob.glob(d + "/**/*results.db", recursive=True)[0]
        c = sqlite3.connect(db)
        for did, n, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
            k = short(n)
            agg[k][cn] += v
            disp[k][cn].add(did)
    for k in sorted(agg, key=lambda k: -max(agg[k].values())):
        parts = []
        for cn, v in sorted(agg[k].items()):
            nd = len(disp[k][cn])
            parts.append(f"{cn}={v:.3e} ({nd} disp, {v / max(nd, 1):.3e}/disp)")
        print(f"{k[:34]:34s} " + "  ".join(parts))


if __name__ == "__main__":
    main()
