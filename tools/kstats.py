"""Per-kernel totals from a rocprofv3 SQLite result (gpurun_out/<dir>/run_results.db),
and optionally the dispatch sequence of a few kernels.  Measurement tool.
usage: python tools/kstats.py gpurun_out/<dir> [seq-substring ...]
"""
import glob
import sqlite3
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def main():
    db = glob.glob(sys.argv[1] + "/**/*results.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e3 from kernels group by name "
                     "order by 3 desc").fetchall()
    for name, n, tot, avg in rows[:16]:
        print(f"{short(name)[-48:]:48s} {n:6d} {tot:10.2f} ms {avg:10.1f} us")
    subs = sys.argv[2:]
    if subs:
        seq = c.execute("select name, (end-start)/1e3 from kernels order by start").fetchall()
        out = [f"{short(n).split('::')[-1][:10]}:{d:.0f}" for n, d in seq if any(s in n for s in subs)]
        print(" ".join(out[:400]))


if __name__ == "__main__":
    main()
