"""Timeline of the last build in a rocprofv3 kernel trace (SQLite results):
kernels in start order with queue, duration and the gap since the previous
kernel ended, collapsed into runs of the same kernel.  Measurement tool.
usage: python tools/timeline.py gpurun_out/<dir> [min_gap_us_to_split_builds]
"""
import glob
import sqlite3
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void srt::", "").replace("srt::", "")
    return n.split("(")[0].replace("unsigned short", "u16").replace("unsigned int", "u32")[:48]


def main():
    db = glob.glob(sys.argv[1] + "/**/*results.db", recursive=True)[0]
    split = float(sys.argv[2]) if len(sys.argv) > 2 else 20000.0
    c = sqlite3.connect(db)
    ev = c.execute("select name, start, end from kernels order by start").fetchall()
    # builds are separated by host gaps > split us
    builds, cur, last_end = [], [], None
    for n, s, e in ev:
        if last_end is not None and (s - last_end) / 1e3 > split:
            builds.append(cur)
            cur = []
        cur.append((short(n), s, e))
        last_end = e if last_end is None else max(last_end, e)
    builds.append(cur)
    b = builds[-1]
    t0 = b[0][1]
    print(f"{len(builds)} builds; last: {(max(e for _, _, e in b) - t0) / 1e6:.3f} ms, {len(b)} kernels")
    runs = []
    for n, s, e in b:
        if runs and runs[-1][0] == n:
            r = runs[-1]
            r[2] = max(r[2], e)
            r[3] += 1
            r[4] += e - s
        else:
            runs.append([n, s, e, 1, e - s])
    for n, s, e, k, busy in runs:
        print(f"{(s - t0) / 1e3:10.1f} us  {n:48s} x{k:<4d} span {(e - s) / 1e3:9.1f} us  busy {busy / 1e3:9.1f} us")


if __name__ == "__main__":
    main()
