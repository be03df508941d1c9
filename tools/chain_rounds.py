"""Round-by-round look-ahead chain of a dense-FW kernel trace (rocprofv3
--kernel-trace CSV), e.g. an emulated N-rank build (tools/emu_trace.sh).

usage: python tools/chain_rounds.py <run_kernel_trace.csv> [rounds_to_show]
For the last build in the trace: every kernel on the chain queue between two
consecutive rest launches (name, duration, gap before it), and the averages
per kernel kind over all rounds -- where the round period goes.
"""
import csv
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void srt::", "").replace("srt::", "")
    base = n.split("(")[0]
    return base.replace("unsigned short", "u16").replace("unsigned int", "u32")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    show = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
                for r in rows)
    rest = [e for e in ev if "minplus_u16_kernel<0, 3" in e[2] or "minplus_u16_kernel<0, 1" in e[2]]
    if not rest:
        print("no rest launches")
        return
    # the last build: rest launches after the largest gap between rest launches
    gaps = [(b[0] - a[1], i + 1) for i, (a, b) in enumerate(zip(rest, rest[1:]))]
    start = max(gaps)[1] if gaps else 0
    rest = rest[start:]
    mq = rest[0][3]
    t_first, t_last = rest[0][0], rest[-1][1]
    side = [e for e in ev if e[3] != mq and t_first - 200_000 <= e[0] <= t_last]
    per_kind = defaultdict(list)
    periods = [(b[0] - a[0]) / 1e3 for a, b in zip(rest, rest[1:])]
    for r, (a, b) in enumerate(zip(rest, rest[1:])):
        chain = [e for e in side if a[0] <= e[0] < b[0]]
        prev_end = a[0]
        for s, e, name, q in chain:
            per_kind[name].append(((e - s) / 1e3, (s - prev_end) / 1e3))
            prev_end = e
        if r < show or r == len(rest) // 2:
            print(f"round {r}: rest {(a[1] - a[0]) / 1e3:.1f} us, period {(b[0] - a[0]) / 1e3:.1f} us, "
                  f"rest start -> next rest start")
            pe = a[0]
            for s, e, name, q in chain:
                print(f"    +{(s - a[0]) / 1e3:7.1f} gap {(s - pe) / 1e3:6.1f} dur {(e - s) / 1e3:6.1f}  {name}")
                pe = e
            print(f"    next rest starts +{(b[0] - a[0]) / 1e3:.1f}, gap after chain {(b[0] - pe) / 1e3:.1f}")
    print(f"\n{len(rest)} rest launches, build span {(t_last - t_first) / 1e6:.2f} ms, "
          f"avg period {sum(periods) / max(1, len(periods)):.1f} us, avg rest "
          f"{sum((e[1] - e[0]) for e in rest) / len(rest) / 1e3:.1f} us")
    for name, v in sorted(per_kind.items(), key=lambda kv: -sum(x[0] + x[1] for x in kv[1])):
        n = len(v)
        print(f"  {name[:60]:60s} n={n:4d} dur {sum(x[0] for x in v) / n:7.1f} us  gap-before {sum(x[1] for x in v) / n:6.1f} us")


if __name__ == "__main__":
    main()
