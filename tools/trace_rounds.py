"""Per-round timeline of a dense-FW kernel trace (rocprofv3 --kernel-trace CSV).

usage: python tools/trace_rounds.py <run_kernel_trace.csv> [n_rows]
Prints a window of kernels around the middle of the run and the average gap
between the phase-3 rest kernels and the look-ahead cross kernels.
"""
import csv
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").split("(")[0].replace("void srt::", "")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    nshow = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    ev = sorted((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, short(r["Kernel_Name"]),
                 r["Queue_Id"], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])) for r in rows)
    fw = [e for e in ev if "minplus" in e[2] or "phase1" in e[2]]
    mid = len(fw) // 2
    for s, e, name, q, wg in fw[mid:mid + nshow]:
        print(f"{s / 1e3:10.1f} {e / 1e3:10.1f} dur={(e - s) / 1e3:7.1f} {name:40s} q={q} wg={wg}")
    # main-queue gaps: consecutive kernels on the queue of the rest kernels
    rest = [e for e in fw if e[2].endswith(", 0>")]
    if not rest:
        return
    q = rest[0][3]
    mq = [e for e in fw if e[3] == q]
    gaps = [b[0] - a[1] for a, b in zip(mq, mq[1:])]
    per_round = [(b[0] - a[0]) for a, b in zip(rest, rest[1:])]
    print(f"rest kernels {len(rest)}: avg dur {sum(e[1] - e[0] for e in rest) / len(rest) / 1e3:.1f} us, "
          f"round period {sum(per_round) / max(1, len(per_round)) / 1e3:.1f} us, "
          f"main-queue gap avg {sum(gaps) / max(1, len(gaps)) / 1e3:.1f} us over {len(gaps)}")


if __name__ == "__main__":
    main()
