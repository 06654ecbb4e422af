"""Idle time between consecutive kernels of a rocprofv3 kernel trace, per (previous, next) pair.

    python tools/trace_gaps.py gpurun_out/prof [min_steps]

Reads <dir>/run_kernel_trace.csv, keeps the dad_* kernels, sorts them by start time and reports,
for every (previous kernel, next kernel) pair, the count and the median / p10 / p90 of
start(next) - end(previous) in microseconds.  A step's idle time is the sum of its seams; the
optimizer -> next-encoder seam is the inter-step gap.
"""
import collections
import csv
import os
import sys


def gaps(prof):
    rows = list(csv.DictReader(open(os.path.join(prof, "run_kernel_trace.csv"))))
    rows = [r for r in rows if r["Kernel_Name"].startswith("dad_")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = collections.defaultdict(list)
    for a, b in zip(rows, rows[1:]):
        na, nb = a["Kernel_Name"].split("(")[0], b["Kernel_Name"].split("(")[0]
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        if g < 50.0:                      # seams inside a stream of back-to-back launches only
            out[(na, nb)].append(g)
    return out


def main():
    prof = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
    need = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    res = gaps(prof)
    print("| previous | next | seams | median us | p10 | p90 |")
    print("|---|---|---|---|---|---|")
    for (a, b), v in sorted(res.items(), key=lambda kv: -len(kv[1])):
        if len(v) < need:
            continue
        v = sorted(v)
        q = lambda f: v[min(len(v) - 1, int(f * len(v)))]
        print("| `%s` | `%s` | %d | %.2f | %.2f | %.2f |" % (a, b, len(v), q(0.5), q(0.1), q(0.9)))


if __name__ == "__main__":
    main()
