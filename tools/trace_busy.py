"""Busy fraction of a rocprofv3 kernel trace: per kernel name the count and median duration, the
summed kernel time against the span of the last N kernels, and the idle seams by size.

    python tools/trace_busy.py gpurun_out/lprof/run_kernel_trace.csv [last_n]
"""
import collections
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-last:]
    dur = collections.defaultdict(list)
    for r in rows:
        dur[r["Kernel_Name"].split("(")[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    busy = sum(sum(v) for v in dur.values())
    print("kernels %d  span %.1f us  busy %.1f us (%.0f%%)" % (len(rows), span, busy, 100 * busy / span))
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print("  %-60s n %5d  median %7.2f us  total %9.1f us" % (k, len(v), statistics.median(v), sum(v)))
    seams = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
    for lo, hi in ((-1e9, 1), (1, 5), (5, 20), (20, 100), (100, 1e9)):
        s = [g for g in seams if lo <= g < hi]
        print("  seams [%g, %g) us: %5d  sum %9.1f us" % (max(lo, -1e9), hi, len(s), sum(s)))


if __name__ == "__main__":
    main()
