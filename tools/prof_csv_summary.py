"""rocprofv3 --stats CSV (run_kernel_stats.csv) -> markdown table for profiles/."""
import csv
import sys


def summary(path, title):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = ["# %s" % title, "", "| kernel | calls | avg us | min us | max us | total % |", "|---|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        out.append("| `%s` | %s | %.1f | %.1f | %.1f | %.1f |" % (
            r["Name"].split("(")[0][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
            float(r["MaxNs"]) / 1e3, 100.0 * float(r["TotalDurationNs"]) / tot))
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    src, dst, title = sys.argv[1], sys.argv[2], sys.argv[3]
    open(dst, "w").write(summary(src, title))
