"""Summarise a rocprofv3 --kernel-trace database (results.db) into a markdown table."""
import sqlite3
import sys


def summary(db, steps=None):
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), avg(end-start), min(end-start), max(end-start), sum(end-start) "
                       "from kernels group by name order by sum(end-start) desc").fetchall()
    out = ["| kernel | calls | avg us | min us | max us | total us |", "|---|---|---|---|---|---|"]
    for n, c, a, mn, mx, s in rows:
        out.append("| %s | %d | %.2f | %.2f | %.2f | %.1f |" % (n.split("(")[0][:70], c, a / 1e3, mn / 1e3, mx / 1e3,
                                                              s / 1e3))
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1]))
