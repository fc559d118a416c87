"""Kernel summary (name, calls, total / average / min / max ns, share) of a
rocprofv3 rocpd database (results.db, the default output format), written as the
CSV `rocprofv3 --stats --output-format csv` gives: python scripts/prof_db.py DB [OUT.csv]"""
import csv
import sqlite3
import sys


def summary(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                          "max(end - start) from kernels group by name order by sum(end - start) desc"))
    tot = sum(r[2] for r in rows) or 1
    return [(r[0], r[1], r[2], r[3], 100.0 * r[2] / tot, r[4], r[5]) for r in rows]


def main():
    rows = summary(sys.argv[1])
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in rows:
        w.writerow(r)


if __name__ == "__main__":
    main()
