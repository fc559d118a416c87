"""Per-kernel dispatch count / mean / total ms from a rocprofv3 results database."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kt = [t for t in tabs if "kernel_dispatch" in t.lower()][0]
ks = [t for t in tabs if "kernel_symbol" in t.lower()][0]
q = (f"select s.kernel_name, count(*), avg(d.end-d.start)/1e6, sum(d.end-d.start)/1e6 from {kt} d "
     f"join {ks} s on d.kernel_id=s.id group by s.kernel_name order by 4 desc limit {int(sys.argv[2]) if len(sys.argv) > 2 else 14}")
print(f"{'kernel':60s} {'calls':>5s} {'avg ms':>8s} {'total ms':>9s}")
for r in c.execute(q):
    print(f"{r[0][:60]:60s} {r[1]:5d} {r[2]:8.3f} {r[3]:9.2f}")
