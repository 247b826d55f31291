"""Print the top kernels of a rocprofv3 results database (argument: directory or .db)."""
import glob
import sqlite3
import sys

p = sys.argv[1]
db = p if p.endswith(".db") else glob.glob(p + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
for name, calls, tot, avg, pct in c.execute("select * from top_kernels limit %d" % int(sys.argv[2] if len(sys.argv) > 2 else 10)):
    print(f"{avg:12.1f} us avg {calls:5d} calls {pct:6.2f}%  {name[:110]}")
