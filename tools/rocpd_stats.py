"""Per-kernel, per-grid duration summary from a rocprofv3 rocpd database (run_results.db):
name, grid_x, dispatches, mean/min/max us. Usage: python tools/rocpd_stats.py DB [substr]"""
import sqlite3
import sys

db = sys.argv[1]
pat = f"%{sys.argv[2]}%" if len(sys.argv) > 2 else "%"
c = sqlite3.connect(db)
q = ("select name, grid_x, count(*), avg(duration)/1000.0, min(duration)/1000.0, "
     "max(duration)/1000.0 from kernels where name like ? group by name, grid_x "
     "order by sum(duration) desc")
print("kernel,grid_x,dispatches,mean_us,min_us,max_us")
for name, g, n, mean, lo, hi in c.execute(q, (pat,)):
    short = name.replace("(anonymous namespace)", "").split("(")[0].split("::")[-1]
    print(f"{short},{g},{n},{mean:.2f},{lo:.2f},{hi:.2f}")
