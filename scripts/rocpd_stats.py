"""Per-(kernel, grid) dispatch statistics from a rocprofv3 results database (rocpd SQLite, the default output of
`rocprofv3 --kernel-trace -d DIR -o NAME`): count, average / min / max duration in microseconds, CSV on stdout.
usage: python scripts/rocpd_stats.py DIR_OR_DB [NAME_FILTER]"""
import glob
import os
import sqlite3
import sys


def main():
    path = sys.argv[1]
    dbs = [path] if path.endswith(".db") else sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    print("kernel,workgroups,dispatches,avg_us,min_us,max_us")
    for db in dbs:
        cur = sqlite3.connect(db).cursor()
        q = ("select name, grid_x / workgroup_x, count(*), avg(duration) / 1e3, min(duration) / 1e3, "
             "max(duration) / 1e3 from kernels where name like ? group by name, grid_x order by name, grid_x")
        for name, g, c, a, lo, hi in cur.execute(q, (f"%{filt}%",)):
            print(f"\"{name}\",{g},{c},{a:.2f},{lo:.2f},{hi:.2f}")


if __name__ == "__main__":
    main()
