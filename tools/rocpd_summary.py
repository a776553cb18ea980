"""Summarise a rocprofv3 rocpd SQLite output (kernel name, calls, total/avg us)."""
import sqlite3
import sys


def summary(db, top=40):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end-start)/1e3, avg(end-start)/1e3 from kernels "
                     "group by name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = [f"{'total_us':>12} {'calls':>6} {'avg_us':>9} {'pct':>6}  kernel"]
    for name, n, t, a in rows[:top]:
        out.append(f"{t:12.1f} {n:6d} {a:9.2f} {100 * t / tot:6.2f}  {name[:150]}")
    out.append(f"{tot:12.1f} total kernel time (us)")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40))
