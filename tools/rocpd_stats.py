"""Summarise a rocprofv3 rocpd database (--kernel-trace) per kernel: calls, total/avg/min/max duration, and per
grid shape when --by-grid is given.  Usage: python tools/rocpd_stats.py <db> [--by-grid] [--top N]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    by_grid = "--by-grid" in sys.argv
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    c = sqlite3.connect(db)
    key = "k.name, k.grid_x, k.grid_y" if by_grid else "k.name"
    q = (f"select {key}, count(*), sum(k.duration), avg(k.duration), min(k.duration), max(k.duration) "
         f"from kernels k group by {key} order by sum(k.duration) desc limit {top}")
    rows = c.execute(q).fetchall()
    tot = c.execute("select sum(duration) from kernels").fetchone()[0]
    print(f"total kernel time {tot / 1e6:.3f} ms")
    for r in rows:
        name = r[0][:70]
        extra = f" grid=({r[1]},{r[2]})" if by_grid else ""
        n, s, a, mn, mx = r[-5:]
        print(f"{s / 1e6:9.3f} ms {100 * s / tot:5.1f}% n={n:7d} avg={a / 1e3:8.2f}us min={mn / 1e3:8.2f} "
              f"max={mx / 1e3:8.2f}  {name}{extra}")


if __name__ == "__main__":
    main()
