"""Summarise a rocprofv3 kernel-trace database (.db) or kernel_stats CSV into a per-kernel table."""
import sqlite3
import sys


def main(path, top=40):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                      f"from kernels group by {name_col} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print("%-70s %7s %12s %12s %12s %6s" % ("kernel", "calls", "total_ms", "avg_us", "max_us", "pct"))
    for r in rows[:top]:
        n = r[0]
        n = n if len(n) < 70 else n[:67] + "..."
        print("%-70s %7d %12.3f %12.2f %12.2f %6.2f" % (n, r[1], r[2] / 1e6, r[3] / 1e3, r[5] / 1e3, 100 * r[2] / tot))


if __name__ == "__main__":
    main(sys.argv[1])
