"""Per-kernel summary (calls, total ms, average ms) from a rocprofv3 rocpd database
(run_results.db), for runs made without --output-format csv.

    python tools/db_kernels.py gpurun_out/prof/run_results.db [name-filter ...]"""
import sqlite3
import sys


def main(path, filters):
    db = sqlite3.connect(path)
    rows = db.execute("select name, count(*), sum(end - start) / 1e6, avg(end - start) / 1e6 from kernels "
                      "group by name order by sum(end - start) desc").fetchall()
    for name, n, tot, avg in rows:
        if filters and not any(f in name for f in filters):
            continue
        print(f"{n:5d} {tot:10.3f} ms {avg:8.4f} ms  {name[:110]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
