"""Per-kernel summary of a rocprofv3 (ROCm 7) rocpd SQLite database: the `--stats` table
that rocprofv3 writes as CSV for other output formats.  usage: rocpd_summary.py results.db"""
import sqlite3
import sys


def main(path: str) -> None:
    c = sqlite3.connect(path)
    print(f"# rocprofv3 --kernel-trace --stats: {path}")
    print(f"{'calls':>7} {'total_us':>12} {'avg_us':>10} {'pct':>7}  kernel")
    for name, calls, total, avg, pct in c.execute("select name, total_calls, total_duration, average, percentage "
                                                  "from top_kernels order by total_duration desc"):
        print(f"{calls:7d} {total:12.1f} {avg:10.3f} {pct:6.2f}%  {name[:140]}")


if __name__ == "__main__":
    main(sys.argv[1])
