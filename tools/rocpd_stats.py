"""Per-kernel totals from a rocprofv3 run:
  python tools/rocpd_stats.py DB [TOP]            rocpd database (the default output format)
  python tools/rocpd_stats.py --csv STATS [TOP]   a --stats kernel_stats.csv"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    q = f"select {name}, count(*), sum(end - start) from kernels group by {name}"
    return [(n, k, t) for n, k, t in c.execute(q)]


def stats_csv(path):
    with open(path) as f:
        return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(f)]


if __name__ == "__main__":
    args = sys.argv[1:]
    rows = stats_csv(args[1]) if args[0] == "--csv" else stats(args[0])
    rest = args[2:] if args[0] == "--csv" else args[1:]
    top = int(rest[0]) if rest else 12
    tot = sum(t for _, _, t in rows)
    print(f"total {tot / 1e6:.2f} ms")
    for n, k, t in sorted(rows, key=lambda r: -r[2])[:top]:
        short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
        print(f"{t / tot * 100:5.1f}% {t / 1e6:8.2f} ms {k:5d} x {t / k / 1e3:8.1f} us  {short}")
