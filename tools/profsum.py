"""Summarise a rocprofv3 SQLite (.db) or kernel_stats CSV: per-kernel total/avg time and share."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = 'kernel_name' if 'kernel_name' in cols else 'name'
    q = "select %s, start, end from kernels" % name_col
    agg = {}
    for name, s, e in db.execute(q):
        d = agg.setdefault(name, [0, 0.0])
        d[0] += 1
        d[1] += (e - s)
    return agg


def from_csv(path):
    agg = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get('Kernel_Name') or r.get('Name')
            s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            d = agg.setdefault(name, [0, 0.0])
            d[0] += 1
            d[1] += e - s
    return agg


def main(path, top=25, width=90):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, '**', '*.db'), recursive=True)
        csvs = glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True)
        path = (dbs or csvs)[0]
    agg = from_db(path) if path.endswith('.db') else from_csv(path)
    total = sum(v[1] for v in agg.values())
    print("%-*s %6s %10s %10s %6s" % (width, "kernel", "calls", "total_us", "avg_us", "pct"))
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print("%-*s %6d %10.1f %10.2f %5.1f%%" % (width, name[:width], n, t / 1e3, t / 1e3 / n,
                                                   100 * t / total))
    print("TOTAL GPU kernel time: %.1f us over %d dispatches" % (total / 1e3,
                                                                 sum(v[0] for v in agg.values())))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
