"""Per-step kernel time of a training step from a rocprofv3 kernel trace (CSV, or the rocpd
SQLite database rocprofv3 writes by default): steps are delimited by the input-packing kernel;
prints the median step's kernels (time, count) and the step's busy fraction."""
import csv
import sys


def load(path):
    """(start ns, end ns, kernel name) from a rocprofv3 kernel-trace CSV or rocpd database."""
    if path.endswith(".db"):
        import sqlite3
        c = sqlite3.connect(path)
        return sorted((int(s), int(e), n) for s, e, n in
                      c.execute("select start, end, name from kernels"))
    rows = list(csv.DictReader(open(path)))
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in rows)


def main(path, marker="pack_input"):
    ks = load(path)
    starts = [s for s, e, n in ks if marker in n]
    steps = list(zip(starts, starts[1:]))[-8:]
    a, b = sorted(steps, key=lambda ab: ab[1] - ab[0])[len(steps) // 2]
    by = {}
    busy = 0
    for s, e, n in ks:
        if s >= a and s < b:
            k = n.replace("void ", "").replace("(anonymous namespace)::", "")
            k = k[:k.index("(")] if "(" in k else k
            c, t = by.get(k, (0, 0))
            by[k] = (c + 1, t + e - s)
            busy += min(e, b) - s
    print("step %.1f us, kernels %.1f us (%.1f %% busy)" % ((b - a) / 1e3, busy / 1e3,
                                                            100.0 * busy / (b - a)))
    for k, (c, t) in sorted(by.items(), key=lambda x: -x[1][1]):
        print("%9.1f us %4d  %s" % (t / 1e3, c, k[:90]))


if __name__ == "__main__":
    main(*sys.argv[1:])
