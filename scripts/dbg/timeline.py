"""Summarise a rocprofv3 kernel trace: busy/idle time of the GPU, per-class kernel time and the
overlap of long-running (rollout) kernels with the rest, over the last `--window` seconds."""
import argparse
import csv


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=0.25)
    ap.add_argument("--long", default="rollout")
    a = ap.parse_args()
    if a.trace.endswith(".db"):  # rocpd SQLite (rocprofv3's default output)
        import sqlite3
        ks = [(int(s), int(e), n) for s, e, n in
              sqlite3.connect(a.trace).execute("select start, end, name from kernels")]
    else:
        rows = list(csv.DictReader(open(a.trace)))
        ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in rows]
    end = max(e for _, e, _ in ks)
    t0 = end - int(a.window * 1e9)
    ks = [(max(s, t0), e, n) for s, e, n in ks if e > t0]
    span = end - t0
    longk = [(s, e) for s, e, n in ks if a.long in n]
    rest = [(s, e) for s, e, n in ks if a.long not in n]
    print("window %.1f ms: kernels %d (%s %d)" % (span / 1e6, len(ks), a.long, len(longk)))
    print("busy any %.1f%%  busy %s %.1f%%  busy other %.1f%%" % (
        100 * union([(s, e) for s, e, _ in ks]) / span, a.long, 100 * union(longk) / span,
        100 * union(rest) / span))
    if longk:
        d = sorted(e - s for s, e in longk)
        print("%s durations ms: min %.2f med %.2f max %.2f; mean concurrency %.2f" % (
            a.long, d[0] / 1e6, d[len(d) // 2] / 1e6, d[-1] / 1e6, sum(d) / span))
    by = {}
    for s, e, n in ks:
        k = n.replace("void ", "").replace("(anonymous namespace)::", "")
        k = k[:k.index("(")] if "(" in k else k
        k = k[:60]
        c, t = by.get(k, (0, 0))
        by[k] = (c + 1, t + e - s)
    for k, (c, t) in sorted(by.items(), key=lambda x: -x[1][1])[:12]:
        print("%8.2f ms %5d  %7.1f us  %s" % (t / 1e6, c, t / c / 1e3, k))


if __name__ == "__main__":
    main()
