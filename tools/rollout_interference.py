"""Rollout / conv co-residency from a rocprofv3 kernel trace: the search's conv
launches split by the fraction of their span that overlaps a running rollout kernel, and the
feature kernel's time per pass.

    python tools/rollout_interference.py TRACE.csv [TRACE2.csv ...] [--conv conv_wino]

Only the part of the trace from the first rollout launch on is counted (warm-up passes before
the search starts have no rollouts to overlap).
"""
import argparse
import csv
import statistics


def load(path):
    if path.endswith(".db"):  # rocpd SQLite
        import sqlite3
        return [(int(s), int(e), n) for s, e, n in
                sqlite3.connect(path).execute("select start, end, name from kernels")]
    return [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(path))]


def overlap(s, e, iv, lo):
    """Nanoseconds of [s, e) covered by the union of the sorted intervals iv (from index lo)."""
    tot, cur = 0, s
    for a, b in iv[lo:]:
        if a >= e:
            break
        if b <= cur:
            continue
        a = max(a, cur)
        tot += min(b, e) - a
        cur = min(b, e)
        if cur >= e:
            break
    return tot


def analyse(path, conv, rollout, feats):
    ks = load(path)
    ro = sorted((s, e) for s, e, n in ks if rollout in n)
    if not ro:
        return None
    t0 = ro[0][0]
    ks = [k for k in ks if k[1] > t0]
    convs = sorted((s, e) for s, e, n in ks if conv in n)
    bins = {"none (< 1 %)": [], "1-50 %": [], "> 50 %": []}
    j = 0
    for s, e in convs:
        while j < len(ro) and ro[j][1] <= s - 10**8:
            j += 1  # rollouts that ended long before this launch (none last 0.1 s)
        f = overlap(s, e, ro, j) / max(1, e - s)
        key = "none (< 1 %)" if f < 0.01 else ("1-50 %" if f <= 0.5 else "> 50 %")
        bins[key].append((e - s) / 1e3)
    allc = [(e - s) / 1e3 for s, e in convs]
    fe = [(e - s) / 1e3 for s, e, n in ks if feats in n]
    rd = sorted((e - s) / 1e3 for s, e in ro)
    return {"trace": path, "bins": bins, "conv_total_ms": sum(allc) / 1e3,
            "conv_median_us": statistics.median(allc) if allc else 0.0,
            "features": fe, "rollout_launches": len(rd),
            "rollout_median_us": rd[len(rd) // 2], "rollout_max_us": rd[-1],
            "span_ms": (max(e for _, e, _ in ks) - t0) / 1e6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--conv", default="conv_wino_kernel")
    ap.add_argument("--rollout", default="rollout_kernel")
    ap.add_argument("--features", default="features_kernel")
    a = ap.parse_args()
    for p in a.traces:
        r = analyse(p, a.conv, a.rollout, a.features)
        if r is None:
            print("# %s: no rollout kernels" % p)
            continue
        print("# %s: %.1f ms from the first rollout launch; %d rollout launches (median %.0f us, "
              "max %.0f us)" % (p, r["span_ms"], r["rollout_launches"], r["rollout_median_us"],
                               r["rollout_max_us"]))
        print("overlap with rollouts   launches   median_us   mean_us   total_ms")
        for k, v in r["bins"].items():
            if v:
                print("%-22s %9d %11.1f %9.1f %10.2f" % (k, len(v), statistics.median(v),
                                                         sum(v) / len(v), sum(v) / 1e3))
            else:
                print("%-22s %9d" % (k, 0))
        hi = r["bins"]["> 50 %"]
        if hi and r["conv_median_us"]:
            print("overlapping mean / overall median: %.2fx" % (
                (sum(hi) / len(hi)) / r["conv_median_us"]))
        if r["features"]:
            f = r["features"]
            print("%s: %d passes, median %.1f us, mean %.1f us" % (
                a.features, len(f), statistics.median(f), sum(f) / len(f)))


if __name__ == "__main__":
    main()
