"""Split a rocprofv3 kernel-trace (.db) of the SL step into 3x3 forward / dgrad / 5x5 conv and
wgrad launch averages (forward = conv launches before the step's first wgrad launch; direct
conv_tap_pp and Winograd conv_wino launches alike).

    python tools/convsplit.py gpurun_out/<job>/trace-sl/sl_results.db [...]
"""
import re
import sqlite3
import statistics as st
import sys


def split(path):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    nc = 'kernel_name' if 'kernel_name' in cols else 'name'
    fw, dg, f5, wg = [], [], [], []
    state = 'f'
    for n, s, e in db.execute("select %s, start, end from kernels order by start" % nc):
        d = (e - s) / 1e3
        if 'wgrad_slab_kernel' in n:
            state = 'b'
            wg.append(d)
            continue
        if 'conv_wino_kernel' in n:
            (fw if state == 'f' else dg).append(d)
            continue
        m = re.search(r'conv_tap_pp_kernel<([^>]*)>', n)
        if not m:
            continue
        a = [x.strip() for x in m.group(1).split(',')]
        if a[3] == '5':  # <NB, NT, BNP, KS, ...> (round 5 template)
            f5.append(d)
            state = 'f'
            continue
        (fw if state == 'f' else dg).append(d)
    mean = lambda v: st.mean(v) if v else float('nan')
    med = lambda v: st.median(v) if v else float('nan')
    return ("fwd3x3 %.2f us (median %.2f, n=%d)  dgrad %.2f us (median %.2f, n=%d)  5x5 %.2f us"
            "  wgrad %.2f us (n=%d)" % (mean(fw), med(fw), len(fw), mean(dg), med(dg), len(dg),
                                       mean(f5), mean(wg), len(wg)))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p, split(p))
