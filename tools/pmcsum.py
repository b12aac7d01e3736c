"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel.

  python tools/pmcsum.py <counter_collection.csv> [name-filter ...]

Per kernel name (truncated): dispatch count, mean duration (us) and mean value of every counter.
Derived, where the counters are present (MI355X_MICROARCH.md 'DVFS give-back', cycle constants):
  clk_GHz      = GRBM_GUI_ACTIVE / 8 XCDs / duration   (reads high for dispatches < ~0.3 ms)
  mfma_util    = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 4 SIMD * 256 CU / 8 XCD ...)
                 reported as busy cycles per SIMD over the kernel's cycles.
"""
import csv
import sys
from collections import OrderedDict, defaultdict


def load(path):
    per = OrderedDict()
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            key = (name, r["Dispatch_Id"])
            d = per.setdefault(key, {"dur": (int(r["End_Timestamp"]) -
                                              int(r["Start_Timestamp"])) / 1e3,
                                     "vgpr": r.get("VGPR_Count"), "agpr": r.get("Accum_VGPR_Count"),
                                     "lds": r.get("LDS_Block_Size")})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = OrderedDict()
    for (name, _), d in per.items():
        a = agg.setdefault(name, defaultdict(float))
        a["_n"] += 1
        for k, v in d.items():
            if isinstance(v, float) or k == "dur":
                a[k] += v
        a["_vgpr"], a["_agpr"], a["_lds"] = d["vgpr"], d["agpr"], d["lds"]
    return agg


def short(name, n=70):
    name = name.replace("(anonymous namespace)::", "")
    return name[:n]


def main(path, filters):
    agg = load(path)
    for name, a in agg.items():
        if filters and not any(f in name for f in filters):
            continue
        n = a["_n"]
        m = {k: v / n for k, v in a.items() if not k.startswith("_")}
        out = ["%-70s n=%-4d dur_us=%.1f vgpr=%s agpr=%s lds=%s" % (
            short(name), n, m["dur"], a["_vgpr"], a["_agpr"], a["_lds"])]
        if "SQ_BUSY_CYCLES" in m and m["dur"] > 0:
            # SQ_BUSY_CYCLES is summed over the 32 shader engines' SQs (shader clock): kernel
            # cycles = SQ_BUSY / 32 (the long elementwise kernels read 2.29-2.39 GHz this way, the
            # GRBM-based quotient reads high below ~0.3 ms); MFMA busy cycles are summed over the
            # 1024 SIMDs at 16 per v_mfma_f32_16x16x32_bf16 (checked against the conv's MFMA count)
            cyc = m["SQ_BUSY_CYCLES"] / 32
            out.append("clk_GHz=%.2f" % (cyc / (m["dur"] * 1e-6) / 1e9))
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                out.append("mfma_busy=%.1f%%" % (100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc))
        elif "GRBM_GUI_ACTIVE" in m and m["dur"] > 0:
            clk = m["GRBM_GUI_ACTIVE"] / 8 / (m["dur"] * 1e-6) / 1e9
            out.append("clk_GHz(grbm)=%.2f" % clk)
        out.append(" ".join("%s=%.0f" % (k, v) for k, v in sorted(m.items()) if k != "dur"))
        print("  ".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
