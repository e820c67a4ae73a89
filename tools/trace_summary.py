"""Summarise a rocprofv3 kernel trace / PMC collection of bench.py (per-bounce kernel times)."""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", name)
    if not m:
        return name.split("(")[0][:40]
    return m.group(1) + (m.group(2) or "").replace(" ", "")


def trace(path, bounces=16):
    rows = list(csv.DictReader(open(path)))
    seq = [(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in rows]
    by = collections.OrderedDict()
    for n, d in seq:
        by.setdefault(n, []).append(d)
    for n, ds in by.items():
        print("%-40s calls %4d  total %9.3f ms  mean %8.4f ms" % (n, len(ds), sum(ds), sum(ds) / len(ds)))
    for n, ds in by.items():
        if ("trace_kernel" in n or "shade_kernel" in n or "process_kernel" in n) and len(ds) >= bounces:
            for i in range(0, len(ds) - bounces + 1, bounces):
                print(n, " ".join("%.2f" % x for x in ds[i:i + bounces]), " sum %.2f" % sum(ds[i:i + bounces]))


def pmc(path, match="trace_kernel"):
    rows = list(csv.DictReader(open(path)))
    agg = collections.OrderedDict()
    for r in rows:
        if match not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    for k, v in agg.items():
        out = [k]
        wc = v.get("SQ_WAVE_CYCLES")
        for c in sorted(v):
            out.append("%s=%.3g" % (c, v[c]))
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in v:
                    out.append("%s/wc=%.2f" % (c[3:], v[c] / wc))
        if v.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in v:
            out.append("lane_util=%.2f" % (v["SQ_THREAD_CYCLES_VALU"] / (v["SQ_ACTIVE_INST_VALU"] * 64)))
        print(" ".join(out))


if __name__ == "__main__":
    kind, path = sys.argv[1], sys.argv[2]
    if kind == "trace":
        trace(path, int(sys.argv[3]) if len(sys.argv) > 3 else 16)
    else:
        pmc(path, sys.argv[3] if len(sys.argv) > 3 else "trace_kernel")
