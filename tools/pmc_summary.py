"""Summarise tools/pmc.sh output per kernel and per bounce: HBM traffic (FETCH_SIZE doubled per
MI355X_MICROARCH.md §HBM for wide streaming reads is NOT applied to gather traffic; both the raw
and the corrected figure are printed), L2 hit rate, effective clock, wave stats.

    python tools/pmc_summary.py TAG [bounces] [--json out.json --workload "..."]"""
import collections
import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(n):
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", n)
    return (m.group(1) + (m.group(2) or "").replace(" ", "")) if m else n[:30]


def main():
    tag = sys.argv[1]
    bounces = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 16
    disp = collections.OrderedDict()     # (kernel, k-th dispatch) -> counters
    for path in sorted(glob.glob(os.path.join(REPO, "gpurun_out", "pmc_%s_*" % tag, "run_counter_collection.csv"))):
        seen = collections.Counter()
        last = None
        for r in csv.DictReader(open(path)):
            k = kname(r["Kernel_Name"])
            did = r["Dispatch_Id"]
            if (k, did) != last:
                seen[k] += 1
                last = (k, did)
            d = disp.setdefault((k, seen[k]), {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    per_kernel = collections.OrderedDict()
    for (k, i), d in disp.items():
        per_kernel.setdefault(k, []).append(d)
    summary = {}
    for k, ds in per_kernel.items():
        tot = collections.Counter()
        for d in ds:
            tot.update(d)
        n = len(ds)
        fetch = tot.get("FETCH_SIZE", 0) * 1024
        write = tot.get("WRITE_SIZE", 0) * 1024
        hit, miss = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
        rd, dram = tot.get("TCC_EA0_RDREQ_sum", 0), tot.get("TCC_EA0_RDREQ_DRAM_sum", 0)
        clk = tot.get("GRBM_GUI_ACTIVE", 0) / 8 / (tot["dur_ms"] / 1e3) / 1e9 if tot.get("GRBM_GUI_ACTIVE") else 0
        summary[k] = dict(dispatches=n, fetch_bytes_per_dispatch=fetch / n, write_bytes_per_dispatch=write / n,
                          l2_hit=hit / (hit + miss) if hit + miss else None,
                          dram_rdreq_frac=dram / rd if rd else None, clock_ghz=clk)
        print("%-28s n=%3d  FETCH %.3g B/disp  WRITE %.3g B/disp  L2 hit %s  EA rd->DRAM %s  clk %.2f GHz" % (
            k, n, fetch / n, write / n, "%.3f" % (hit / (hit + miss)) if hit + miss else "-",
            "%.3f" % (dram / rd) if rd else "-", clk))
        if "trace_kernel" in k and n >= bounces:
            for b in range(bounces):
                d = ds[b]
                print("   bounce %2d  %.3f ms  fetch %.3g  write %.3g  L2hit %s" % (
                    b, d["dur_ms"], d.get("FETCH_SIZE", 0) * 1024, d.get("WRITE_SIZE", 0) * 1024,
                    "%.3f" % (d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])) if d.get("TCC_HIT_sum") else "-"))
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        wl = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else ""
        tr, sh = summary.get("trace_kernel<true,false>"), summary.get("shade_kernel<true,false>")
        rec = {"workload": wl, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/pmc.sh %s)" % tag,
               "kernels": summary}
        if tr and sh:
            rec["hbm_bytes_per_launch"] = int(tr["fetch_bytes_per_dispatch"] + tr["write_bytes_per_dispatch"] +
                                              sh["fetch_bytes_per_dispatch"] + sh["write_bytes_per_dispatch"])
            rec["note"] = ("per process launch = one trace_kernel + one shade_kernel dispatch, averaged over the "
                           "16 bounces of one pass; FETCH_SIZE/WRITE_SIZE as reported (KiB x 1024), no 2x gfx950 "
                           "streaming correction applied (gather traffic, not wide streaming)")
        json.dump(rec, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
