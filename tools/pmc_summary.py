"""Summarise tools/pmc.sh output per kernel: every collected counter averaged per dispatch, plus
derived figures (HBM-side bytes, L2 hit rate, VALU utilisation, TA busy).

    python tools/pmc_summary.py TAG [TAG ...] [--json profiles/pmc_traffic.json --workload "..." --run "..."]

HBM-side bytes: FETCH_SIZE/WRITE_SIZE as reported, and the request-size-priced figure
128*RDREQ_128B + 64*RDREQ_64B + 32*RDREQ_32B (MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE
tallies 128-B requests at 64 B).  Both count Infinity-Cache hits (L2 -> fabric requests)."""
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


def collect(tags):
    """(kernel, k-th dispatch of that kernel in the run) -> {counter: value, dur_ms}."""
    disp = collections.OrderedDict()
    for tag in tags:
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
    return disp


def derive(avg):
    out = {}
    if "FETCH_SIZE" in avg:
        out["fetch_size_bytes"] = avg["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in avg:
        out["write_size_bytes"] = avg["WRITE_SIZE"] * 1024
    if "TCC_EA0_RDREQ_128B_sum" in avg and "TCC_EA0_RDREQ_64B_sum" in avg:
        n128, n64, n32 = avg["TCC_EA0_RDREQ_128B_sum"], avg["TCC_EA0_RDREQ_64B_sum"], avg.get("TCC_EA0_RDREQ_32B_sum", 0)
        out["read_bytes_by_size"] = 128 * n128 + 64 * n64 + 32 * n32
        if "TCC_EA0_RDREQ_sum" in avg:
            out["rdreq_unclassified"] = avg["TCC_EA0_RDREQ_sum"] - n128 - n64 - n32
    if "TCC_EA0_WRREQ_sum" in avg and "TCC_EA0_WRREQ_64B_sum" in avg:
        n, n64 = avg["TCC_EA0_WRREQ_sum"], avg["TCC_EA0_WRREQ_64B_sum"]
        out["write_bytes_by_size"] = 64 * n64 + 32 * (n - n64)
    if avg.get("TCC_HIT_sum", 0) + avg.get("TCC_MISS_sum", 0):
        out["l2_hit"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if avg.get("SQ_ACTIVE_INST_VALU") and avg.get("SQ_BUSY_CYCLES"):
        out["valu_active_per_busy_cycle"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_BUSY_CYCLES"]
    if avg.get("SQ_THREAD_CYCLES_VALU") and avg.get("SQ_ACTIVE_INST_VALU"):
        out["valu_lane_util"] = avg["SQ_THREAD_CYCLES_VALU"] / (64 * avg["SQ_ACTIVE_INST_VALU"])
    if avg.get("SQ_WAIT_INST_ANY") and avg.get("SQ_WAVE_CYCLES"):
        out["wait_inst_frac"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
    if avg.get("SQ_WAVE_CYCLES") and avg.get("SQ_BUSY_CYCLES"):
        out["avg_waves"] = avg["SQ_WAVE_CYCLES"] / avg["SQ_BUSY_CYCLES"]
    if avg.get("TCP_TCC_READ_REQ_LATENCY_sum") and avg.get("TCP_TCC_READ_REQ_sum"):
        out["l1_to_l2_read_latency_cycles"] = avg["TCP_TCC_READ_REQ_LATENCY_sum"] / avg["TCP_TCC_READ_REQ_sum"]
    if avg.get("GRBM_GUI_ACTIVE"):
        out["gpu_cycles"] = avg["GRBM_GUI_ACTIVE"]
        if avg.get("TA_BUSY_avr"):
            out["ta_busy_frac"] = avg["TA_BUSY_avr"] / avg["GRBM_GUI_ACTIVE"]
    return out


def main():
    argv = sys.argv[1:]
    opts = {}
    for flag in ("--json", "--workload", "--run"):
        if flag in argv:
            i = argv.index(flag)
            opts[flag] = argv[i + 1]
            del argv[i:i + 2]
    disp = collect(argv)
    per_kernel = collections.OrderedDict()
    for (k, i), d in disp.items():
        per_kernel.setdefault(k, []).append(d)
    summary = {}
    for k, ds in per_kernel.items():
        keys = set().union(*ds)
        avg = {c: sum(d.get(c, 0.0) for d in ds) / len(ds) for c in keys}
        rec = {"dispatches": len(ds), "counters_per_dispatch": avg, "derived": derive(avg)}
        summary[k] = rec
        print("%-30s n=%3d %s" % (k, len(ds), "  ".join("%s=%.4g" % kv for kv in sorted(rec["derived"].items()))))
    if "--json" in opts:
        # profiles/pmc_traffic.json: {workload: record}; bench.py reads the record of its workload
        path = opts["--json"]
        try:
            allrec = json.load(open(path))
        except (OSError, ValueError):
            allrec = {}
        passes = summary.get("fill_live_kernel", {}).get("dispatches", 0)   # one per rendered pass
        trace = [k for k in summary if k.startswith("trace_kernel")]

        def total(keys, field):
            return sum(summary[k]["derived"].get(field, 0) * summary[k]["dispatches"] for k in keys)

        def hbm(keys):
            rd = total(keys, "read_bytes_by_size") or 2 * total(keys, "fetch_size_bytes")
            wr = total(keys, "write_bytes_by_size") or total(keys, "write_size_bytes")
            return rd, wr
        rec = {"source": "rocprofv3 --pmc, one invocation per counter group (tools/pmc.sh; tags %s)" % ",".join(argv),
               "run": opts.get("--run", ""), "passes_profiled": passes, "kernels": summary}
        n_trace = sum(summary[k]["dispatches"] for k in trace)
        if passes and n_trace:
            rd, wr = hbm(trace)
            rec["trace_launches"] = n_trace
            rec["trace_bytes_per_launch"] = int((rd + wr) / n_trace)
            rec["trace_read_bytes_per_launch"] = int(rd / n_trace)
            rec["trace_write_bytes_per_launch"] = int(wr / n_trace)
            rec["trace_fetch_size_bytes_per_launch"] = int(total(trace, "fetch_size_bytes") / n_trace)
            # exclusive launch durations of the same profiled run (the profiler serialises dispatches),
            # in dispatch order per trace kernel variant: the denominator of the fabric-bytes rate
            durs = [round(d["dur_ms"], 5) for (k, _), d in disp.items() if k in trace and "dur_ms" in d]
            # the same bytes launch by launch (bounce b = the b-th trace dispatch of the pass)
            per = []
            for (k, _), d in disp.items():
                if k not in trace:
                    continue
                dd = derive(d)
                rd1 = dd.get("read_bytes_by_size") or 2 * dd.get("fetch_size_bytes", 0)
                wr1 = dd.get("write_bytes_by_size") or dd.get("write_size_bytes", 0)
                per.append(int(rd1 + wr1))
            if per and passes == 1:
                rec["trace_bytes_by_launch"] = per
            if durs:
                rec["trace_dur_ms_per_launch"] = durs
                rec["trace_dur_ms_avg"] = sum(durs) / len(durs)
                rec["trace_fabric_gbs"] = (rd + wr) / n_trace / (rec["trace_dur_ms_avg"] / 1e3) / 1e9
            rd, wr = hbm(list(summary))
            rec["pass_bytes"] = int((rd + wr) / passes)
            rec["note"] = ("trace_bytes_per_launch: summed over every trace_kernel dispatch of the profiled passes and "
                           "divided by their number; pass_bytes: every kernel's bytes divided by the passes profiled "
                           "(fill_live_kernel dispatches).  Reads priced by request size (TCC_EA0_RDREQ_{128B,64B,32B}; "
                           "2 x FETCH_SIZE where those are missing, MI355X_MICROARCH.md §HBM), writes by "
                           "TCC_EA0_WRREQ{,_64B}; L2->fabric requests, so Infinity-Cache hits are included (an upper "
                           "bound on HBM bytes).  The profiler serialises dispatches.")
        allrec[opts.get("--workload", "")] = rec
        json.dump(allrec, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
