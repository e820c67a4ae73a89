"""Occupancy timeline of a timed pass batch from a rocprofv3 --kernel-trace CSV (e.g. of
`bench.py --steps 20 --warmup 5 --no-extras`): the last BATCH passes (one fill_live_kernel each) are the
timed batch; per BIN-ms bin it prints the passes in flight, the trace kernels running (time-weighted),
their workgroups as a share of the chip's resident trace workgroups, and the share of the bin in which
any kernel of the batch runs.  The first and last bins show the ramp-up and ramp-down of the batch.

    python tools/timeline_occupancy.py run_kernel_trace.csv [BATCH=20] [BIN=2] [RESIDENT=2048]"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    binms = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
    resident = int(sys.argv[4]) if len(sys.argv) > 4 else 2048   # 256 CUs x 8 trace workgroups
    ks = []
    for r in csv.DictReader(open(path)):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:24]
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, wg, r.get("Queue_Id", "")))
    ks.sort()
    fills = [k for k in ks if k[2] == "fill_live_kernel"]
    if len(fills) < batch:
        sys.exit("fewer than %d passes in the trace" % batch)
    t0 = fills[-batch][0]
    accs = [k for k in ks if k[2] == "accumulate_kernel" and k[0] >= t0]
    t1 = max(k[1] for k in ks if k[0] >= t0 and k[2] not in ("__amd_rocclr_copyBuffer",))
    span = (t1 - t0) / 1e6
    nb = int(span / binms) + 1
    trace_n = [0.0] * nb
    trace_wg = [0.0] * nb
    busy = [[] for _ in range(nb)]
    passes = [0] * nb
    for s, e, name, wg, _ in ks:
        if e <= t0:
            continue
        a, b = (max(s, t0) - t0) / 1e6, (e - t0) / 1e6
        i = int(a / binms)
        while i < nb and i * binms < b:
            lo, hi = max(a, i * binms), min(b, (i + 1) * binms)
            if hi > lo:
                busy[i].append((lo, hi))
                if name == "trace_kernel":
                    trace_n[i] += (hi - lo) / binms
                    trace_wg[i] += (hi - lo) / binms * min(wg, resident) / resident
            i += 1
    # passes in flight: from its fill_live start to its accumulate end (matched in order)
    pstart = [(k[0] - t0) / 1e6 for k in fills[-batch:]]
    pend = sorted((k[1] - t0) / 1e6 for k in accs)[:batch]
    for i in range(nb):
        mid = (i + 0.5) * binms
        passes[i] = sum(1 for p in pstart if p <= mid) - sum(1 for p in pend if p <= mid)
    print("batch of %d passes: %.2f ms (first pass start to last kernel end); bins of %.1f ms" % (batch, span, binms))
    print("%8s %7s %8s %10s %6s" % ("t ms", "passes", "traces", "trace WG%", "busy%"))
    tot_busy = 0.0
    for i in range(nb):
        iv = sorted(busy[i])
        cov, cur_lo, cur_hi = 0.0, None, None
        for lo, hi in iv:
            if cur_hi is None or lo > cur_hi:
                if cur_hi is not None:
                    cov += cur_hi - cur_lo
                cur_lo, cur_hi = lo, hi
            else:
                cur_hi = max(cur_hi, hi)
        if cur_hi is not None:
            cov += cur_hi - cur_lo
        width = min(binms, span - i * binms)
        tot_busy += cov
        print("%8.1f %7d %8.2f %9.0f%% %5.0f%%" % (i * binms, passes[i], trace_n[i], 100 * trace_wg[i],
                                                  100 * cov / width if width > 0 else 0))
    print("ends of passes (ms):", " ".join("%.1f" % p for p in pend))


if __name__ == "__main__":
    main()
