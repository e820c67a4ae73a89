"""End-of-batch ramp of a rank's pass share: from a rocprofv3 --kernel-trace CSV of a short run
(e.g. `bench.py --steps 13 --dist --no-extras`, a 13-pass share of the teapot frame), the pass that
ends last is split bounce by bounce into kernel time and inter-launch gaps on its stream, and the
part of it that ran ALONE (after every other pass had finished) is reported -- that is the ramp a
short pass list cannot overlap.

    python tools/ramp_breakdown.py gpurun_out/<dir>/run_kernel_trace.csv [oracle_profile.json]

The optional oracle profile (tools/oracle_bounce_profile.py) adds the longest ray's trace steps per
bounce: the latency floor of a tail bounce is that ray's chain of dependent steps."""
import collections
import csv
import json
import re
import sys


def kname(n):
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", n)
    return (m.group(1) + (m.group(2) or "").replace(" ", "")) if m else n[:30]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    prof = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else None
    by_stream = collections.defaultdict(list)
    for r in rows:
        by_stream[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"])))
    passes = []                         # (stream, [(start, end, kernel)])
    for sid, ks in by_stream.items():
        ks.sort()
        cur = None
        for k in ks:
            if k[2].startswith("fill_live"):
                cur = []
                passes.append((sid, cur))
            if cur is not None:
                cur.append(k)
    passes = [p for p in passes if any(k[2].startswith("trace_kernel") or k[2].startswith("shade_kernel") for k in p[1])]
    if not passes:
        sys.exit("no passes found")
    ends = sorted((max(k[1] for k in p[1]), i) for i, p in enumerate(passes))
    last_end, last_i = ends[-1]
    alone_from = ends[-2][0] if len(ends) > 1 else min(k[0] for k in passes[last_i][1])
    t0 = min(k[0] for p in passes for k in p[1])
    ks = passes[last_i][1]
    # bounces: a trace (or inline shade) launch opens each bounce
    opener = "trace_kernel" if any(k[2].startswith("trace_kernel") for k in ks) else "shade_kernel"
    bounces = []
    for k in ks:
        if k[2].startswith(opener):
            bounces.append([])
        if bounces:
            bounces[-1].append(k)
    out = {"passes": len(passes), "frame_ms": (last_end - t0) / 1e6, "last_pass_stream": passes[last_i][0],
           "alone_ms": (last_end - alone_from) / 1e6, "bounces": []}
    prev_end = None
    for b, bk in enumerate(bounces):
        start, end = bk[0][0], bk[-1][1]
        busy = sum(k[1] - k[0] for k in bk)
        trace = sum(k[1] - k[0] for k in bk if k[2].startswith("trace_kernel"))
        gap_before = (start - prev_end) if prev_end is not None else 0
        rec = {"bounce": b, "start_ms": round((start - t0) / 1e6, 3), "trace_ms": round(trace / 1e6, 4),
               "other_kernels_ms": round((busy - trace) / 1e6, 4), "gaps_ms": round((end - start - busy + gap_before) / 1e6, 4),
               "alone": start >= alone_from}
        if prof:
            pp = next(iter(prof["passes"].values()))
            if b < len(pp["max_steps"]):
                rec["oracle_longest_ray_steps"] = pp["max_steps"][b]
                rec["oracle_live"] = pp["live"][b]
        out["bounces"].append(rec)
        prev_end = end
    alone = [x for x in out["bounces"] if x["alone"]]
    out["alone_split"] = {"bounces": len(alone), "trace_ms": round(sum(x["trace_ms"] for x in alone), 3),
                          "other_kernels_ms": round(sum(x["other_kernels_ms"] for x in alone), 3),
                          "gaps_ms": round(sum(x["gaps_ms"] for x in alone), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
