"""Per-kernel time of the last pass in a serialized (RT_INFLIGHT=1) rocprofv3 kernel trace.
usage: python tools/pass_breakdown.py gpurun_out/<dir>/run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = []
for r in rows:
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", r["Kernel_Name"])
    k = (m.group(1) + (m.group(2) or "").replace(" ", "")) if m else r["Kernel_Name"][:30]
    seq.append((int(r["Start_Timestamp"]), k, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
seq.sort()
passes, cur = [], None
for t, k, d in seq:
    if k.startswith("fill_live"):
        cur = []
        passes.append(cur)
    if cur is not None:
        cur.append((k, d))
p = passes[-1]
tot = collections.defaultdict(float)
for k, d in p:
    tot[k] += d
print("last pass: %.3f ms of kernels" % sum(d for k, d in p))
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print("  %-36s %.3f" % (k, v))
for name in ("trace", "shade", "sort_scatter", "compact"):
    xs = [d for k, d in p if k.startswith(name)]
    if xs:
        print("%-12s per bounce: %s" % (name, " ".join("%.2f" % x for x in xs)))
