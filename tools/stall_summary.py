"""Wave time breakdown of the trace/shade kernels from tools/pmc.sh TAG tools/pmc_groups/stall.txt.
usage: python tools/stall_summary.py TAG [--json profiles/pmc_issue.json --workload "..." --run "..."]
(fractions of SQ_WAVE_CYCLES; counts summed over launches).  --json records the pass's instruction
counts (every kernel; per pass = totals / fill_live_kernel dispatches), which bench.py prices against
the chip's VALU issue rate (roofline.valu)."""
import collections
import json
import os
import sys

from pmc_summary import REPO, collect

argv = sys.argv[1:]
opts = {}
for flag in ("--json", "--workload", "--run"):
    if flag in argv:
        i = argv.index(flag)
        opts[flag] = argv[i + 1]
        del argv[i:i + 2]
disp = collect(argv)
per = collections.OrderedDict()
for (k, i), d in disp.items():
    if k.startswith(("trace_kernel", "trace2_kernel", "shade_kernel")):
        per.setdefault(k, []).append(d)
print("# Wave time breakdown (tools/pmc.sh %s tools/pmc_groups/stall.txt; one teapot pass at 1080p, kernels\n"
      "# serialised by the profiler).  Fractions are of SQ_WAVE_CYCLES (the waves' resident time); instruction\n"
      "# counts are totals over the pass's launches of that kernel." % " ".join(argv))
for k, ds in per.items():
    s = collections.Counter()
    for d in ds:
        s.update(d)
    wc = s["SQ_WAVE_CYCLES"] or 1
    f = lambda c: s.get(c, 0) / wc
    print("%s  launches %d  kernel time %.2f ms  waves %d" % (k, len(ds), s["dur_ms"], s["SQ_WAVES"]))
    print("   waiting (SQ_WAIT_ANY) %.3f   ready, not issued (SQ_WAIT_INST_ANY) %.3f   issuing (SQ_ACTIVE_INST_ANY) %.3f"
          % (f("SQ_WAIT_ANY"), f("SQ_WAIT_INST_ANY"), f("SQ_ACTIVE_INST_ANY")))
    print("   issuing by unit: VALU %.3f  SALU %.3f  misc/branch %.3f  LDS %.3f"
          % (f("SQ_ACTIVE_INST_VALU"), f("SQ_ACTIVE_INST_SCA"), f("SQ_ACTIVE_INST_MISC"), f("SQ_ACTIVE_INST_LDS")))
    print("   instructions: VALU %.3g  SALU %.3g  branch %.3g  VMEM read %.3g  LDS %.3g   TA addr/cmd FIFO full %d/%d  "
          "LDS bank conflicts %d" % (s["SQ_INSTS_VALU"], s["SQ_INSTS_SALU"], s["SQ_INSTS_BRANCH"], s["SQ_INSTS_VMEM_RD"],
                                     s["SQ_INSTS_LDS"], s["SQ_VMEM_TA_ADDR_FIFO_FULL"], s["SQ_VMEM_TA_CMD_FIFO_FULL"],
                                     s["SQ_LDS_BANK_CONFLICT"]))

if "--json" in opts:
    passes = sum(1 for (k, i) in disp if k.startswith("fill_live_kernel")) or 1
    tot, trace = collections.Counter(), collections.Counter()
    for (k, i), d in disp.items():
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS",
                  "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
            tot[c] += d.get(c, 0)
            if k.startswith(("trace_kernel", "trace2_kernel")):
                trace[c] += d.get(c, 0)
    path = opts["--json"] if os.path.isabs(opts["--json"]) else os.path.join(REPO, opts["--json"])
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    doc[opts.get("--workload", "unnamed")] = {
        "passes_profiled": passes,
        "per_pass": {c: v / passes for c, v in tot.items()},
        "trace_per_pass": {c: v / passes for c, v in trace.items()},
        "run": opts.get("--run", ""),
        "source": "tools/pmc.sh %s tools/pmc_groups/stall.txt + tools/stall_summary.py" % " ".join(argv),
        "note": "wave-instructions summed over every dispatch of the profiled pass(es), chip-wide; "
                "SQ_WAVE_CYCLES (quad-cycles of resident waves) summed the same way, so trace / all is the trace "
                "kernel's share of the pass's wave residency (bench.py roofline.timed)",
    }
    with open(path, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
