"""Wave time breakdown of the trace/shade kernels from tools/pmc.sh TAG tools/pmc_groups/stall.txt.
usage: python tools/stall_summary.py TAG   (fractions of SQ_WAVE_CYCLES; counts summed over launches)"""
import collections
import sys

from pmc_summary import collect

disp = collect(sys.argv[1:])
per = collections.OrderedDict()
for (k, i), d in disp.items():
    if k.startswith("trace_kernel") or k.startswith("shade_kernel"):
        per.setdefault(k, []).append(d)
print("# Wave time breakdown (tools/pmc.sh %s tools/pmc_groups/stall.txt; one teapot pass at 1080p, kernels\n"
      "# serialised by the profiler).  Fractions are of SQ_WAVE_CYCLES (the waves' resident time); instruction\n"
      "# counts are totals over the pass's launches of that kernel." % " ".join(sys.argv[1:]))
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
