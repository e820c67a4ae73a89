"""Instruction-fetch counters per kernel from rocprofv3 --pmc CSVs (gpurun_out/pmc_<tag>_*/run_counter_collection.csv):
I-cache hit rate and the share of wave time spent waiting for an instruction to issue.
    python tools/icache_summary.py TAG [TAG ...]"""
import csv
import glob
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for tag in sys.argv[1:]:
    tot = {}
    for path in sorted(glob.glob(os.path.join(REPO, "gpurun_out", "pmc_%s_*" % tag, "run_counter_collection.csv"))):
        for r in csv.DictReader(open(path)):
            k = re.sub(r"\(.*", "", re.sub(r"^void (\(anonymous namespace\)::)?", "", r["Kernel_Name"]))
            k = re.sub(r"\s+", "", k)[:60]
            d = tot.setdefault(k, {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print("== %s" % tag)
    for k, d in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        h, m = d.get("SQC_ICACHE_HITS", 0), d.get("SQC_ICACHE_MISSES", 0)
        wc = d.get("SQ_WAVE_CYCLES", 0)
        print("%-60s icache_hit %.4f misses %.3g ifetch %.3g wait_inst %.3f wave_cycles %.3g" % (
            k, h / (h + m) if h + m else float("nan"), m, d.get("SQ_IFETCH", 0),
            d.get("SQ_WAIT_INST_ANY", 0) / wc if wc else float("nan"), wc))
