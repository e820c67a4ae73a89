"""BASELINE.md's results table from committed files only (DESIGN.md §6 "Results table"): one row per
BASELINE config x GPUs.  1-GPU cells come from profiles/<round>/bench_*.json and profiles/pmc_traffic.json;
N > 1 has no hardware measurement (the driver's SCALE run is the only one), so those rows say so.

    python tools/results_table.py [profiles/r06/final]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "r05", "final"))
ROWS = [("1 cornell 256² × 64 × 4", "bench_cornell.json"),
        ("2 cornell_plus 512² × 256 × 8", "bench_cornell_plus.json"),
        ("3 spheres 1024² × 1024 × 8", "bench_spheres.json"),
        ("4 teapot 1080p × 2048 × 16", "bench_teapot.json"),
        ("4 teapot, no_sort", "bench_teapotnosort.json"),
        ("5 lamp 1080p × 4096 × 32", "bench_lamp.json"),
        ("5 lamp, no_sort", "bench_lampnosort.json")]


def line(f):
    with open(os.path.join(D, f)) as fh:
        return json.loads(fh.read().strip().splitlines()[-1])


def pass_kernel_ms(workload):
    try:
        rec = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))[workload]
    except (OSError, KeyError, ValueError):
        return None
    tot = 0.0
    for k in rec["kernels"].values():
        tot += k["counters_per_dispatch"].get("dur_ms", 0.0) * k["dispatches"]
    return tot / max(rec.get("passes_profiled", 1), 1)


def main():
    print("| config | GPUs | render-wall ms | serialised kernel ms / pass | live Mrays/s | nominal Mrays/s | "
          "fabric GB/s (frac of 8 TB/s) | VALU frac | trace occupancy | bit-exact | CPU s (threads) | file |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for name, f in ROWS:
        try:
            d = line(f)
        except OSError:
            continue
        r = d.get("roofline") or {}
        fr = r.get("frame") or {}
        va = r.get("valu") or {}
        cb = d.get("cpu_baseline") or {}
        km = pass_kernel_ms(d["config"]["workload"])
        occ = "8 waves/SIMD (64 VGPRs)" if r else "— (no trace kernel)" if "spheres" in name else "8 waves/SIMD"
        cpu = "%.1f (%d, %s)" % (cb["frame_s"], cb["cores"], "extrapolated" if cb.get("extrapolated") else "full frame") \
            if cb.get("frame_s") is not None else "—"
        print("| %s | 1 | %s | %s | %.0f | %.0f | %s | %s | %s | %s | %s | %s |" % (
            name, d.get("render_wall_ms"), "%.1f" % km if km else "—", d["value"], d["config"]["nominal_mrays_per_s"],
            "%.0f (%.3f)" % (fr["achieved"], fr["frac"]) if fr else "—", "%.3f" % va["frac"] if va else "—", occ,
            d.get("bit_exact_vs_oracle"), cpu, os.path.relpath(os.path.join(D, f), REPO)))
        print("| %s | 2 / 4 / 8 | unmeasured on hardware (no multi-GPU node here; the driver's SCALE run) "
              "| | | | | | | | | |" % name)


if __name__ == "__main__":
    main()
