#!/usr/bin/env python3
"""Benchmark of the MI355X path tracer (BASELINE.json metric: Mrays/s per scene at 1/2/4/8 GPUs).

Workload (default): teapot.scene at 1920x1080, 2048 spp, 16 bounces, sort on (BASELINE.json
configs[3], the config the north star's roofline target is stated on).  A step is one 20-spp
pass of the hot path on every GPU: ray generation, 16 x (BVH traversal + shading + reorder
key, stable reorder), ordered accumulation.  Multi-GPU runs shard whole passes round-robin
over the GPUs (GPU r renders pass r + N*k); the pass framebuffers are exchanged as pixel slices
(one RCCL all-to-all: GPU j owns slice j and adds the slices in pass order, bit-identical to
1 GPU) and the finished slices are gathered to GPU 0.  By default the timed region is one
full frame (strong scaling); `--steps K` times K passes per GPU (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene teapot] [--no-sort]
    torchrun --nproc-per-node N bench.py --gpus N ...

`--gpus N` is honoured however bench.py is started:
  * under torchrun (WORLD_SIZE set): one process per GPU, collectives through torch.distributed
    (RCCL); WORLD_SIZE must equal N, or the run exits with status 2;
  * without it (WORLD_SIZE unset), N > 1: one process drives the N GPUs through the library's own
    multi-GPU renderer (rt_multi: ncclCommInitAll over GPUs 0..N-1, one host thread per GPU, the
    same pass sharding and slice exchange); N above the visible HIP devices exits with status 2.
Every line carries n_gpus = N and config.n_ranks_seen = the ranks the collective backend counted.

Rank 0 prints ONE JSON line.  `value` = live ray segments (process_ray calls on live slots)
per second over all GPUs, inputs resident in HBM.  `render_wall_ms` = one full frame (the
metric's second column); `bit_exact_vs_oracle` = this run's pass-0 framebuffer hashed against
the oracle's (tests/golden/bench_pass0.json).  `roofline` prices the dominant kernel
(trace_kernel) inside the timed step (its wave-residency share of a pass x ms_per_step):
algorithmic HBM bytes and the measured PMC traffic against HBM, with the exclusive-launch
figures, the per-launch table and SURVEY.md §8(d)'s logical cache-inclusive bytes (against the
L2) as labelled secondary fields; `cpu_baseline` times the oracle's restatement of the
reference `cpu` path on the host cores (§8(d): first pass + remainder pass, extrapolated).
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# The renderer keeps up to 20 passes in flight on their own streams; HIP's default of 4 hardware
# queues would make them share queues (20 in flight: 24 queues beat 16 by 1.5 % on teapot, 3.4 %
# on lamp).  With torch.distributed (RCCL) in the process its streams need queues too (16 passes
# and 16 queues cost the 1-GPU --dist run 11 %).  Set before HIP initialises.
def _argv_gpus(argv):
    """--gpus N from the command line before argparse runs (the queue count must be set before HIP starts)."""
    for i, a in enumerate(argv):
        try:
            if a == "--gpus" and i + 1 < len(argv):
                return int(argv[i + 1])
            if a.startswith("--gpus="):
                return int(a.split("=", 1)[1])
        except ValueError:
            return 1
    return 1


_DIST = (int(os.environ.get("WORLD_SIZE", "1")) > 1 or "--dist" in sys.argv or "--inlib" in sys.argv or
         _argv_gpus(sys.argv) > 1)
_HWQ = os.environ.get("RTAMD_HW_QUEUES")            # RTAMD_HW_QUEUES: sweeps only
if _HWQ is not None and not (_HWQ.isdigit() and 1 <= int(_HWQ) <= 32):
    sys.exit("bench.py: RTAMD_HW_QUEUES=%r: expected a queue count in 1..32" % _HWQ)
_QUEUES = int(_HWQ) if _HWQ else (28 if _DIST else 24)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _QUEUES or _HWQ:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_QUEUES)
# Next to RCCL, 16 passes in flight beat 20 (1-GPU --dist: 7.63 vs 7.76 ms/pass for a frame, 8.10
# vs 9.0-12.7 for a 13-pass share); alone, 20 are faster.
if _DIST:
    os.environ.setdefault("RTAMD_INFLIGHT", "16")
sys.path.insert(0, os.path.join(REPO, "cuda-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
if os.environ.get("RTAMD_TORCH_FIRST") == "1" and __name__ == "__main__":
    # diagnostic: torch (and its bundled HIP runtime) loaded first, as in the torch.distributed path
    import torch
    torch.cuda.set_device(0)

import numpy as np  # noqa: E402

import rtamd  # noqa: E402

def hip_runtimes():
    """The HIP runtime and RCCL files mapped into this process (diagnostic: the torch.distributed path runs the
    renderer on torch's bundled runtime, which torch loads first; librtamd loaded first does not make torch use
    /opt/rocm's -- torch's copy has another soname, and the renderer then finds no device)."""
    seen = set()
    try:
        for line in open("/proc/self/maps"):
            f = line.split()[-1]
            if "libamdhip64" in f or "librccl" in f:
                seen.add(f)
    except OSError:
        pass
    return sorted(seen)

CONFIGS = {
    # name: (scene file, W, H, spp, bounces, sort, use_bvh)
    "teapot": ("teapot.scene", 1920, 1080, 2048, 16, True, True),
    "cornell_plus": ("cornell_plus.scene", 512, 512, 256, 8, True, True),
    "spheres": ("spheres.scene", 1024, 1024, 1024, 8, True, False),
    "lamp": ("lamp_available.scene", 1920, 1080, 4096, 32, True, True),
    "cornell": ("cornell.scene", 256, 256, 64, 4, True, True),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
CPU_FULL_FRAME_S = 30.0  # cpu_baseline: frames estimated within this many seconds are timed whole
TILE_ROWS = 8          # pixel-tile stripe height (--shard tiles; SURVEY §8e: interleaved 8-row stripes)


L2_PEAK_GBS = 34500.0  # MI355X aggregate L2 (8 XCDs x 4 MiB), MI355X_MICROARCH.md §L2: ~34.5 TB/s
# wave64 VALU instruction issue: 256 CUs x 4 SIMD-32 x 2.4 GHz / 2 cycles per wave64 instruction
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles"; max clock 2400 MHz)
VALU_PEAK_GWIS = 256 * 4 * 2.4 / 2


def logical_trace_bytes(st, spheres):
    """SURVEY.md §8(d)'s logical (cache-inclusive) bytes of the traversal part of process_ray over
    the counted launches: per live segment the ray (24 B) and S spheres, 32 B per node pop, 64 B
    per internal visit (two child nodes), 48 B per triangle test, 8 B hit written."""
    return (st["live_segments"] * (24 + 16 * spheres + 8) + 32 * st["nodes_popped"] +
            64 * st["internal_visits"] + 48 * st["triangle_tests"])


XCDS = 8   # MI355X: 8 XCDs, each with its own non-coherent 4 MB L2 (MI355X_MICROARCH.md)


def compulsory_trace_bytes(st, scene_bytes, launches, per_xcd=False):
    """Algorithmic HBM bytes of the trace launches: what a launch cannot avoid moving from or to
    HBM.  Each live segment's ray (o, d: 24 B) is read once, except at bounce 0 where the primary
    ray is computed in place (every generated ray is live there); its hit {t, index} (8 B) is
    written once; the scene's node and triangle arrays (reference layouts, 32 B / 48 B / 16 B per
    sphere) are read once per launch, or once per XCD (per_xcd: every XCD's L2 fetches them)."""
    live, gen = st["live_segments"], st["generated_rays"]
    return 24 * (live - gen) + 8 * live + launches * scene_bytes * (XCDS if per_xcd else 1)


def load_pmc(workload):
    """Measured HBM-side traffic for this workload from the committed rocprofv3 PMC summary
    (tools/pmc.sh + tools/pmc_summary.py, one profiled pass)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    d = d.get(workload)
    if d:
        d["file"] = "profiles/pmc_traffic.json"
    return d


def load_issue(workload):
    """Wave-instruction counts of one pass from the committed PMC stall run (profiles/pmc_issue.json,
    tools/pmc.sh ... stall.txt + tools/stall_summary.py --json)."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_issue.json")) as f:
            return json.load(f).get(workload)
    except (OSError, ValueError):
        return None


def load_golden(scene, sort):
    path = os.path.join(REPO, "tests", "golden", "bench_pass0.json")
    try:
        with open(path) as f:
            return json.load(f).get("%s sort=%s" % (scene, "on" if sort else "off"))
    except (OSError, ValueError):
        return None


def run_cpu(exe, cfg, spp, pass_limit, threads):
    scene, w, h, _, bounces = cfg[:5]
    cmd = [exe, os.path.join(rtamd.ASSETS, scene), rtamd.ASSETS, str(w), str(h), str(spp), str(bounces),
           str(pass_limit), str(threads)]
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, env=env).stdout
    return json.loads(out.strip().splitlines()[-1])


def cpu_baseline(cfg, args):
    """Times the oracle's restatement of cpu_raytrace (raytracing.cu:122-163, OpenMP
    schedule(dynamic, 1000) at :136,144, bounce-invariant seed :148; built with the reference's
    -O3 -ffast-math -fopenmp) as SURVEY.md §8(d) specifies: configs of up to 4 passes in full,
    larger ones as the first full 20-spp pass plus the remainder pass, extrapolated linearly to
    the frame (passes cost the same: the remainder pass is the only short one)."""
    exe = os.path.join(REPO, "oracle", "build", "cpu_baseline")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    nproc = os.cpu_count() or 1
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    # The GPU pool sets OMP_NUM_THREADS to the box's CPU share for one GPU (16) and asks jobs to size
    # worker pools to it, although the affinity mask shows the whole host (256): the baseline runs on
    # that share.  Elsewhere (no OMP_NUM_THREADS): every thread of the affinity mask.
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = args.cpu_threads or env_threads or affinity
    scene, w, h, spp, bounces = cfg[:5]
    P = -(-spp // 20)
    full = P <= 4
    if not full:
        first = run_cpu(exe, cfg, spp, 1, threads)                  # pass 0: 20 spp
        # a frame that fits the sample budget is timed whole (cornell_plus: ~4 s on 16 threads)
        full = first["seconds"] * P <= CPU_FULL_FRAME_S
    if full:
        rec = run_cpu(exe, cfg, spp, -1, threads)
        secs, live = rec["seconds"], rec["live_segments"]
        sample = "%s %dx%d %d spp %d bounces, the whole frame (%d passes) timed: %.2f s" % (scene, w, h, spp, bounces,
                                                                                             P, secs)
    else:
        rem = spp - 20 * (P - 1)
        last = run_cpu(exe, cfg, rem, 1, threads)                   # the remainder pass (remaining = 0)
        secs = first["seconds"] * (P - 1) + last["seconds"]
        live = first["live_segments"] * (P - 1) + last["live_segments"]
        sample = ("%s %dx%d %d bounces: 2 of the frame's %d passes timed -- the first full 20-spp pass %.2f s and the "
                  "remainder %d-spp pass %.2f s -- and the frame extrapolated linearly (passes are i.i.d. in cost, "
                  "SURVEY 8(d)): %.1f s" % (scene, w, h, bounces, P, first["seconds"], rem, last["seconds"], secs))
    if env_threads and not args.cpu_threads and env_threads < affinity:
        sample += ("; %d threads, not all %d of the affinity mask: the GPU pool gives a one-GPU job a %d-CPU share "
                   "(it sets OMP_NUM_THREADS=%d and asks jobs to size worker pools to it) although nproc shows the "
                   "whole host" % (threads, affinity, env_threads, env_threads))
    return {
        "value": round(live / secs / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": sample + " (oracle cpu_raytrace restatement, -O3 -ffast-math -fopenmp, %d OpenMP threads)" % threads,
        "frame_s": round(secs, 3),
        "extrapolated": not full,
        "host_nproc": nproc,
        "affinity_threads": affinity,
        "threads_from": "--cpu-threads" if args.cpu_threads else ("OMP_NUM_THREADS (the pool's CPU share per GPU; "
                                                                  "the affinity mask allows %d)" % affinity
                                                                  if env_threads else "the affinity mask"),
    }


def roofline(excl, counted, launches, trace_ms, scene_bytes, spheres, workload, elapsed, steps):
    """The dominant kernel (trace_kernel) against HBM, reproducible from committed files.  Headline (round 6):
    the kernel inside the timed step (timed_regime: its wave-residency share of a pass x ms_per_step, so its
    time never exceeds the step): achieved = one pass's algorithmic trace bytes / that time, traffic = the
    PMC fabric bytes of one pass's trace launches (profiles/pmc_traffic.json) over the same time.  Secondary,
    labelled: `exclusive` (pass 0 alone on the chip, per launch; 16 such launches take longer than a timed
    step, so they describe another regime), `shared` (the timed steps' launch spans, which overlap), the
    per-launch table, the L2 and VALU figures."""
    xc = excl["counted"]
    n_ex = excl["launches"]
    ms_ex = excl["ms_per_launch"]
    comp_ex = compulsory_trace_bytes(xc, scene_bytes, n_ex, per_xcd=True) / n_ex
    logical_ex = logical_trace_bytes(xc, spheres) / n_ex
    achieved_ex = comp_ex / (ms_ex / 1e3) / 1e9
    pmc = load_pmc(workload)
    traffic_ex = pmc["trace_bytes_per_launch"] if pmc else None
    kernel = "trace_kernel (BVH traversal + Moller-Trumbore + slab + sphere loop)"
    exclusive = {
        "achieved": round(achieved_ex, 1), "frac": round(achieved_ex / HBM_PEAK_GBS, 4), "traffic": traffic_ex,
        "bytes_per_launch": int(comp_ex), "ms_per_launch": round(ms_ex, 4), "launches": n_ex,
        "exclusive_pass_kernel_ms": round(excl["kernel_ms"], 3),
        "achieved_def": "secondary, another regime than the timed step: algorithmic HBM bytes per trace launch of "
                        "pass 0 run alone on the chip (24 B ray read per live segment past bounce 0 + 8 B hit write "
                        "per live segment + the scene's node and triangle arrays (reference layouts, 32 / 48 B) "
                        "once per XCD: 8 non-coherent 4 MB L2s each fetch the scene) / its exclusive average launch "
                        "duration (device wall clock, first wave start to last wave end, one pass context, trace "
                        "grid = every resident workgroup, best of 3, measured before the warmup; bench.py "
                        "exclusive_pass)",
        "traffic_def": None if not pmc else
        "measured fabric-side bytes per trace launch, rocprofv3 --pmc over exactly pass 0 with dispatches "
        "serialised (%s; reads priced by request size TCC_EA0_RDREQ_{128B,64B,32B}, = 2 x FETCH_SIZE for 128-B "
        "requests per MI355X_MICROARCH.md §HBM; writes TCC_EA0_WRREQ{,_64B}; Infinity-Cache hits included, "
        "an upper bound on HBM bytes); %s" % (pmc["file"], pmc.get("run", "")),
        "traffic_frac": round(traffic_ex / (ms_ex / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if traffic_ex else None,
        "traffic_over_algorithmic": round(traffic_ex / comp_ex, 3) if traffic_ex else None}
    if pmc and pmc.get("trace_dur_ms_avg"):
        exclusive["pmc_run"] = {"ms_per_launch": round(pmc["trace_dur_ms_avg"], 4),
                                "fabric_gbs": round(pmc["trace_fabric_gbs"], 1),
                                "frac": round(pmc["trace_fabric_gbs"] / HBM_PEAK_GBS, 4),
                                "def": "the PMC run's own numbers: fabric bytes per trace launch / the profiler's "
                                       "average trace dispatch duration (profiles/pmc_traffic.json "
                                       "trace_dur_ms_per_launch)"}
    iss = load_issue(workload)
    # the timed regime's own PMC records (the driver's 20 concurrent passes) where they exist; one pass's otherwise
    iss_t, pmc_t = load_issue(workload + TIMED_PMC), load_pmc(workload + TIMED_PMC)
    if iss_t and steps >= 2:
        timed = timed_regime(iss_t, pmc_t or pmc, counted, launches, scene_bytes, elapsed, steps, one_pass=iss)
    else:
        timed = timed_regime(iss, pmc, counted, launches, scene_bytes, elapsed, steps)
    if timed:
        roof = {"bound": "hbm", "achieved": timed["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": timed["frac"], "traffic": timed.get("measured_bytes_per_step"),
                "traffic_frac": timed.get("measured_frac"), "regime": "timed step",
                "kernel": kernel + ", inside the timed step",
                "bytes_per_step": timed["algorithmic_bytes_per_step"], "kernel_ms_per_step": timed["ms_per_step"],
                "traffic_unit": "bytes per step (one pass's trace launches, rocprofv3 --pmc, %s)" % timed["regime"],
                "achieved_def": "one pass's algorithmic trace bytes (24 B ray read per live segment past bounce 0 + "
                                "8 B hit write per live segment + the scene once per XCD per launch) / the trace "
                                "kernel's time per step (its SQ_WAVE_CYCLES share of the timed regime's wave "
                                "residency x ms_per_step, roofline.timed); traffic = the PMC fabric bytes of a "
                                "pass's trace launches in that regime over the same time (traffic_frac)"}
    else:
        roof = {"bound": "hbm", "achieved": exclusive["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": exclusive["frac"], "traffic": traffic_ex, "traffic_frac": exclusive["traffic_frac"],
                "regime": "exclusive launch (no committed PMC issue record for this workload)",
                "kernel": kernel + ", per exclusive launch", "bytes_per_launch": int(comp_ex),
                "ms_per_launch": round(ms_ex, 4), "achieved_def": exclusive["achieved_def"]}
    roof["exclusive"] = exclusive
    comp_sh = compulsory_trace_bytes(counted, scene_bytes, launches, per_xcd=True) / launches
    roof["shared"] = {"ms_per_launch": round(trace_ms, 4), "launches": launches,
                      "achieved": round(comp_sh / (trace_ms / 1e3) / 1e9, 1),
                      "frac": round(comp_sh / (trace_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                      "def": "secondary: the timed steps' trace launches, re-run untimed with event timing; up to 20 "
                             "passes share the chip, so a launch's span includes time it shared (what rocprofv3's "
                             "kernel trace of the bench command reports as the average trace duration)"}
    roof["l2"] = {"achieved": round(logical_ex / (ms_ex / 1e3) / 1e9, 1), "peak": L2_PEAK_GBS, "unit": "GB/s",
                  "frac": round(logical_ex / (ms_ex / 1e3) / 1e9 / L2_PEAK_GBS, 4), "bytes_per_launch": int(logical_ex),
                  "def": "SURVEY.md 8(d) logical cache-inclusive bytes of the traversal (24 B ray + 16 B x S + 32 B x "
                         "node pops + 64 B x internal visits + 48 B x triangle tests + 8 B hit) per exclusive launch / "
                         "its duration, against the aggregate L2 rate (MI355X_MICROARCH.md §L2)"}
    if steps and elapsed > 0:
        ms_pass = elapsed / steps * 1e3
        lg = logical_trace_bytes(counted, spheres) / max(steps, 1)
        roof["logical_per_step"] = {"bytes_per_step": int(lg), "ms_per_step": round(ms_pass, 3),
                                    "achieved": round(lg / (ms_pass / 1e3) / 1e9, 1),
                                    "def": "cross-check, cache-inclusive (NOT HBM): SURVEY.md 8(d) logical traversal "
                                           "bytes per pass / ms_per_step; above the HBM peak because traversal reuse "
                                           "is served by the L1/L2/Infinity Cache"}
    if pmc and pmc.get("pass_bytes") and steps:
        ms_pass = elapsed / max(steps, 1) * 1e3
        roof["frame"] = {"hbm_bytes_per_pass": pmc["pass_bytes"], "ms_per_pass": round(ms_pass, 3),
                         "achieved": round(pmc["pass_bytes"] / (ms_pass / 1e3) / 1e9, 1),
                         "frac": round(pmc["pass_bytes"] / (ms_pass / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "def": "measured fabric-side bytes of one pass (every kernel, same PMC run) / timed "
                                "wall per pass (one GPU's passes overlap 20 at a time)"}
    table = per_launch_table(excl, scene_bytes, pmc)
    if table:
        roof.update(table)
    if timed:
        roof["timed"] = timed
    if iss and steps:
        ms_pass = elapsed / steps * 1e3
        v_all, v_tr = iss["per_pass"]["SQ_INSTS_VALU"], iss["trace_per_pass"]["SQ_INSTS_VALU"]
        rate = v_all / (ms_pass / 1e3) / 1e9
        roof["valu"] = {"wave_instructions_per_pass": int(v_all), "trace_share": round(v_tr / v_all, 3),
                        "achieved": round(rate, 1), "peak": VALU_PEAK_GWIS, "unit": "G wave64 VALU instr/s",
                        "frac": round(rate / VALU_PEAK_GWIS, 4),
                        "def": "VALU wave-instructions of one pass, every kernel (rocprofv3 --pmc SQ_INSTS_VALU, "
                               "profiles/pmc_issue.json: %s) / timed wall per pass, against the chip's issue "
                               "rate (1024 SIMD-32 x 2.4 GHz / 2 cycles)" % iss.get("run", "")}
    return roof


TIMED_PMC = " | timed 20 passes"     # profiles/pmc_*.json key suffix: PMC runs of the driver's 20 concurrent passes


def timed_regime(iss, pmc, counted, launches, scene_bytes, elapsed, steps, one_pass=None):
    """The dominant kernel inside the timed step (up to 20 passes sharing the chip): its time per step is
    taken as its share of one pass's wave residency (rocprofv3 --pmc SQ_WAVE_CYCLES of the trace launches
    over every kernel's, profiles/pmc_issue.json) times ms_per_step, so it never exceeds the step; over
    that time, one pass's algorithmic trace bytes, its measured fabric bytes (profiles/pmc_traffic.json)
    and its VALU wave-instructions, against the HBM peak and the chip's VALU issue rate."""
    if not (iss and steps and elapsed > 0 and launches and counted):
        return None
    wc_all = iss.get("per_pass", {}).get("SQ_WAVE_CYCLES")
    wc_tr = iss.get("trace_per_pass", {}).get("SQ_WAVE_CYCLES")
    if not (wc_all and wc_tr):
        return None
    share = wc_tr / wc_all
    ms_pass = elapsed / steps * 1e3
    t = share * ms_pass / 1e3                       # s of trace per step
    alg = compulsory_trace_bytes(counted, scene_bytes, launches, per_xcd=True) / steps
    concurrent = iss.get("passes_profiled", 1) > 1
    out = {"wave_cycle_share": round(share, 4), "ms_per_step": round(share * ms_pass, 4),
           "step_ms": round(ms_pass, 3),
           "regime": ("the driver's %d concurrent passes" % iss["passes_profiled"]) if concurrent else "one pass alone",
           "algorithmic_bytes_per_step": int(alg), "achieved": round(alg / t / 1e9, 1),
           "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4)}
    if pmc and pmc.get("trace_bytes_per_launch") and pmc.get("passes_profiled"):
        meas = pmc["trace_bytes_per_launch"] * pmc["trace_launches"] / pmc["passes_profiled"]
        out.update({"measured_bytes_per_step": int(meas), "measured_achieved": round(meas / t / 1e9, 1),
                    "measured_frac": round(meas / t / 1e9 / HBM_PEAK_GBS, 4)})
    v_tr = iss.get("trace_per_pass", {}).get("SQ_INSTS_VALU")
    if v_tr:
        out["valu_frac"] = round(v_tr / t / 1e9 / VALU_PEAK_GWIS, 4)
    if one_pass and one_pass.get("per_pass", {}).get("SQ_WAVE_CYCLES") and \
            one_pass.get("trace_per_pass", {}).get("SQ_WAVE_CYCLES"):
        s1 = one_pass["trace_per_pass"]["SQ_WAVE_CYCLES"] / one_pass["per_pass"]["SQ_WAVE_CYCLES"]
        out["one_pass"] = {"wave_cycle_share": round(s1, 4), "ms_per_step": round(s1 * ms_pass, 4),
                           "frac": round(alg / (s1 * ms_pass / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                           "def": "the same with the share of ONE pass profiled alone (profiles/pmc_issue.json: %s)"
                                  % one_pass.get("run", "")}
    out["def"] = ("trace_kernel within the timed step: its share of the wave residency (SQ_WAVE_CYCLES of the "
                  "trace launches / every kernel's) in %s (profiles/pmc_issue.json: %s) x ms_per_step = its time "
                  "per step (<= ms_per_step); frac = one pass's algorithmic trace bytes (as achieved_def) / that "
                  "time / HBM peak; measured_frac = the PMC fabric bytes of a pass's trace launches in the same "
                  "regime (profiles/pmc_traffic.json) / that time / HBM peak; valu_frac = a pass's trace VALU "
                  "wave-instructions / that time / the chip's VALU issue rate" % (out["regime"], iss.get("run", "")))
    return out


def per_launch_table(excl, scene_bytes, pmc):
    """The exclusive pass's trace launches one by one (bounce b = launch b): device-clock duration,
    live rays, algorithmic HBM bytes (24 B ray read past bounce 0 + 8 B hit write per live ray + the
    scene once per XCD) and their fraction of the HBM peak, with the measured fabric bytes of the
    same launch from the PMC run when it recorded them per launch.  The heavy launches (bounces 0-1,
    >90 % of the rays) and the latency-bound tail are summarised apart."""
    prof = excl.get("launch_profile") if excl else None
    if not prof:
        return None
    meas = (pmc or {}).get("trace_bytes_by_launch")
    meas_ms = (pmc or {}).get("trace_dur_ms_per_launch")
    rows = []
    for b, (ms, live) in enumerate(prof):
        alg = (24 if b else 0) * live + 8 * live + XCDS * scene_bytes
        row = {"bounce": b, "ms": round(ms, 4), "live": int(live), "algorithmic_bytes": int(alg),
               "frac": round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if ms > 0 else None}
        if meas and b < len(meas):
            row["measured_bytes"] = int(meas[b])
            if meas_ms and b < len(meas_ms) and meas_ms[b] > 0:
                row["measured_frac"] = round(meas[b] / (meas_ms[b] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
        rows.append(row)

    def group(sel, name):
        r = [x for x in rows if sel(x["bounce"])]
        if not r:
            return None
        ms = sum(x["ms"] for x in r)
        alg = sum(x["algorithmic_bytes"] for x in r)
        g = {"launches": len(r), "ms": round(ms, 4), "live": sum(x["live"] for x in r), "algorithmic_bytes": alg,
             "frac": round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if ms > 0 else None, "def": name}
        if all("measured_bytes" in x for x in r):
            g["measured_bytes"] = sum(x["measured_bytes"] for x in r)
        return g
    return {"per_launch": rows,
            "heavy": group(lambda b: b <= 1, "bounces 0-1: every primary ray and the first bounce's survivors"),
            "tail": group(lambda b: b >= 2, "bounces >= 2: latency-bound, the longest ray's chain of fetches")}


class RtamdBackend:
    """The product path: librtamd.so renderers (HIP kernels through the C ABI) on this process's GPU,
    collectives through torch.distributed over RCCL (backend "nccl") when the run is distributed."""

    def __init__(self, use_dist):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = self.torch = self.device = None
        self.use_dist = use_dist
        if use_dist:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            import torch
            import torch.distributed as dist
            torch.cuda.set_device(self.local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            self.dist, self.torch, self.device = dist, torch, torch.device("cuda", self.local)
        self.probe = None

    def scene(self, scene_file, use_bvh, image):
        return rtamd.Scene(os.path.join(rtamd.ASSETS, scene_file), use_bvh=use_bvh, image=image)

    def renderer(self, scene, sort, tiles):
        return rtamd.Renderer(scene, sort=sort, device=self.local, tiles=tiles)

    def attach_tile_exchange(self, ren, emulated):
        """Pixel tiles with the reorder on: one byte per global live ray per bounce, summed
        over the owners on the device.  N > 1 ranks: the renderer joins an RCCL communicator of its own
        (rt_renderer_set_exchange_rccl; rank 0's id is broadcast over torch.distributed) and all-reduces
        the bytes in place on each pass's stream.  The 1-GPU --tile-share probe has no other owners:
        tests/native/xchg.hip emulates their slots on the device (live with the own rays' live fraction,
        else terminated), so rank 0 ranks its rays in a global order of a realistic size; its seeds (and
        image) are not a real N-GPU run's, so no parity is claimed."""
        if not emulated:
            import rtamd_dist
            rtamd_dist.join_tile_exchange(self.dist, ren, rtamd)
        else:
            import xchg_lib
            self.probe = xchg_lib.EmulatedPeers()
            self.probe.attach(ren)

    def exclusive_pass(self, scene, sort):
        """Pass 0 alone on the chip (untimed): a renderer with one pass context (RTAMD_INFLIGHT=1, so its
        trace grid is every resident workgroup), per-launch device wall-clock spans of its trace launches
        (rt_stats.trace_ms / trace_launches, event timing on; rt_renderer_launch_profile per launch),
        then the same pass with the work counters.  This is the exclusive launch duration the dominant
        kernel's roofline is priced on, the same serialised situation as the rocprofv3 --pmc pass
        (tools/pmc.sh: one pass, dispatches serialised by the profiler)."""
        old = os.environ.get("RTAMD_INFLIGHT")
        os.environ["RTAMD_INFLIGHT"] = "1"
        try:
            r1 = rtamd.Renderer(scene, sort=sort, device=self.local)
        finally:
            if old is None:
                del os.environ["RTAMD_INFLIGHT"]
            else:
                os.environ["RTAMD_INFLIGHT"] = old
        try:
            r1.set_event_timing(True)
            r1.run(0, 1)                        # warm
            runs = []
            for _ in range(3):
                st = r1.run(0, 1)
                runs.append((st, r1.launch_profile()))
            best, prof = min(runs, key=lambda x: x[0]["trace_ms"])
            r1.set_counters(True)
            counted = r1.run(0, 1)
            r1.set_counters(False)
        finally:
            r1.close()
        n = best["trace_launches"]
        return {"trace_ms": best["trace_ms"], "launches": n, "ms_per_launch": best["trace_ms"] / n if n else 0.0,
                "kernel_ms": best["kernel_ms"], "launch_profile": prof,
                "counted": {k: int(v) for k, v in counted.items() if isinstance(v, int)}}

    def render_pass0(self, scene, sort):
        fb0, _ = rtamd.render(scene, sort=sort, device=self.local, pass_begin=0, pass_count=1)
        return fb0

    def async_render(self, ren, on_stats):
        """The renderer's asynchronous form for rtamd_dist.PassShardedFrame: the slices of finished passes
        are exchanged while later passes render (RTAMD_XCHG_OVERLAP=0: one exchange after the batch)."""
        if os.environ.get("RTAMD_XCHG_OVERLAP", "1") == "0":
            return None
        torch = self.torch

        class AsyncPasses:
            def start(self, passes, out):
                stride = passes[1] - passes[0] if len(passes) > 1 else 1
                ren.run_async(passes[0], len(passes), stride, out.data_ptr())

            def wait(self, j):
                ren.wait_pass(j, torch.cuda.current_stream().cuda_stream)

            def finish(self):
                on_stats(ren.finish())
        return AsyncPasses()

    def barrier_sync(self):
        if self.use_dist:
            self.dist.barrier()
            self.torch.cuda.synchronize()

    def close(self):
        if self.probe:
            self.probe.close()
        if self.use_dist:
            self.dist.barrier()
            self.dist.destroy_process_group()


class InLibBackend(RtamdBackend):
    """--gpus N without torchrun: one process drives N GPUs through the library's own multi-GPU renderer
    (rt_multi: one RCCL communicator from ncclCommInitAll, one host thread and renderer per GPU, the pass
    sharding and overlapped slice exchange of rt_render's device_count path).  The frame is
    gathered on GPU 0; the stats are summed over the GPUs.  With the test build (RTAMD_LIB =
    librtamd_test.so) and RTAMD_MULTI_LOOPBACK=1 the N "GPUs" are the box's one GPU (tests only)."""
    inlib = True

    def __init__(self, n):
        self.world, self.rank, self.local = n, 0, 0
        self.dist = self.torch = self.device = None
        self.use_dist = False
        self.probe = None
        loopback = os.environ.get("RTAMD_MULTI_LOOPBACK") == "1" and rtamd.LIB_PATH == rtamd.TEST_LIB_PATH
        visible = rtamd.device_count()
        if not loopback and n > visible:
            raise SystemExit2("bench.py: --gpus %d but %d HIP device(s) visible" % (n, visible))
        self.devices = [0] * n if loopback else list(range(n))
        self.loopback = loopback

    def renderer(self, scene, sort, tiles):
        if tiles:
            raise SystemExit2("bench.py: --shard tiles / --tile-share need one process per GPU (torchrun)")
        return rtamd.MultiRenderer(scene, self.devices, sort=sort)


class SystemExit2(SystemExit):
    """A usage error that ends the run with exit status 2 (message on stderr)."""

    def __init__(self, msg):
        print(msg, file=sys.stderr)
        super().__init__(2)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (default: WORLD_SIZE under torchrun, else 1); without torchrun N > 1 runs the "
                         "library's in-process multi-GPU renderer")
    ap.add_argument("--steps", type=int, default=None,
                    help="passes per GPU to time (default: one full frame, ceil(passes/N) per GPU)")
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--scene", default="teapot", choices=sorted(CONFIGS))
    ap.add_argument("--no-sort", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-counters", action="store_true", help="skip the byte-model counting rerun")
    ap.add_argument("--no-extras", action="store_true",
                    help="only the warmup and timed steps (profiling: --steps 1 --warmup 0 renders exactly one pass)")
    ap.add_argument("--dist", action="store_true", help="use the torch.distributed path even at N=1")
    ap.add_argument("--inlib", action="store_true",
                    help="use the library's in-process multi-GPU renderer (rt_multi) even at N=1 (without torchrun)")
    ap.add_argument("--shard", choices=("passes", "tiles"), default="passes",
                    help="multi-GPU decomposition: whole passes per GPU or 8-row pixel stripes per GPU over "
                         "every pass (sort on: one byte per live ray all-reduced after every bounce); both exact")
    ap.add_argument("--tile-share", type=int, default=0, metavar="N",
                    help="1-GPU probe of --shard tiles: render only rank 0's stripes of an N-GPU split")
    args = ap.parse_args(argv)
    if args.no_extras:
        args.no_counters = args.no_cpu_baseline = True
    return args


def run(args, backend, cfg=None, json_out=None, golden=None):
    """The benchmark's orchestration, over any backend that renders passes and runs collectives
    (RtamdBackend: the HIP renderer and RCCL; tests/test_bench_orchestration.py: the oracle's pass
    sums over gloo).  Rank 0 writes the JSON line to json_out and gets it back with the timed
    region's framebuffer (the assembled frame of the distributed path); other ranks get None."""
    world, rank = backend.world, backend.rank
    dist, torch = backend.dist, backend.torch
    use_dist = dist is not None
    inlib = getattr(backend, "inlib", False)     # one process, N GPUs through rt_multi
    name = args.scene
    cfg = cfg or CONFIGS[name]
    scene_file, W, H, spp, bounces, sort, use_bvh = cfg
    if args.no_sort:
        sort = False
    tiles = args.shard == "tiles" or args.tile_share > 1
    # Weak scaling (--steps K over N ranks, pass sharding): every GPU renders K whole passes.  When the
    # frame has fewer than N*K passes, it is extended to N*K passes (spp = 20*N*K, every pass a full
    # 20-spp pass as before; only the per-pass `remaining` seeds differ), so each GPU renders its K
    # passes in one batch instead of wrapping round to the frame's first pass and paying the
    # pipeline ramp twice.
    frame_spp = spp
    if args.steps is not None and not tiles and -(-spp // 20) < world * args.steps:
        frame_spp = 20 * world * args.steps
    t_load = time.perf_counter()
    scene = backend.scene(scene_file, use_bvh, (W, H, frame_spp, bounces))
    load_s = time.perf_counter() - t_load
    P = scene.passes
    tile_split = (args.tile_share, 0) if args.tile_share > 1 else (world, rank)
    ren = backend.renderer(scene, sort, tile_split + (TILE_ROWS,) if tiles else None)
    if tiles and sort and tile_split[0] > 1:
        backend.attach_tile_exchange(ren, emulated=not (use_dist and world > 1))

    px3 = W * H * 3
    frame = None
    stats_acc = {}

    def accumulate_stats(st):
        for k, v in st.items():
            if isinstance(v, (int, float)):
                stats_acc[k] = stats_acc.get(k, 0) + v

    def render_passes(passes, out):
        # passes are r, r+N, r+2N, ...: one renderer call keeps several of them in flight
        stride = passes[1] - passes[0] if len(passes) > 1 else 1
        accumulate_stats(ren.run(pass_begin=passes[0], count=len(passes), stride=stride,
                                 d_pass_sums=out.data_ptr()))

    # rounds (one pass per GPU each) per frame; pixel tiles: every GPU renders every pass
    R = P if tiles else -(-P // world)
    full_frame = args.steps is None
    steps = R if full_frame else args.steps
    if use_dist:
        import rtamd_dist
        if tiles:
            frame = rtamd_dist.TileShardedFrame(dist, torch, W, H, backend.device,
                                                lambda out: ren.copy_framebuffer(out.data_ptr()), rows=TILE_ROWS)
        else:
            # the owners add the pass slices themselves: the renderer's own framebuffer add chain (each
            # pass's add waits for the previous pass's, across streams) is turned off
            if hasattr(ren, "set_accumulate"):
                ren.set_accumulate(False)
            async_render = backend.async_render(ren, accumulate_stats) if hasattr(backend, "async_render") else None
            frame = rtamd_dist.PassShardedFrame(dist, torch, px3, P, backend.device, render_passes,
                                                async_render=async_render)

    def run_steps(k, stats):
        """k steps from the first pass of the frame, wrapping at its end; one pass per GPU per
        step (rank r renders passes r, r+N, ...).  Returns the passes this rank rendered."""
        stats_acc.clear()
        done = mine = 0
        while done < k:
            m = min(k - done, R)
            if tiles:
                # every pass over this GPU's row stripes, then one RCCL gather of the owned rows
                # to rank 0 (rtamd_dist.TileShardedFrame)
                ren.clear()
                accumulate_stats(ren.run(pass_begin=0, count=m, stride=1))
                if use_dist:
                    frame.run_all()
                mine += m
            elif use_dist:
                # this rank's passes of those rounds in one renderer call, then one RCCL all-to-all
                # of pixel slices to their owners, which add them in pass order, and a gather of the
                # finished slices to rank 0 (rtamd_dist.PassShardedFrame)
                frame.reset()
                mine += frame.run_rounds(0, m)
                frame.collect()
            elif inlib:
                # the first m rounds of the frame over the N GPUs in one library call (rt_multi_run: pass
                # p on GPU p mod N, the slice exchange overlapped, the frame gathered on GPU 0)
                n = min(P, world * m)
                accumulate_stats(ren.run(pass_count=n))
                mine += n
            else:
                accumulate_stats(ren.run(pass_begin=0, count=m, stride=1))
                mine += m
            done += m
        for key, v in stats_acc.items():
            stats[key] = stats.get(key, 0) + v
        return mine

    def reduce(vals, op="sum"):
        """Sum (or max) of per-rank floats over the ranks (every rank calls it)."""
        if not use_dist:
            return list(vals)
        t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=backend.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return [float(x) for x in t.tolist()]

    # No per-bounce HIP events in the timed steps (five marker packets per bounce in every pass's
    # stream cost ~2 %); the per-launch kernel times come from an untimed re-run below.
    ren.set_event_timing(False)
    # the dominant kernel's exclusive launch durations (roofline), before the warmup: measured in the
    # same state as the one-pass PMC run they are compared with, not after minutes of full load
    excl = None
    if not args.no_extras and not args.no_counters and not tiles and rank == 0:
        excl = backend.exclusive_pass(scene, sort)
    warm = {}
    run_steps(args.warmup, warm)
    backend.barrier_sync()
    single = not use_dist and not inlib and not tiles
    if single and full_frame:
        ren.clear()                     # the renderer's framebuffer then holds exactly the timed frame
    timed = {}
    t0 = time.perf_counter()
    my_passes = run_steps(steps, timed)
    backend.barrier_sync()
    elapsed = time.perf_counter() - t0
    timed_fb = None
    if use_dist and rank == 0 and frame.fb is not None:
        timed_fb = frame.fb.detach().to("cpu").numpy().copy()
    elif (inlib or single) and full_frame and rank == 0:
        timed_fb = ren.framebuffer()

    # ---- untimed legs (every rank takes part: they contain collectives)
    evrun, counted, frame_s, parity = {}, None, None, None
    if not args.no_extras:
        # per-launch kernel times: the same steps again with per-bounce HIP events on each pass's stream
        ren.set_event_timing(True)
        run_steps(steps, evrun)
        ren.set_event_timing(False)
        if not args.no_counters and steps > 0:
            # byte model: the same steps with the counting kernel variant
            ren.set_counters(True)
            counted = {}
            run_steps(steps, counted)
            counted = {k: int(v) for k, v in counted.items() if isinstance(v, int)}
            ren.set_counters(False)
        if full_frame:
            frame_s = elapsed
        else:
            # the metric's render-wall column is a full frame: time one (untimed for `value`); with the
            # weak-scaling extension, the configured frame's number of rounds of the extended one
            backend.barrier_sync()
            f0 = time.perf_counter()
            run_steps(R if frame_spp == spp else -(-(-(-spp // 20)) // world), {})
            backend.barrier_sync()
            frame_s = time.perf_counter() - f0
        if not tiles and rank == 0:
            # parity: pass 0 of this workload, hashed against the oracle's (tests/golden/bench_pass0.json)
            # (a one-shot rt_render of pass 0 of the configured frame: its generate seed depends on the
            # frame's spp, which the weak-scaling extension above may have raised)
            import hashlib
            pscene = scene if frame_spp == spp else backend.scene(scene_file, use_bvh, (W, H, spp, bounces))
            fb0 = backend.render_pass0(pscene, sort)
            digest = hashlib.sha256(np.asarray(fb0, dtype="<f4").tobytes()).hexdigest()
            gold = golden if golden is not None else load_golden(name, sort)
            parity = {"bit_exact_vs_oracle": (digest == gold["sha256"]) if gold else None,
                      "sha256_pass0": digest,
                      "oracle": "tests/golden/bench_pass0.json (CPU oracle, tests/golden/make_bench_hashes.py)"
                      if gold else "no golden hash for this workload",
                      **frame_parity(timed_fb, name, sort, (W, H, spp, bounces) if full_frame and frame_spp == spp
                                     else None),
                      "reference_rms": "parity unpinned: the reference's GPU path cannot run here (SURVEY.md §8c), "
                                       "the oracle is a cited restatement; image error vs the reference is not "
                                       "measured (DESIGN.md: the fast-math floor)"}
    elapsed, frame_s_max = reduce([elapsed, frame_s or 0.0], "max")
    # ranks that took part, as the collective backend counts them (a SCALE run can be checked for
    # RCCL seeing N ranks): an all-reduce of 1 per rank (in-library: per GPU, done by rt_multi_create)
    n_ranks_seen = ren.ranks if inlib else int(reduce([1.0])[0])
    live, gen = reduce([timed.get("live_segments", 0), timed.get("generated_rays", 0)])

    out = None
    if rank == 0:
        workload = "%s %dx%d %dspp %d bounces sort=%s" % (scene_file, W, H, spp, bounces, "on" if sort else "off")
        v = scene.view
        scene_bytes = 32 * v.bvh_node_count + 48 * v.triangle_count + 16 * v.sphere_count
        launches = int(evrun.get("trace_launches", 0))
        trace_ms = evrun.get("trace_ms", 0.0) / launches if launches else 0.0
        roof = None
        if counted and launches and trace_ms > 0 and excl:
            pg_counted, pg_launches = counted, launches
            if inlib and world > 1:
                # the counters and launches are summed over the N GPUs: one GPU's share per step (passes cost
                # the same), as the per-process path reports rank 0's own
                pg_counted = {k: v // world for k, v in counted.items()}
                pg_launches = max(1, launches // world)
            roof = roofline(excl, pg_counted, pg_launches, trace_ms, scene_bytes, v.sphere_count, workload, elapsed,
                            steps)
        value = live / elapsed / 1e6 if elapsed > 0 else 0.0
        nominal = gen * bounces / elapsed / 1e6 if elapsed > 0 else 0.0
        ms_step = elapsed / steps * 1e3 if steps else 0.0
        out = {
            "metric": "Mrays/s (live ray segments/s, %s)" % name,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if full_frame or tiles else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: reference scene + assets, procedural stand-in env map (assets missing upstream)",
            "render_wall_ms": round(frame_s_max * 1e3, 1) if frame_s_max else None,
            "bit_exact_vs_oracle": parity["bit_exact_vs_oracle"] if parity else None,
            "config": {
                "workload": workload,
                "step": ("one 20-spp pass (%d rays x %d bounces) over this GPU's %d-row pixel stripes; "
                         "every GPU renders every pass" % (20 * W * H, bounces, TILE_ROWS)) if tiles else
                        ("one 20-spp pass (%d rays x %d bounces) per GPU; pass-sharded over GPUs" % (20 * W * H, bounces)),
                "timed": ("one full frame (%d passes)" % P) if full_frame else ("%d passes per GPU" % steps),
                "parallelism": ("pixel-tile x%d (%d-row stripes) + RCCL gather" % (world, TILE_ROWS) if tiles else
                                "pass-shard x%d + RCCL all-to-all/gather" % world) if world > 1 else "single GPU",
                "launch": ("one process, %d GPUs through the library's rt_multi (ncclCommInitAll)%s"
                           % (world, ", loopback test transport on one GPU" if getattr(backend, "loopback", False)
                              else "")) if inlib else ("one process per GPU (torch.distributed over RCCL)"
                                                       if use_dist else "one process"),
                "nominal_mrays_per_s": round(nominal, 2),
                "render_wall_def": "one full frame (%d passes), first pass to the accumulated framebuffer on the "
                                   "GPU, inputs resident (%s)" % (-(-spp // 20), "the timed region" if full_frame else
                                                                  "an untimed full-frame leg after the timed steps" +
                                                                  ("; its rounds of full 20-spp passes of the extended "
                                                                   "frame" if frame_spp != spp else "")),
                "passes_per_frame": P,
                "n_ranks_seen": n_ranks_seen,
                "hip_runtime": hip_runtimes(),
                "passes_in_flight": passes_in_flight(inlib),
                **({"frame_extended": "%d spp (%d passes) instead of %d, so that each of the %d GPUs renders its %d "
                                      "passes in one batch" % (frame_spp, P, spp, world, steps)}
                   if frame_spp != spp else {}),
                # launch spans of the event-timed re-run, summed over this rank's passes: up to 20 passes
                # run concurrently, so these sums exceed ms_per_step (they are not a per-step kernel time;
                # the exclusive per-pass kernel time is exclusive_pass_kernel_ms)
                "summed_concurrent_spans_per_pass": {
                    "process_ms": round(evrun.get("process_ms", 0.0) / max(my_passes, 1), 3),
                    "trace_ms": round(evrun.get("trace_ms", 0.0) / max(my_passes, 1), 3),
                    "sort_ms": round(evrun.get("sort_ms", 0.0) / max(my_passes, 1), 3),
                    "def": "HIP-event spans of every launch of a pass, summed, per pass; up to 20 passes share the "
                           "chip at once, so the sum exceeds ms_per_step (not a kernel time per step)"},
                **({"exclusive_pass_kernel_ms": round(excl["kernel_ms"], 3),
                    "exclusive_pass_def": "pass 0 alone on the chip (one pass context): every kernel of the pass, "
                                          "HIP events around the pass loop"} if excl else {}),
                "scene_load_s": round(load_s, 3),
                "bvh_ms": round(scene.bvh_ms, 1),
                **({"tile_share_probe": "rank 0's %d-row stripes of a %d-GPU split, on one GPU"
                    % (TILE_ROWS, args.tile_share) + (" (sort on: the other owners' global slots emulated on the "
                                                      "device by tests/native/xchg.hip, live with the own rays' "
                                                      "live fraction else terminated; an approximation of the "
                                                      "N-GPU share's work, not its image)" if sort else "")}
                   if args.tile_share > 1 else {}),
            },
            "parity": parity,
            "roofline": roof,
            "cpu_baseline": None,
        }
        if counted:
            out["config"]["counters"] = {k: counted[k] for k in ("live_segments", "nodes_popped", "internal_visits",
                                                                 "triangle_tests", "hits", "misses", "dead_slots")}
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(cfg, args)
            except Exception as e:  # reported, never fatal for the GPU numbers
                out["cpu_baseline"] = {"error": str(e)}
        if json_out is not None:
            print(json.dumps(out), file=json_out, flush=True)
    ren.close()
    return {"line": out, "timed_fb": timed_fb, "my_passes": my_passes, "frame_passes": P} if rank == 0 else None


def passes_in_flight(inlib):
    """The passes a renderer keeps in flight (per GPU): 20, 16 inside rt_multi, at most RTAMD_INFLIGHT (bench.py sets
    16 next to RCCL) and at most GPU_MAX_HW_QUEUES (rt_render.hip queues_granted)."""
    cap = 16 if inlib else 20
    e = os.environ.get("RTAMD_INFLIGHT")
    if e and e.isdigit():
        cap = min(cap, max(1, int(e)))
    q = os.environ.get("GPU_MAX_HW_QUEUES", "")
    return {"cap": min(cap, int(q) if q.isdigit() and int(q) > 0 else 4), "hw_queues": q or None}


def frame_parity(fb, name, sort, image):
    """The timed region's whole frame (when it is the configured frame) hashed against the oracle's
    (tests/golden/bench_frames.json: cornell, cornell_plus, spheres, teapot in both sort modes)."""
    if fb is None or image is None:
        return {}
    try:
        with open(os.path.join(REPO, "tests", "golden", "bench_frames.json")) as f:
            gold = json.load(f).get("%s frame sort=%s" % (name, "on" if sort else "off"))
    except (OSError, ValueError):
        gold = None
    if not gold or list(gold["image"]) != list(image):
        return {}
    import hashlib
    digest = hashlib.sha256(np.asarray(fb, dtype="<f4").tobytes()).hexdigest()
    return {"frame_bit_exact_vs_oracle": digest == gold["sha256"], "sha256_frame": digest,
            "frame_oracle": "tests/golden/bench_frames.json (the timed frame, assembled over the GPUs)"}


def make_backend(args):
    """The backend `--gpus N` asks for (see the module docstring); exits with status 2 on a mismatch."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        world = int(ws)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit2("bench.py: --gpus %d but WORLD_SIZE=%d (torchrun --nproc-per-node must equal --gpus)"
                              % (args.gpus, world))
        return RtamdBackend(use_dist=world > 1 or args.dist)
    n = args.gpus if args.gpus is not None else 1
    if n < 1:
        raise SystemExit2("bench.py: --gpus must be at least 1")
    if args.dist and args.inlib:
        raise SystemExit2("bench.py: --dist and --inlib are exclusive")
    if n > 1 or args.inlib:
        if args.dist:
            raise SystemExit2("bench.py: --dist with --gpus > 1 needs torchrun (one process per GPU)")
        return InLibBackend(n)
    return RtamdBackend(use_dist=args.dist)


def main():
    args = parse_args()
    # The JSON line is the only thing on stdout: native libraries (RCCL prints a version banner)
    # write to stdout too, so fd 1 is pointed at stderr and the line goes to a saved copy of it.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    backend = make_backend(args)
    import make_envmap
    make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
    run(args, backend, json_out=json_out)
    backend.close()


if __name__ == "__main__":
    main()
